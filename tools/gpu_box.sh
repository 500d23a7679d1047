#!/bin/bash
# box-row layout check: smoke, the structured-kernel parity tests without the duals test, a short
# bench; then (only if all passed) the duals test on its own.
set -o pipefail
OUT=gpurun_out/box2
mkdir -p $OUT
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_ocp.py tests/test_gpu_fp32.py -q -x -k "not duals and not restatement" --timeout 120 --timeout-method thread > $OUT/pytest_a.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu > $OUT/bench.log 2>&1 && \
timeout -k 10 120 python -u -m pytest tests/test_gpu_ocp.py -q -x -k "duals" --timeout 60 --timeout-method thread > $OUT/pytest_b.log 2>&1
rc=$?
for f in smoke pytest_a pytest_b; do [ -f $OUT/$f.log ] && tail -n 5 $OUT/$f.log; done
[ -f $OUT/bench.log ] && tail -c 600 $OUT/bench.log
exit $rc
