#!/bin/bash
# Long-horizon layout check: structured GPU tests, C2 and C5 (fp64 / mixed) benches.
set -o pipefail
OUT=gpurun_out/${1:-lng}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ocp.py tests/test_gpu_mixed.py tests/test_gpu_fp32.py tests/test_gpu_duals.py tests/test_gpu_closed_loop.py tests/test_gpu_lbmpc_loop.py tests/test_gpu_ocp_poly.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/c2.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu > $OUT/c5.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --precision mixed > $OUT/c5m.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --steps 10 --warmup 2 --no-cpu > $OUT/c3.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest.log | tail -2
for f in c2 c5 c5m c3; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | cut -c1-200; done
exit $rc
