#!/bin/bash
# Kernel iteration loop: structured-solver GPU tests, phase stamps, C2 bench line (no CPU leg).
# usage (on the GPU box, via gpurun): bash tools/gpu_perf.sh OUTDIR [extra pytest files]
set -o pipefail
OUT=gpurun_out/${1:-perf}
shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ocp.py tests/test_gpu_duals.py tests/test_gpu_fp32.py tests/test_gpu_closed_loop.py "$@" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/bench.log 2>&1
rc=$?
tail -n 4 $OUT/pytest.log; cat $OUT/stamps.log; tail -n 1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], d['check'])"
exit $rc
