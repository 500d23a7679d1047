#!/bin/bash
# GPU check of the mixed-precision path: its tests, then C5 in fp64 / mixed / fp32 (no CPU leg).
# usage (on the GPU box, via gpurun): bash tools/gpu_mixed.sh OUTDIR
set -o pipefail
OUT=gpurun_out/${1:-mixed}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_fp32.py tests/test_mex_gateway.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest_mixed.log 2>&1 && \
timeout -k 10 180 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu > $OUT/c5.log 2>&1 && \
timeout -k 10 180 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --precision mixed > $OUT/c5_mixed.log 2>&1 && \
timeout -k 10 180 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --precision fp32 > $OUT/c5_fp32.log 2>&1 && \
timeout -k 10 180 python bench.py --steps 20 --warmup 3 --no-cpu > $OUT/c2.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/pytest_mixed.log | tail -3
for f in c5 c5_mixed c5_fp32 c2; do tail -n 1 $OUT/$f.log | cut -c1-260; done
exit $rc
