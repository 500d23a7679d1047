#!/bin/bash
# GPU check of the tree: every gpu test, smoke(), the C2 bench line (with the CPU leg).
# usage (on the GPU box, via gpurun): bash tools/gpu_check.sh OUTDIR
set -o pipefail
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.log 2>&1
rc=$?
tail -n 5 $OUT/pytest_gpu.log; tail -n 1 $OUT/smoke.log; tail -n 1 $OUT/bench.log
exit $rc
