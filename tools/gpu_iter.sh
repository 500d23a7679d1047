#!/bin/bash
# Quick GPU iteration: parity tests, per-phase stamps breakdown, short bench (no CPU leg).
# Each GPU step has its own limit; steps are chained with && so the first failure ends the call.
# usage: tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python tools/stamps.py 1024 > $OUT/stamps.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu > $OUT/bench.log 2>&1
rc=$?
tail -n 4 $OUT/pytest_gpu.log
[ -f $OUT/stamps.log ] && tail -n 18 $OUT/stamps.log
[ -f $OUT/bench.log ] && tail -c 900 $OUT/bench.log
exit $rc
