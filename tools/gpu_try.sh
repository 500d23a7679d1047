#!/bin/bash
# Cautious first run of a restructured kernel: smoke (8 instances) under a short limit, then
# the parity tests, the stamps breakdown and a short bench.  Steps chained with &&.
# usage: tools/gpu_try.sh TAG
set -o pipefail
TAG=${1:-try}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu > $OUT/bench.log 2>&1
rc=$?
for f in smoke pytest_gpu stamps; do [ -f $OUT/$f.log ] && tail -n 24 $OUT/$f.log; done
[ -f $OUT/bench.log ] && tail -c 700 $OUT/bench.log
exit $rc
