#!/bin/bash
# round-4 GPU run: smoke, every gpu test, A/B of the in-tree library against BASE_SO (C2 C4 C3
# C5), then the CLL line; logs under gpurun_out/TAG.  usage: bash tools/gpu_r04_run.sh TAG BASE_SO
set -o pipefail
TAG=${1:-r04_run}; BASE=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BASE" ]; then bash tools/gpu_r03_ab.sh $TAG/ab $BASE C2 C4 C3 C5 || exit $?; fi
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1
rc2=$?
tail -n 1 $OUT/bench_cll.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
exit $rc2
