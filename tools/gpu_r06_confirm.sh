#!/bin/bash
# round-6 last check of the shipped library: smoke, every GPU test, the default bench line
set -o pipefail
TAG=${1:-r06_confirm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 || exit $?
tail -n 1 $OUT/bench_c2.log | cut -c1-700
exit $rc
