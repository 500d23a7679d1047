#!/bin/bash
# Bench lines of every config (C2 default + C3/C4/C5) on one GPU; each step time-limited,
# chained with && so the first failure ends the session.  usage: tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-configs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_C2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 3 > $OUT/bench_C3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 2 > $OUT/bench_C4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 > $OUT/bench_C5.log 2>&1
rc=$?
for f in $OUT/bench_C*.log; do tail -n 1 $f; done
exit $rc
