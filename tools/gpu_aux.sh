#!/bin/bash
# Measurements of the §8(f) paths (C1 LBMPC SQP, CL closed loop) + a kernel-trace profile of each.
set -o pipefail
TAG=${1:-aux}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C1 --steps 20 --warmup 2 > $OUT/bench_C1.log 2>&1 && \
timeout -k 10 300 python bench.py --config C1 --batch 1024 --steps 5 --warmup 1 > $OUT/bench_C1_b1024.log 2>&1 && \
timeout -k 10 300 python bench.py --config CL --batch 1024 --steps 50 > $OUT/bench_CL.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_C1 -o run -- python3 bench.py --config C1 --batch 1024 --steps 3 --warmup 1 > $OUT/trace_C1.log 2>&1
rc=$?
for f in $OUT/bench_*.log; do tail -n 1 $f; done
exit $rc
