#!/bin/bash
# Phase stamps of the C2 kernel + one bench line per config (no CPU legs).
# usage (on the GPU box, via gpurun): bash tools/gpu_stamps_configs.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-sc}
mkdir -p $OUT
timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --steps 20 --warmup 3 --no-cpu > $OUT/bench_C3.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 10 --warmup 2 --no-cpu > $OUT/bench_C4.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_C5.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --precision fp32 --steps 10 --warmup 2 --no-cpu > $OUT/bench_C5f.log 2>&1 && \
timeout -k 10 200 python bench.py --config C1 --steps 10 --warmup 2 --no-cpu > $OUT/bench_C1.log 2>&1
rc=$?
cat $OUT/stamps.log
for f in $OUT/bench_C*.log; do echo $f; tail -n 1 $f | cut -c1-400; done
exit $rc
