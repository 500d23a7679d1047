#!/bin/bash
# round-5 check of the tree: smoke + every GPU test, then the bench lines of C2 (with its CPU
# sweep), C3, C4, C5 and CLL; logs under gpurun_out/TAG
set -o pipefail
TAG=${1:-r05_full}
OUT=gpurun_out/$TAG
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1
rc=$?
for f in bench_c2 bench_c3 bench_c4 bench_c5 bench_cll; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'kernel_ms', r.get('kernel_ms', d.get('kernel_ms')), 'frac', r.get('frac'), 'iters', c.get('iterations_mean', c.get('sqp_iterations_mean')), 'flags', c.get('exitflag_hist_all_ranks'))"; done
exit $rc
