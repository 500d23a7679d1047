#!/bin/bash
# round-6 first check: smoke + every GPU test, the mixed-repair diagnostic,
# the bench lines at one stream and the C2 rocprofv3 kernel trace of the
# default bench command; logs under gpurun_out/TAG
set -o pipefail
TAG=${1:-r06_a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_mixed_repair.py > $OUT/diag_mixed_repair.log 2>&1 || exit $?
cat $OUT/diag_mixed_repair.log | cut -c1-600
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 || exit $?
# A/B: the same configs with one instance per slot (no work queue)
BQP_NO_QUEUE=1 timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3_noq.log 2>&1 && \
BQP_NO_QUEUE=1 timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4_noq.log 2>&1 && \
BQP_NO_QUEUE=1 timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5_noq.log 2>&1 || exit $?
for f in bench_c2 bench_c3 bench_c4 bench_c5 bench_c3_noq bench_c4_noq bench_c5_noq; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'alone', r.get('kernel_ms_alone'), 'frac', r.get('frac'), 'two_groups', c.get('value_two_groups'), 'iters', c.get('iterations_mean'), c.get('iterations_max'), 'flags', c.get('exitflag_hist_all_ranks'), 'pol', c.get('polished_count'))"; done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=$OUT/C2
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
head -6 $D/trace/run_kernel_stats.csv | cut -d, -f1-6
exit $rc
