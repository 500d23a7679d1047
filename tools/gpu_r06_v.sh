#!/bin/bash
# round-6 call n: the exact-Hessian kernel's Cholesky tests at two pivots per barrier pair: every GPU
# test, CLL A/B against the library before (build/abship/libbqp_pre2p.so),
# the n = 101 sub-problem alone, CLL kernel trace
set -o pipefail
TAG=${1:-r06_v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 && \
BQP_LIB=learning-based-mpc_amd/build/abship/libbqp_pre2p.so timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_pre2p.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_b.log 2>&1 || exit $?
for f in bench_cll bench_cll_pre2p bench_cll_b; do tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'dense_ms', r.get('kernel_ms'), 'sqp', c.get('sqp_iterations_mean'), 'slow', c.get('x_init_vs_stored_q100_slow_max'))"; done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=$OUT/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('$D/trace/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,4))
" > $D/summary.txt
head -8 $D/summary.txt
exit $rc
