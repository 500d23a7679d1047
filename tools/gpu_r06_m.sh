#!/bin/bash
# round-6 call m: polish phase stamps (diagnostic library build/stamps_ship/libbqp_dstamps.so, a
# short CLL run), then every GPU test and a CLL A/B of the update kernel's coalesced A_in' lam
# against the library before it (build/abship/libbqp_preupd.so)
set -o pipefail
TAG=${1:-r06_m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BQP_LIB=learning-based-mpc_amd/build/stamps_ship/libbqp_dstamps.so timeout -k 10 300 python -u bench.py --config CLL --steps 2 --warmup 0 --batch 256 --no-cpu > $OUT/cll_pst.log 2>&1 || exit $?
grep PSTAMPS $OUT/cll_pst.log | head -3
python3 - $OUT/cll_pst.log <<'PY' || true
import sys, re, collections
tot = collections.Counter(); c = 0; rounds = 0
for l in open(sys.argv[1]):
    if l.startswith('PSTAMPS'):
        f = l.split()
        d = dict(zip(f[1::2], f[2::2]))
        c += 1; rounds += int(d['rounds'])
        for k in ('actlist', 'K', 'cholK', 'Y', 'S', 'cholS', 'mult', 'checks', 'corr'):
            tot[k] += int(d[k])
print('polish launches %d mean rounds %.2f' % (c, rounds / max(c, 1)))
for k, v in tot.items(): print('  %-8s %10d cyc per polish' % (k, v // max(c, 1)))
PY
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 && \
BQP_LIB=learning-based-mpc_amd/build/abship/libbqp_preupd.so timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_preupd.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_b.log 2>&1 || exit $?
for f in bench_cll bench_cll_preupd bench_cll_b; do tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'dense_ms', r.get('kernel_ms'), 'sqp', c.get('sqp_iterations_mean'), 'slow', c.get('x_init_vs_stored_q100_slow_max'))"; done
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
head -10 $D/summary.txt
exit $rc
