#!/bin/bash
# round-6 call o: phase stamps of the dense polish (diagnostic library build/stamps_ship, short CLL
# run; every 16th instance of each polish launch prints its phases)
set -o pipefail
TAG=${1:-r06_o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BQP_LIB=learning-based-mpc_amd/build/stamps_ship/libbqp_dstamps.so timeout -k 10 300 python -u bench.py --config CLL --steps 2 --warmup 0 --batch 256 --no-cpu > $OUT/cll_pst.log 2>&1 || exit $?
python3 - $OUT/cll_pst.log <<'PY'
import sys, collections
tot = collections.Counter(); c = 0; rounds = 0; mx = collections.Counter()
for l in open(sys.argv[1]):
    if l.startswith('PSTAMPS'):
        f = l.split()
        d = dict(zip(f[1::2], f[2::2]))
        c += 1; rounds += int(d['rounds'])
        s = 0
        for k in ('actlist', 'K', 'cholK', 'Y', 'S', 'cholS', 'mult', 'checks', 'corr'):
            tot[k] += int(d[k]); s += int(d[k])
        mx['total'] = max(mx['total'], s)
print('polish samples %d mean rounds %.2f max total %d' % (c, rounds / max(c, 1), mx['total']))
for k, v in tot.items(): print('  %-8s %10d cyc per polish' % (k, v // max(c, 1)))
PY
exit 0
