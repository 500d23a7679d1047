#!/bin/bash
# round-6 call q: exact-Hessian kernel stamps (diagnostic library build/stamps_ship/libbqp_rstamps.so:
# row products, assembly, Cholesky tests and their count, every 16th instance) in a short CLL run
set -o pipefail
TAG=${1:-r06_q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BQP_LIB=learning-based-mpc_amd/build/stamps_ship/libbqp_rstamps.so timeout -k 10 300 python -u bench.py --config CLL --steps 2 --warmup 0 --batch 256 --no-cpu --streams 1 > $OUT/cll_hst.log 2>&1 || exit $?
python3 - $OUT/cll_hst.log <<'PY'
import sys, collections
v = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('HSTAMPS'):
        f = l.split(); d = dict(zip(f[1::2], f[2::2]))
        for k in d: v[k].append(int(d[k]))
import statistics
for k, x in v.items(): print('%-9s n %d mean %.0f max %d' % (k, len(x), statistics.mean(x), max(x)))
att = collections.Counter(v['attempts']); print('attempts histogram', dict(att))
PY
exit 0
