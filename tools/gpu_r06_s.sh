#!/bin/bash
# round-6 call s: learned-rollout phase stamps (diagnostic library build/stamps_ship/libbqp_rstamps.so)
set -o pipefail
TAG=${1:-r06_s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BQP_LIB=learning-based-mpc_amd/build/stamps_ship/libbqp_rstamps.so timeout -k 10 300 python -u bench.py --config CLL --steps 3 --warmup 0 --batch 256 --no-cpu --streams 1 > $OUT/cll_rst.log 2>&1 || exit $?
python - $OUT/cll_rst.log <<'PY'
import sys, re, collections
acc = collections.defaultdict(lambda: [0, [0] * 6])
for l in open(sys.argv[1]):
    m = re.match(r'RSTAMPS rollout gn (\d) pre (\d+) nw (\d+) post (\d+) term (\d+) costate (\d+) pass2 (\d+)', l)
    if m:
        g = int(m.group(1)); v = [int(x) for x in m.groups()[1:]]
        acc[g][0] += 1
        acc[g][1] = [a + b for a, b in zip(acc[g][1], v)]
for g, (c, v) in sorted(acc.items()):
    print('gn %d launches %d mean cycles: pre %d nw %d post %d term %d costate %d pass2 %d' % ((g, c) + tuple(x // max(c, 1) for x in v)))
PY
exit 0
