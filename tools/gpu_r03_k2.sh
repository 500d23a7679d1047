#!/bin/bash
# C2 / C5 bench with and without the active-set polish (round-3 kernel cost split)
set -o pipefail
OUT=gpurun_out/${1:-r03_k2}
mkdir -p $OUT
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/c2_pol.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-polish > $OUT/c2_nopol.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/c5_pol.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu --no-polish > $OUT/c5_nopol.log 2>&1
rc=$?
for f in c2_pol c2_nopol c5_pol c5_nopol; do python -c "
import json; d=json.loads(open('$OUT/$f.log').read().strip().split('\n')[-1]); c=d['check']
print('$f', d['value'], d['roofline']['kernel_ms'], 'it mean', c['iterations_mean'], 'max', c.get('iterations_max'), 'polished', c.get('polished_count'))"; done
exit $rc
