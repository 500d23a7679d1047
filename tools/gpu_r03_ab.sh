#!/bin/bash
# A/B timing on one box: the in-tree library against another build (BQP_LIB), alternating runs
# usage: bash tools/gpu_r03_ab.sh TAG BASE_SO [CONFIGS...]
set -o pipefail
OUT=gpurun_out/${1:-r03_ab}; BASE=$2; shift 2
CFGS=${@:-C2 C4}
mkdir -p $OUT
for c in $CFGS; do
  case $c in C4) S="--steps 5 --warmup 1";; C5) S="--steps 10 --warmup 2";; *) S="--steps 50 --warmup 5";; esac
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --config $c $S --no-cpu > $OUT/${c}_new_$rep.log 2>&1 || exit $?
    BQP_LIB=$BASE timeout -k 10 200 python bench.py --config $c $S --no-cpu > $OUT/${c}_base_$rep.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do python -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); c=d['check']
print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms'], c.get('iterations_mean'), c.get('exitflag_hist_all_ranks'))" || true; done
