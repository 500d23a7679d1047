#!/bin/bash
# C5 regression hunt: A/B of the in-tree library against other builds on C5 (and C2), then a
# rocprofv3 kernel trace of the in-tree C5 bench.  usage: bash tools/gpu_r04_c5.sh TAG SO...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/C5_new_$rep.log 2>&1 || exit $?
  for so in "$@"; do
    b=$(basename $so .so)
    BQP_LIB=$so timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/C5_${b}_$rep.log 2>&1 || exit $?
  done
done
for so in "$@"; do
  b=$(basename $so .so)
  BQP_LIB=$so timeout -k 10 200 python bench.py --config C2 --steps 50 --warmup 5 --no-cpu > $OUT/C2_${b}.log 2>&1 || exit $?
done
for f in $OUT/*.log; do python -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); c=d['check']
print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms'], c.get('iterations_mean'))" || true; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/$OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-300 | head -20
