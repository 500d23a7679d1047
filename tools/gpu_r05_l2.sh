#!/bin/bash
# dense sub-problem time against its L2 footprint; the headline with 3 / 4 streams
set -o pipefail
OUT=gpurun_out/${1:-r05_l2}
mkdir -p $OUT
timeout -k 10 300 python -u tools/diag_dense_l2.py > $OUT/dense_l2.log 2>&1 || exit $?
grep "batch" $OUT/dense_l2.log
for s in 2 3 4; do
  timeout -k 10 300 python bench.py --config C2 --streams $s --steps 400 --warmup 20 --no-cpu > $OUT/bench_c2_s$s.log 2>&1 || exit $?
  tail -1 $OUT/bench_c2_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C2 streams $s', d['value'], d['ms_per_step'], r['kernel_ms'], r['kernel_ms_alone'])"
done
for c in C3 C5; do for s in 2 3; do
  timeout -k 10 300 python bench.py --config $c --streams $s --no-cpu > $OUT/bench_${c}_s$s.log 2>&1 || exit $?
  tail -1 $OUT/bench_${c}_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c streams $s', d['value'], d['ms_per_step'], r['kernel_ms'], r['kernel_ms_alone'])"
done; done
