#!/bin/bash
# the closed-loop lines with the rank's instances in 1 / 2 / 4 concurrent groups (own stream each)
set -o pipefail
OUT=gpurun_out/${1:-r05_cs}
mkdir -p $OUT
for s in 1 2 4; do
  timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 --no-cpu --streams $s > $OUT/bench_cll_s$s.log 2>&1 || exit $?
  tail -1 $OUT/bench_cll_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('CLL streams $s', d['value'], d['ms_per_step'], d['check'].get('sqp_iterations_mean'), d['check'].get('x_init_vs_stored_q100_all_max'))"
done
for s in 1 2; do
  timeout -k 10 300 python bench.py --config CL --no-cpu --streams $s > $OUT/bench_cl_s$s.log 2>&1 || exit $?
  tail -1 $OUT/bench_cl_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('CL streams $s', d['value'], d['ms_per_step'])"
done
