#!/bin/bash
# C2 / C4 / C5 / C3 throughput with consecutive steps on 1, 2, 3 and 4 HIP streams (bench.py --streams)
set -o pipefail
OUT=gpurun_out/${1:-r05_str}
mkdir -p $OUT
for cfg in C2 C3 C5; do
  for s in 1 2 3 4; do
    timeout -k 10 200 python bench.py --config $cfg --streams $s --no-cpu --steps 40 --warmup 5 > $OUT/${cfg}_s$s.log 2>&1 || exit $?
    tail -1 $OUT/${cfg}_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg streams $s', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
