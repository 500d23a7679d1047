#!/bin/bash
# kernel-trace stats of the learned-model NLP loop (bench --config CLL)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03_cll}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config CLL --steps 3 --batch 256 > $OUT/bench.log 2>&1
rc=$?
head -20 $OUT/trace/run_kernel_stats.csv | cut -d, -f1-5
exit $rc
