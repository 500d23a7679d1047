#!/bin/bash
# round-4 final pass: smoke + every GPU test + the CLL line (tools/gpu_r04_run.sh without A/B),
# the default bench line, then the profiling pass (tools/gpu_r04_prof.sh)
set -o pipefail
TAG=$1
bash tools/gpu_r04_run.sh $TAG || exit $?
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench_default.log 2>&1 || exit $?
tail -n 1 gpurun_out/$TAG/bench_default.log | cut -c1-600
bash tools/gpu_r04_prof.sh ${TAG}_prof C2 C3 C4 C5 || exit $?
