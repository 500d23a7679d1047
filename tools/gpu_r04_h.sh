#!/bin/bash
# row-replicated factor check: smoke + every GPU test + A/B vs BASE on C2 C4 C3 C5 + the CLL line
# (tools/gpu_r04_run.sh), then the C2 phase stamps of the in-tree kernel
set -o pipefail
TAG=$1; BASE=$2
bash tools/gpu_r04_run.sh $TAG $BASE || exit $?
timeout -k 10 120 python tools/stamps.py 1024 > gpurun_out/$TAG/stamps.log 2>&1 || exit $?
cat gpurun_out/$TAG/stamps.log
