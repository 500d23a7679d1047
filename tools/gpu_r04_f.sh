#!/bin/bash
# round-4 check: full GPU tests + A/B vs BASE (tools/gpu_r04_run.sh), then the DPP-sweep variant:
# C2 stamps of both builds and an alternating A/B on C2 C5 C3.
# usage: bash tools/gpu_r04_f.sh TAG BASE_SO VARIANT_SO VARIANT_STAMPS_SO
set -o pipefail
TAG=$1; BASE=$2; VAR=$3; VST=$4
bash tools/gpu_r04_run.sh $TAG $BASE || exit $?
bash tools/gpu_r04_ab.sh ${TAG}_dpp $VAR $VST || exit $?
