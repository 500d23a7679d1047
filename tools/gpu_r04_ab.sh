#!/bin/bash
# round-4 A/B of structured-kernel variants on one box: C2 phase stamps of the in-tree kernel and of
# a variant stamp build, then alternating bench runs of the in-tree library against variant builds.
# usage: bash tools/gpu_r04_ab.sh TAG VARIANT_SO VARIANT_STAMPS_SO [PREV_SO]
set -o pipefail
TAG=$1; VAR=$2; VST=$3; PREV=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps_new.log 2>&1 || exit $?
BQP_STAMPS_LIB=$VST timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps_var.log 2>&1 || exit $?
bash tools/gpu_r03_ab.sh $TAG/ab $VAR C2 C5 C3 || exit $?
if [ -n "$PREV" ]; then bash tools/gpu_r03_ab.sh $TAG/ab_prev $PREV C2 || exit $?; fi
