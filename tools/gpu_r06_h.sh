#!/bin/bash
# round-6 call h: phase stamps of the LDL' tree (C3, C2) from the shipped stamps build, and the
# C5 bench line of the current library
set -o pipefail
TAG=${1:-r06_h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export BQP_STAMPS_LIB=learning-based-mpc_amd/build/stamps_ship/libbqp_stamps.so
timeout -k 10 180 python tools/stamps.py --config C3 --json $OUT/stamps_C3.json > $OUT/stamps_c3.log 2>&1 && \
timeout -k 10 180 python tools/stamps.py --config C2 --json $OUT/stamps_C2.json > $OUT/stamps_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --no-cpu > $OUT/bench_c5.log 2>&1
rc=$?
cat $OUT/stamps_c3.log $OUT/stamps_c2.log
tail -n 1 $OUT/bench_c5.log | cut -c1-600
exit $rc
