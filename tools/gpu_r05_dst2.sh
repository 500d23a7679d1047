#!/bin/bash
# dense workgroup kernel phase stamps from the locally built diagnostic library (build/dstamps,
# shipped for this run): tools/diag_dense_qp.py with it
set -o pipefail
OUT=gpurun_out/${1:-r05_dstx}
mkdir -p $OUT
BQP_LIB=learning-based-mpc_amd/build/dstamps/libbqp_dstamps.so timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_dst.log 2>&1 || exit $?
grep DSTAMPS $OUT/dq_dst.log | tail -2
