#!/bin/bash
# dense workgroup kernel phase stamps: builds the diagnostic library on the box (build/dstamps is
# not shipped), then tools/diag_dense_qp.py with it (instance 0's per-phase cycles printed by the
# kernel) and without it (kernel times)
set -o pipefail
OUT=gpurun_out/${1:-r05_dst}
mkdir -p $OUT
make -s -j16 -C learning-based-mpc_amd dstamps > $OUT/make.log 2>&1 || { tail $OUT/make.log; exit 1; }
BQP_LIB=learning-based-mpc_amd/build/dstamps/libbqp_dstamps.so timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_dst.log 2>&1 || exit $?
grep DSTAMPS $OUT/dq_dst.log | tail -4
timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq.log 2>&1 || exit $?
tail -4 $OUT/dq.log
