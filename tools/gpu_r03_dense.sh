#!/bin/bash
# dense workgroup kernel change check: the dense / LBMPC / condensed-route GPU tests, then the
# n = 101 sub-problem diagnostic and the CLL loop, new library vs BASE (A/B on one box)
set -o pipefail
OUT=gpurun_out/${1:-r03_dense}; BASE=$2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_quadprog.py tests/test_gpu_quadprog_status.py tests/test_gpu_condensed_route.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_pinned.py tests/test_gpu_lbmpc_dms.py tests/test_gpu_ocp.py tests/test_mex_gateway.py -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_new.log 2>&1 || exit $?
BQP_LIB=$BASE timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_base.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config CLL --steps 5 --batch 256 > $OUT/cll_new.log 2>&1 || exit $?
BQP_LIB=$BASE timeout -k 10 300 python bench.py --config CLL --steps 5 --batch 256 > $OUT/cll_base.log 2>&1 || exit $?
tail -3 $OUT/dq_new.log; tail -3 $OUT/dq_base.log
for f in cll_new cll_base; do grep '^{' $OUT/$f.log | cut -c1-260; done
exit $rc
