#!/bin/bash
# dense kernel iteration: its GPU tests, the stamps (locally built build/dstamps), the n = 101 QP
# time, and the CLL line
set -o pipefail
OUT=gpurun_out/${1:-r05_dn}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_quadprog.py tests/test_gpu_quadprog_status.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_pinned.py tests/test_gpu_lbmpc_dms.py tests/test_gpu_condensed_route.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
BQP_LIB=learning-based-mpc_amd/build/dstamps/libbqp_dstamps.so timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_dst.log 2>&1 || exit $?
grep DSTAMPS $OUT/dq_dst.log | tail -1
timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq.log 2>&1 || exit $?
grep "batch" $OUT/dq.log
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 || exit $?
tail -1 $OUT/bench_cll.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('CLL', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['check'])"
