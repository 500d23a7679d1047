#!/bin/bash
# dense kernels (workgroup + wave): every GPU test, the n = 101 QP stamps and time, the C1 and CLL lines
set -o pipefail
OUT=gpurun_out/${1:-r05_dnw}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
BQP_LIB=learning-based-mpc_amd/build/dstamps/libbqp_dstamps.so timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq_dst.log 2>&1 || exit $?
grep DSTAMPS $OUT/dq_dst.log | tail -1
timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq.log 2>&1 || exit $?
grep "batch" $OUT/dq.log
timeout -k 10 300 python bench.py --config C1 --no-cpu > $OUT/bench_c1.log 2>&1 || exit $?
tail -1 $OUT/bench_c1.log | cut -c1-400
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 || exit $?
tail -1 $OUT/bench_cll.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('CLL', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['check'])"
