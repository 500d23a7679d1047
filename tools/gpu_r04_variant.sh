#!/bin/bash
# A/B of a variant library (BQP_LIB=$2) on the dense / loop GPU tests, the n = 101 QP and the CLL line
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export BQP_LIB=$GRAFT_REPO_ROOT/$2
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "quadprog or lbmpc or dense or condensed or closed_loop or learned or dms" > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/diag_dense_qp.py > $OUT/dq.log 2>&1 || exit $?
tail -n 4 $OUT/dq.log
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 || exit $?
tail -n 1 $OUT/bench_cll.log | cut -c1-300
