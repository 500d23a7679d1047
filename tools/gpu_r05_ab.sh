#!/bin/bash
# A/B of dense-kernel variants on the failing / key dense tests (libraries under build/dstamps)
set -o pipefail
OUT=gpurun_out/${1:-r05_ab}
mkdir -p $OUT
for v in ${VARIANTS:-vA vB main}; do
  lib=learning-based-mpc_amd/build/dstamps/libbqp_$v.so; [ $v = main ] && lib=learning-based-mpc_amd/bqp/libbqp.so
  BQP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_quadprog.py tests/test_gpu_quadprog_status.py -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  echo "$v rc=$? $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
done
