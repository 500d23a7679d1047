#!/bin/bash
# new GPU tests of this step, then the C5 regression A/B (tools/gpu_r04_c5.sh)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -k "ode23 or c_restatement or end_to_end" > $OUT/pytest_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|loop" $OUT/pytest_new.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_r04_c5.sh "$(basename $OUT)_c5" "$@"
