#!/bin/bash
# learned-model NLP loop check: the new DMS LBMPC GPU tests and the existing LBMPC kernel tests
set -o pipefail
OUT=gpurun_out/${1:-r03_dms}
mkdir -p $OUT
export OMP_NUM_THREADS=4
timeout -k 10 900 python -u -m pytest tests/test_gpu_lbmpc_dms.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_pinned.py tests/test_gpu_lbmpc_loop.py -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
exit $rc
