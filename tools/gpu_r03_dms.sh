#!/bin/bash
# learned-model NLP loop check: the DMS LBMPC GPU tests, the existing LBMPC kernel tests, the
# iteration diagnostic
set -o pipefail
OUT=gpurun_out/${1:-r03_dms}
mkdir -p $OUT
export OMP_NUM_THREADS=4
timeout -k 10 900 python -u -m pytest tests/test_gpu_lbmpc_dms.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_pinned.py tests/test_gpu_lbmpc_loop.py -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/diag_dms_gpu.py > $OUT/diag.log 2>&1
rc2=$?
cat $OUT/diag.log
exit $rc
