#!/bin/bash
# the asynchronous learned-model loop: its parity test against the step-synchronous form, the
# learned-loop GPU tests, and the CLL line
set -o pipefail
OUT=gpurun_out/${1:-r05_async}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lbmpc_dms.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_loop.py tests/test_gpu_lbmpc_pinned.py tests/test_mex_gateway.py -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -8
grep "async vs" $OUT/pytest.log | head -2
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 || exit $?
tail -1 $OUT/bench_cll.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('CLL', d['value'], d['ms_per_step'], d['check'])"
exit $rc
