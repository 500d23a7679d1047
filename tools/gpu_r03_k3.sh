#!/bin/bash
# round-3 GPU check: every gpu test (crash stops the script), then the C2 bench line
set -o pipefail
OUT=gpurun_out/${1:-r03_k3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "PASSED|FAILED|ERROR" $OUT/pytest_gpu.log | grep -v PASSED | head -20; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1
rc=$?
tail -1 $OUT/smoke.log
for f in bench_c2 bench_c4 bench_c5; do python -c "
import json; d=json.loads(open('$OUT/$f.log').read().strip().split('\n')[-1]); c=d['check']
print('$f', d['value'], d['roofline']['kernel_ms'], 'it', c.get('iterations_mean'), c.get('iterations_max'), 'pol', c.get('polished_count'), c.get('exitflag_hist_all_ranks'))" || true; done
exit $rc
