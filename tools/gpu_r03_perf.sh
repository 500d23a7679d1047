#!/bin/bash
# structured-kernel change check: every gpu test (a crash stops the script), then the C2 / C3 /
# C4 / C5 bench lines (no CPU legs)
set -o pipefail
OUT=gpurun_out/${1:-r03_perf}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --steps 20 --warmup 3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1
rc2=$?
for f in bench_c2 bench_c3 bench_c4 bench_c5; do python -c "
import json; d=json.loads([l for l in open('$OUT/$f.log') if l.startswith('{')][-1]); c=d['check']
print('$f', d['value'], d['roofline']['kernel_ms'], 'it', c.get('iterations_mean'), c.get('exitflag_hist_all_ranks'), c.get('max_abs_du0_vs_exact'))" || true; done
[ $rc -ne 0 ] && exit $rc
exit $rc2
