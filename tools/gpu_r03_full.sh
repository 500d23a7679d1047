#!/bin/bash
# round-3 full GPU check: every gpu test (a crash stops the script), smoke(), the default bench line
# (with its CPU leg), and the C1 / CLL / C3 aux lines
set -o pipefail
OUT=gpurun_out/${1:-r03_full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 200 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1 && \
timeout -k 10 200 python bench.py --config C1 --steps 10 --warmup 2 > $OUT/bench_c1.log 2>&1 && \
timeout -k 10 200 python bench.py --config C1 --steps 10 --warmup 2 --batch 1024 --no-cpu > $OUT/bench_c1b.log 2>&1
rc2=$?
tail -1 $OUT/smoke.log
for f in bench_c2 bench_cll bench_c1 bench_c1b; do tail -n 1 $OUT/$f.log | cut -c1-900; echo; done
[ $rc -ne 0 ] && exit $rc
exit $rc2
