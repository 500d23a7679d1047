#!/bin/bash
# round-4 GPU check: smoke(), every gpu test (a crash or hang stops the script), the default bench
# line (C2 with its CPU leg) and the C4 / C3 / C5 / CLL lines; logs under gpurun_out/TAG
set -o pipefail
TAG=${1:-r04_check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 && \
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1
rc2=$?
for f in bench_c2 bench_c4 bench_c3 bench_c5 bench_cll; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | cut -c1-700; echo; done
[ $rc -ne 0 ] && exit $rc
exit $rc2
