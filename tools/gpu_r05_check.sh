#!/bin/bash
# round-5 GPU check: smoke(), every gpu test (a crash or hang stops the script), the default bench
# line (C2 with its CPU thread sweep) and the CLL line; logs under gpurun_out/TAG
set -o pipefail
TAG=${1:-r05_check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1
rc2=$?
for f in bench_c2 bench_cll; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | cut -c1-1500; echo; done
[ $rc -ne 0 ] && exit $rc
exit $rc2
