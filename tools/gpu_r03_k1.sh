#!/bin/bash
# round-3 GPU check of the robust kernel: gpu tests (failures reported, crashes stop the script),
# C4 full-generator exit flags vs the C restatement, C2/C5/C4 bench lines (no CPU leg)
set -o pipefail
OUT=gpurun_out/${1:-r03_k1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/c4_check.py > $OUT/c4.log 2>&1
rc=$?; cat $OUT/c4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1
rc=$?
tail -c 700 $OUT/bench_c2.log; tail -c 500 $OUT/bench_c5.log; tail -c 500 $OUT/bench_c4.log
exit $rc
