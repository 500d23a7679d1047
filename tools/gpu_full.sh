#!/bin/bash
# full GPU check of the tree: all gpu tests, smoke, C2 bench (with CPU leg), C3 / C4 / C5 lines
# (phase stamps: tools/gpu_stamps_configs.sh, needs `make -C learning-based-mpc_amd stamps`)
set -o pipefail
OUT=gpurun_out/${1:-full}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu > $OUT/c5.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --precision fp32 --steps 5 --warmup 1 --no-cpu > $OUT/c5_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --steps 10 --warmup 2 --no-cpu > $OUT/c3.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > $OUT/c4.log 2>&1
rc=$?
tail -n 3 $OUT/pytest_gpu.log; tail -n 1 $OUT/smoke.log
for f in bench c5 c5_fp32 c3 c4; do [ -f $OUT/$f.log ] && echo "$f: $(grep -o '"value": [0-9.]*' $OUT/$f.log) $(grep -o '"kernel_ms": [0-9.]*' $OUT/$f.log)"; done
exit $rc
