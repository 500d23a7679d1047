#!/bin/bash
# Dense-path GPU check: quadprog / LBMPC / MEX tests, the C2D (F1 via quadprog) and C1 benches,
# rocprofv3 kernel stats of C2D and C1, MFMA busy-cycle PMC pass of C2D.
# usage (GPU box, via gpurun): bash tools/gpu_dense.sh OUTDIR
set -o pipefail
OUT=gpurun_out/${1:-dense}
mkdir -p $OUT
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_quadprog.py tests/test_gpu_quadprog_status.py tests/test_gpu_lbmpc.py tests/test_gpu_lbmpc_pinned.py tests/test_mex_gateway.py tests/test_gpu_duals.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --config C2D --steps 20 --warmup 3 > $OUT/c2d.log 2>&1 && \
timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 > $OUT/c1.log 2>&1 && \
timeout -k 10 200 python bench.py --config C1 --batch 1024 --steps 10 --warmup 2 > $OUT/c1_1024.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2d -o run -- python3 bench.py --config C2D --steps 10 --warmup 2 > $OUT/trace_c2d.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o run -- python3 bench.py --config C1 --steps 10 --warmup 2 > $OUT/trace_c1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py --config C2D --steps 3 --warmup 1 > $OUT/pmc_mfma.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest.log | tail -2
for f in c2d c1 c1_1024; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | cut -c1-300; done
exit $rc
