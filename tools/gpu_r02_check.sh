#!/bin/bash
# Round-2 GPU check: every gpu test, smoke(), the C2 bench line (with CPU leg), the other
# configs (C3, C4, C5 fp64 / mixed / fp32), and rocprofv3 kernel-trace stats of C2, C5 mixed and C5 fp64.
# usage (GPU box, via gpurun): bash tools/gpu_r02_check.sh OUTDIR
set -o pipefail
OUT=gpurun_out/${1:-r02}
mkdir -p $OUT
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --steps 10 --warmup 2 --no-cpu > $OUT/c3.log 2>&1 && \
timeout -k 10 200 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > $OUT/c4.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu > $OUT/c5.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --precision mixed > $OUT/c5_mixed.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu --precision fp32 > $OUT/c5_fp32.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c2 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_trace_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5m -o run -- python3 bench.py --config C5 --precision mixed --steps 5 --warmup 1 --no-cpu > $OUT/bench_trace_c5m.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o run -- python3 bench.py --config C5 --steps 5 --warmup 1 --no-cpu > $OUT/bench_trace_c5.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2; tail -n 1 $OUT/smoke.log
for f in bench c3 c4 c5 c5_mixed c5_fp32; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | cut -c1-200; done
exit $rc
