#!/bin/bash
# rocprofv3 kernel-trace stats of the bench workload (no PMC in this pass), then an HBM PMC pass.
# usage: [BENCH_ARGS='--config C5'] tools/gpu_prof.sh TAG
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu $BENCH_ARGS > gpurun_out/$TAG/bench_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/$TAG/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/$TAG/pmc_write.log 2>&1
rc=$?
find gpurun_out/$TAG -name "*.csv" | head -20
exit $rc
