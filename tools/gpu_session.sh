#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel-trace stats, HBM PMC passes and
# (if built) the per-phase stamps diagnostic.  Every GPU step has its own time limit; the steps
# are chained with && so the first failure (fault, abort, timeout) ends the session.
# usage: tools/gpu_session.sh TAG [pytest-args]
set -o pipefail
TAG=${1:-session}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/pmc_write.log 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -f learning-based-mpc_amd/build/stamps/libbqp_stamps.so ]; then
  timeout -k 10 120 python tools/stamps.py 1024 > $OUT/stamps.log 2>&1
  rc=$?
fi
tail -n 5 $OUT/pytest_gpu.log
for f in smoke bench stamps; do [ -f $OUT/$f.log ] && tail -n 20 $OUT/$f.log; done
exit $rc
