#!/bin/bash
# One GPU session: parity tests, smoke, quick numbers, bench.  Each GPU step has its own limit;
# steps are chained with && so the first failure ends the session.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python tools/gpu_quick.py > gpurun_out/quick.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
for f in smoke quick bench; do tail -n 3 gpurun_out/$f.log; done
exit $rc
