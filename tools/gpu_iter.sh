#!/bin/bash
# quick GPU iteration: parity tests, stamps breakdown, short bench
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -n 6 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/stamps.py 1024 > gpurun_out/stamps.log 2>&1; tail -n 18 gpurun_out/stamps.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; tail -c 900 gpurun_out/bench.log
