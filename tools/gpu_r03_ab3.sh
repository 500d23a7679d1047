set -o pipefail
mkdir -p gpurun_out/r03_ab3
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_ab3/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_ab3/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r03_ab.sh r03_ab3 learning-based-mpc_amd/build/ab/libbqp_prev.so C2 C4
timeout -k 10 120 python tools/stamps.py 1024 --json gpurun_out/r03_ab3/stamps_C2.json > gpurun_out/r03_ab3/stamps.log 2>&1
tail -30 gpurun_out/r03_ab3/stamps.log
