set -o pipefail
mkdir -p gpurun_out/r03_ab2
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ocp.py tests/test_gpu_duals.py -q --timeout 300 --timeout-method thread > gpurun_out/r03_ab2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_ab2/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r03_ab.sh r03_ab2 learning-based-mpc_amd/build/ab/libbqp_base.so C2 C4
