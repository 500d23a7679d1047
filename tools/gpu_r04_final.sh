#!/bin/bash
# round-4 final check of the tree: smoke + every GPU test + the default bench line + the CLL line
# (with its CPU baseline), then the CLL profile passes (kernel trace, MFMA busy, HBM)
set -o pipefail
TAG=${1:-r04_final}
OUT=gpurun_out/$TAG
bash tools/gpu_r04_run.sh $TAG || exit $?
timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1 || exit $?
tail -n 1 $OUT/bench_default.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=$OUT/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_write.log 2>&1 || exit $?
head -6 $D/trace/run_kernel_stats.csv | cut -d, -f1-5
