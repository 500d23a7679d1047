#!/bin/bash
# round-4 profiling: tools/gpu_r03_prof.sh for the structured configs (kernel-trace stats, HBM
# FETCH_SIZE / WRITE_SIZE passes, C2 phase stamps), then the learned-model loop (CLL): kernel
# trace of the bench command and a counter pass with the MFMA busy cycles of the dense kernel.
# usage (on the GPU box, via gpurun): bash tools/gpu_r04_prof.sh TAG [CFG ...]
set -o pipefail
TAG=${1:-r04_prof}; shift
bash tools/gpu_r03_prof.sh $TAG "$@" || exit $?
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/$TAG/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_write.log 2>&1 || exit $?
head -12 $D/trace/run_kernel_stats.csv | cut -d, -f1-5
