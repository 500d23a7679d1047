#!/bin/bash
# round-5 profiling of the final tree: C2 phase stamps (build/stamps/libbqp_stamps.so, built on
# the CPU side and shipped for this call), then per config the rocprofv3 kernel-trace stats of the
# default bench command (2 streams) and the HBM PMC passes (FETCH_SIZE, WRITE_SIZE; one counter
# group per run), then the learned-model loop (CLL): trace, MFMA busy, HBM.  Summarise afterwards
# on the CPU with tools/pmc_summary.py / tools/cll_pmc_summary.py.
# usage (on the GPU box, via gpurun): bash tools/gpu_r05_prof.sh TAG [CFG ...]
set -o pipefail
TAG=${1:-r05_prof}; shift
CFGS=${@:-C2 C3 C4 C5}
[ "$CFGS" = "none" ] && CFGS=""   # CLL only
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
if [ -f learning-based-mpc_amd/build/stamps/libbqp_stamps.so ]; then
  timeout -k 10 120 python3 tools/stamps.py 1024 --json gpurun_out/$TAG/stamps_C2.json > gpurun_out/$TAG/stamps.log 2>&1 || exit $?
  tail -3 gpurun_out/$TAG/stamps.log
fi
for c in $CFGS; do
  case $c in
    C4) S="--steps 3 --warmup 1";;
    C5*) S="--steps 5 --warmup 1";;
    *) S="--steps 20 --warmup 3";;
  esac
  A="--config ${c%%_*}"
  [ "$c" != "${c%%_*}" ] && A="$A --precision ${c#*_}"
  D=gpurun_out/$TAG/$c
  mkdir -p $D
  echo "== $c: $A $S"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $S --no-cpu $A > $D/bench_trace.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu $A > $D/pmc_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu $A > $D/pmc_write.log 2>&1 || exit $?
  tail -n 1 $D/bench_trace.log | cut -c1-300
done
D=gpurun_out/$TAG/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_write.log 2>&1 || exit $?
head -8 $D/trace/run_kernel_stats.csv | cut -d, -f1-5
