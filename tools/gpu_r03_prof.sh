#!/bin/bash
# round-3 profiling: for each config, rocprofv3 kernel-trace stats of the bench command, then the
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run), and the C2 phase stamps
# (diagnostic build, make -C learning-based-mpc_amd stamps).  Summarise afterwards on the CPU with
#   python tools/pmc_summary.py gpurun_out/TAG/CFG profiles/TAG/CFG --config CFG
# usage (on the GPU box, via gpurun): bash tools/gpu_r03_prof.sh TAG [CFG ...]
set -o pipefail
TAG=${1:-r03_prof}; shift
CFGS=${@:-C2 C3 C4 C5}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
if [ -f learning-based-mpc_amd/build/stamps/libbqp_stamps.so ]; then
  timeout -k 10 120 python3 tools/stamps.py 1024 --json gpurun_out/$TAG/stamps_C2.json > gpurun_out/$TAG/stamps.log 2>&1 || exit $?
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
find gpurun_out/$TAG -name "*.csv" | head -40
