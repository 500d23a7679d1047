#!/bin/bash
# round-6 call c: (1) the r06_b fault replayed once with serialised launches (tools/diag_n127.py),
# stopping there if it faults; (2) smoke + every GPU test; (3) C3 A/B of the DI occupancy-3
# variant (five instances per workgroup, three waves per SIMD; build/abship) and phase stamps of
# C3 / C2 (diagnostic library, build/stamps_ship); (4) rocprofv3 traces + HBM PMC passes of the
# default bench commands of C2..C5 (one stream).  Logs under gpurun_out/TAG.
set -o pipefail
TAG=${1:-r06_c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 180 python -u tools/diag_n127.py > $OUT/diag_n127.log 2>&1
rc=$?
cat $OUT/diag_n127.log | grep -v "^$" | tail -12
[ $rc -ne 0 ] && { echo "diag_n127 rc=$rc"; exit $rc; }
[ -n "$ONLY_DIAG" ] && exit 0
rc=0
if [ -z "$SKIP_TESTS" ]; then
  NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu --no-polish > $OUT/bench_c3_nopol.log 2>&1 && \
BQP_LIB=learning-based-mpc_amd/build/abship/libbqp_di3.so BQP_OCP_WPB=5 timeout -k 10 300 python bench.py --config C3 --no-cpu --no-polish > $OUT/bench_c3_occ3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 || exit $?
for f in bench_c2 bench_c3 bench_c3_nopol bench_c3_occ3 bench_c4 bench_c5; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'alone', r.get('kernel_ms_alone'), 'frac', r.get('frac'), 'two_groups', c.get('value_two_groups'), 'iters', c.get('iterations_mean'), c.get('iterations_max'), 'flags', c.get('exitflag_hist_all_ranks'), 'pol', c.get('polished_count'), 'all', c.get('value_all_instances'))"; done
# CLL A/B of the dense-kernel variants (build/abship): tile-Cholesky lookahead; + four-wave solves
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 || exit $?
for v in olddense chollook; do
  VL=learning-based-mpc_amd/build/abship/libbqp_$v.so
  [ -f $VL ] && { BQP_LIB=$VL timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_$v.log 2>&1 || exit $?; }
done
for f in bench_cll bench_cll_olddense bench_cll_chollook; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'dense_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'sqp', c.get('sqp_iterations_mean'), 'slow', c.get('x_init_vs_stored_q100_slow_max'), 'gather_dev', c.get('gather_from_device'))"; done
SL=learning-based-mpc_amd/build/stamps_ship/libbqp_stamps.so
if [ -f $SL ]; then
  BQP_STAMPS_LIB=$SL timeout -k 10 120 python3 tools/stamps.py --config C3 --json $OUT/stamps_C3.json > $OUT/stamps_c3.log 2>&1 && \
  BQP_STAMPS_LIB=$SL BQP_NO_QUEUE=1 timeout -k 10 120 python3 tools/stamps.py --config C3 --json $OUT/stamps_C3_noq.json > $OUT/stamps_c3_noq.log 2>&1 && \
  BQP_STAMPS_LIB=$SL timeout -k 10 120 python3 tools/stamps.py --json $OUT/stamps_C2.json > $OUT/stamps_c2.log 2>&1 || exit $?
  tail -14 $OUT/stamps_c3.log
fi
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for c in C2 C3 C4 C5; do
  case $c in
    C4) S="--steps 3 --warmup 1";;
    C5) S="--steps 5 --warmup 1";;
    *) S="--steps 20 --warmup 3";;
  esac
  D=$OUT/$c
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $S --no-cpu --no-two-groups --config $c > $D/bench_trace.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-two-groups --config $c > $D/pmc_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-two-groups --config $c > $D/pmc_write.log 2>&1 || exit $?
  echo "== $c"; head -4 $D/trace/run_kernel_stats.csv | cut -d, -f1-4
done
D=$OUT/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_write.log 2>&1 || exit $?
head -8 $D/trace/run_kernel_stats.csv | cut -d, -f1-5
exit $rc
