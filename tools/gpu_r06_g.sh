#!/bin/bash
# round-6 call g: the DI 2 x 2 LDL' factor - every GPU test, C3 bench A/B against the library
# before it (build/abship/libbqp_preldl.so), the C3 kernel trace + HBM passes of the new library
set -o pipefail
TAG=${1:-r06_g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
BQP_LIB=learning-based-mpc_amd/build/abship/libbqp_preldl.so timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3_preldl.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3_b.log 2>&1 || exit $?
for f in bench_c3 bench_c3_preldl bench_c3_b; do [ -f $OUT/$f.log ] && tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'alone', r.get('kernel_ms_alone'), 'frac', r.get('frac'), 'two_groups', c.get('value_two_groups'), 'iters', c.get('iterations_mean'), c.get('iterations_max'), 'flags', c.get('exitflag_hist_all_ranks'))"; done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=$OUT/C3
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-two-groups --config C3 > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-two-groups --config C3 > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-two-groups --config C3 > $D/pmc_write.log 2>&1 || exit $?
head -3 $D/trace/run_kernel_stats.csv | cut -d, -f1-4
exit $rc
