#!/bin/bash
# round-6 call i: every GPU test on the tree (DI reciprocals by frcp; dense kernel with the row
# state in registers), C3 A/B against the library before frcp (build/abship/libbqp_prefrcp.so),
# CLL A/B of the register row state (BQP_DENSE_NO_RG=1: the workspace form), CLL trace + PMC
set -o pipefail
TAG=${1:-r06_i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
BQP_LIB=learning-based-mpc_amd/build/abship/libbqp_prefrcp.so timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3_prefrcp.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3_b.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll.log 2>&1 && \
BQP_DENSE_NO_RG=1 timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_norg.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 --no-cpu > $OUT/bench_cll_b.log 2>&1 || exit $?
for f in bench_c3 bench_c3_prefrcp bench_c3_b; do tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'two_groups', c.get('value_two_groups'), 'iters', c.get('iterations_mean'), c.get('iterations_max'), 'flags', c.get('exitflag_hist_all_ranks'))"; done
for f in bench_cll bench_cll_norg bench_cll_b; do tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); print('$f', d['value'], 'ms/step', d['ms_per_step'], 'dense_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'sqp', c.get('sqp_iterations_mean'), 'slow', c.get('x_init_vs_stored_q100_slow_max'))"; done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
D=$OUT/CLL
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config CLL --steps 5 --batch 256 --no-cpu > $D/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_mfma -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py --config CLL --steps 2 --batch 256 --no-cpu > $D/pmc_write.log 2>&1 || exit $?
head -8 $D/trace/run_kernel_stats.csv | cut -d, -f1-5
exit $rc
