#!/bin/bash
# round-6 final check on the final tree: smoke, every GPU test, the default bench line (C2 with
# its CPU leg), the C3 / C4 / C5 / CLL lines, rocprofv3 kernel traces + HBM PMC passes of C2, C3
# and CLL (the kernels that changed this round; C4 / C5 run the unchanged MG instantiations)
set -o pipefail
TAG=${1:-r06_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NO_BENCH=1 bash tools/gpu_r05_check.sh $TAG
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --config C3 --no-cpu > $OUT/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu > $OUT/bench_c4.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c5.log 2>&1 && \
timeout -k 10 600 python bench.py --config CLL --steps 20 --batch 256 > $OUT/bench_cll.log 2>&1 || exit $?
for f in bench_c2 bench_c3 bench_c4 bench_c5 bench_cll; do tail -n 1 $OUT/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('check',{}); cb=d.get('cpu_baseline') or {}; print('$f', d['value'], 'ms/step', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'two_groups', c.get('value_two_groups'), 'all', c.get('value_all_instances'), 'iters', c.get('iterations_mean'), c.get('iterations_max'), 'cpu', cb.get('value'))"; done
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for c in C2 C3; do
  D=$OUT/$c
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-two-groups --config $c > $D/bench_trace.log 2>&1 || exit $?
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
exit $rc
