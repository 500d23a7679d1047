#!/bin/bash
# instruction-supply counters of the C2 solve kernel: the counter list, then SQ wave-cycle buckets
# and (if present) the SQC instruction-cache counters, one pass each
set -o pipefail
OUT=gpurun_out/${1:-r04_ic}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o -E "(SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_WAIT_INST[A-Z_]*|SQ_INST_LEVEL[A-Z_]*|SQC_TC_INST[A-Z_]*)" $OUT/counters.txt | sort -u > $OUT/ic_names.txt
cat $OUT/ic_names.txt | tr '\n' ' '; echo
for cfg in C2 CLL; do
  if [ $cfg = CLL ]; then B="python3 bench.py --config CLL --steps 1 --batch 256 --no-cpu"; else B="python3 bench.py --steps 2 --warmup 1 --no-cpu"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $OUT/$cfg/sq -o run -- $B > $OUT/$cfg.sq.log 2>&1 || exit $?
  if grep -q SQC_ICACHE_MISSES $OUT/ic_names.txt; then
    timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES --output-format csv -d $OUT/$cfg/ic -o run -- $B > $OUT/$cfg.ic.log 2>&1 || exit $?
  fi
  if grep -q SQ_IFETCH $OUT/ic_names.txt; then
    timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/$cfg/sq2 -o run -- $B > $OUT/$cfg.sq2.log 2>&1 || exit $?
  fi
done
for f in $(find $OUT -name "run_counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'ocp_ipm_kernel' in r['Kernel_Name'] or 'dense_ipm_kernel' in r['Kernel_Name']:
        acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
print(sys.argv[1], {k: '%.4g' % (v / n[k]) for k, v in acc.items()})
PY
done
