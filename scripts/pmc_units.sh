#!/bin/bash
# usage: pmc.sh LIB TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
LIB=$1; TAG=$2
OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p $OUT
export TMPDIR=/tmp H2S_LIB=$ROOT/$LIB
cd /tmp
ARGS="--steps 4 --warmup 1 --cpu-seconds 0 --no-alt"
i=0
for set in "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'k_tile' not in row.get('Kernel_Name', '') and 'k_quad' not in row.get('Kernel_Name', ''): continue
        acc[(row['Counter_Name'], row['Dispatch_Id'])].append(float(row['Counter_Value']))
tot = collections.defaultdict(list)
for (name, d), v in acc.items(): tot[name].append(sum(v))
for name in sorted(tot): print(f'{name:40s} {sum(tot[name])/len(tot[name]):16.1f}  (n={len(tot[name])})')
PY
