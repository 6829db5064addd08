#!/bin/bash
# Round-2 evidence for the bench workload, each GPU step under its own limit:
# (1) PMC passes (traffic + instruction mix -> profiles/<tag>/traffic.json);
# (2) bench.py and rocprofv3 --kernel-trace --stats on ONE run (the same
#     command: bench's HIP-event kernel_ms beside rocprof's average);
# (3) L1->L2 request counters for smooth vs uniform content.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/final_r02
mkdir -p "$OUT"
bash "$ROOT/scripts/profile.sh" r02 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/same_cmd" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --no-alt --cpu-seconds 0 > "$OUT/same_cmd.log" 2>&1 || { echo "same_cmd failed"; exit 1; }
for kind in smooth uniform; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
    -d "$OUT/pmc_l1l2_$kind" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-alt --cpu-seconds 0 --kind $kind --steps 3 --warmup 1 > "$OUT/pmc_l1l2_$kind.log" 2>&1 \
    || { echo "pmc $kind failed"; exit 1; }
done
echo done
