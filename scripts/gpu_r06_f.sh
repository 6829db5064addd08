#!/bin/bash
# Round 6: the GPU suite (parity / float reports), the default bench and the
# peak-statistics timing (plain and under a kernel trace).  Stops at the
# first failure.  Usage: scripts/gpu_r06_f.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r06_f}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
BENCH=0 bash scripts/gpu_r06_e.sh "$TAG" scripts/variants/libh2s_r06a.so || exit $?
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 200 python -u scripts/bench_peak_stats.py > "$OUT/bench_peak.log" 2>&1 || { tail -5 "$OUT/bench_peak.log"; exit 1; }
tail -1 "$OUT/bench_peak.log"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 scripts/bench_peak_stats.py \
  > "$OUT/trace.log" 2>&1 || { tail -5 "$OUT/trace.log"; exit 1; }
python3 scripts/trace_by_grid.py $(find "$OUT/trace" -name "*kernel_trace.csv" | head -1) peak | tee "$OUT/trace_by_grid.txt"
