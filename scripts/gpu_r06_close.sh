#!/bin/bash
# Round-6 closing run at the final tree.  Part A (default): the -m gpu suite
# with the parity and float reports, smoke(), the default bench line, the
# peak-statistics kernel trace.  Part B (PART=B): scripts/profile.sh for C2
# and for C3 (warm kernel trace + PMC passes).  Outputs under
# gpurun_out/TAG/.  Stops at the first failure.  Usage: scripts/gpu_r06_close.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-closing}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${PART:-A}" = A ]; then
  export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
  export H2S_PARITY_REPORT=$OUT/parity_report.jsonl
  rm -f "$H2S_FLOAT_REPORT" "$H2S_PARITY_REPORT"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
  echo "=== smoke"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  echo "=== bench"
  timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"
  cut -c1-300 "$OUT/bench.json"
  echo "=== peak statistics trace"
  export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/peak_trace" -o run --output-format csv -- python3 scripts/bench_peak_stats.py \
    > "$OUT/peak_trace.log" 2>&1 || { tail -5 "$OUT/peak_trace.log"; exit 1; }
  python3 scripts/trace_by_grid.py $(find "$OUT/peak_trace" -name "*kernel_trace.csv" | head -1) peak | tee "$OUT/peak_trace_by_grid.txt"
else
  bash scripts/profile.sh "${TAG}_c2" || exit 1
  H2S_PROF_KERNEL='k_tile<0, 7, 0, 1, 0>' bash scripts/profile.sh "${TAG}_c3" --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo || exit 1
  # keep the summaries, the kernel-trace CSVs and the logs (the PMC CSVs are large)
  for t in c2 c3; do
    find "$ROOT/gpurun_out/prof_${TAG}_$t" -type f -name '*counter_collection.csv' -delete
  done
fi
