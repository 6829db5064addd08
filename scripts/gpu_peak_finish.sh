# dynamic-peak tests, then the C3 static / dynamic A/B under a kernel trace
# (per-kernel durations of k_peak_stats_v / k_peak_finish / k_tile)
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pk_finish}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/raw" -o run --output-format csv -- python3 -u "$R/scripts/bench_peak_chunk.py" 0:64 > "$OUT/ab.log" 2>&1 || { tail -5 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log"
f=$(find "$OUT/raw" -name "*kernel_stats.csv" -print -quit)
cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/raw"
grep -E "peak|k_tile" "$OUT/kernel_stats.csv" | cut -c1-160
