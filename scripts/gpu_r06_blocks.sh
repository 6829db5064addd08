set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for nb in 64 256 128; do
  d=gpurun_out/r06_k6/blocks_$nb
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 scripts/bench_peak_kernel.py smooth $nb > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
  echo "== blocks $nb"
  python3 scripts/trace_by_grid.py $(find "$d" -name "*kernel_trace.csv" | head -1) k_peak_stats_q | tee "gpurun_out/r06_k6/by_grid_blocks_$nb.txt"
done
