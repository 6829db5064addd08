# final check at the final tree: the -m gpu suite, smoke(), then the
# tiles-per-block sweep (scripts/bench_tpb.py)
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_final}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -8 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > "$OUT/smoke.log" 2>&1 || { tail -8 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u scripts/bench_tpb.py > "$OUT/tpb.log" 2>&1 || { tail -5 "$OUT/tpb.log"; exit 1; }
tail -1 "$OUT/tpb.log"
