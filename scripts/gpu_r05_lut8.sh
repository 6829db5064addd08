# round-5 A/Bs: the LP lut3d 8-bit coordinate table (base = per pixel, tab =
# table) and the peak statistics' loads in flight (base 2, inf4, inf8)
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_lut8}
mkdir -p "$OUT"
cd "$R"
V=scripts/variants
timeout -k 10 400 python -u scripts/time_lp_variants.py $V/libh2s_base.so $V/libh2s_tab.so $V/libh2s_base.so $V/libh2s_tab.so > "$OUT/lp.log" 2>&1 || { tail -5 "$OUT/lp.log"; exit 1; }
cat "$OUT/lp.log"
for v in base inf4 inf8; do
  H2S_LIB=$R/$V/libh2s_$v.so timeout -k 10 200 python -u scripts/bench_peak_chunk.py 0:64 > "$OUT/peak_$v.log" 2>&1 || { tail -5 "$OUT/peak_$v.log"; exit 1; }
  echo "$v $(tail -1 "$OUT/peak_$v.log")"
done
timeout -k 10 600 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_peak_detect.py tests/test_gpu_switches.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
