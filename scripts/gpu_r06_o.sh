#!/bin/bash
# Dynamic-peak overhead of a library variant (profiles/r06/ab_patches/*.patch,
# scripts/build_ablation.sh): the peak-detect GPU tests on the variant, then
# scripts/bench_peak_stats.py under a kernel trace for product and variant,
# alternating, two rounds (per-kernel averages by launch shape).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_o}
V=${2:-peak_fastpow}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
H2S_LIB=$ROOT/scripts/variants/libh2s_$V.so timeout -k 10 400 python -u -m pytest tests/test_peak_detect.py tests/test_dist_gpu.py \
  tests/test_website_fixture.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$V.log" 2>&1 || { tail -30 "$OUT/pytest_$V.log"; exit 1; }
echo "$V: $(tail -1 "$OUT/pytest_$V.log")"
for i in 1 2; do
  for v in product $V; do
    lib=""; [ $v != product ] && lib=$ROOT/scripts/variants/libh2s_$v.so
    d=$OUT/trace_${v}_$i
    H2S_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 scripts/bench_peak_stats.py \
      > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
    echo "== $v $i $(tail -1 "$d.log" | cut -c1-200)"
    python3 scripts/trace_by_grid.py $(find "$d" -name "*kernel_trace.csv" | head -1) k_peak_finish | tee "$OUT/by_grid_${v}_$i.txt"
  done
done
