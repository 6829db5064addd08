#!/bin/bash
# Peak statistics kernel variants (profiles/r06/ab_patches/peak_*.patch, built
# by scripts/build_ablation.sh): the peak-detect GPU tests on each variant
# that changes results, then a kernel trace per library, alternating with the
# product.  Usage: [KINDS="smooth website"] bash scripts/gpu_r06_k.sh OUTNAME "VARIANT..." [PARITY_VARIANT...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_k}
VARS=${2:-}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
for v in ${3:-}; do
  H2S_LIB=$ROOT/scripts/variants/libh2s_$v.so timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || { tail -30 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/pytest_$v.log")"
done
for kind in ${KINDS:-smooth}; do
for round in 1 2; do
  for v in product $VARS; do
    lib=""; [ "$v" = product ] || lib=$ROOT/scripts/variants/libh2s_$v.so
    d=$OUT/trace_${kind}_${v}_$round
    H2S_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 scripts/bench_peak_kernel.py $kind \
      > "$d.log" 2>&1 || { tail -5 "$d.log"; exit 1; }
    echo "== $kind $v round $round"
    python3 scripts/trace_by_grid.py $(find "$d" -name "*kernel_trace.csv" | head -1) k_peak_stats_q | tee "$OUT/by_grid_${kind}_${v}_$round.txt"
  done
done
done
