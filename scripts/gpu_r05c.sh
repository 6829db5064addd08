#!/bin/bash
# Round-5 GPU call, third form: the -m gpu suite with the C3 diagnostics
# (scripts/gpu_r05.sh), the H2S_OPT_LP_EXACT modes (scripts/bench_lp_exact.py),
# the libplacebo k_tile variants (scripts/time_lp_variants.py, prebuilt under
# scripts/variants/), the peak A/B and the bench.  Each step under its own
# limit; stop at the first failure.  Usage: scripts/gpu_r05c.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}
OUT=$ROOT/gpurun_out/$TAG
cd "$ROOT"
bash scripts/gpu_r05.sh "$TAG" tests/diag/diag_c3_kernels.py tests/diag/diag_c3_bound.py || exit $?
echo "=== bench_lp_exact"
timeout -k 10 400 python -u scripts/bench_lp_exact.py --windows ${NT_WINDOWS:-3000,6000,12000} > "$OUT/bench_lp_exact.log" 2>&1 \
  || { echo "bench_lp_exact failed"; tail -20 "$OUT/bench_lp_exact.log"; exit 1; }
cat "$OUT/bench_lp_exact.log"
if [ -n "${VARIANTS:-}" ]; then
  echo "=== lp variants"
  timeout -k 10 600 python -u scripts/time_lp_variants.py $VARIANTS > "$OUT/lp_variants.log" 2>&1 \
    || { echo "lp variants failed"; tail -20 "$OUT/lp_variants.log"; exit 1; }
  cat "$OUT/lp_variants.log"
fi
if [ -n "${C2VARIANTS:-}" ]; then
  echo "=== C2 variants"
  KINDS=smooth,uniform,website TM=hable timeout -k 10 600 python -u scripts/time_variants.py $C2VARIANTS > "$OUT/c2_variants.log" 2>&1 \
    || { echo "C2 variants failed"; tail -20 "$OUT/c2_variants.log"; exit 1; }
  cat "$OUT/c2_variants.log"
fi
bash scripts/gpu_peak_ab.sh "$TAG/peak_ab" || exit $?
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
