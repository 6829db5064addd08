#!/bin/bash
# Round-5 GPU call, fourth form: the -m gpu suite with diagnostics
# (scripts/gpu_r05.sh), the libplacebo k_tile variants (VARIANTS, prebuilt
# under scripts/variants/), and the bench.  Usage: scripts/gpu_r05d.sh TAG [diag...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
OUT=$ROOT/gpurun_out/$TAG
cd "$ROOT"
bash scripts/gpu_r05.sh "$TAG" "$@" || exit $?
if [ -n "${VARIANTS:-}" ]; then
  echo "=== lp variants"
  timeout -k 10 600 python -u scripts/time_lp_variants.py $VARIANTS > "$OUT/lp_variants.log" 2>&1 \
    || { echo "lp variants failed"; tail -20 "$OUT/lp_variants.log"; exit 1; }
  cat "$OUT/lp_variants.log"
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
