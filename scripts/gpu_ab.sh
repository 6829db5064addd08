#!/bin/bash
# One GPU call timing prebuilt libh2s variants (scripts/build_variants.sh) on
# the C2 workload (and, with TMS, other operators), outputs diffed against the
# first variant.  Usage: scripts/gpu_ab.sh TAG lib1.so lib2.so ...
# env: TMS (default "hable"), KINDS (default smooth,uniform,website), BENCH=1
# to also run the default bench line first.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-ab}; shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log"
fi
export KINDS=${KINDS:-smooth,uniform,website}
for tm in ${TMS:-hable}; do
  rm -f /tmp/ref_${tm}_*.npy
  TM=$tm timeout -k 10 600 python -u scripts/time_variants.py "$@" > "$OUT/ab_$tm.log" 2>&1 \
    || { echo "time_variants $tm failed"; tail -20 "$OUT/ab_$tm.log"; exit 1; }
  echo "== $tm"; cat "$OUT/ab_$tm.log"
done
