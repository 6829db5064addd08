#!/bin/bash
# Round-6: the tile kernel's data-path ceiling (H2S_SKELETON build: no
# per-pixel arithmetic) against the product build on C2, same box, then the
# C3 libplacebo instance's PMC profile (scripts/profile.sh).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r06_skel
mkdir -p "$OUT"
cd "$ROOT"
A="--steps 300 --warmup 10 --cpu-seconds 0 --no-alt --no-sharded"
timeout -k 10 300 python -u bench.py $A > "$OUT/product.log" 2>&1 || { tail -5 "$OUT/product.log"; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/product.log').read().strip().splitlines()[-1]); print('product', d['roofline']['kernel_ms'], d['roofline']['achieved'])"
timeout -k 10 300 env H2S_LIB=$ROOT/scripts/variants/libh2s_skel.so python -u bench.py $A > "$OUT/skel.log" 2>&1 || { tail -5 "$OUT/skel.log"; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/skel.log').read().strip().splitlines()[-1]); print('skeleton', d['roofline']['kernel_ms'], d['roofline']['achieved'])"
if [ "${PROF:-1}" = 1 ]; then
  H2S_PROF_KERNEL='k_tile<0, 7, 0, 1, 0>' bash scripts/profile.sh r06_c3 --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo \
    > "$OUT/prof_c3.log" 2>&1 || { tail -20 "$OUT/prof_c3.log"; exit 1; }
  find "$ROOT/gpurun_out/prof_r06_c3" -type f ! -name '*kernel_stats.csv' ! -name 'summary.txt' ! -name 'traffic.json' ! -name '*.log' -delete
  head -50 "$ROOT/gpurun_out/prof_r06_c3/summary.txt"
fi
