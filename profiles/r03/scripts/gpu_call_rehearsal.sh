#!/bin/bash
# two ranks sharing the box's one GPU over gloo (the N>1 flow incl. the
# sharded C4 / C5 lines; not a scaling figure), then smoke()
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_rehearsal
mkdir -p "$OUT"
cd "$ROOT"
H2S_DIST_BACKEND=gloo H2S_BENCH_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus 2 --steps 50 --warmup 5 \
  > "$OUT/bench_2rank_gloo.log" 2>&1 || { echo "rehearsal failed"; tail -20 "$OUT/bench_2rank_gloo.log"; exit 1; }
tail -1 "$OUT/bench_2rank_gloo.log" | cut -c1-600
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
