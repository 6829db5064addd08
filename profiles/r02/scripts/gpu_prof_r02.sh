#!/bin/bash
# PMC traffic + kernel-trace evidence for the bench workload, then the
# multi-rank launcher rehearsal (2 ranks sharing GPU 0 over gloo).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
bash scripts/profile.sh r02 || exit $?
mkdir -p gpurun_out
H2S_DIST_BACKEND=gloo H2S_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 \
  --frames 16 --cpu-seconds 0 --no-alt > gpurun_out/bench_2rank_gloo.log 2>&1
echo "rehearsal rc=$?"
tail -3 gpurun_out/bench_2rank_gloo.log
