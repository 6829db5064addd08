#!/bin/bash
# Round-5 closing run, part B: rocprofv3 kernel-trace stats and the PMC
# passes (scripts/profile.sh, one pass per run) for the C2 headline and the
# C3 libplacebo instance; the raw per-dispatch CSVs are pruned afterwards (the
# summaries, kernel stats and traffic.json stay), so that gpurun_out stays
# under the copy-back limit.  Usage: scripts/gpu_r05_prof.sh TAG
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-closing}
cd "$ROOT"
prune() {
  find "$ROOT/gpurun_out/prof_$1" -type f ! -name '*kernel_stats.csv' ! -name 'summary.txt' ! -name 'traffic.json' \
    ! -name '*.log' -delete
}
bash scripts/profile.sh "${TAG}_c2" | grep -E "^(===|.* rc=)" || exit 1
prune "${TAG}_c2"
cat "$ROOT/gpurun_out/prof_${TAG}_c2/summary.txt"
H2S_PROF_KERNEL='k_tile<0, 7, 0, 1, 0>' bash scripts/profile.sh "${TAG}_c3" --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo | grep -E "^(===|.* rc=)" || exit 1
prune "${TAG}_c3"
cat "$ROOT/gpurun_out/prof_${TAG}_c3/summary.txt"
