#!/bin/bash
# Round-5 closing run, part B: rocprofv3 kernel-trace stats and the PMC
# passes (scripts/profile.sh, one pass per run) for the C2 headline and the
# C3 libplacebo instance.  Usage: scripts/gpu_r05_prof.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-closing}
cd "$ROOT"
bash scripts/profile.sh "${TAG}_c2" || exit $?
H2S_PROF_KERNEL='k_tile<0, 7, 0, 1, 0>' bash scripts/profile.sh "${TAG}_c3" --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo || exit $?
