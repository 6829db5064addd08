#!/bin/bash
# Round-5 GPU call, second form: the -m gpu suite (scripts/gpu_r05.sh), then
# the peak A/B (scripts/gpu_peak_ab.sh) and the bench.  Usage: scripts/gpu_r05b.sh TAG [diag...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
cd "$ROOT"
bash scripts/gpu_r05.sh "$TAG" "$@" || exit $?
bash scripts/gpu_peak_ab.sh "$TAG/peak_ab" || exit $?
timeout -k 10 400 python -u bench.py > "gpurun_out/$TAG/bench.log" 2>&1 || { echo "bench failed"; tail -5 "gpurun_out/$TAG/bench.log"; exit 1; }
tail -1 "gpurun_out/$TAG/bench.log" | cut -c1-300
