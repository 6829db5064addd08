#!/bin/bash
# round-3 evidence: the rocprofv3 kernel-trace + PMC passes of the bench
# command (scripts/profile.sh), then the list of available counters
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
bash scripts/profile.sh r03 || exit $?
cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > "$ROOT/gpurun_out/prof_r03/list_avail.txt" 2>&1 || true
