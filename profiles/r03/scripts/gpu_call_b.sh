#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$ROOT/scripts/gpu_wave_ab.sh" r03_b_wave || exit $?
bash "$ROOT/scripts/gpu_suite.sh" r03_b_suite
