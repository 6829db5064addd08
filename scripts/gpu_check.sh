#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout (exit != 0/1) stops
# the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD... ; tolerate pytest's "tests failed" (1)
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -x -q"}
step pytest_gpu 900 python -m pytest $PYTEST_ARGS
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  cd /tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --no-alt
fi
echo ALLDONE
