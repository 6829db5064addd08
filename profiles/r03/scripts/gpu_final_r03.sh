#!/bin/bash
# round-3 closing evidence at HEAD: smoke(), the -m gpu suite, the default
# bench line (the driver's command), then the rocprofv3 kernel-trace + PMC
# passes of the bench workload (scripts/profile.sh).  Each GPU step under its
# own limit; stop at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_final_head
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
rm -f "$H2S_FLOAT_REPORT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -20 "$OUT/pytest_gpu.log"; exit 1; }
unset H2S_FLOAT_REPORT
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
bash scripts/profile.sh r03h > "$OUT/profile.log" 2>&1 || { echo "profile failed"; tail -30 "$OUT/profile.log"; exit 1; }
tail -45 "$OUT/profile.log"
