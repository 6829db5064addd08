#!/bin/bash
# Round 6: a libplacebo-instance change (argument 2: the variant library it
# is compared against, same box, alternating), then the GPU suite with the
# parity report and the default bench.  Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r06_e}
OLD=$ROOT/${2:-scripts/variants/libh2s_r06a.so}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
NEW=$ROOT/hdr-to-sdr_amd/hdr2sdr/libh2s.so
for i in 1 2; do
  for v in new old; do
    lib=$NEW; [ $v = old ] && lib=$OLD
    timeout -k 10 200 env H2S_LIB=$lib python -u scripts/time_lp_variants_r06.py ${v}_$i >> "$OUT/lp_ab.log" 2>&1 ||
      { echo "lp $v failed"; tail -5 "$OUT/lp_ab.log"; exit 1; }
  done
done
grep '^{' "$OUT/lp_ab.log"
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
export H2S_PARITY_REPORT=$OUT/parity_report.jsonl
rm -f "$H2S_FLOAT_REPORT" "$H2S_PARITY_REPORT"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=60 -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" | cut -c1-400
fi
