#!/bin/bash
# Round-6 A/B: the packed 8-byte Y'CbCr lattice (H2S_PACKED_LUT variant,
# scripts/build_variants.sh) against the product build on C2 (smooth,
# uniform, the website frame) and the sharded C4 / C5 workloads, plus the
# variant's parity on the CPU-chain GPU tests.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r06_packed
mkdir -p "$OUT"
cd "$ROOT"
V=$ROOT/scripts/variants/libh2s_packed.so
timeout -k 10 400 env H2S_LIB=$V python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -k "not libplacebo and not lp_exact and not C3 and not spline and not bt2390" \
  > "$OUT/pytest_packed.log" 2>&1 || { tail -30 "$OUT/pytest_packed.log"; exit 1; }
tail -2 "$OUT/pytest_packed.log"
A="--steps 300 --warmup 10 --cpu-seconds 0"
for r in 1 2; do
  for lib in product packed; do
    L=""; [ $lib = packed ] && L="H2S_LIB=$V"
    timeout -k 10 300 env $L python -u bench.py $A > "$OUT/${lib}_$r.log" 2>&1 || { tail -5 "$OUT/${lib}_$r.log"; exit 1; }
    python3 - "$OUT/${lib}_$r.log" $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d['config']
print(sys.argv[2], 'C2', d['roofline']['kernel_ms'], 'uniform', c['alt_content']['kernel_ms'], 'website', c['real_content']['kernel_ms'],
      'C4', c['other_configs']['C4']['kernel_ms'], 'C5', c['other_configs']['C5']['kernel_ms'], 'C1', c['other_configs']['C1']['kernel_ms'])
PY
  done
done
