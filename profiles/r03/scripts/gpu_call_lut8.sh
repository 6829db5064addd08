#!/bin/bash
# libplacebo branch: lut3d's 8-bit path as a 2^24-entry table (one 4-byte
# gather per pixel) — the bench's other_configs lines (C3 and the LP
# variants) for HEAD's library and the new one, then the GPU suite on the new one
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_lut8
mkdir -p "$OUT"
cd "$ROOT"
for lib in scripts/variants/libh2s_base.so hdr-to-sdr_amd/hdr2sdr/libh2s.so; do
  log=$OUT/bench_$(basename $(dirname $lib)).log
  H2S_LIB=$ROOT/$lib timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-sharded > "$log" 2>&1 \
    || { echo "bench failed"; tail -5 "$log"; exit 1; }
  tail -1 "$log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], {k: v['kernel_ms'] for k, v in d['config']['other_configs'].items()})"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -4 "$OUT/pytest_gpu.log"
exit $rc
