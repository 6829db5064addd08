#!/bin/bash
# Effective clock of k_tile per variant: rocprofv3 --pmc GRBM_GUI_ACTIVE
# (sum over 8 XCDs) next to the bench's own HIP-event kernel time.
# usage: bash scripts/clock_probe.sh lib1.so lib2.so ...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "$lib" .so)
  OUT=$ROOT/gpurun_out/clk_$name; mkdir -p "$OUT"
  (cd /tmp && H2S_LIB=$ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d "$OUT" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --steps 6 --warmup 1 --cpu-seconds 0 --no-alt > "$OUT/bench.log" 2>&1) \
    || { echo "$name failed"; tail -3 "$OUT/bench.log"; exit 1; }
  python3 - "$OUT" "$name" <<'PY'
import collections, csv, glob, json, sys
out, name = sys.argv[1], sys.argv[2]
line = [l for l in open(out + '/bench.log') if l.startswith('{')][-1]
ms = json.loads(line)['roofline']['kernel_ms']
acc = collections.defaultdict(float)
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'k_tile' in row['Kernel_Name'] or 'k_quad' in row['Kernel_Name']:
            acc[(row['Counter_Name'], row['Dispatch_Id'])] += float(row['Counter_Value'])
g = sorted(v for (k, d), v in acc.items() if k == 'GRBM_GUI_ACTIVE')
b = sorted(v for (k, d), v in acc.items() if k == 'SQ_BUSY_CYCLES')
gm = g[len(g) // 2]
print(f'{name:20s} kernel {ms:.4f} ms  GRBM/8 {gm / 8:.0f} cyc  eff clock {gm / 8 / ms / 1e6:.3f} GHz  '
      f'SQ_BUSY/GRBM {b[len(b) // 2] / gm:.3f}')
PY
done
