# one PMC pass (VALU / CVT / LDS instruction counts) of the C3 k_tile instance
# per library variant: scripts/gpu_pmc_ab.sh TAG lib_a.so lib_b.so ...
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  H2S_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_CVT SQ_WAVES -d "$OUT/$n" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-alt --cpu-seconds 0 --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo > "$OUT/$n.log" 2>&1 || { tail -5 "$OUT/$n.log"; exit 1; }
  f=$(find "$OUT/$n" -name "*counter_collection.csv" -print -quit)
  python3 - "$f" "$n" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_tile<0, 7, 0, 1, 0>' in r.get('Kernel_Name', ''):
        v[r['Counter_Name']].append(float(r['Counter_Value']))
px = 64 * 3840 * 2160
print(sys.argv[2], {k: round(sum(x) / len(x) * 64 / px, 2) for k, x in v.items()})
PY
  rm -rf "$OUT/$n"
done
