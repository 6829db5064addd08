# LDS bank conflicts: the luma / chroma staging row stride
# (68 floats = bank shift 4 per row: 8 rows x 8 columns of a step overlap 2-way)
# against 72 / 76; conflict counters per variant, then time
set -u
OUT=$PWD/gpurun_out/r04_lds
mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/scripts/variants
for v in base st72 st76; do
  (cd /tmp && H2S_LIB=$V/libh2s_$v.so timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d $OUT/pmc_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 1 --cpu-seconds 0 --no-alt --no-sharded \
    > $OUT/pmc_$v.log 2>&1) || { echo "pmc $v failed"; tail -20 $OUT/pmc_$v.log; exit 1; }
  python3 - "$OUT/pmc_$v" "$v" <<'PY'
import csv, glob, sys
vals = {}
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_tile' in r.get('Kernel_Name', ''):
            vals.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
m = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
print(sys.argv[2], {k: round(v) for k, v in m.items()},
      'conflict share %.3f' % (m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']))
PY
done
TMS='hable' bash scripts/gpu_ab.sh r04_lds_t $V/libh2s_base.so $V/libh2s_st72.so $V/libh2s_st76.so $V/libh2s_base.so $V/libh2s_st72.so || exit 1
