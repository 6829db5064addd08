# A/B of the round-4 VALU trims and the dark-exact path: timing (C2 Hable,
# C3 BT.2390) and the k_tile float-stage report on the ramp, per variant
set -u
V=scripts/variants
OUT=gpurun_out/r04_ab4
mkdir -p $OUT
TMS='hable bt.2390' bash scripts/gpu_ab.sh r04_ab4 $V/libh2s_base.so $V/libh2s_dark.so $V/libh2s_base.so $V/libh2s_dark.so || exit 1
for v in base dark; do
  H2S_LIB=$PWD/$V/libh2s_$v.so H2S_FLOAT_REPORT=$OUT/float_$v.jsonl H2S_FLOOR_ONLY_MAX=1 \
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
    -k "float_intermediates and k_tile and (ramp or uniform)" > $OUT/float_$v.log 2>&1
  rc=$?   # 1 = assertion failures (a report, go on); anything else stops the call
  [ $rc -le 1 ] || { echo "float $v rc=$rc"; tail -5 $OUT/float_$v.log; exit 1; }
  tail -1 $OUT/float_$v.log
done
timeout -k 10 300 python -u tests/diag/diag_c3_flips.py > $OUT/diag_c3_flips.log 2>&1 || { echo diag failed; tail -20 $OUT/diag_c3_flips.log; exit 1; }
cat $OUT/diag_c3_flips.log
