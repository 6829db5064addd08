set -u
OUT=gpurun_out/r04_float
mkdir -p $OUT
H2S_FLOAT_DEBUG=1 H2S_FLOAT_REPORT=$OUT/float_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py \
  -m gpu -q --timeout 120 --timeout-method thread -k "float" > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
grep -E "^E  +AssertionError" $OUT/pytest.log | sort | uniq -c | sort -rn | head -20
[ $rc -le 1 ] || exit $rc
grep -E "^  \[k_" $OUT/pytest.log | head -40
