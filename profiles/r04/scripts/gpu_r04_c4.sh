set -u
mkdir -p gpurun_out/r04_c4
rm -f gpurun_out/r04_c4/diag_lut177.log
for v in ${VARIANTS:-in-tree}; do
  if [ $v = in-tree ]; then unset H2S_LIB; else export H2S_LIB=$PWD/$v; fi
  timeout -k 10 120 python -u tests/diag/diag_lut177.py >> gpurun_out/r04_c4/diag_lut177.log 2>&1 || { echo "diag failed ($v)"; tail -20 gpurun_out/r04_c4/diag_lut177.log; exit 1; }
done
cat gpurun_out/r04_c4/diag_lut177.log
