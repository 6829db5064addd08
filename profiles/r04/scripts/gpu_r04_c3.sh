set -u
mkdir -p gpurun_out/r04_ab2
timeout -k 10 120 python -u tests/diag/diag_lut177.py > gpurun_out/r04_ab2/diag_lut177.log 2>&1 || { echo diag177 failed; tail -20 gpurun_out/r04_ab2/diag_lut177.log; exit 1; }
head -3 gpurun_out/r04_ab2/diag_lut177.log
bash scripts/gpu_suite.sh r04_suite2 || exit 1
V=scripts/variants
TMS='hable bt.2390' bash scripts/gpu_ab.sh r04_ab2 $V/libh2s_notrim.so $V/libh2s_base.so $V/libh2s_dark.so $V/libh2s_notrim.so $V/libh2s_base.so $V/libh2s_dark.so || exit 1
timeout -k 10 300 python -u tests/diag/diag_c3_flips.py > gpurun_out/r04_ab2/diag_c3_flips.log 2>&1 || { echo diag failed; tail -20 gpurun_out/r04_ab2/diag_c3_flips.log; exit 1; }
cat gpurun_out/r04_ab2/diag_c3_flips.log
