set -u
mkdir -p gpurun_out/r04_drift
V=scripts/variants
timeout -k 10 600 python -u tests/diag/diag_trim_drift.py $V/libh2s_notrim.so $V/libh2s_base.so > gpurun_out/r04_drift/trim_drift.log 2>&1 || { echo drift failed; tail -20 gpurun_out/r04_drift/trim_drift.log; exit 1; }
cat gpurun_out/r04_drift/trim_drift.log
