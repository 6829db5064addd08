set -u
bash scripts/gpu_suite.sh r04_suite3 || exit 1
bash scripts/gpu_r04_c6.sh || exit 1
