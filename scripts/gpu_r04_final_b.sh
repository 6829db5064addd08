# round-4 closing evidence, part B: rocprofv3 kernel trace + PMC passes of the
# bench command (TD busy, LDS bank conflicts, VALU / TRANS per pixel), then the
# C3 lattice-refetch split and the frame cache-policy A/B
set -u
bash scripts/profile.sh r04 || exit 1
bash scripts/gpu_r04_c6.sh || exit 1
