# scheduler strategy for the CPU-chain tile TU, re-checked after round 4's changes
set -u
V=scripts/variants
TMS='hable mobius' bash scripts/gpu_ab.sh r04_sched $V/libh2s_base.so $V/libh2s_schdef.so $V/libh2s_schilp.so $V/libh2s_base.so $V/libh2s_schdef.so $V/libh2s_schilp.so || exit 1
