# C3 (libplacebo branch, BT.2390, IPT) counters at the final tree
set -u
bash scripts/profile.sh r04c3 --tonemapper bt.2390 --gamma 1.0 || exit 1
