# C3's lattice refetch: FETCH_SIZE with the 65^3 and the
# 2^3 lattice for C2, C3 (libplacebo), C3 on the CPU chain and C3 max-rgb;
# then frame load / store cache policies on C3 (FETCH and time)
set -u
V=scripts/variants
FETCH_CFGS="c2 c3 c3cpu c3max c2web c3web" FETCH_CTRS=FETCH_SIZE bash scripts/prof_fetch_split.sh r04_fetch || exit 1
FETCH_CFGS="c3" FETCH_CTRS=FETCH_SIZE FETCH_LIBS="nts19=$V/libh2s_nts19.so ntl19=$V/libh2s_ntl19.so nt19=$V/libh2s_nt19.so" \
  bash scripts/prof_fetch_split.sh r04_fetch_nt || exit 1
TMS='bt.2390 hable' bash scripts/gpu_ab.sh r04_nt $V/libh2s_base.so $V/libh2s_nts19.so $V/libh2s_ntl19.so $V/libh2s_nt19.so $V/libh2s_base.so || exit 1
