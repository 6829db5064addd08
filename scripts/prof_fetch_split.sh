#!/bin/bash
# Split k_tile's FETCH_SIZE into frame streaming and lattice refetches
# (VERDICT r03 item 6): the same 64-frame launch with the 65^3 lattice and
# with a 2^3 lattice (96 B: always cache-resident), for C2 (Hable) and C3
# (BT.2390, libplacebo branch).  FETCH_SIZE counts Infinity-Cache hits too
# (MI355X_MICROARCH.md, HBM section), so the difference is the lattice lines
# the L2 re-fetched, wherever they were served from.  One --pmc pass per run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-fetch_split}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
CFGS=${FETCH_CFGS:-"c2 c3"}
# FETCH_LIBS: "tag=path ..." library variants (H2S_LIB), default the in-tree one
for lv in ${FETCH_LIBS:-base=}; do
lt=${lv%%=*}; lp=${lv#*=}
if [ -n "$lp" ]; then export H2S_LIB=$ROOT/$lp; else unset H2S_LIB; fi
for name in $CFGS; do
  case $name in
    c2) cfg="c2 --tonemapper hable --gamma 2.2" ;;
    c3) cfg="c3 --tonemapper bt.2390 --gamma 1.0" ;;
    c3cpu) cfg="c3cpu --tonemapper bt.2390 --gamma 1.0 --pipeline cpu" ;;
    c3max) cfg="c3max --tonemapper bt.2390 --gamma 1.0 --lp-tone max-rgb" ;;
    c3hable) cfg="c3hable --tonemapper hable --gamma 1.0 --pipeline libplacebo" ;;
    c2web) cfg="c2web --tonemapper hable --gamma 2.2 --kind website" ;;
    c3web) cfg="c3web --tonemapper bt.2390 --gamma 1.0 --kind website" ;;
  esac
  set -- $cfg; name=$1; shift
  for lut in 65 2; do
    for ctr in ${FETCH_CTRS:-FETCH_SIZE WRITE_SIZE}; do
      tag=${lt}.${name}_lut${lut}_${ctr}
      timeout -k 10 240 rocprofv3 --pmc $ctr -d "$OUT/$tag" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --steps 6 --warmup 1 --cpu-seconds 0 --no-alt --no-sharded --lut $lut "$@" \
        > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -20 "$OUT/$tag.log"; exit 1; }
      echo "$tag done"
    done
  done
done
done
python3 "$ROOT/scripts/fetch_split_summary.py" "$OUT" | tee "$OUT/summary.txt"
