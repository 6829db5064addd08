// h2s_fast_lp.hip — the tile kernel's product instances for the libplacebo
// branch (k_tile<..., LP = 1>), in their own translation unit so that they
// compile with LLVM's default scheduler, which measured 2-3 % faster for them
// than the max-memory-clause schedule the CPU chain's instances use
// (profiles/r03/ablations/fast_body_scheduler_*.log).
#include <hip/hip_runtime.h>

#include "h2s_tile.h"

namespace h2s {

H2S_TILE_INSTANCE(0, 1)

}  // namespace h2s
