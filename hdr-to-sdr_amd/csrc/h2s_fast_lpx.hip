// h2s_fast_lpx.hip — the tile kernel's near-tie instances for the libplacebo
// branch (k_tile<..., LP = 2>: BT.2390 / spline on the IPT form, listing the
// quads whose rgba8 download may round the other way for k_process's exact
// pass; H2S_OPT_LP_EXACT 1), in their own translation unit beside the LP = 1
// instances (same scheduler).
#include <hip/hip_runtime.h>

#include "h2s_tile.h"

namespace h2s {

H2S_TILE_INSTANCE(0, 2)

}  // namespace h2s
