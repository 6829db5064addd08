// h2s_fast_dbg12.hip — debug instances of k_tile (h2s_stage 1, 2): the tile kernel's own
// arithmetic with its stage planes exported (h2s_debug_float).
#include <hip/hip_runtime.h>

#include "h2s_tile.h"

namespace h2s {

H2S_TILE_INSTANCE(1, 0)
H2S_TILE_INSTANCE(1, 1)
H2S_TILE_INSTANCE(2, 0)
H2S_TILE_INSTANCE(2, 1)

}  // namespace h2s
