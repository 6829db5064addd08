// h2s_fast_dbg345.hip — debug instances of k_tile (h2s_stage 3, 4, 5): the tile kernel's own
// arithmetic with its stage planes exported (h2s_debug_float).
#include <hip/hip_runtime.h>

#include "h2s_tile.h"

namespace h2s {

H2S_TILE_INSTANCE(3, 0)
H2S_TILE_INSTANCE(3, 1)
H2S_TILE_INSTANCE(4, 0)
H2S_TILE_INSTANCE(4, 1)
H2S_TILE_INSTANCE(5, 0)
H2S_TILE_INSTANCE(5, 1)

}  // namespace h2s
