// k_knn_r4.hip — kNN kernels for 0.25 m y/z grid cells (R = 4 cells per side), plain kNN pass (flat queue, wide mode, per-row loop).
// One translation unit per (R, fused) so the instantiations compile in parallel (fbr_gn.h).
#include "fbr_gn.h"

namespace fbr {
template void launch_gn_knn_r<4, false>(hipStream_t, const GnArgs&, int, int);
}  // namespace fbr
