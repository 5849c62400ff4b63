// k_knn_r4f.hip — kNN kernels for 0.25 m y/z grid cells (R = 4 cells per side), fused kNN + residual row + item partial (the GN tail mode).
// One translation unit per (R, fused) so the instantiations compile in parallel (fbr_gn.h).
#include "fbr_gn.h"

namespace fbr {
template void launch_gn_knn_r<4, true>(hipStream_t, const GnArgs&, int, int);
}  // namespace fbr
