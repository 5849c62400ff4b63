// k_knn_r1f.hip — kNN kernels for 1 m y/z grid cells (R = 1 cells per side), fused kNN + residual row + item partial (the GN tail mode).
// One translation unit per (R, fused) so the instantiations compile in parallel (fbr_gn.h).
#include "fbr_gn.h"

namespace fbr {
template void launch_gn_knn_r<1, true>(hipStream_t, const GnArgs&, int, int);
}  // namespace fbr
