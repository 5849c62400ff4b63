// k_knn_r2f.hip — kNN kernels for 0.5 m y/z grid cells (R = 2 cells per side), fused kNN + residual row + item partial (the GN tail mode).
// One translation unit per (R, fused) so the instantiations compile in parallel (fbr_gn.h).
#include "fbr_gn.h"

namespace fbr {
template void launch_gn_knn_r<2, true>(hipStream_t, const GnArgs&, int, int);
}  // namespace fbr
