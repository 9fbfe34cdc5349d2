// mhada_gemm kernels for one (compute, A, C) dtype combination: float, float, float.
#include "gemm_impl.h"

namespace mhada {
int gemm_dispatch_f32(int mode, const GemmP& p, int nz, hipStream_t s) {
  return dispatch_mode<float, float, float>(mode, p, nz, s);
}
}  // namespace mhada
