// mhada_gemm kernels for one (compute, A, C) dtype combination: bf16, float, bf16.
#include "gemm_impl.h"

namespace mhada {
int gemm_dispatch_bf16_a32_o16(int mode, const GemmP& p, int nz, hipStream_t s) {
  return dispatch_mode<bf16, float, bf16>(mode, p, nz, s);
}
}  // namespace mhada
