// mhada_gemm kernels for one (compute, A, C) dtype combination: bf16, float, float.
#include "gemm_impl.h"

namespace mhada {
int gemm_dispatch_bf16_a32_o32(int mode, const GemmP& p, int nz, hipStream_t s) {
  return dispatch_mode<bf16, float, float>(mode, p, nz, s);
}
}  // namespace mhada
