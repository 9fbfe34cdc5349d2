// mhada_gemm kernels for one (compute, A, C) dtype combination: bf16, bf16, float.
#include "gemm_impl.h"

namespace mhada {
int gemm_dispatch_bf16_a16_o32(int mode, const GemmP& p, int nz, hipStream_t s) {
  return dispatch_mode<bf16, bf16, float>(mode, p, nz, s);
}
}  // namespace mhada
