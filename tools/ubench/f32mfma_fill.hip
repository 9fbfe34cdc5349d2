// Microbenchmark: does VALU work issued by the SAME wave hide under v_mfma_f32_32x32x2_f32?
// One wave per SIMD (4 waves per workgroup, one workgroup per CU); each wave runs ITERS
// iterations of 4 independent-accumulator MFMAs with F independent v_add_f32 after each MFMA.
// Reports shader cycles per MFMA (s_memtime deltas, clock-independent).  Also the bf16
// 32x32x16 and the f32 16x16x4 forms for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int F, int KIND>
__global__ void __launch_bounds__(256, 1) kern(float* out, unsigned long long* cyc, int iters) {
  f32x16 acc[4];
  f32x4 acc4[4];
  for (int i = 0; i < 4; ++i) { acc[i] = (f32x16)0.f; acc4[i] = (f32x4)0.f; }
  float a = threadIdx.x * 1e-3f, b = 1.f + threadIdx.x * 1e-4f;
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = i * 0.5f + threadIdx.x;
  bf16x8 ab, bb;
  for (int i = 0; i < 8; ++i) { ab[i] = (__bf16)(a + i); bb[i] = (__bf16)(b - i); }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if constexpr (KIND == 0) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m], 0, 0, 0);
      else if constexpr (KIND == 1) acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc[m], 0, 0, 0);
      else acc4[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc4[m], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < F; ++f) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[f & 15]) : "v"(b));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][15] + acc4[i][0];
  for (int i = 0; i < 16; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int F, int KIND>
void run(float* out, unsigned long long* cyc, int ncu, const char* name) {
  const int iters = 2000;
  hipLaunchKernelGGL((kern<F, KIND>), dim3(ncu), dim3(256), 0, 0, out, cyc, iters);
  hipLaunchKernelGGL((kern<F, KIND>), dim3(ncu), dim3(256), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(ncu * 4);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto x : h) s += (double)x;
  s /= h.size();
  printf("%-22s fillers/MFMA %2d: %7.1f cycles per MFMA\n", name, F, s / (iters * 4.0));
}

int main() {
  int ncu = 256;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, ncu * 256 * 4);
  hipMalloc(&cyc, ncu * 4 * 8);
  run<0, 0>(out, cyc, ncu, "f32 32x32x2");
  run<2, 0>(out, cyc, ncu, "f32 32x32x2");
  run<4, 0>(out, cyc, ncu, "f32 32x32x2");
  run<8, 0>(out, cyc, ncu, "f32 32x32x2");
  run<12, 0>(out, cyc, ncu, "f32 32x32x2");
  run<16, 0>(out, cyc, ncu, "f32 32x32x2");
  run<0, 1>(out, cyc, ncu, "bf16 32x32x16");
  run<4, 1>(out, cyc, ncu, "bf16 32x32x16");
  run<8, 1>(out, cyc, ncu, "bf16 32x32x16");
  run<0, 2>(out, cyc, ncu, "f32 16x16x4");
  run<4, 2>(out, cyc, ncu, "f32 16x16x4");
  run<8, 2>(out, cyc, ncu, "f32 16x16x4");
  hipFree(out);
  hipFree(cyc);
  return 0;
}
