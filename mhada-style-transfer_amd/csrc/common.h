// Shared definitions for the MHAda HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/mhada_hip.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define MHADA_DEV __device__ __forceinline__

namespace mhada {

// ---- error reporting (thread-local message, see mhada_last_error) -----------------------
void set_error(const std::string& msg);
int fail(const std::string& msg);  // sets message, returns MHADA_ERR_ARG
int check_launch(const char* what);  // hipGetLastError -> MHADA_ERR_LAUNCH

// ---- scalar conversions -----------------------------------------------------------------
template <typename T> MHADA_DEV float to_f32(T x);
template <> MHADA_DEV float to_f32<float>(float x) { return x; }
template <> MHADA_DEV float to_f32<bf16>(bf16 x) { return (float)x; }

template <typename T> MHADA_DEV T from_f32(float x);
template <> MHADA_DEV float from_f32<float>(float x) { return x; }
template <> MHADA_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

// 16-byte vector of T: 4 f32 or 8 bf16
template <typename T> struct Vec16;
template <> struct Vec16<float> { typedef f32x4 type; static constexpr int N = 4; };
template <> struct Vec16<bf16> { typedef bf16x8 type; static constexpr int N = 8; };

MHADA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MHADA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b, b+8, b+16 ... are dealt to one XCD; give each XCD a contiguous
// range of logical ids so neighbouring tiles (which share operands) share its L2.
MHADA_DEV int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8;
  const int xcd = bid % 8, k = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

}  // namespace mhada
