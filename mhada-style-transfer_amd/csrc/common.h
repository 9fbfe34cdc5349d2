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

// ---- kernel-variant selection -------------------------------------------------------------
// The defaults are the measured winners.  The non-default variants exist for A/B measurements
// and for tests that force a rare path (e.g. the online-max bf16 attention).  The values are
// read ONCE, at the first launch, from MHADA_* environment variables, and can be changed only
// through mhada_set_tuning() (include/mhada_hip.h) — never per launch from the environment.
struct Tuning {
  int attn_fixed_shift = 1;  // bf16 softmax attention: fixed-shift kernel (0: online-max kernel)
  int attn_waves = 0;        // attention waves per workgroup: 4 | 8 as set; 0 = 8, or 4 when the 8-wave grid is smaller than the CU count
  int attn_tk = 128;         // bf16 attention keys per tile (64 | 128)
  int attn_prio = 1;         // fixed-shift kernel: s_setprio(1) for the younger wave half
  int vit_attn_vec = 1;      // bf16 batch-axis attention: vectorised form
  int out3_mfma = 1;         // bf16 last decoder layer: MFMA tile kernel (0: per-pixel VALU)
  int out3_tile = 1;         // fp32 last decoder layer: LDS-tiled kernel (0: per-pixel)
  int gemm_pp = 1;           // ping-pong GEMM kernels
  int gemm_persist = 1;      // persistent form of the ping-pong GEMM
  int gemm_pp128 = 1;        // 256x128 persistent ping-pong form for 65..128 columns
  int gemm_ldsepi = 1;       // ping-pong epilogue staged through LDS
  int gemm_n64 = 128;        // N <= 64 tile rows (128 | 256)
  int conv_c64 = 1;          // bf16 64->64 3x3 conv (+ fused upsample): direct tile kernel
  int conv_dir = 1;          // bf16 128->64 / 128->128 / 256->128 3x3 conv: direct tile kernel with a streamed weight ring (round 5)
  int gemm_rinit = 1;        // persistent ping-pong GEMM: residual + bias loaded into the accumulators
  int tn_skinny_lds = 1;     // M <= 4 conv weight gradient: LDS-tiled kernel (0: the gather kernel)
  int wino4 = 1;             // fp32 Winograd conv: 4-wave kernel (round 5; 0: the 8-wave kernel, also the fallback for inputs >= 2 GiB)
  int train_dkv_dma = 1;     // training dK/dV' with the dS spill: LDS-DMA kernel, one wave per SIMD, software-pipelined (0: round 3's)
  int upsample_quad = 1;     // bf16 bilinear x2: 2 x 2-output-block kernel (0: the 16-B per-pixel kernel)
  int xknob = 0;             // scratch knob for one-off A/B builds; no shipped kernel or dispatch reads it
};
const Tuning& tuning();

// conv_tile.hip: bf16 3x3 conv, Cin = Cout = 64, reflect pad, optional fused bilinear x2
// upsample of the input; H, W = output size.  Dispatched from mhada_gemm.
int conv3x3_c64(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, bool up, int relu,
                hipStream_t s);
// conv_tile.hip: bf16 3x3 conv, (Cin, Cout) in {(128, 64), (128, 128), (256, 128)}, reflect pad, no upsample.
int conv3x3_dir(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int cin, int cout,
                int relu, hipStream_t s);

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

// Bilinear blend in PyTorch's order, h0 * (w0 * x00 + w1 * x01) + h1 * (w0 * x10 + w1 * x11), with the
// fp32 contraction pinned (explicit fmaf), so every kernel that upsamples — the standalone
// upsample kernels, the conv tile kernel's fused halo and the implicit GEMM's UP2 gather —
// produces the same bits.
MHADA_DEV float bilerp(float ly0, float ly1, float lx0, float lx1, float x00, float x01, float x10, float x11) {
  return fmaf(ly1, fmaf(lx0, x10, lx1 * x11), ly0 * fmaf(lx0, x00, lx1 * x01));
}

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
