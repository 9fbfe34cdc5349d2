// fp32 3x3 convolution as Winograd F(2x2, 3x3) on the fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the fp32 Conv2d(k=3) calls of the decoder (ReflectionPad2d(1) + conv, conv.py:23-33,
// 36-45, 61-72) and of VGG19 (zero padding 1, vgg19.py:15-70), and the input-gradient convs of
// the training step (zero padding 1 / the pad-2 full correlation, train_image.py:139).
//
// Why: fp32 MFMA is 1/16 of the bf16 rate, so at fp32 the direct product is MFMA bound (the
// implicit GEMM runs these layers at ~76 % of the 157 TF/s fp32 peak).  F(2x2,3x3) computes a
// 2x2 output tile from a 4x4 input tile with 16 products per (input channel, output channel)
// instead of 36: 2.25x fewer MFMA FLOPs.  Transforms (Lavin & Gray 2016):
//   V = B^T d B  (input 4x4)   U = G g G^T  (3x3 filter -> 4x4)   Y = A^T (U . V) A  (2x2)
// and for each of the 16 positions xi the channel reduction M_xi[tile][co] = sum_ci V_xi[tile][ci]
// U_xi[ci][co] is a GEMM; all 16 run here inside one workgroup, so V and M never touch HBM.
// The transforms only add/subtract (G's 1/2 is exact), so the result is the direct
// correlation up to fp32 rounding of 4-term sums.
//
// Workgroup = 4 waves (one per SIMD) = 32 Winograd tiles (4 x 8 tiles = 8 x 16 output pixels)
// x 64 output channels.  Wave w owns the four positions xi = (i = w, j = 0..3): 8 accumulator
// blocks (32 tiles x 32 channels) = 128 registers.  Per 8-channel chunk of the input:
//   * each thread loads its (tile, channel) 4x4 input patch (padding resolved on load) and the
//     U slice [16][64 co][8 ci] (contiguous 32 KiB, prepacked by mhada_wino_weights), issued one
//     chunk ahead into registers;
//   * after the current chunk's MFMAs it transforms the patch and writes V[16][32][8] and U into
//     the other LDS buffer (rows padded to 48 B: conflict-free ds_read_b128 down 16 rows);
//   * per chunk a wave runs 32 MFMAs (4 k-steps x 4 xi x 2 channel blocks; k-step s of lane half
//     h takes channel 4h + s, read as one ds_read_b128 for A and for B).
// Epilogue: each wave reduces its row i of the 4x4 grid along j (P_i = M_i. A), the four row
// partials meet in LDS, and Y = A^T P + bias (+ReLU) is stored as 64-channel pixel rows.
#include "common.h"

#ifndef WINO_DBG
#define WINO_DBG 0  // ablation builds (tools/wino_dbg.py): 1 no MFMA, 2 no loads, 4 no transform/LDS stores
#endif

namespace mhada {

namespace {
constexpr int kTY = 4, kTX = 8, kTT = kTY * kTX;  // tiles per workgroup
constexpr int kCO = 64;                            // output channels per workgroup
constexpr int kCK = 8;                             // input channels per chunk
constexpr int kLR = 12;                            // LDS row: 8 floats + 4 pad (48 B)
constexpr int kVS = 16 * kTT * kLR;                // V buffer (floats)
constexpr int kUS = 16 * kCO * kLR;                // U buffer (floats)
constexpr int kStage = kVS + kUS;                  // 18432 floats = 72 KiB
constexpr int kLE = kCO + 4;                       // epilogue row stride (floats)
static_assert(8 * kTT * kLE <= 2 * kStage, "epilogue exchange must fit the staging buffers");

struct WinoP {
  const float* x;     // NHWC [B][H][W][Cin]
  const float* u;     // [Cin/8][16][Cout][8]
  const float* bias;  // [Cout] or null
  float* y;           // NHWC [B][Ho][Wo][ldc]
  int B, H, W, Cin, Cout, Ho, Wo, pad, zero, relu;
  long long ldc;
  int nbx, nby, nbn, nblk;
};

MHADA_DEV int reflect_clamp(int v, int n) {
  v = v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
  return min(max(v, 0), n - 1);
}

__global__ void __launch_bounds__(256, 1) wino_kernel(const WinoP p) {
  __shared__ __attribute__((aligned(16))) float lds[2 * kStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;

  // logical block: output-channel block fastest (neighbours share the input patch in L2)
  int id = xcd_remap(blockIdx.x, p.nblk);
  const int nb = id % p.nbn;
  id /= p.nbn;
  const int bx = id % p.nbx;
  id /= p.nbx;
  const int by = id % p.nby;
  const int b = id / p.nby;
  const int co0 = nb * kCO;

  // this thread's transform item: tile t, channel c of the chunk
  const int tc = tid & 7, tt = tid >> 3;
  const int ty = by * kTY + (tt >> 3), tx = bx * kTX + (tt & 7);
  const int P = p.zero ? p.pad : 1;
  int off[16];
  bool inb[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int iy = 2 * ty - P + i, ix = 2 * tx - P + j;
      bool ok = true;
      if (p.zero) {
        ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
        iy = min(max(iy, 0), p.H - 1);
        ix = min(max(ix, 0), p.W - 1);
      } else {
        iy = reflect_clamp(iy, p.H);
        ix = reflect_clamp(ix, p.W);
      }
      off[4 * i + j] = ((b * p.H + iy) * p.W + ix) * p.Cin + tc;
      inb[4 * i + j] = ok;
    }

  struct Stage {
    float d[16];
    f32x4 us[8];
  };
  const float* ub = p.u + (long long)co0 * 8;
  const long long ustride = (long long)16 * p.Cout * 8;  // floats per 8-channel chunk
  const int nck = p.Cin / kCK;
  // loads of chunk min(k, nck-1): clamped so every issue is unconditional (straight-line code
  // keeps the compiler's vmcnt tracking exact); surplus chunks land in a buffer nobody reads
  auto issue = [&](Stage& r, int k) {
#if WINO_DBG & 2
    return;
#endif
    k = min(k, nck - 1);
    const float* xc = p.x + k * kCK;
#pragma unroll
    for (int e = 0; e < 16; ++e) r.d[e] = xc[off[e]];  // clamped address, unconditional load
    const float* uc = ub + k * ustride;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 256 * i;  // (xi, co, half): 16 x 64 x 2 chunks of 16 B
      const int xi = idx >> 7, rem = idx & 127;
      r.us[i] = *reinterpret_cast<const f32x4*>(uc + (long long)xi * p.Cout * 8 + rem * 4);
    }
  };
  auto commit = [&](Stage& r, float* st) {
#if WINO_DBG & 4
    return;
#endif
    // zero padding applied here, not at the load: nothing consumes the loads before the MFMAs,
    // so they stay in flight across them (a select next to the load made the compiler wait)
    float d[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) d[e] = inb[e] ? r.d[e] : 0.f;
    // V = B^T d B
    float t[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[0 * 4 + j] = d[0 * 4 + j] - d[2 * 4 + j];
      t[1 * 4 + j] = d[1 * 4 + j] + d[2 * 4 + j];
      t[2 * 4 + j] = d[2 * 4 + j] - d[1 * 4 + j];
      t[3 * 4 + j] = d[1 * 4 + j] - d[3 * 4 + j];
    }
    float* sv = st + tt * kLR + tc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v0 = t[4 * i + 0] - t[4 * i + 2];
      const float v1 = t[4 * i + 1] + t[4 * i + 2];
      const float v2 = t[4 * i + 2] - t[4 * i + 1];
      const float v3 = t[4 * i + 1] - t[4 * i + 3];
      sv[(4 * i + 0) * kTT * kLR] = v0;
      sv[(4 * i + 1) * kTT * kLR] = v1;
      sv[(4 * i + 2) * kTT * kLR] = v2;
      sv[(4 * i + 3) * kTT * kLR] = v3;
    }
    float* su = st + kVS;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + 256 * i;
      const int xi = idx >> 7, co = (idx >> 1) & 63, half = idx & 1;
      *reinterpret_cast<f32x4*>(su + (xi * kCO + co) * kLR + 4 * half) = r.us[i];
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][n][e] = 0.f;

  auto mfmas = [&](const float* st) {
#if WINO_DBG & 1
    return;
#endif
    f32x4 av[4], bv[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int xi = 4 * wave + j;
      av[j] = *reinterpret_cast<const f32x4*>(st + (xi * kTT + r32) * kLR + 4 * h);
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bv[j][n] = *reinterpret_cast<const f32x4*>(st + kVS + (xi * kCO + 32 * n + r32) * kLR + 4 * h);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[j][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j][s], bv[j][n][s], acc[j][n], 0, 0, 0);
  };
  // Two chunks of loads in flight (one MFMA phase does not cover an L2-miss latency): chunk c is
  // staged in register set c & 1; step k runs chunk k's MFMAs, then commits chunk k+1 (loaded
  // two steps earlier) and reuses its registers for chunk k+3.  The loop is unrolled by two so
  // the register sets stay static.
  Stage r0, r1;
  float* buf0 = lds;
  float* buf1 = lds + kStage;
  issue(r0, 0);
  commit(r0, buf0);
  issue(r1, 1);
  issue(r0, 2);
  __syncthreads();
  auto step = [&](const float* cur, Stage& r, float* nxt, int knext) {
    __builtin_amdgcn_sched_barrier(0);
    mfmas(cur);
    __builtin_amdgcn_sched_barrier(0);
    commit(r, nxt);
    issue(r, knext);
    __syncthreads();
  };
  for (int k = 0; k + 1 < nck; k += 2) {
    step(buf0, r1, buf1, k + 3);
    step(buf1, r0, buf0, k + 4);
  }
  if (nck & 1) mfmas(buf0);
  __syncthreads();

  // row partials P_w[q] = sum_j M[w][j] A[j][q]  (A^T = [[1,1,1,0],[0,1,-1,-1]])
  float* ex = lds;  // [w*2+q][tile][kLE]
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int tile = (r & 3) + 8 * (r >> 2) + 4 * h, co = 32 * n + r32;
      const float m0 = acc[0][n][r], m1 = acc[1][n][r], m2 = acc[2][n][r], m3 = acc[3][n][r];
      ex[((2 * wave + 0) * kTT + tile) * kLE + co] = m0 + m1 + m2;
      ex[((2 * wave + 1) * kTT + tile) * kLE + co] = m1 - m2 - m3;
    }
  __syncthreads();
  const int co = tid & 63;
  const float bias = p.bias ? p.bias[co0 + co] : 0.f;
#pragma unroll
  for (int it = 0; it < kTT / 4; ++it) {
    const int tile = (tid >> 6) + 4 * it;
    const int oy0 = 2 * (by * kTY + (tile >> 3)), ox0 = 2 * (bx * kTX + (tile & 7));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float p0 = ex[((0 + q) * kTT + tile) * kLE + co];
      const float p1 = ex[((2 + q) * kTT + tile) * kLE + co];
      const float p2 = ex[((4 + q) * kTT + tile) * kLE + co];
      const float p3 = ex[((6 + q) * kTT + tile) * kLE + co];
      float y0 = p0 + p1 + p2 + bias, y1 = p1 - p2 - p3 + bias;
      if (p.relu) {
        y0 = fmaxf(y0, 0.f);
        y1 = fmaxf(y1, 0.f);
      }
      const int ox = ox0 + q;
      if (ox < p.Wo) {
        if (oy0 < p.Ho) p.y[((long long)(b * p.Ho + oy0) * p.Wo + ox) * p.ldc + co0 + co] = y0;
        if (oy0 + 1 < p.Ho) p.y[((long long)(b * p.Ho + oy0 + 1) * p.Wo + ox) * p.ldc + co0 + co] = y1;
      }
    }
  }
}

// U = G g G^T per (co, ci); w [Cout][3][3][Cin] -> u [Cin/8][16][Cout][8]
__global__ void wino_weights_kernel(const float* __restrict__ w, float* __restrict__ u, int Cout, int Cin) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)Cout * Cin) return;
  const int ci = (int)(i % Cin), co = (int)(i / Cin);
  float g[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t] = w[((long long)co * 9 + t) * Cin + ci];
  float gg[12];  // (G g)[i][kx]
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float a = g[kx], bb = g[3 + kx], c = g[6 + kx];
    gg[0 * 3 + kx] = a;
    gg[1 * 3 + kx] = 0.5f * (a + bb + c);
    gg[2 * 3 + kx] = 0.5f * (a - bb + c);
    gg[3 * 3 + kx] = c;
  }
  float* ub = u + ((long long)(ci >> 3) * 16 * Cout + co) * 8 + (ci & 7);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float a = gg[3 * r], bb = gg[3 * r + 1], c = gg[3 * r + 2];
    const float v[4] = {a, 0.5f * (a + bb + c), 0.5f * (a - bb + c), c};
#pragma unroll
    for (int j = 0; j < 4; ++j) ub[(long long)(4 * r + j) * Cout * 8] = v[j];
  }
}
}  // namespace

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_wino_weights(const float* w, float* u, int Cout, int Cin, mhada_stream_t s_) {
  if (!w || !u || Cout <= 0 || Cin <= 0 || Cin % 8) return fail("mhada_wino_weights: bad args (Cin % 8 == 0)");
  const long long n = (long long)Cout * Cin;
  hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s_, w, u,
                     Cout, Cin);
  return check_launch("mhada_wino_weights");
}

extern "C" int mhada_conv3x3_wino(const float* x, const float* u, const float* bias, float* y, int B, int H, int W,
                                  int Cin, int Cout, long long ldc, int pad_mode, int pad, int relu,
                                  mhada_stream_t s_) {
  if (!x || !u || !y || B <= 0 || H < 2 || W < 2 || Cin <= 0 || Cout <= 0)
    return fail("mhada_conv3x3_wino: bad args");
  if (Cin % kCK || Cout % kCO) return fail("mhada_conv3x3_wino: needs Cin % 8 == 0 and Cout % 64 == 0");
  if (pad_mode != MHADA_PAD_REFLECT && pad_mode != MHADA_PAD_ZERO) return fail("mhada_conv3x3_wino: bad pad_mode");
  if (pad_mode == MHADA_PAD_ZERO && pad != 1 && pad != 2) return fail("mhada_conv3x3_wino: zero pad must be 1 or 2");
  if (ldc < Cout) return fail("mhada_conv3x3_wino: ldc < Cout");
  WinoP p;
  p.x = x; p.u = u; p.bias = bias; p.y = y;
  p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.zero = pad_mode == MHADA_PAD_ZERO;
  p.pad = p.zero ? pad : 1;
  p.Ho = p.zero ? H + 2 * (pad - 1) : H;
  p.Wo = p.zero ? W + 2 * (pad - 1) : W;
  p.relu = relu;
  p.ldc = ldc;
  const int TY = (p.Ho + 1) / 2, TX = (p.Wo + 1) / 2;
  p.nby = (TY + kTY - 1) / kTY;
  p.nbx = (TX + kTX - 1) / kTX;
  p.nbn = Cout / kCO;
  const long long nblk = (long long)B * p.nby * p.nbx * p.nbn;
  if (nblk > (1LL << 31) - 1 || (long long)B * H * W * Cin > (1LL << 31) - 1)
    return fail("mhada_conv3x3_wino: problem too large for 32-bit indexing");
  p.nblk = (int)nblk;
  hipLaunchKernelGGL(wino_kernel, dim3(p.nblk), dim3(256), 0, (hipStream_t)s_, p);
  return check_launch("mhada_conv3x3_wino");
}
