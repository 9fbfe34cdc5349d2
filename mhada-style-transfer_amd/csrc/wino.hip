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
// U_xi[ci][co] is a GEMM; all 16 run inside one workgroup, so V and M never touch HBM.  The
// transforms only add / subtract (G's 1/2 is exact): the direct correlation up to fp32 rounding
// of 4-term sums.
//
// Workgroup = 8 waves (two per SIMD) = 64 Winograd tiles (8 x 8 tiles = 16 x 16 output pixels)
// x 64 output channels.  Wave w = (e, th, ch) = (w >> 2, w & 1, (w >> 1) & 1) accumulates the
// 8 positions xi = 8e .. 8e+7 for tiles 32 th.. x channels 32 ch.. (8 accumulator blocks = 128
// registers); positions 8..15 reach waves 0-3 through LDS for the output transform.  The input
// channels stream in chunks of 8; per chunk k:
//   * LDS-DMA (global_load_lds) brings U(k+1) [16][64 co][8 ci] (32 KiB, prepacked
//     [Cin/8][16][Cout][8] by mhada_wino_weights) and the raw 18 x 18-pixel patch of chunk k+2
//     (32 B per pixel; padding pixels load a clamped pixel and are zeroed in the transform);
//   * the wave's 32 MFMAs of chunk k (8 positions x 4 k-steps) run beside every thread's
//     transform V = B^T d B of one (tile, channel) of chunk k+1 into the other V buffer;
//   * one counted vmcnt(0) + workgroup barrier.
// Earlier forms, measured and replaced: 4 waves x 32 tiles with scalar gathers
// (L2 bound), and 4 waves x 64 tiles holding all 16 positions in 256 AGPRs (one wave per SIMD:
// the transform and loads serialised with the MFMAs).  Round 5: the default is wino4_kernel
// below (the same tile and MFMA sequence, bit-identical, 13-15 % faster); this 8-wave kernel
// remains the fallback for inputs of 2 GiB and more (wino4 addresses x by a buffer resource).
// LDS operand rows are 32 B (8 channels) with the two 16-B halves swapped on rows with bit 3
// set (swz), so the ds_read_b128 of 32 consecutive rows is conflict-free; the raw patch's 16-B
// slots are XOR-swizzled (rswz) so the transform's ds_read_b32 hit distinct banks.
#include "common.h"

#include <algorithm>
#include <utility>

#ifndef WINO_DBG
#define WINO_DBG 0  // ablation builds (tools/wino_dbg.py): 1 no MFMA, 2 no loads, 4 no transform
#endif
#ifndef WINO4_DBG
#define WINO4_DBG 0  // 4-wave kernel ablation builds (results invalid): 1 no DMA, 2 no transform, 4 no MFMA, 8 no DMA wait
#endif

namespace mhada {

namespace {
constexpr int kT = 8;                  // tiles per side: 8 x 8 tiles, 16 x 16 output pixels
constexpr int kTT = kT * kT;           // 64 tiles
constexpr int kCO = 64;                // output channels per workgroup
constexpr int kCK = 8;                 // input channels per chunk
constexpr int kRP = 2 * kT + 2;        // raw patch side: 18 pixels
constexpr int kRaw = kRP * kRP;        // 324 pixels x 32 B
constexpr int kRDma = (2 * kRaw + 63) / 64;  // LDS-DMA instructions for the raw patch (11)
constexpr int kVS = 16 * kTT * kCK;    // V buffer (floats): [16][64 tiles][8]
constexpr int kUS = 16 * kCO * kCK;    // U buffer (floats): [16][64 co][8]
constexpr int kRS = kRDma * 64 * 4;    // raw buffer (floats): 704 16-B slots, 648 used

struct WinoP {
  const float* x;     // NHWC [B][H][W][Cin]
  const float* u;     // [Cin/8][16][Cout][8]
  const float* bias;  // [Cout] or null
  float* y;           // NHWC [B][Ho][Wo][ldc]
  const float* mask;  // null, or [B][Ho][Wo][ldc]: y = 0 where mask <= 0 (a ReLU adjoint folded into a dgrad)
  int B, H, W, Cin, Cout, Ho, Wo, pad, zero, relu;
  long long ldc;
  int nbx, nby, nbn, nblk;
};

MHADA_DEV int reflect_clamp(int v, int n) {
  v = v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
  return min(max(v, 0), n - 1);
}
// float offset of the 16-B half `half` (channels 4*half .. 4*half+3) of 32-B row `row`: halves
// swapped on rows with bit 3 set, so ds_read_b128 of 32 consecutive rows is conflict-free
MHADA_DEV int swz(int row, int half) { return row * 8 + ((half ^ ((row >> 3) & 1)) << 2); }
// Raw-patch 16-B slot swizzle (an involution): bit 1 of the slot flips with bit 3, so the
// transform's ds_read_b32 of 4 tiles x 8 channels (slots s0 + 4 tx + {0, 1}) hit 8 distinct
// 4-bank groups (ds_read_b32 serves 32 lanes over 32 banks; unswizzled, tiles tx and tx + 2 met).
MHADA_DEV int rswz(int slot) { return slot ^ (((slot >> 3) & 1) << 1); }
// The 4-wave kernel's raw-patch swizzle: its transform reads 64-bit channel pairs of 8 tiles of one
// tile row per half-wave (pixels 2 apart = 4 slots): bit 1 of the slot flips with bit 4, so tiles
// t and t + 4 (16 slots apart) land on different 16-B bank groups.
MHADA_DEV int rswz4(int slot) { return slot ^ (((slot >> 4) & 1) << 1); }
MHADA_DEV void glds16(const float* src, float* lds) {  // LDS-DMA: lane l -> lds + 16 l bytes
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}


__global__ void __launch_bounds__(512, 1) wino_kernel(const WinoP p) {
  __shared__ __attribute__((aligned(16))) float lds[2 * (kVS + kUS + kRS)];  // 150 KiB
  auto sV = [&](int i) { return lds + i * kVS; };
  auto sU = [&](int i) { return lds + 2 * kVS + i * kUS; };
  auto sR = [&](int i) { return lds + 2 * (kVS + kUS) + i * kRS; };
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wave w: positions xi = 8e .. 8e+7 (rows 2e, 2e+1 of the 4x4 grid, e = w >> 2) x tiles
  // 32(w & 1).. x channels 32((w >> 1) & 1)..; every thread also transforms one (tile, channel)
  // and every wave issues a share of the LDS-DMA
  const int e = wave >> 2, th = wave & 1, ch = (wave >> 1) & 1;

  // logical block: output-channel block fastest (neighbours share the input patch in L2)
  int id = xcd_remap(blockIdx.x, p.nblk);
  const int nb = id % p.nbn;
  id /= p.nbn;
  const int bx = id % p.nbx;
  id /= p.nbx;
  const int by = id % p.nby;
  const int b = id / p.nby;
  const int co0 = nb * kCO;
  const int P = p.zero ? p.pad : 1;
  const int nck = p.Cin / kCK;

  // raw patch DMA: instruction j (wave j % 8, j < 11) fills 16-B slots 64 j + lane = pixel
  // (slot >> 1), channel half (slot & 1); padding pixels load a clamped pixel (zeroed later)
  int roff[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int slot = rswz(64 * (wave + 8 * t) + lane);  // logical slot stored at this position
    const int px = min(slot >> 1, kRaw - 1);
    int iy = 2 * by * kT - P + px / kRP, ix = 2 * bx * kT - P + px % kRP;
    if (p.zero) {
      iy = min(max(iy, 0), p.H - 1);
      ix = min(max(ix, 0), p.W - 1);
    } else {
      iy = reflect_clamp(iy, p.H);
      ix = reflect_clamp(ix, p.W);
    }
    roff[t] = ((b * p.H + iy) * p.W + ix) * p.Cin + 4 * (slot & 1);
  }
  // U DMA: instructions 4w .. 4w+3 of 32; slot 64 j + lane = (xi, co row, stored half); the
  // source half is the logical one (swz)
  int uoff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int slot = 64 * (4 * wave + t) + lane;
    const int xi = slot >> 7, row = (slot >> 1) & 63, sh = slot & 1;
    uoff[t] = (xi * p.Cout + co0 + row) * kCK + 4 * (sh ^ ((row >> 3) & 1));
  }
  const long long ustride = (long long)16 * p.Cout * kCK;  // floats per chunk
  auto dma = [&](int cu, float* su, int cr, float* sr) {
#if WINO_DBG & 2
    return;
#endif
    cu = min(cu, nck - 1);
    cr = min(cr, nck - 1);
    const float* uc = p.u + cu * ustride;
#pragma unroll
    for (int t = 0; t < 4; ++t) glds16(uc + uoff[t], su + (4 * wave + t) * 256);
    glds16(p.x + roff[0] + cr * kCK, sr + wave * 256);
    if (wave + 8 < kRDma) glds16(p.x + roff[1] + cr * kCK, sr + (wave + 8) * 256);
  };
  // transform item: channel tc of tile tt; zero-padding positions of its 4x4 patch
  const int tc = tid & 7, tt = tid >> 3;
  // LDS float offsets of the item's 16 raw values (swizzled 16-B slots, see rswz)
  int roffs[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = (2 * (tt >> 3) + i) * kRP + 2 * (tt & 7) + j;
      roffs[4 * i + j] = rswz(2 * pix + (tc >> 2)) * 4 + (tc & 3);
    }
  const int vdst = swz(tt, tc >> 2) + (tc & 3);
  unsigned zmask = 0;
  if (p.zero) {
    const int y0 = 2 * (by * kT + (tt >> 3)) - P, x0 = 2 * (bx * kT + (tt & 7)) - P;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (y0 + i < 0 || y0 + i >= p.H || x0 + j < 0 || x0 + j >= p.W) zmask |= 1u << (4 * i + j);
  }
  auto transform = [&](const float* sr, float* sv) {
#if WINO_DBG & 4
    return;
#endif
    float d[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = sr[roffs[4 * i + j]];
        d[4 * i + j] = (zmask >> (4 * i + j)) & 1 ? 0.f : v;
      }
    float t[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[0 * 4 + j] = d[0 * 4 + j] - d[2 * 4 + j];
      t[1 * 4 + j] = d[1 * 4 + j] + d[2 * 4 + j];
      t[2 * 4 + j] = d[2 * 4 + j] - d[1 * 4 + j];
      t[3 * 4 + j] = d[1 * 4 + j] - d[3 * 4 + j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sv[(4 * i + 0) * kTT * kCK + vdst] = t[4 * i + 0] - t[4 * i + 2];
      sv[(4 * i + 1) * kTT * kCK + vdst] = t[4 * i + 1] + t[4 * i + 2];
      sv[(4 * i + 2) * kTT * kCK + vdst] = t[4 * i + 2] - t[4 * i + 1];
      sv[(4 * i + 3) * kTT * kCK + vdst] = t[4 * i + 1] - t[4 * i + 3];
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[x][q] = 0.f;
  // operands: A rows = tiles 32 th + r32, B rows = channels 32 ch + r32, positions 8e + x;
  // k-step s of lane half h takes channel 4h + s
  const int arow = swz(32 * th + r32, h) + 8 * e * (kTT * kCK), brow = swz(32 * ch + r32, h) + 8 * e * (kCO * kCK);
  auto mfmas = [&](const float* sv, const float* su) {
#if WINO_DBG & 1
    return;
#endif
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const f32x4 av = *reinterpret_cast<const f32x4*>(sv + x * (kTT * kCK) + arow);
      const f32x4 bv = *reinterpret_cast<const f32x4*>(su + x * (kCO * kCK) + brow);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc[x], 0, 0, 0);
    }
  };
  auto publish = [&]() {  // this wave's DMA landed, then the workgroup barrier
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  // prologue: U(0) and raw(0) -> transform into V[0]; raw(1) in R[1]
  dma(0, sU(0), 0, sR(0));
  dma(0, sU(0), 1, sR(1));
  publish();
  transform(sR(0), sV(0));
  __syncthreads();
  // chunk k: DMA of U(k+1) into U[(k+1)&1] and raw(k+2) into R[k&1]; MFMAs on V/U[k&1]; the
  // transform of raw(k+1) into V[(k+1)&1]; one barrier
  for (int k = 0; k < nck; ++k) {
    const int c = k & 1, n = c ^ 1;
    dma(k + 1, sU(n), k + 2, sR(c));
    mfmas(sV(c), sU(c));
    transform(sR(n), sV(n));
    publish();
  }

  // output transform Y = A^T M A (A^T = [[1,1,1,0],[0,1,-1,-1]]): row partials
  // P_i[q] = sum_j M[i][j] A[j][q]; Y[0][q] = P0 + P1 + P2, Y[1][q] = P1 - P2 - P3.  Waves
  // 4-7 (rows 2, 3) hand their share (P2, -P2 - P3) to waves 0-3 through LDS.
  float* ex = lds + (wave & 3) * (16 * 4 * 64) + lane;  // [w&3][r][4][64 lanes] (64 KiB)
  static_assert(4 * 16 * 4 * 64 <= 2 * kVS, "epilogue exchange must fit sV");
  if (e) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float m[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float m0 = acc[4 * i][r], m1 = acc[4 * i + 1][r], m2 = acc[4 * i + 2][r], m3 = acc[4 * i + 3][r];
        m[i][0] = m0 + m1 + m2;
        m[i][1] = m1 - m2 - m3;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ex[(r * 4 + 2 * q) * 64] = m[0][q];
        ex[(r * 4 + 2 * q + 1) * 64] = -m[0][q] - m[1][q];
      }
    }
  }
  __syncthreads();
  if (e) return;
  const int co = co0 + 32 * ch + r32;
  const float bias = p.bias ? p.bias[co] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tile = 32 * th + (r & 3) + 8 * (r >> 2) + 4 * h;
    float m[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float m0 = acc[4 * i][r], m1 = acc[4 * i + 1][r], m2 = acc[4 * i + 2][r], m3 = acc[4 * i + 3][r];
      m[i][0] = m0 + m1 + m2;
      m[i][1] = m1 - m2 - m3;
    }
    const int oy0 = 2 * (by * kT + (tile >> 3)), ox0 = 2 * (bx * kT + (tile & 7));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float y0 = m[0][q] + m[1][q] + ex[(r * 4 + 2 * q) * 64] + bias;
      float y1 = m[1][q] + ex[(r * 4 + 2 * q + 1) * 64] + bias;
      if (p.relu) {
        y0 = fmaxf(y0, 0.f);
        y1 = fmaxf(y1, 0.f);
      }
      const int ox = ox0 + q;
      if (ox < p.Wo) {
        const long long i0 = ((long long)(b * p.Ho + oy0) * p.Wo + ox) * p.ldc + co;
        const long long i1 = i0 + (long long)p.Wo * p.ldc;
        if (p.mask) {
          if (oy0 < p.Ho && !(p.mask[i0] > 0.f)) y0 = 0.f;
          if (oy0 + 1 < p.Ho && !(p.mask[i1] > 0.f)) y1 = 0.f;
        }
        if (oy0 < p.Ho) p.y[i0] = y0;
        if (oy0 + 1 < p.Ho) p.y[i1] = y1;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// 4-wave form (round 5, tuning wino4): the same workgroup tile, LDS images and chunk pipeline as
// wino_kernel, one wave per SIMD with ALL 16 positions of its 32 tiles x 32 channels in 256
// accumulator registers (wave w: tiles 32 (w & 1).., channels 32 (w >> 1)..), and the chunk's
// non-MFMA work cut to the transform arithmetic.  Measured (tools/ubench/f32mfma_fill.hip,
// profiles/r05_f32mfma_fill.log): v_mfma_f32_32x32x2_f32 holds the SIMD's vector issue for its
// whole 64 cycles, so every VALU instruction of an fp32 MFMA kernel adds its issue cost to the
// MFMA time whichever wave issues it — only fewer vector instructions help.  Hence:
//   * LDS-DMA through buffer resources (buffer_load ... lds): the per-chunk advance is the scalar
//     soffset, no 64-bit address VALU per piece; zero padding comes from out-of-range offsets
//     (the buffer returns 0), so the transform has no per-value select;
//   * the chunk loop unrolled by two, so every LDS address of the transform, the operand reads
//     and the V writes is a per-lane base plus an immediate;
//   * a chunk is 16 stages of 4 MFMAs, fenced per stage: operand reads two stages ahead, one
//     LDS-DMA piece in each of stages 0-10, the transform (one item per thread: a channel pair of
//     one tile, packed f32 arithmetic) loaded in stage 2 and finished in stages 4-5.
// Every MFMA (accumulator, operand bits and order) is the 8-wave kernel's and the output transform
// keeps its association: bit-identical to wino_kernel.
// ------------------------------------------------------------------------------------
template <int DBG>
__global__ void __launch_bounds__(256, 1) wino4_kernel(const WinoP p) {
  __shared__ __attribute__((aligned(16))) float lds[2 * (kVS + kUS + kRS)];  // 150 KiB
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int th = wave & 1, ch = wave >> 1;

  int id = xcd_remap(blockIdx.x, p.nblk);
  const int nb = id % p.nbn;
  id /= p.nbn;
  const int bx = id % p.nbx;
  id /= p.nbx;
  const int by = id % p.nby;
  const int b = id / p.nby;
  const int co0 = nb * kCO;
  const int P = p.zero ? p.pad : 1;
  const int nck = p.Cin / kCK;

  // buffer resources (sizes < 2^31 bytes, checked on the host): offsets at or past the size read 0
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x), 0, (int)((long long)p.B * p.H * p.W * p.Cin * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.u), 0, p.Cin * 16 * p.Cout * 4, 0x00020000);
  // raw patch DMA: instruction j = wave + 4 t (j < 11), slots as wino_kernel's; byte offsets,
  // 0x7ff00000 (past the buffer) for zero-padding pixels
  int rvo[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int slot = rswz4(64 * min(wave + 4 * t, kRDma - 1) + lane);
    const int px = min(slot >> 1, kRaw - 1);
    int iy = 2 * by * kT - P + px / kRP, ix = 2 * bx * kT - P + px % kRP;
    bool inside = true;
    if (p.zero) {
      inside = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W;
    } else {
      iy = reflect_clamp(iy, p.H);
      ix = reflect_clamp(ix, p.W);
    }
    rvo[t] = inside ? (((b * p.H + iy) * p.W + ix) * p.Cin + 4 * (slot & 1)) * 4 : 0x7ff00000;
  }
  const bool raw2 = wave + 8 < kRDma;
  // U DMA: instructions 8w .. 8w+7 of 32 (byte offsets inside one chunk)
  int uvo[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int slot = 64 * (8 * wave + t) + lane;
    const int xi = slot >> 7, row = (slot >> 1) & 63, sh = slot & 1;
    uvo[t] = ((xi * p.Cout + co0 + row) * kCK + 4 * (sh ^ ((row >> 3) & 1))) * 4;
  }
  const int ucb = 16 * p.Cout * kCK * 4;  // bytes per U chunk
  typedef __attribute__((address_space(3))) void* LdsP;
  // DMA piece i (0-7: U of chunk cu into U buffer su, 8-10: raw of chunk cr into raw buffer sr)
  auto dma_piece = [&](int i, int cu, int su, int cr, int sr) {
    if constexpr ((DBG & 1) != 0) return;
    if (i < 8) {
      float* dst = lds + 2 * kVS + su * kUS + (8 * wave + i) * 256;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ur, (LdsP)dst, 16, uvo[i], min(cu, nck - 1) * ucb, 0, 0);
    } else if (i < 10 || raw2) {
      float* dst = lds + 2 * (kVS + kUS) + sr * kRS + (wave + 4 * (i - 8)) * 256;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (LdsP)dst, 16, rvo[i - 8], min(cr, nck - 1) * kCK * 4, 0, 0);
    }
  };
  // transform item: channels 2 tp, 2 tp + 1 of tile tt (one item per thread, both channels in one
  // 64-bit LDS word: ds_read_b64 / v_pk_add_f32 / ds_write2st64_b64, half the instructions of
  // one channel per item)
  const int tp = tid & 3, tt = tid >> 2;
  // LDS float offsets of the item's 16 raw pairs (raw buffer 0; buffer 1 is + kRS); & 0xffff: the
  // sign bit is known zero, so hipcc folds the buffer constant into the ds_read immediate
  int roffs[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pix = (2 * (tt >> 3) + i) * kRP + 2 * (tt & 7) + j;
      roffs[4 * i + j] = (2 * (kVS + kUS) + rswz4(2 * pix + (tp >> 1)) * 4 + 2 * (tp & 1)) & 0xffff;
    }
  const int vdst = (swz(tt, tp >> 1) + 2 * (tp & 1)) & 0x7fff;
  f32x2 d[16], tv[16];
  auto tload = [&](int rbuf) {
    if constexpr ((DBG & 2) != 0) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = *reinterpret_cast<const f32x2*>(lds + roffs[q] + rbuf * kRS);
  };
  auto tcols = [&]() {
    if constexpr ((DBG & 2) != 0) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tv[0 * 4 + j] = d[0 * 4 + j] - d[2 * 4 + j];
      tv[1 * 4 + j] = d[1 * 4 + j] + d[2 * 4 + j];
      tv[2 * 4 + j] = d[2 * 4 + j] - d[1 * 4 + j];
      tv[3 * 4 + j] = d[1 * 4 + j] - d[3 * 4 + j];
    }
  };
  auto trows = [&](int vbuf, int i0) {  // rows i0, i0 + 1 of V = t B
    if constexpr ((DBG & 2) != 0) return;
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i) {
      float* o = lds + vbuf * kVS + vdst;
      *reinterpret_cast<f32x2*>(o + (4 * i + 0) * kTT * kCK) = tv[4 * i + 0] - tv[4 * i + 2];
      *reinterpret_cast<f32x2*>(o + (4 * i + 1) * kTT * kCK) = tv[4 * i + 1] + tv[4 * i + 2];
      *reinterpret_cast<f32x2*>(o + (4 * i + 2) * kTT * kCK) = tv[4 * i + 2] - tv[4 * i + 1];
      *reinterpret_cast<f32x2*>(o + (4 * i + 3) * kTT * kCK) = tv[4 * i + 1] - tv[4 * i + 3];
    }
  };

  f32x16 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[x][q] = 0.f;
  const int arow = swz(32 * th + r32, h) & 0x7fff, brow = (2 * kVS + swz(32 * ch + r32, h)) & 0xffff;
  f32x4 oa[3], ob[3];
  auto rdop = [&](int xi, int buf, f32x4& a, f32x4& bb) {
    a = *reinterpret_cast<const f32x4*>(lds + buf * kVS + xi * (kTT * kCK) + arow);
    bb = *reinterpret_cast<const f32x4*>(lds + buf * kUS + xi * (kCO * kCK) + brow);
  };
  auto publish = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((DBG & 8) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto fence = [&]() { __builtin_amdgcn_sched_barrier(0); };

  // prologue: U(0), raw(0), raw(1); transform raw(0) into V[0]
#pragma unroll
  for (int i = 0; i < 11; ++i) dma_piece(i, 0, 0, 0, 0);
#pragma unroll
  for (int i = 8; i < 11; ++i) dma_piece(i, 0, 0, 1, 1);
  publish();
  tload(0);
  tcols();
  trows(0, 0);
  trows(0, 2);
  __syncthreads();
  // chunk k (buffer parity C = k & 1, a compile-time constant in each unrolled copy)
  auto chunk = [&](int k, auto cc) {
    constexpr int C = decltype(cc)::value, N = C ^ 1;
    rdop(0, C, oa[0], ob[0]);
    rdop(1, C, oa[1], ob[1]);
    fence();
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      if (xi + 2 < 16) rdop(xi + 2, C, oa[(xi + 2) % 3], ob[(xi + 2) % 3]);
      if constexpr ((DBG & 4) == 0) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(oa[xi % 3][s], ob[xi % 3][s], acc[xi], 0, 0, 0);
      }
      if (xi < 11) dma_piece(xi, k + 1, N, k + 2, C);
      if (xi == 2) tload(N);
      if (xi == 4) { tcols(); trows(N, 0); }
      if (xi == 5) trows(N, 2);
      fence();
    }
    publish();
  };
  int k = 0;
  for (; k + 1 < nck; k += 2) {
    chunk(k, std::integral_constant<int, 0>());
    chunk(k + 1, std::integral_constant<int, 1>());
  }
  if (k < nck) chunk(k, std::integral_constant<int, 0>());

  // output transform Y = A^T M A, every position in this wave; the association of wino_kernel's
  // two-wave form (row partials P_i; Y0 = (P0 + P1) + P2, Y1 = P1 + (-P2 - P3))
  const int co = co0 + 32 * ch + r32;
  const float bias = p.bias ? p.bias[co] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tile = 32 * th + (r & 3) + 8 * (r >> 2) + 4 * h;
    float m[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float m0 = acc[4 * i][r], m1 = acc[4 * i + 1][r], m2 = acc[4 * i + 2][r], m3 = acc[4 * i + 3][r];
      m[i][0] = m0 + m1 + m2;
      m[i][1] = m1 - m2 - m3;
    }
    const int oy0 = 2 * (by * kT + (tile >> 3)), ox0 = 2 * (bx * kT + (tile & 7));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float e1 = -m[2][q] - m[3][q];
      float y0 = m[0][q] + m[1][q] + m[2][q] + bias;
      float y1 = m[1][q] + e1 + bias;
      if (p.relu) {
        y0 = fmaxf(y0, 0.f);
        y1 = fmaxf(y1, 0.f);
      }
      const int ox = ox0 + q;
      if (ox < p.Wo) {
        const long long i0 = ((long long)(b * p.Ho + oy0) * p.Wo + ox) * p.ldc + co;
        const long long i1 = i0 + (long long)p.Wo * p.ldc;
        if (p.mask) {
          if (oy0 < p.Ho && !(p.mask[i0] > 0.f)) y0 = 0.f;
          if (oy0 + 1 < p.Ho && !(p.mask[i1] > 0.f)) y1 = 0.f;
        }
        if (oy0 < p.Ho) p.y[i0] = y0;
        if (oy0 + 1 < p.Ho) p.y[i1] = y1;
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
  float* ub = u + ((long long)(ci / kCK) * 16 * Cout + co) * kCK + (ci % kCK);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float a = gg[3 * r], bb = gg[3 * r + 1], c = gg[3 * r + 2];
    const float v[4] = {a, 0.5f * (a + bb + c), 0.5f * (a - bb + c), c};
#pragma unroll
    for (int j = 0; j < 4; ++j) ub[(long long)(4 * r + j) * Cout * kCK] = v[j];
  }
}
// ------------------------------------------------------------------------------------
// Weight gradient of the same conv, Winograd F(2x2, 3x3) (the decoder's Conv2d weight / bias
// gradients in train_image.py:139; replaces the im2col TN GEMM, 2.25x fewer products).
// With U = G g G^T and Y_t = A^T (U . V_t) A for output tile t (V_t = B^T d_t B):
//   dU[co][ci] = sum_t (A dY_t A^T)[co] . V_t[ci]      (16 positions, elementwise in xi)
//   dg = G^T dU G                                        (4x4 -> 3x3 per (co, ci))
// so per position xi the tile sum is a GEMM [Cout x tiles] x [tiles x Cin]: the forward kernel's
// MFMA structure with the tiles as the reduction axis.  Workgroup = (64 co, 64 ci) x a split of the
// tile chunks; a chunk = 8 consecutive tiles of one tile row (16 output columns).  Per chunk:
//   * LDS-DMA of the output-gradient rows (2 x 16 px x 64 co, 8 KiB) and the input patch
//     (4 x 18 px x 64 ci, 18 KiB), one chunk ahead, single-buffered (consumed by the transforms of
//     the next chunk, after the barrier);
//   * every thread transforms one (tile, co) item Yh = A dY A^T and one (tile, ci) item
//     V = B^T d B of the NEXT chunk into the other buffers (raw pixels' 64 channels XOR-swizzled by
//     pixel so the 8 tiles' reads hit distinct banks);
//   * 32 MFMAs per wave of this chunk (8 positions x 4 k-steps of 2 tiles), one barrier.
// Partial dU of each split goes to work [S][16][Cout][Cin], the bias gradient (sum of dY, from the
// dY transform of the ci-block-0 workgroups) to [S][Cout]; wgrad_finish sums the splits in a fixed
// order and applies G^T . G.  Deterministic.
// ------------------------------------------------------------------------------------
constexpr int kWgT = 8;                 // tiles per chunk (the MFMA reduction axis)
constexpr int kWgS = 16 * 64 * kWgT;    // Yh / V buffer (floats): [16][64 rows][8 tiles]
constexpr int kWgRX = 4 * 18 * 64;      // raw input patch (floats): [72 px][64 ci]
constexpr int kWgRY = 2 * 16 * 64;      // raw output gradient (floats): [32 px][64 co]

struct WgP {
  const float* x;    // NHWC [B][H][W][Cin] (the conv input)
  const float* g;    // NHWC [B][H][W][ldg] (the output gradient, ReLU mask applied)
  float* slab;       // [S][16][Cout][Cin]
  float* cslab;      // [S][Cout] or null
  int B, H, W, Cin, Cout, zero;
  long long ldg;
  int crow, nchunk, cps;  // chunks per tile row, all chunks, chunks per split
};

// 64-channel pixel rows XOR-swizzled in units of 8 floats by pixel: channel c of pixel px at
// px * 64 + (c ^ (8 * ((px >> 1) & 7)))
MHADA_DEV int wg_px(int px, int c) { return px * 64 + (c ^ (8 * ((px >> 1) & 7))); }

// ZERO: zero padding (VGG-style), else reflect (the decoder).  Per-chunk work is scalar where it
// can be: the chunk coordinates are stepped (no divisions), interior chunks (the patch and the
// dY rows inside the image) load through a per-chunk base plus per-lane constant offsets, and the
// transforms' LDS offsets (per-lane XOR swizzles) are computed once — every VALU instruction here
// costs its full issue time beside the fp32 MFMAs (profiles/r05_f32mfma_fill.log).
template <bool ZERO>
__global__ void __launch_bounds__(512, 1) wino_wgrad_kernel(const WgP p) {
  __shared__ __attribute__((aligned(16))) float lds[4 * kWgS + kWgRX + kWgRY];  // 154 KiB
  auto sYh = [&](int i) { return lds + i * kWgS; };
  auto sVb = [&](int i) { return lds + (2 + i) * kWgS; };
  float* sRX = lds + 4 * kWgS;
  float* sRY = sRX + kWgRX;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int e = wave >> 2, coh = wave & 1, cih = (wave >> 1) & 1;
  const int nib = p.Cin / 64;
  const int cb = blockIdx.x / nib, ib = blockIdx.x - cb * nib;
  const int co0 = cb * 64, ci0 = ib * 64;
  const int c_beg = blockIdx.y * p.cps, c_end = min(p.nchunk, c_beg + p.cps);
  constexpr int P = 1;  // pad 1
  const int TW = p.crow * kWgT, TH = p.H / 2;  // tile columns / rows per image

  // chunk coordinates, stepped along the chunk order (b, ty, tx0 / 8)
  struct Pos { int b, ty, tx0; };
  auto step_pos = [&](Pos& q) {
    q.tx0 += kWgT;
    if (q.tx0 >= TW) {
      q.tx0 = 0;
      if (++q.ty >= TH) {
        q.ty = 0;
        ++q.b;
      }
    }
  };
  auto src_pix = [&](int b, int Y, int X) -> long long {
    if (ZERO) {
      Y = min(max(Y, 0), p.H - 1);
      X = min(max(X, 0), p.W - 1);
    } else {
      Y = reflect_clamp(Y, p.H);
      X = reflect_clamp(X, p.W);
    }
    return ((long long)b * p.H + Y) * p.W + X;
  };
  // per-lane constants of the DMA pieces: dY (one piece per wave: px 4w + lane / 16) and X (pieces
  // ins = wave + 8 j < 18: px 4 ins + lane / 16); slot (px, q) holds source quad q ^ (2 ((px >> 1) & 7))
  const int ypx = 4 * wave + (lane >> 4), ysq = (lane & 15) ^ (2 * ((ypx >> 1) & 7));
  const long long yoff = ((long long)(ypx >> 4) * p.W + (ypx & 15)) * p.ldg + 4 * ysq;
  int xpx[3], xsq[3];
  long long xoff[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    xpx[j] = 4 * (wave + 8 * j) + (lane >> 4);
    xsq[j] = (lane & 15) ^ (2 * ((xpx[j] >> 1) & 7));
    xoff[j] = ((long long)(xpx[j] / 18) * p.W + xpx[j] % 18) * p.Cin + 4 * xsq[j];
  }
  // the chunk's patch rows 2ty-1 .. 2ty+2, columns 2tx0-1 .. 2tx0+16 and its dY rows lie in the image
  auto interior = [&](const Pos& q) {
    return q.ty > 0 && 2 * q.ty + 2 < p.H && q.tx0 > 0 && 2 * q.tx0 + 16 < p.W;
  };
  auto dma = [&](const Pos& q) {
#if WINO_DBG & 2
    return;
#endif
    glds16(p.g + (((long long)q.b * p.H + 2 * q.ty) * p.W + 2 * q.tx0) * p.ldg + co0 + yoff, sRY + wave * 256);
    if (interior(q)) {
      const float* xb = p.x + (((long long)q.b * p.H + 2 * q.ty - P) * p.W + 2 * q.tx0 - P) * p.Cin + ci0;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (wave + 8 * j < 18) glds16(xb + xoff[j], sRX + (wave + 8 * j) * 256);
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (wave + 8 * j < 18) {
          const long long pix = src_pix(q.b, 2 * q.ty - P + xpx[j] / 18, 2 * q.tx0 - P + xpx[j] % 18);
          glds16(p.x + pix * p.Cin + ci0 + 4 * xsq[j], sRX + (wave + 8 * j) * 256);
        }
    }
  };
  // transforms of the chunk whose raw rows are in sRY / sRX into buffer slot n: item (t, row) with
  // t = lane & 7 and row = 8 * wave + (lane >> 3) (both the co of Yh and the ci of V)
  const int it = lane & 7, irow = 8 * wave + (lane >> 3);
  const int wdst = swz(irow, it >> 2) + (it & 3);
  int ry[4], rx[16];  // LDS offsets of the item's raw reads (wg_px swizzle, per lane)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) ry[2 * i + j] = wg_px(16 * i + 2 * it + j, irow);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) rx[4 * i + j] = wg_px(18 * i + 2 * it + j, irow);
  float bsum = 0.f;  // bias gradient partial of co = co0 + irow (ci block 0)
  auto transform = [&](const Pos& q, int n) {
#if WINO_DBG & 4
    return;
#endif
    // Yh = A dY A^T, A = [[1,0],[1,1],[1,-1],[0,-1]]
    float d[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) d[i][j] = sRY[ry[2 * i + j]];
    if (ib == 0) bsum += (d[0][0] + d[0][1]) + (d[1][0] + d[1][1]);
    float a[4][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      a[0][j] = d[0][j];
      a[1][j] = d[0][j] + d[1][j];
      a[2][j] = d[0][j] - d[1][j];
      a[3][j] = -d[1][j];
    }
    float* yh = sYh(n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      yh[(4 * i + 0) * 512 + wdst] = a[i][0];
      yh[(4 * i + 1) * 512 + wdst] = a[i][0] + a[i][1];
      yh[(4 * i + 2) * 512 + wdst] = a[i][0] - a[i][1];
      yh[(4 * i + 3) * 512 + wdst] = -a[i][1];
    }
    // V = B^T d B on the 4 x 4 patch of tile it (input rows 2ty-1 .. 2ty+2)
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = sRX[rx[i]];
    if (ZERO && !interior(q)) {  // zero padding: the clamped pixels outside the image read 0
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int Y = 2 * q.ty - P + i, X = 2 * q.tx0 - P + 2 * it + j;
          if (Y < 0 || Y >= p.H || X < 0 || X >= p.W) v[4 * i + j] = 0.f;
        }
    }
    float t[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t[0 * 4 + j] = v[0 * 4 + j] - v[2 * 4 + j];
      t[1 * 4 + j] = v[1 * 4 + j] + v[2 * 4 + j];
      t[2 * 4 + j] = v[2 * 4 + j] - v[1 * 4 + j];
      t[3 * 4 + j] = v[1 * 4 + j] - v[3 * 4 + j];
    }
    float* sv = sVb(n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sv[(4 * i + 0) * 512 + wdst] = t[4 * i + 0] - t[4 * i + 2];
      sv[(4 * i + 1) * 512 + wdst] = t[4 * i + 1] + t[4 * i + 2];
      sv[(4 * i + 2) * 512 + wdst] = t[4 * i + 2] - t[4 * i + 1];
      sv[(4 * i + 3) * 512 + wdst] = t[4 * i + 1] - t[4 * i + 3];
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[x][q] = 0.f;
  // A operand = Yh rows (co 32 coh + r32), B operand = V rows (ci 32 cih + r32); k-step s of lane
  // half h takes tile 4h + s
  const int arow = swz(32 * coh + r32, h) + 8 * e * 512, brow = swz(32 * cih + r32, h) + 8 * e * 512;
  auto mfmas = [&](int n) {
#if WINO_DBG & 1
    return;
#endif
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const f32x4 av = *reinterpret_cast<const f32x4*>(sYh(n) + x * 512 + arow);
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sVb(n) + x * 512 + brow);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc[x], 0, 0, 0);
    }
  };
  auto publish = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  if (c_beg < c_end) {
    Pos q;  // chunk c_beg: the one division of the kernel
    {
      const int per_img = TH * p.crow;
      q.b = c_beg / per_img;
      const int r = c_beg - q.b * per_img;
      q.ty = r / p.crow;
      q.tx0 = (r - q.ty * p.crow) * kWgT;
    }
    dma(q);
    publish();
    transform(q, 0);
    __syncthreads();
    // chunk c: DMA of c+1's raw rows (the raw buffers were last read by transform(c) before the
    // barrier), MFMAs on slot c&1, then (after its DMA landed) transform c+1 into the other slot
    for (int c = c_beg; c < c_end; ++c) {
      const int k = c - c_beg, cur = k & 1;
      const bool more = c + 1 < c_end;
      step_pos(q);  // chunk c + 1
      if (more) dma(q);
      mfmas(cur);
      if (more) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every wave's pieces of c+1 landed
        transform(q, cur ^ 1);
      }
      __syncthreads();
    }
  }
  // partial dU of this split: acc[x] <-> position 8e + x, co = 32 coh + (r & 3) + 8 (r >> 2) + 4h,
  // ci = 32 cih + r32
  float* sl = p.slab + (long long)blockIdx.y * 16 * p.Cout * p.Cin;
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + 32 * coh + (r & 3) + 8 * (r >> 2) + 4 * h, ci = ci0 + 32 * cih + r32;
      sl[((long long)(8 * e + x) * p.Cout + co) * p.Cin + ci] = acc[x][r];
    }
  if (p.cslab && ib == 0) {  // the 8 tile lanes of a co are consecutive lanes: fixed-order xor tree
    bsum += __shfl_xor(bsum, 1, 64);
    bsum += __shfl_xor(bsum, 2, 64);
    bsum += __shfl_xor(bsum, 4, 64);
    if (it == 0) p.cslab[(long long)blockIdx.y * p.Cout + co0 + irow] = bsum;
  }
}

// dW[co][tap][ci] = G^T (sum_s dU[s][.][co][ci]) G, G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]];
// db[co] = sum_s cslab[s][co] (threads with ci == 0)
__global__ void __launch_bounds__(256) wino_wgrad_finish_kernel(const float* __restrict__ slab,
                                                                const float* __restrict__ cslab, float* __restrict__ dw,
                                                                float* __restrict__ db, int Cout, int Cin, int S) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)Cout * Cin) return;
  const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
  const long long st = (long long)Cout * Cin;
  float u[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) u[x] = 0.f;
  for (int s = 0; s < S; ++s) {
    const float* q = slab + (long long)s * 16 * st + i;
#pragma unroll
    for (int x = 0; x < 16; ++x) u[x] += q[x * st];
  }
  // m = G^T u (3 x 4): row a of G^T is column a of G
  float m[3][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    m[0][c] = u[0 * 4 + c] + 0.5f * (u[1 * 4 + c] + u[2 * 4 + c]);
    m[1][c] = 0.5f * (u[1 * 4 + c] - u[2 * 4 + c]);
    m[2][c] = 0.5f * (u[1 * 4 + c] + u[2 * 4 + c]) + u[3 * 4 + c];
  }
  float* o = dw + (long long)co * 9 * Cin + ci;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o[(3 * a + 0) * Cin] = m[a][0] + 0.5f * (m[a][1] + m[a][2]);
    o[(3 * a + 1) * Cin] = 0.5f * (m[a][1] - m[a][2]);
    o[(3 * a + 2) * Cin] = 0.5f * (m[a][1] + m[a][2]) + m[a][3];
  }
  if (db && cslab && ci == 0) {
    float sb = 0.f;
    for (int s = 0; s < S; ++s) sb += cslab[(long long)s * Cout + co];
    db[co] = sb;
  }
}
}  // namespace

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_conv3x3_wgrad_wino_splits(int B, int H, int W, int Cin, int Cout) {
  if (B <= 0 || H < 2 || W < 16 || Cin <= 0 || Cout <= 0 || Cin % 64 || Cout % 64) return 0;
  const long long nchunk = (long long)B * (H / 2) * (W / 16);
  const long long blocks = (long long)(Cout / 64) * (Cin / 64);
  // about two workgroups per CU over the grid, at least 16 chunks per split
  const long long s = std::max<long long>(1, std::min<long long>((512 + blocks - 1) / blocks, nchunk / 16));
  return (int)std::min<long long>(s, 65535);
}

extern "C" int mhada_conv3x3_wgrad_wino(const float* x, const float* g, float* dw, float* db, float* work,
                                        long long work_floats, int B, int H, int W, int Cin, int Cout, long long ldg,
                                        int pad_mode, mhada_stream_t s_) {
  if (!x || !g || !dw || !work || B <= 0 || H < 2 || W < 2 || Cin <= 0 || Cout <= 0)
    return fail("mhada_conv3x3_wgrad_wino: bad args");
  if (Cin % 64 || Cout % 64 || H % 2 || W % 16)
    return fail("mhada_conv3x3_wgrad_wino: needs Cin % 64 == 0, Cout % 64 == 0, H even, W % 16 == 0");
  if (pad_mode != MHADA_PAD_REFLECT && pad_mode != MHADA_PAD_ZERO) return fail("mhada_conv3x3_wgrad_wino: bad pad_mode");
  if (ldg < Cout || ldg % 4) return fail("mhada_conv3x3_wgrad_wino: ldg >= Cout, ldg % 4 == 0");
  if (((uintptr_t)x | (uintptr_t)g | (uintptr_t)work) & 15) return fail("mhada_conv3x3_wgrad_wino: 16-byte aligned x, g, work");
  if ((long long)B * H * W * std::max<long long>(Cin, ldg) > (1LL << 31) - 1)
    return fail("mhada_conv3x3_wgrad_wino: problem too large for 32-bit indexing");
  WgP p;
  p.x = x; p.g = g;
  p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout; p.ldg = ldg;
  p.zero = pad_mode == MHADA_PAD_ZERO;
  p.crow = W / 16;
  p.nchunk = B * (H / 2) * p.crow;
  int S = mhada_conv3x3_wgrad_wino_splits(B, H, W, Cin, Cout);
  const long long per = 16LL * Cout * Cin + (db ? Cout : 0);
  S = (int)std::min<long long>(S, work_floats / per);
  if (S < 1) return fail("mhada_conv3x3_wgrad_wino: workspace smaller than 16*Cout*Cin (+Cout) floats");
  p.cps = (p.nchunk + S - 1) / S;
  S = (p.nchunk + p.cps - 1) / p.cps;
  p.slab = work;
  p.cslab = db ? work + (long long)S * 16 * Cout * Cin : nullptr;
  const dim3 grid((unsigned)((Cout / 64) * (Cin / 64)), (unsigned)S);
  if (p.zero)
    hipLaunchKernelGGL(wino_wgrad_kernel<true>, grid, dim3(512), 0, (hipStream_t)s_, p);
  else
    hipLaunchKernelGGL(wino_wgrad_kernel<false>, grid, dim3(512), 0, (hipStream_t)s_, p);
  if (int rc = check_launch("mhada_conv3x3_wgrad_wino")) return rc;
  const long long n = (long long)Cout * Cin;
  hipLaunchKernelGGL(wino_wgrad_finish_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s_,
                     p.slab, p.cslab, dw, db, Cout, Cin, S);
  return check_launch("mhada_conv3x3_wgrad_wino(finish)");
}

extern "C" int mhada_wino_weights(const float* w, float* u, int Cout, int Cin, mhada_stream_t s_) {
  if (!w || !u || Cout <= 0 || Cin <= 0 || Cin % kCK) return fail("mhada_wino_weights: bad args (Cin % 8 == 0)");
  const long long n = (long long)Cout * Cin;
  hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s_, w, u,
                     Cout, Cin);
  return check_launch("mhada_wino_weights");
}

extern "C" int mhada_conv3x3_wino(const float* x, const float* u, const float* bias, float* y, int B, int H, int W,
                                  int Cin, int Cout, long long ldc, int pad_mode, int pad, int relu,
                                  const float* relu_mask, mhada_stream_t s_) {
  if (!x || !u || !y || B <= 0 || H < 2 || W < 2 || Cin <= 0 || Cout <= 0)
    return fail("mhada_conv3x3_wino: bad args");
  if (Cin % kCK || Cout % kCO) return fail("mhada_conv3x3_wino: needs Cin % 8 == 0 and Cout % 64 == 0");
  if (pad_mode != MHADA_PAD_REFLECT && pad_mode != MHADA_PAD_ZERO) return fail("mhada_conv3x3_wino: bad pad_mode");
  if (pad_mode == MHADA_PAD_ZERO && pad != 1 && pad != 2) return fail("mhada_conv3x3_wino: zero pad must be 1 or 2");
  if (ldc < Cout) return fail("mhada_conv3x3_wino: ldc < Cout");
  if (((uintptr_t)x | (uintptr_t)u) & 15) return fail("mhada_conv3x3_wino: x and u must be 16-byte aligned");
  WinoP p;
  p.x = x; p.u = u; p.bias = bias; p.y = y; p.mask = relu_mask;
  p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.zero = pad_mode == MHADA_PAD_ZERO;
  p.pad = p.zero ? pad : 1;
  p.Ho = p.zero ? H + 2 * (pad - 1) : H;
  p.Wo = p.zero ? W + 2 * (pad - 1) : W;
  p.relu = relu;
  p.ldc = ldc;
  const int TY = (p.Ho + 1) / 2, TX = (p.Wo + 1) / 2;
  p.nby = (TY + kT - 1) / kT;
  p.nbx = (TX + kT - 1) / kT;
  p.nbn = Cout / kCO;
  const long long nblk = (long long)B * p.nby * p.nbx * p.nbn;
  if (nblk > (1LL << 31) - 1 || (long long)B * H * W * Cin > (1LL << 31) - 1)
    return fail("mhada_conv3x3_wino: problem too large for 32-bit indexing");
  p.nblk = (int)nblk;
  // the 4-wave form addresses x through a buffer resource: byte size below the out-of-range offset
  if (tuning().wino4 && (long long)B * H * W * Cin * 4 < 0x7ff00000LL) {
    hipLaunchKernelGGL(wino4_kernel<WINO4_DBG>, dim3(p.nblk), dim3(256), 0, (hipStream_t)s_, p);
  } else
    hipLaunchKernelGGL(wino_kernel, dim3(p.nblk), dim3(512), 0, (hipStream_t)s_, p);
  return check_launch("mhada_conv3x3_wino");
}
