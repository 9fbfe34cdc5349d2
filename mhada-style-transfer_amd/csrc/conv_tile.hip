// Direct 3x3 convolution for the decoder's 64-channel layer (conv.py:75-100, the last
// ConvReluBlock: upsample x2 -> ReflectionPad2d(1) -> conv 64->64 -> ReLU at the full output
// resolution), bf16 MFMA with fp32 accumulation.
//
// Why not the implicit GEMM (gemm.hip): with N = Cout = 64 a GEMM tile re-gathers every input
// pixel nine times (once per tap) from L2 and runs 64-column tiles; at 1024^2 batch 4 the
// separate upsample + GEMM pair took ~1.1 ms (283 TFLOP/s) for 309 GFLOP.  Here:
//   * all 9 x 64 x 64 weights stay resident in LDS for the whole (persistent) block;
//   * an output tile of 8 x 32 pixels stages its 10 x 34 halo ONCE into LDS; the nine taps
//     are shifted reads of that image (16-B chunk swizzle: chunk c of LDS row r sits at
//     c ^ ((r>>1)&7), conflict-free ds_read_b128 over 16 consecutive pixel / channel rows);
//   * UP: the halo is the bilinear x2 upsample of a 6 x 18 source window, staged into LDS and
//     blended there in upsample2x_kernel's exact fp32 order (bit-identical to the separate
//     upsample), so the 4x larger upsampled image never goes through HBM;
//   * orientation D[co][px] = W[co][k] . X[k][px]: a lane owns one pixel and 4 consecutive
//     output channels per register group; each output row goes out through LDS as 1-KiB
//     contiguous 16-B-per-lane stores.
// 4 waves (one per SIMD, 512 registers): wave w computes output rows 2w, 2w+1 x 64 channels,
// 144 v_mfma_f32_32x32x16_bf16 per tile against 144 ds_read_b128 (1 per MFMA, inside the
// 2-per-gap LDS budget of MI355X_MICROARCH.md "LDS").  The next tile's global loads are issued
// before the current tile's MFMAs.
#include "common.h"

#include <type_traits>
#include <utility>

namespace mhada {

namespace {
constexpr int kTH = 8, kTW = 32;                  // output tile
constexpr int kHH = kTH + 2, kHW = kTW + 2;       // halo tile
constexpr int kHPIX = kHH * kHW;                  // 340
constexpr int kHCH = kHPIX * 8;                   // 16-B chunks of the halo image (64 ch)
constexpr int kSRH = kTH / 2 + 4, kSRW = kTW / 2 + 4;  // UP: source window 8 x 20 from (Y0/2-2, X0/2-2)
constexpr int kSCH = kSRH * kSRW * 8;
constexpr int kNT = 256;
constexpr int kXJ = (kHCH + kNT - 1) / kNT;       // halo chunks per thread (11)
constexpr int kSJ = (kSCH + kNT - 1) / kNT;       // source chunks per thread (5)
constexpr int kPBY = kTH / 2 + 2, kPBX = kTW / 2 + 2;  // UP interior: 2x2 output blocks covering the halo (6 x 18)
constexpr int kPB = kPBY * kPBX * 8;                  // (block, 8-channel chunk) items

// 128-B rows: 16 consecutive rows (a ds_read_b128 cycle) must hit 16 distinct 16-B bank
// groups = 8 * (row & 1) + chunk', hence chunk' = chunk ^ ((row >> 1) & 7)
MHADA_DEV int swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }
// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a release fence as well, which
// makes every wave drain its outstanding GLOBAL stores (vmcnt(0) counts stores on CDNA4) before
// the barrier: the tile's 16 epilogue stores per lane would then serialise with the next tile.
MHADA_DEV void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
MHADA_DEV int reflect_clamp(int v, int n) {
  v = v < 0 ? -v : (v >= n ? 2 * n - 2 - v : v);
  return min(max(v, 0), n - 1);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct ConvTileP {
  const bf16* x;      // NHWC [B][Hs][Ws][64]
  const bf16* w;      // [64][9*64], k = tap*64 + ci
  const float* bias;  // [64]
  bf16* y;            // NHWC [B][H][W][64]
  int B, H, W, Hs, Ws, tiles_x, tiles_y, ntiles, relu;
};
}  // namespace

template <bool UP>
__global__ void __launch_bounds__(kNT, 1) conv3x3_c64_kernel(const ConvTileP p) {
  __shared__ __attribute__((aligned(16))) bf16 sW[9 * 64 * 64];
  __shared__ __attribute__((aligned(16))) bf16 sX[kHPIX * 64];
  __shared__ __attribute__((aligned(16))) bf16 sS[UP ? kSRH * kSRW * 64 : 8];
  __shared__ __attribute__((aligned(16))) bf16 sO[4 * 32 * 64];  // per-wave output row staging
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;

  for (int i = tid; i < 9 * 64 * 8; i += kNT) {  // weights: LDS row = tap*64 + co
    const int row = i >> 3, c = i & 7, tap = row >> 6, co = row & 63;
    *reinterpret_cast<bf16x8*>(sW + swz(row, c)) =
        *reinterpret_cast<const bf16x8*>(p.w + (long long)co * 576 + tap * 64 + c * 8);
  }

  constexpr int NJ = UP ? kSJ : kXJ;
  bf16x8 stage[NJ];
  int hy_j[UP ? 1 : NJ], hx_j[UP ? 1 : NJ], c_j[UP ? 1 : NJ];  // tile-independent halo chunk coordinates
  if constexpr (!UP) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = min(tid + kNT * j, kHCH - 1), px = i >> 3;
      hy_j[j] = px / kHW;
      hx_j[j] = px - hy_j[j] * kHW;
      c_j[j] = (i & 7) * 8;
    }
  }
  auto tile_origin = [&](int t, int& b, int& Y0, int& X0) {
    const int per = p.tiles_x * p.tiles_y;
    b = t / per;
    const int r = t - b * per, ty = r / p.tiles_x;
    Y0 = ty * kTH;
    X0 = (r - ty * p.tiles_x) * kTW;
  };
  auto fetch = [&](int t) {  // global -> registers for tile t
    int b, Y0, X0;
    tile_origin(t, b, Y0, X0);
    if constexpr (UP) {
      const int sr0 = Y0 / 2 - 2, sc0 = X0 / 2 - 2;
      const bf16* xb = p.x + (long long)b * p.Hs * p.Ws * 64;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = min(tid + kNT * j, kSCH - 1), px = i >> 3, c = i & 7;
        const int sr = px / kSRW, sc = px - sr * kSRW;
        const int gy = min(max(sr0 + sr, 0), p.Hs - 1), gx = min(max(sc0 + sc, 0), p.Ws - 1);
        stage[j] = *reinterpret_cast<const bf16x8*>(xb + ((long long)gy * p.Ws + gx) * 64 + c * 8);
      }
    } else {
      const bf16* xb = p.x + (long long)b * p.H * p.W * 64;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gy = reflect_clamp(Y0 - 1 + hy_j[j], p.H), gx = reflect_clamp(X0 - 1 + hx_j[j], p.W);
        stage[j] = *reinterpret_cast<const bf16x8*>(xb + ((long long)gy * p.W + gx) * 64 + c_j[j]);
      }
    }
  };
  auto commit = [&](int t) {  // registers -> LDS halo image (UP: source window, then blend)
    if constexpr (UP) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = min(tid + kNT * j, kSCH - 1);
        *reinterpret_cast<bf16x8*>(sS + swz(i >> 3, i & 7)) = stage[j];
      }
      lds_barrier();
      int b, Y0, X0;
      tile_origin(t, b, Y0, X0);
      const int sr0 = Y0 / 2 - 2, sc0 = X0 / 2 - 2;
      // interior tile: every halo pixel's bilinear taps are the unclamped x2 pattern, so each
      // 2x2 output block (rows 2i, 2i+1, cols 2j, 2j+1 of the upsampled image) blends the 3x3
      // source neighbourhood of (i, j) with the constant weights 1/4, 3/4 -- 9 chunk reads for 4
      // outputs instead of 16; same expression (and rounding) as upsample2x_kernel
      const bool interior = Y0 >= 8 && Y0 + 12 <= p.H && X0 >= 32 && X0 + 36 <= p.W;
      if (interior) {
        for (int it = tid; it < kPB; it += kNT) {
          const int blk = it >> 3, c = it & 7, by = blk / kPBX, bx = blk - by * kPBX;
          // block (by, bx) covers upsampled rows Y0-2+2by .., cols X0-2+2bx ..; its centre source
          // pixel (Y0/2-1+by, X0/2-1+bx) is window pixel (by+1, bx+1)
          float v[3][3][8];
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(sS + swz((by + dy) * kSRW + bx + dx, c));
#pragma unroll
              for (int e = 0; e < 8; ++e) v[dy][dx][e] = (float)a[e];
            }
#pragma unroll
          for (int ey = 0; ey < 2; ++ey) {
            const int hy = 2 * by + ey - 1;  // halo row (upsampled row Y0 - 1 + hy)
            if (hy < 0 || hy >= kHH) continue;
            const float ly0 = ey ? 0.75f : 0.25f, ly1 = ey ? 0.25f : 0.75f;
#pragma unroll
            for (int ex = 0; ex < 2; ++ex) {
              const int hx = 2 * bx + ex - 1;
              if (hx < 0 || hx >= kHW) continue;
              const float lx0 = ex ? 0.75f : 0.25f, lx1 = ex ? 0.25f : 0.75f;
              bf16x8 o;
#pragma unroll
              for (int e = 0; e < 8; ++e)
                o[e] = (bf16)bilerp(ly0, ly1, lx0, lx1, v[ey][ex][e], v[ey][ex + 1][e], v[ey + 1][ex][e],
                                    v[ey + 1][ex + 1][e]);
              *reinterpret_cast<bf16x8*>(sX + swz(hy * kHW + hx, c)) = o;
            }
          }
        }
        return;
      }
      for (int i = tid; i < kHCH; i += kNT) {
        const int px = i >> 3, c = i & 7, hy = px / kHW, hx = px - hy * kHW;
        const int uy = reflect_clamp(Y0 - 1 + hy, p.H), ux = reflect_clamp(X0 - 1 + hx, p.W);
        // upsample2x_kernel's coordinates and blend order (align_corners = False)
        const float sy = fmaxf(((float)uy + 0.5f) * 0.5f - 0.5f, 0.f);
        const float sx = fmaxf(((float)ux + 0.5f) * 0.5f - 0.5f, 0.f);
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < p.Hs - 1 ? 1 : 0), x1 = x0 + (x0 < p.Ws - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
        const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
        const int r0 = (y0 - sr0) * kSRW, r1 = (y1 - sr0) * kSRW, c0 = x0 - sc0, c1 = x1 - sc0;
        const bf16x8 a00 = *reinterpret_cast<const bf16x8*>(sS + swz(r0 + c0, c));
        const bf16x8 a01 = *reinterpret_cast<const bf16x8*>(sS + swz(r0 + c1, c));
        const bf16x8 a10 = *reinterpret_cast<const bf16x8*>(sS + swz(r1 + c0, c));
        const bf16x8 a11 = *reinterpret_cast<const bf16x8*>(sS + swz(r1 + c1, c));
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          o[e] = (bf16)bilerp(ly0, ly1, lx0, lx1, (float)a00[e], (float)a01[e], (float)a10[e], (float)a11[e]);
        *reinterpret_cast<bf16x8*>(sX + swz(px, c)) = o;
      }
    } else {
      // unconditional: lanes past the end hold (and rewrite) the last chunk -- a conditional
      // store splits the block and hipcc then drains every outstanding store (vmcnt(0)) first
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = min(tid + kNT * j, kHCH - 1);
        *reinterpret_cast<bf16x8*>(sX + swz(i >> 3, i & 7)) = stage[j];
      }
    }
  };

  // bias of this lane's output channels: co = cb*32 + 8*g + 4*h + (0..3)
  f32x4 bias4[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) bias4[cb][g] = *reinterpret_cast<const f32x4*>(p.bias + cb * 32 + 8 * g + 4 * h);

  // operand fragments of k-step s (tap = s / 4, 16 input channels 16*(s % 4) ..): read one
  // k-step ahead of their MFMAs (one wave per SIMD has no partner to cover the LDS latency)
  auto frag = [&](const int s, bf16x8 (&wa)[2], bf16x8 (&xb)[2]) __attribute__((always_inline)) {
    const int tap = s >> 2, dy = tap / 3, dx = tap - 3 * dy, c = 2 * (s & 3) + h;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) wa[cb] = *reinterpret_cast<const bf16x8*>(sW + swz(tap * 64 + cb * 32 + r32, c));
#pragma unroll
    for (int pb = 0; pb < 2; ++pb)
      xb[pb] = *reinterpret_cast<const bf16x8*>(sX + swz((2 * wave + pb + dy) * kHW + r32 + dx, c));
  };

  int t = blockIdx.x;
  if (t < p.ntiles) fetch(t);
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(stage[j]));  // no loads pending at the loop head
  for (; t < p.ntiles; t += gridDim.x) {
    lds_barrier();  // every wave is done reading the previous tile's halo image
    commit(t);
    lds_barrier();
    // next tile's loads (clamped: the last tile re-fetches itself, unused), in the same basic
    // block as the MFMA stream so their address VALU can fill MFMA gaps
    fetch(min(t + (int)gridDim.x, p.ntiles - 1));

    f32x16 acc[2][2];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][pb][e] = 0.f;
    bf16x8 wa[2][2], xb[2][2];
    frag(0, wa[0], xb[0]);
#pragma unroll
    for (int s = 0; s < 36; ++s) {
      if (s + 1 < 36) frag(s + 1, wa[(s + 1) & 1], xb[(s + 1) & 1]);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int pb = 0; pb < 2; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s & 1][cb], xb[s & 1][pb], acc[cb][pb], 0, 0, 0);
    }
    // consume the next tile's staged loads HERE, before this tile's stores are issued: hipcc
    // treats loads and stores as completing out of order, so a wait placed after the stores
    // (in the next commit) becomes vmcnt(0) and drains them; here the loads are long complete
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(stage[j]));
    int b, Y0, X0;
    tile_origin(t, b, Y0, X0);
    // Output: each wave stages one 32-pixel output row (32 x 128 B) in its private LDS slab and
    // writes it back as whole 16-B chunks (one contiguous 1 KiB per store instruction); direct
    // 8-byte per-lane stores at a 128-B pixel stride ran the store path at ~1.4 TB/s.
    // Buffer-descriptor stores: chunks outside the image get an offset past num_records and are
    // dropped by the hardware (no branch around the stores).
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        p.y + (long long)b * p.H * p.W * 64, 0, p.H * p.W * 64 * 2, 0x00020000);
    bf16* so = sO + wave * (32 * 64);
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[cb][pb][4 * g + e] + bias4[cb][g][e];
            if (p.relu) v = fmaxf(v, 0.f);
            o[e] = (bf16)v;
          }
          *reinterpret_cast<bf16x4*>(so + swz(r32, cb * 4 + g) + 4 * h) = o;
        }
      const int oy = Y0 + 2 * wave + pb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = lane + 64 * i, px = q >> 3, c = q & 7, ox = X0 + px;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(so + swz(px, c));
        const int off = (oy < p.H && ox < p.W) ? ((oy * p.W + ox) * 64 + c * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yr, off, 0, 0);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Direct 3x3 convolution for the decoder's 128 / 256-input-channel layers (conv.py:75-100: conv2.0
// 128 -> 128 and conv2.1 128 -> 64 at half the output resolution, conv1.4 256 -> 128), bf16 MFMA,
// fp32 accumulation, reflect pad 1, bias + ReLU, NHWC.  The implicit GEMM ran the first two at
// 14-16 % of the bf16 peak (K = 1152, N <= 128: per-tile prologue / epilogue, every input pixel
// gathered 9 times).  Here (Cin = 128; Cin = 256 uses 4-row tiles, see below):
//   * the output tile of 8 x 32 pixels stages its 10 x 34 x 128-channel halo ONCE in LDS
//     (85 KiB; 256-B pixel rows, chunk c at c ^ (row & 15): conflict-free ds_read_b128 over 16
//     consecutive pixels), prefetched into registers during the previous tile's MFMAs;
//   * the weights (147 / 295 KiB: too large to stay resident next to the halo) stream through a
//     3-slot LDS-DMA ring of 16-KiB stages — one tap (Cout = 64) or half a tap (Cout = 128) — by
//     buffer loads with per-lane constant offsets; the stage sequence repeats per tile, so the
//     ring runs on across tiles.  ONE barrier per stage, placed before the stage's last k-step:
//     it proves every wave has read the stage's slot (the last k-step's fragments are already
//     in registers) and publishes the next stage, whose first fragments are then read beside
//     that last k-step's MFMAs.  The slots are three separate __shared__ objects and the DMA
//     issue is pinned after the barrier (see the comments at sW0 and at the DMA call);
//   * 4 waves (one per SIMD), wave w = output rows 2w, 2w+1 x all Cout: per 16-channel k-step
//     Cout/32 + 2 ds_read_b128 per 2 Cout/32 MFMAs (v_mfma_f32_32x32x16_bf16), within the LDS
//     budget of one read per MFMA; output rows staged in LDS (aliasing the halo after a barrier)
//     and stored as 16-B chunks through a buffer descriptor, as conv3x3_c64_kernel.
// ---------------------------------------------------------------------------------------------
namespace {
template <typename F, int... I>
MHADA_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(std::integral_constant<int, i>) for i = 0 .. N-1, unrolled at compile time
template <int N, typename F>
MHADA_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
constexpr int kDStage = 8192;                                 // bf16 elements per weight stage (16 KiB)
constexpr int kDSlots = 3;
}  // namespace

// CIN = 128: 8 x 32-pixel tiles (10 x 34 halo, 85 KiB), wave w = output rows 2w, 2w+1;
// CIN = 256: 4 x 32-pixel tiles (6 x 34 halo, 102 KiB), wave w = output row w.
template <int CIN, int COUT>
__global__ void __launch_bounds__(kNT, 1) conv3x3_dir_kernel(const ConvTileP p) {
  constexpr int TH = CIN == 128 ? 8 : 4, PB = TH / 4;   // tile rows, output rows per wave
  constexpr int HPIX = (TH + 2) * kHW;                  // halo pixels
  constexpr int CCH = CIN / 8;                          // 16-B chunks per halo pixel
  constexpr int XJ = (HPIX * CCH + kNT - 1) / kNT;      // halo chunks per thread (22 / 26)
  static_assert(CIN == 128 || CIN == 256, "Cin");
  // halo pixel rows of CIN channels, chunk c at c ^ (row & 15): 16 consecutive pixels hit 16
  // distinct 16-B bank groups (the row stride is a multiple of the 256-B bank width)
  auto hswz = [](int row, int chunk) { return row * CIN + ((chunk ^ (row & 15)) << 3); };
  constexpr int KS = kDStage / COUT;        // input channels per stage: 128 (a tap) or 64 (half a tap)
  constexpr int SPT = CIN / KS;             // stages per tap
  constexpr int NST = 9 * SPT;              // stages per tile
  constexpr int WCH = KS / 8;               // 16-B chunks per weight row (16 or 8)
  constexpr int KSTEP = KS / 16;            // k-steps per stage
  constexpr int CB = COUT / 32;             // 32-channel output blocks
  constexpr int RPI = 64 / WCH;             // weight rows per DMA instruction (1 KiB)
  constexpr int DPW = kDStage * 2 / 1024 / 4;  // DMA instructions per wave per stage (4)
  constexpr int ST = PB * (COUT / 16);         // output stores per lane and tile
  static_assert(KS * COUT == kDStage && (WCH == 16 || WCH == 8), "stage shape");
  // NST is a multiple of the ring depth, so every tile's stage s sits in slot s % kDSlots: the
  // slots are compile-time constants (with runtime slots hipcc cannot prove the DMA's LDS writes
  // disjoint from the fragment reads and drains every DMA with vmcnt(0) before the next read)
  static_assert(NST % kDSlots == 0, "ring depth must divide the stage count");
  __shared__ __attribute__((aligned(16))) bf16 sX[HPIX * CIN];
  // the ring slots are three separate LDS objects: hipcc's wait insertion tells an LDS-DMA write
  // and a later ds_read apart only by the object they address (within one array it drains the DMA
  // with vmcnt(0) before every fragment read)
  __shared__ __attribute__((aligned(16))) bf16 sW0[kDStage];
  __shared__ __attribute__((aligned(16))) bf16 sW1[kDStage];
  __shared__ __attribute__((aligned(16))) bf16 sW2[kDStage];
  static_assert(kDSlots == 3, "three ring objects");
  auto slot = [&](auto S_) -> bf16* {
    constexpr int k = decltype(S_)::value % kDSlots;
    if constexpr (k == 0) return sW0;
    else if constexpr (k == 1) return sW1;
    else return sW2;
  };
  __shared__ __attribute__((aligned(16))) float sB[COUT];  // bias (the epilogue reads LDS, not HBM: a
                                                          // global load there would wait on the DMA ahead)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  typedef __attribute__((address_space(3))) void* LdsP;
  // weight rows: 128-B rows (KS = 64) use conv3x3_c64's swizzle, 256-B rows the halo's
  auto wswz = [](int row, int chunk) {
    return WCH == 8 ? swz(row, chunk) : row * 128 + ((chunk ^ (row & 15)) << 3);
  };
  // DMA: instruction j = DPW * wave + i covers weight rows RPI j .. + RPI; lane -> row RPI j + lane / WCH,
  // LDS slot lane % WCH, which holds chunk (slot ^ swizzle(row)) of the row.  Offsets in bytes into w
  // (row co of the packed [Cout][9 * 128] weights); the stage adds tap * 128 + part * KS channels.
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p.w), 0, COUT * 9 * CIN * 2, 0x00020000);
  unsigned wvo[DPW];
#pragma unroll
  for (int i = 0; i < DPW; ++i) {
    const int row = RPI * (DPW * wave + i) + lane / WCH, slot = lane % WCH;
    const int chunk = WCH == 8 ? slot ^ ((row >> 1) & 7) : slot ^ (row & 15);
    wvo[i] = (unsigned)(row * 9 * CIN + chunk * 8) * 2u;
  }
  auto dma = [&](auto G_) {  // stage G (mod NST) into slot G % kDSlots
    constexpr int gs = decltype(G_)::value % NST, tap = gs / SPT, part = gs - tap * SPT;
    bf16* dst = slot(G_);
#pragma unroll
    for (int i = 0; i < DPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (LdsP)(dst + 512 * (DPW * wave + i)), 16, wvo[i],
                                               (tap * CIN + part * KS) * 2, 0, 0);
  };

  bf16x8 stage[XJ];
  auto tile_origin = [&](int t, int& b, int& Y0, int& X0) {
    const int per = p.tiles_x * p.tiles_y;
    b = t / per;
    const int r = t - b * per, ty = r / p.tiles_x;
    Y0 = ty * TH;
    X0 = (r - ty * p.tiles_x) * kTW;
  };
  auto fetch = [&](int t) {
    int b, Y0, X0;
    tile_origin(t, b, Y0, X0);
    const bf16* xb = p.x + (long long)b * p.H * p.W * CIN;
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int i = min(tid + kNT * j, HPIX * CCH - 1), px = i / CCH, hy = px / kHW, hx = px - hy * kHW;
      const int gy = reflect_clamp(Y0 - 1 + hy, p.H), gx = reflect_clamp(X0 - 1 + hx, p.W);
      stage[j] = *reinterpret_cast<const bf16x8*>(xb + ((long long)gy * p.W + gx) * CIN + (i % CCH) * 8);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
      const int i = min(tid + kNT * j, HPIX * CCH - 1);
      *reinterpret_cast<bf16x8*>(sX + hswz(i / CCH, i % CCH)) = stage[j];
    }
  };

  // fragments of k-step ks of stage s (slot sl): weights co = cb*32 + r32, the lane half's 8 channels;
  // pixels of output rows 2 wave + pb, column r32, shifted by the stage's tap
  auto frag = [&](auto S_, const int ks, bf16x8 (&wa)[CB], bf16x8 (&xb)[PB]) __attribute__((always_inline)) {
    constexpr int s = decltype(S_)::value, tap = s / SPT, part = s - tap * SPT, dy = tap / 3, dx = tap - 3 * dy;
    const bf16* ws = slot(S_);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) wa[cb] = *reinterpret_cast<const bf16x8*>(ws + wswz(cb * 32 + r32, 2 * ks + h));
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
      xb[pb] = *reinterpret_cast<const bf16x8*>(
          sX + hswz((PB * wave + pb + dy) * kHW + r32 + dx, part * (KS / 8) + 2 * ks + h));
  };

  int t = blockIdx.x;
  const int first = t;
  if (t >= p.ntiles) return;
  for (int i = tid; i < COUT; i += kNT) sB[i] = p.bias[i];
  dma(std::integral_constant<int, 0>{});
  dma(std::integral_constant<int, 1>{});
  dma(std::integral_constant<int, 2>{});
  fetch(t);
  for (; t < p.ntiles; t += gridDim.x) {
    if (t != first) lds_barrier();  // every wave is done with the previous tile's output staging (halo alias)
    commit();
    // the first tile: the halo loads are waited for above (the newest loads), so stages 0..2 have landed
    lds_barrier();
    fetch(min(t + (int)gridDim.x, p.ntiles - 1));

    f32x16 acc[CB][PB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int pb = 0; pb < PB; ++pb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[cb][pb][e] = 0.f;
    bf16x8 wa[2][CB], xb[2][PB];
    frag(std::integral_constant<int, 0>{}, 0, wa[0], xb[0]);
    // NST stages x KSTEP k-steps, fully unrolled: every ring slot, buffer and wait count is a constant
    auto step = [&](auto S_, auto K_) __attribute__((always_inline)) {
      constexpr int s = decltype(S_)::value, ks = decltype(K_)::value, q = (s * KSTEP + ks) & 1;
      if constexpr (ks + 1 < KSTEP) {
        frag(S_, ks + 1, wa[q ^ 1], xb[q ^ 1]);
      } else {
        // this stage's slot is fully read by this wave: wait for our DMA of stage s + 1, barrier
        // (publishes it; every wave is past stage s's reads), refill the slot of stage s with s + 3
        // (stages 0 and 1: the ops issued since that DMA include the previous tile's ST output
        // stores and this tile's kDXJ halo loads; vmcnt counts both, in issue order)
        if constexpr (s < 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW + ST + XJ) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // bare: a __syncthreads() would drain the DMA ahead (vmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
        dma(std::integral_constant<int, s + 3>{});
        __builtin_amdgcn_sched_barrier(0);  // issue the DMA here, two stages ahead (not sunk to the next wait)
        if constexpr (s + 1 < NST) frag(std::integral_constant<int, s + 1>{}, 0, wa[q ^ 1], xb[q ^ 1]);
      }
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int pb = 0; pb < PB; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[q][cb], xb[q][pb], acc[cb][pb], 0, 0, 0);
    };
    static_for<NST>([&](auto S_) { static_for<KSTEP>([&](auto K_) { step(S_, K_); }); });
    // the next tile's halo loads complete here, before this tile's stores (see conv3x3_c64_kernel)
#pragma unroll
    for (int j = 0; j < XJ; ++j) asm volatile("" ::"v"(stage[j]));
    lds_barrier();  // every wave's last halo reads are done: the output staging may alias the halo
    int b, Y0, X0;
    tile_origin(t, b, Y0, X0);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        p.y + (long long)b * p.H * p.W * COUT, 0, p.H * p.W * COUT * 2, 0x00020000);
    bf16* so = sX + wave * (32 * COUT);
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      // row r32 (pixel) of the staging slab, COUT channels = COUT / 8 chunks (swizzled by pixel)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          // bias from LDS per tile: 4 x CB registers of bias would not fit beside the halo
          // prefetch and the accumulators at Cout = 128
          const f32x4 bb = *reinterpret_cast<const f32x4*>(sB + cb * 32 + 8 * gq + 4 * h);
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[cb][pb][4 * gq + e] + bb[e];
            if (p.relu) v = fmaxf(v, 0.f);
            o[e] = (bf16)v;
          }
          const int ch = cb * 4 + gq;  // 16-B chunk of the pixel's COUT channels
          *reinterpret_cast<bf16x4*>(so + r32 * COUT + ((ch ^ (r32 & (COUT / 8 - 1))) << 3) + 4 * h) = o;
        }
      const int oy = Y0 + PB * wave + pb;
#pragma unroll
      for (int i = 0; i < COUT / 16; ++i) {  // one output row: 32 pixels x COUT channels in 16-B chunks
        const int qd = lane + 64 * i, px = qd / (COUT / 8), c = qd % (COUT / 8), ox = X0 + px;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(so + px * COUT + ((c ^ (px & (COUT / 8 - 1))) << 3));
        const int off = (oy < p.H && ox < p.W) ? ((oy * p.W + ox) * COUT + c * 8) * 2 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yr, off, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA left in flight at exit
}

// Host side, called from mhada_gemm for a bf16 CONV3X3 GEMM with (Cin, Cout) in {(128, 64), (128, 128),
// (256, 128)}.
int conv3x3_dir(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int cin, int cout,
                int relu, hipStream_t s) {
  ConvTileP p;
  p.x = (const bf16*)x; p.w = (const bf16*)w; p.bias = bias; p.y = (bf16*)y;
  p.B = B; p.H = H; p.W = W; p.relu = relu;
  p.Hs = H; p.Ws = W;
  const int th = cin == 128 ? 8 : 4;
  p.tiles_x = (W + kTW - 1) / kTW;
  p.tiles_y = (H + th - 1) / th;
  const long long nt = (long long)B * p.tiles_x * p.tiles_y;
  if (nt >= (1LL << 31)) return fail("conv3x3_dir: too many tiles");
  if ((long long)H * W * cin * 2 >= 0x7ff00000LL) return fail("conv3x3_dir: image too large for 32-bit offsets");
  p.ntiles = (int)nt;
  const int grid = (int)std::min<long long>(nt, 256);
  if (cin == 128 && cout == 64) hipLaunchKernelGGL((conv3x3_dir_kernel<128, 64>), dim3(grid), dim3(kNT), 0, s, p);
  else if (cin == 128 && cout == 128) hipLaunchKernelGGL((conv3x3_dir_kernel<128, 128>), dim3(grid), dim3(kNT), 0, s, p);
  else if (cin == 256 && cout == 128) hipLaunchKernelGGL((conv3x3_dir_kernel<256, 128>), dim3(grid), dim3(kNT), 0, s, p);
  else return fail("conv3x3_dir: (Cin, Cout) must be (128, 64), (128, 128) or (256, 128)");
  return check_launch("conv3x3_dir");
}

// Host side, called from mhada_gemm for a bf16 CONV3X3 / CONV3X3_UP2 GEMM with Cin = Cout = 64
// (the caller has validated the GEMM arguments).  H, W: OUTPUT size.
int conv3x3_c64(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, bool up, int relu,
                hipStream_t s) {
  ConvTileP p;
  p.x = (const bf16*)x; p.w = (const bf16*)w; p.bias = bias; p.y = (bf16*)y;
  p.B = B; p.H = H; p.W = W; p.relu = relu;
  p.Hs = up ? H / 2 : H; p.Ws = up ? W / 2 : W;
  p.tiles_x = (W + kTW - 1) / kTW;
  p.tiles_y = (H + kTH - 1) / kTH;
  const long long nt = (long long)B * p.tiles_x * p.tiles_y;
  if (nt >= (1LL << 31)) return fail("conv3x3_c64: too many tiles");
  p.ntiles = (int)nt;
  const int grid = (int)std::min<long long>(nt, 256);
  if (up) hipLaunchKernelGGL(conv3x3_c64_kernel<true>, dim3(grid), dim3(kNT), 0, s, p);
  else hipLaunchKernelGGL(conv3x3_c64_kernel<false>, dim3(grid), dim3(kNT), 0, s, p);
  return check_launch("conv3x3_c64");
}

}  // namespace mhada
