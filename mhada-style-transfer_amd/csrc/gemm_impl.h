// GEMM kernel templates and tile dispatch (included by the per-dtype dispatch units
// gemm_d_*.hip, which instantiate them in parallel translation units, and by gemm.hip for the
// argument checks of the C entry point).
#pragma once
// Batched NT GEMM on MFMA with fused A-gathers (rows / 8x8 patches / reflect-padded 3x3
// taps with optional bilinear x2) and a fused bias/ReLU/residual epilogue.
//
// One kernel body serves every dense contraction of the forward path except the MHAda
// attention itself: ViT patch embedding, QKV/out/MLP projections, the per-head 1x1 convs of
// the MHAda blocks and the implicit-GEMM decoder convolutions (see include/mhada_hip.h).
//
// Tiling (gfx950): 256 threads = 4 waves, each wave owns a 64x64 output sub-tile made of
// 2x2 32x32 MFMA blocks.  Block tile 128x128 (waves 2x2) or 256x64 (waves 4x1, for N=64
// problems).  K is staged 128 bytes per step (BK = 32 fp32 / 64 bf16) through a double-
// buffered LDS image whose rows are padded to 144 B, which makes the per-lane 16-byte row
// reads of both operands conflict-free (rows distinct mod 16 land on distinct 16-B slots).
// Global->register loads of tile k+1 are issued before the MFMAs of tile k and written to
// LDS after them (register-staged async split).
#include "common.h"

#include <algorithm>
#include <mutex>
#include <stdlib.h>

namespace mhada {

struct GemmP {
  int M, N, K, nb2;
  const void* a; long long lda, sa1, sa2;
  const float* a_mu; long long smu1, smu2;
  int img_c, img_h, img_w, out_h, out_w;
  int pad;  // CONV3X3_ZERO: input coordinate = output + tap - pad (zero outside the image)
  const void* w; long long ldw, sw1, sw2;
  const float* bias; long long sb1, sb2;
  const void* r; long long ldr, sr1, sr2;
  void* c; long long ldc, sc1, sc2;
  int relu, tiles_n, ntiles;
  int lds_epi;  // ping-pong kernels: stage the output through LDS (tuning gemm_ldsepi = 0: direct stores)
  int rinit;    // persistent ping-pong, fp32 C, no ReLU: residual + bias loaded into the accumulators
  void* c2; long long ldc2, sc21, sc22;  // optional bf16 copy of an fp32 C
  void* vt; long long ldt, svt1, svt2;   // optional transposed V' image (K|V' projection, N = 128)
  long long spl;  // MHADA_A_SPLIT3: element stride between the three bf16 planes of A (M * lda)
  int c2planes;   // c2 = three bf16 planes [3][M][ldc2] of the fp32 result (C may be null)
};

template <typename TC> struct Cfg {
  static constexpr int E = 16 / sizeof(TC);    // compute elements per 16-B chunk
  static constexpr int BK = 128 / sizeof(TC);  // K per stage (128 B rows)
  static constexpr int LS = BK + E;            // padded LDS row (144 B)
};

// One 16-byte chunk of compute-type elements, as raw global data (converted late).
template <typename TA, typename TC> struct RawChunk;
template <> struct RawChunk<float, float> { f32x4 v; };
template <> struct RawChunk<bf16, bf16> { bf16x8 v; };
template <> struct RawChunk<float, bf16> { f32x4 lo, hi; };

template <typename TA, typename TC>
MHADA_DEV RawChunk<TA, TC> load_raw(const TA* p) {
  RawChunk<TA, TC> r;
  if constexpr (sizeof(TA) == sizeof(TC)) {
    r.v = *reinterpret_cast<const typename Vec16<TA>::type*>(p);
  } else {
    r.lo = *reinterpret_cast<const f32x4*>(p);
    r.hi = *reinterpret_cast<const f32x4*>(p + 4);
  }
  return r;
}

template <typename TA, typename TC>
MHADA_DEV RawChunk<TA, TC> zero_raw() {
  RawChunk<TA, TC> r;
  if constexpr (sizeof(TA) == sizeof(TC)) {
#pragma unroll
    for (int i = 0; i < 16 / (int)sizeof(TA); ++i) r.v[i] = (TA)0.0f;
  } else {
    r.lo = f32x4{0.f, 0.f, 0.f, 0.f};
    r.hi = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  return r;
}

// element i of a raw chunk as fp32
template <typename TA, typename TC>
MHADA_DEV float raw_get(const RawChunk<TA, TC>& r, int i) {
  if constexpr (sizeof(TA) == sizeof(TC)) {
    return (float)r.v[i];
  } else {
    return i < 4 ? r.lo[i] : r.hi[i - 4];
  }
}

template <typename TC>
MHADA_DEV void store_chunk(TC* dst, const float (&f)[Cfg<TC>::E]) {
  typename Vec16<TC>::type v;
#pragma unroll
  for (int i = 0; i < Cfg<TC>::E; ++i) v[i] = from_f32<TC>(f[i]);
  *reinterpret_cast<typename Vec16<TC>::type*>(dst) = v;
}

MHADA_DEV int reflect1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// 16 zero bytes per lane for LDS-DMA staging of zero-padding taps (a glds cannot write zeros)
static __device__ __attribute__((aligned(16))) float g_zero16[4];

// Source pixel of output (y, x) under 3x3 tap offset (dy, dx) in {-1,0,1}: reflect modes fold
// the coordinate back into the (output) grid (ReflectionPad2d(1)); CONV3X3_ZERO shifts by
// 1 - pad and reports taps outside the input as zero padding (returns false).
template <int AMODE>
MHADA_DEV bool conv_src(const GemmP& p, int y, int x, int dy, int dx, int& Y, int& X) {
  if constexpr (AMODE == MHADA_A_CONV3X3_ZERO) {
    Y = y + dy + 1 - p.pad;
    X = x + dx + 1 - p.pad;
    return Y >= 0 && Y < p.img_h && X >= 0 && X < p.img_w;
  } else {
    Y = reflect1(y + dy, p.out_h);
    X = reflect1(x + dx, p.out_w);
    return true;
  }
}

// Internal A mode: ROWS with per-column centring (a_mu != NULL), a separate instantiation so
// the plain ROWS path stages raw chunks with no per-element work.
constexpr int kRowsCentred = 100;
// MHADA_A_SPLIT3 (fp32-accurate products on the bf16 MFMA): A is three bf16 planes p0 + p1 + p2 of
// an fp32 matrix (8 + 8 + 8 mantissa bits), the GEMM's K = 6 K0 is virtual: K-tile 6 kk + t reads
// columns 64 kk .. of plane kSplitPlanes[t] = 1, 2, 0, 1, 0, 0, and W holds the matching [N][6 K0]
// interleave (chunk kk of q1, q0, q2, q0, q1, q0), so the fp32 accumulators sum p1 q1 + p2 q0 +
// p0 q2 + p1 q0 + p0 q1 + p0 q0 chunk by chunk: every cross product p_i q_j with i + j <= 2.  With
// round-to-nearest planes |p1| <= 2^-8 |x|, |p2| <= 2^-16 |x| (likewise q), so the three dropped
// terms are below 2^-24 |x w| (p1 q2 and p2 q1) and 2^-32 |x w| (p2 q2) per product.
constexpr int kRowsSplit3 = 101;
constexpr int kSplitPlanes = 0x001021;  // nibble t = plane of K-block t

// ------------------------------------------------------------------------------------
// A-operand staging for one K step.  Each thread owns A_CH chunks: rows (tid>>3)+32*i,
// 16-byte column kc = tid&7.
// ------------------------------------------------------------------------------------
template <typename TA, typename TC, int AMODE, int A_CH>
struct AStage {
  static constexpr int NT = (AMODE == MHADA_A_CONV3X3_UP2) ? 4 : 1;  // bilinear taps
  RawChunk<TA, TC> raw[A_CH][NT];
  float wt[A_CH][NT];
  float mu[Cfg<TC>::E];
};

struct RowInfo {  // per staged row: CONV -> (b, y, x); ROWS/PATCH -> linear offsets
  int b, y, x;
  bool valid;
};

template <typename TA, typename TC, int AMODE, int A_CH>
MHADA_DEV void issue_a(AStage<TA, TC, AMODE, A_CH>& st, const GemmP& p, const TA* abase,
                       const RowInfo (&ri)[A_CH], int k0, int kc) {
  constexpr int E = Cfg<TC>::E;
  const int k = k0 + kc * E;
  const bool kvalid = k < p.K;
  if constexpr (AMODE == MHADA_A_ROWS || AMODE == kRowsCentred) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const long long m = (long long)ri[i].b;  // row index within the z problem
      st.raw[i][0] = (ri[i].valid && kvalid) ? load_raw<TA, TC>(abase + m * p.lda + k) : zero_raw<TA, TC>();
      st.wt[i][0] = 1.f;
    }
    if constexpr (AMODE == kRowsCentred) {
#pragma unroll
      for (int e = 0; e < E; ++e) st.mu[e] = kvalid ? p.a_mu[k + e] : 0.f;
    }
  } else if constexpr (AMODE == MHADA_A_PATCH8) {
    // k = c*64 + py*8 + px ; E | 8 so a chunk stays inside one image row
    const int cch = k >> 6, py = (k >> 3) & 7, px = k & 7;
    const long long plane = (long long)p.img_h * p.img_w;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const TA* src = abase + cch * plane + (long long)(ri[i].y * 8 + py) * p.img_w + ri[i].x * 8 + px;
      st.raw[i][0] = (ri[i].valid && kvalid) ? load_raw<TA, TC>(src) : zero_raw<TA, TC>();
      st.wt[i][0] = 1.f;
    }
  } else {
    // implicit GEMM 3x3: k = tap*Cin + cin; a K step never straddles a tap (Cin % BK == 0)
    const int cin_n = p.img_c;
    const int tap = k / cin_n, cin = k - tap * cin_n;
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int Y, X;
      const bool inside = conv_src<AMODE>(p, ri[i].y, ri[i].x, dy, dx, Y, X);
      const bool ok = ri[i].valid && kvalid && inside;
      if constexpr (AMODE == MHADA_A_CONV3X3 || AMODE == MHADA_A_CONV3X3_ZERO) {
        const TA* src = abase + (((long long)ri[i].b * p.img_h + Y) * p.img_w + X) * cin_n + cin;
        st.raw[i][0] = ok ? load_raw<TA, TC>(src) : zero_raw<TA, TC>();
        st.wt[i][0] = 1.f;
      } else {
        // bilinear x2, align_corners=False (upsample_bilinear2d): src = 0.5*(dst+0.5)-0.5
        const float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.f);
        const float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.f);
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < p.img_h - 1 ? 1 : 0), x1 = x0 + (x0 < p.img_w - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
        const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
        const long long rb = (long long)ri[i].b * p.img_h;
        const TA* s00 = abase + ((rb + y0) * p.img_w + x0) * cin_n + cin;
        const TA* s01 = abase + ((rb + y0) * p.img_w + x1) * cin_n + cin;
        const TA* s10 = abase + ((rb + y1) * p.img_w + x0) * cin_n + cin;
        const TA* s11 = abase + ((rb + y1) * p.img_w + x1) * cin_n + cin;
        st.raw[i][0] = ok ? load_raw<TA, TC>(s00) : zero_raw<TA, TC>();
        st.raw[i][1] = ok ? load_raw<TA, TC>(s01) : zero_raw<TA, TC>();
        st.raw[i][2] = ok ? load_raw<TA, TC>(s10) : zero_raw<TA, TC>();
        st.raw[i][3] = ok ? load_raw<TA, TC>(s11) : zero_raw<TA, TC>();
        // PyTorch blends h0*(w0*x00 + w1*x01) + h1*(w0*x10 + w1*x11)
        st.wt[i][0] = ly0; st.wt[i][1] = ly1; st.wt[i][2] = lx0; st.wt[i][3] = lx1;
      }
    }
  }
}

template <int RS, typename TA, typename TC, int AMODE, int A_CH>
MHADA_DEV void commit_a(const AStage<TA, TC, AMODE, A_CH>& st, TC* sA, int tid) {
  constexpr int E = Cfg<TC>::E, LS = Cfg<TC>::LS;
  const int kc = tid & 7;
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int row = (tid >> 3) + RS * i;
    float f[E];
    if constexpr (AMODE == MHADA_A_CONV3X3_UP2) {
      const float ly0 = st.wt[i][0], ly1 = st.wt[i][1], lx0 = st.wt[i][2], lx1 = st.wt[i][3];
#pragma unroll
      for (int e = 0; e < E; ++e)
        f[e] = bilerp(ly0, ly1, lx0, lx1, raw_get(st.raw[i][0], e), raw_get(st.raw[i][1], e),
                      raw_get(st.raw[i][2], e), raw_get(st.raw[i][3], e));
    } else if constexpr (AMODE == kRowsCentred || sizeof(TA) != sizeof(TC)) {
#pragma unroll
      for (int e = 0; e < E; ++e) f[e] = raw_get(st.raw[i][0], e) - (AMODE == kRowsCentred ? st.mu[e] : 0.f);
    } else {
      // same type, no centring: the raw 16-byte chunk goes to LDS untouched
      *reinterpret_cast<typename Vec16<TC>::type*>(sA + row * LS + kc * E) = st.raw[i][0].v;
      continue;
    }
    store_chunk<TC>(sA + row * LS + kc * E, f);
  }
}

// Epilogue shared by the GEMM kernels.  The MFMAs take W as the A operand, so each
// accumulator holds C^T: the lane owns ONE output row m (mrow + 32*mi) and registers
// 4g..4g+3 of acc[mi][ni] hold the 4 consecutive columns ncol + 32*ni + 8g + 4h + 0..3 — every
// store moves 4 elements (8-16 B) instead of one (a row-per-lane scalar-store tail is
// store-issue bound).  Fused: + bias[n], ReLU, + residual r[m][n] (after the ReLU).
template <typename TO, int TM, int TN>
MHADA_DEV void store_tile(const GemmP& p, const f32x16 (&acc)[TM][TN], int z1, int z2, int mrow, int ncol, int h) {
  TO* cbase = reinterpret_cast<TO*>(p.c) + z1 * p.sc1 + z2 * p.sc2;
  const TO* rbase = p.r ? reinterpret_cast<const TO*>(p.r) + z1 * p.sr1 + z2 * p.sr2 : nullptr;
  const float* bbase = p.bias ? p.bias + z1 * p.sb1 + z2 * p.sb2 : nullptr;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m = mrow + mi * 32;
    if (m >= p.M) continue;
    TO* crow = cbase + (long long)m * p.ldc;
    const TO* rrow = rbase ? rbase + (long long)m * p.ldr : nullptr;
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = ncol + ni * 32 + 8 * g + 4 * h;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[mi][ni][4 * g + e];
        if (n + 3 < p.N) {
          if (bbase) {
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bbase + n);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bb[e];
          }
          if (p.relu == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if constexpr (sizeof(TO) == 4) {
            if (rrow) {
              const f32x4 rr = *reinterpret_cast<const f32x4*>(rrow + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = p.relu == 2 ? (rr[e] > 0.f ? v[e] : 0.f) : v[e] + rr[e];
            }
            *reinterpret_cast<f32x4*>(crow + n) = f32x4{v[0], v[1], v[2], v[3]};
            if (p.c2)
              *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p.c2) + z1 * p.sc21 + z2 * p.sc22 +
                                         (long long)m * p.ldc2 + n) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          } else {
            if (rrow) {
              const bf16x4 rr = *reinterpret_cast<const bf16x4*>(rrow + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += (float)rr[e];
            }
            *reinterpret_cast<bf16x4*>(crow + n) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (n + e < p.N) {
              float x = v[e] + (bbase ? bbase[n + e] : 0.f);
              if (p.relu == 1) x = fmaxf(x, 0.f);
              if (rrow) x = p.relu == 2 ? (to_f32<TO>(rrow[n + e]) > 0.f ? x : 0.f) : x + to_f32<TO>(rrow[n + e]);
              crow[n + e] = from_f32<TO>(x);
            }
          }
        }
      }
    }
  }
}


// Epilogue through a per-wave LDS scratch (4 KiB = one 32x32 fp32 block): the accumulator
// block (lane = row r32, 4-column groups 8g + 4h) is written raw, read back row-major (lane =
// row 8i + (lane >> 3), columns 4 (lane & 7) .. +3) and stored so that one store instruction
// covers 8 rows x 32 columns (64-128 contiguous bytes per row) instead of 32 rows x 16 B;
// bias, ReLU and the residual (read in the same coalesced layout) are applied in row layout.
// The 16-B chunk c of row r sits at slot c ^ (r & 7) (spreads both the column-group writes and
// the row reads over the banks).  No barrier: each wave owns its scratch.
// PLANES (the SPLIT3 kernel only): c2 may hold the result's three bf16 planes and C may be null.
template <typename TO, int TM, int TN, bool PLANES = false>
MHADA_DEV void store_tile_lds(const GemmP& p, const f32x16 (&acc)[TM][TN], int z1, int z2, int mrow0, int ncol0,
                              int lane, float* scr) {
  TO* cbase = reinterpret_cast<TO*>(p.c) + z1 * p.sc1 + z2 * p.sc2;
  const TO* rbase = p.r ? reinterpret_cast<const TO*>(p.r) + z1 * p.sr1 + z2 * p.sr2 : nullptr;
  const float* bbase = p.bias ? p.bias + z1 * p.sb1 + z2 * p.sb2 : nullptr;
  const int h = lane >> 5, r32 = lane & 31;
  const int rr = lane >> 3, cq = lane & 7;  // read-back: row rr (+ 8i), 16-B chunk cq
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int n = ncol0 + ni * 32 + 4 * cq;
    f32x4 bb = {0.f, 0.f, 0.f, 0.f};
    if (bbase) {
      if (n + 3 < p.N) {
        bb = *reinterpret_cast<const f32x4*>(bbase + n);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) bb[e] = n + e < p.N ? bbase[n + e] : 0.f;
      }
    }
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 2 * g + h;
        *reinterpret_cast<f32x4*>(scr + r32 * 32 + 4 * (c ^ (r32 & 7))) =
            f32x4{acc[mi][ni][4 * g], acc[mi][ni][4 * g + 1], acc[mi][ni][4 * g + 2], acc[mi][ni][4 * g + 3]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      f32x4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 8 * i + rr;
        v[i] = *reinterpret_cast<const f32x4*>(scr + r * 32 + 4 * (cq ^ (r & 7)));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mrow0 + mi * 32 + 8 * i + rr;
        if (m >= p.M) continue;
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = v[i][e] + bb[e];
          if (p.relu == 1) x[e] = fmaxf(x[e], 0.f);
        }
        TO* crow = cbase + (long long)m * p.ldc;
        const TO* rrow = rbase ? rbase + (long long)m * p.ldr : nullptr;
        if (n + 3 < p.N) {
          if constexpr (sizeof(TO) == 4) {
            if (rrow) {
              const f32x4 q = *reinterpret_cast<const f32x4*>(rrow + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) x[e] = p.relu == 2 ? (q[e] > 0.f ? x[e] : 0.f) : x[e] + q[e];
            }
            if (!PLANES || p.c) *reinterpret_cast<f32x4*>(crow + n) = f32x4{x[0], x[1], x[2], x[3]};
            if (p.c2) {
              bf16* c2row = reinterpret_cast<bf16*>(p.c2) + z1 * p.sc21 + z2 * p.sc22 + (long long)m * p.ldc2 + n;
              const bf16x4 h0 = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
              *reinterpret_cast<bf16x4*>(c2row) = h0;
              if (PLANES && p.c2planes) {  // the SPLIT3 operand of the next GEMM: x = p0 + p1 + p2
                const long long pl = (long long)p.M * p.ldc2;
                float r1[4];
                bf16x4 h1, h2;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  r1[e] = x[e] - (float)h0[e];
                  h1[e] = (bf16)r1[e];
                  h2[e] = (bf16)(r1[e] - (float)h1[e]);
                }
                *reinterpret_cast<bf16x4*>(c2row + pl) = h1;
                *reinterpret_cast<bf16x4*>(c2row + 2 * pl) = h2;
              }
            }
          } else {
            if (rrow) {
              const bf16x4 q = *reinterpret_cast<const bf16x4*>(rrow + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) x[e] += (float)q[e];
            }
            *reinterpret_cast<bf16x4*>(crow + n) = bf16x4{(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (n + e < p.N) {
              float y = x[e];
              if (rrow) y = p.relu == 2 ? (to_f32<TO>(rrow[n + e]) > 0.f ? y : 0.f) : y + to_f32<TO>(rrow[n + e]);
              crow[n + e] = from_f32<TO>(y);
            }
          }
        }
      }
    }
  }
}

// The K|V' projection's V' half written as the attention's transposed operand image (replaces
// mhada_transpose_v): for a wave sub-tile of 32*TM keys x 64 channels o (TN = 2),
//   vt[o][pos(m)] = V'[m][o],  vt[64 + o][pos(m)] = V'[m][o]^2,
// bf16: pos permutes keys inside groups of 16 (bits 2 and 3 swapped, the order the 32x32x16 PV
// operand reads) and V'^2 is the square of the bf16-rounded V' (as mhada_transpose_v); fp32:
// natural order.  Each 32 x 32 block is transposed through the wave's 4-KiB scratch and stored
// as 16-B chunks of key positions; positions >= M (up to ldt) are written 0.
template <typename TO, int TM>
MHADA_DEV void store_vt_tile(const GemmP& p, const f32x16 (&acc)[TM][2], int z1, int z2, int mrow0, int ncol0,
                             int lane, float* scr) {
  TO* vbase = reinterpret_cast<TO*>(p.vt) + z1 * p.svt1 + z2 * p.svt2;
  const float* bbase = p.bias ? p.bias + z1 * p.sb1 + z2 * p.sb2 : nullptr;
  const int h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m0 = mrow0 + 32 * mi;
    if (m0 >= p.ldt) break;  // ldt % 64 == 0: a 32-key block is wholly inside or outside
    const bool mv = m0 + r32 < p.M;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      if constexpr (sizeof(TO) == 2) {
        bf16* sb = reinterpret_cast<bf16*>(scr);
        const int pos = (r32 & ~12) | ((r32 & 4) << 1) | ((r32 & 8) >> 1);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ol = 8 * g + 4 * h + e;
            float x = acc[mi][ni][4 * g + e] + (bbase ? bbase[ncol0 + 32 * ni + ol] : 0.f);
            sb[ol * 32 + pos] = mv ? (bf16)x : (bf16)0.0f;
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bf16x8 v[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = lane + 64 * j;
          v[j] = *reinterpret_cast<const bf16x8*>(sb + (c >> 2) * 32 + 8 * (c & 3));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = lane + 64 * j, ol = c >> 2, part = c & 3;
          TO* dst = vbase + (long long)(32 * ni + ol) * p.ldt + m0 + 8 * part;
          *reinterpret_cast<bf16x8*>(dst) = v[j];
          bf16x8 sq;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)v[j][e];
            sq[e] = (bf16)(f * f);
          }
          *reinterpret_cast<bf16x8*>(dst + 64 * p.ldt) = sq;
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ol = 8 * g + 4 * h + e;
            const float x = acc[mi][ni][4 * g + e] + (bbase ? bbase[ncol0 + 32 * ni + ol] : 0.f);
            scr[ol * 32 + r32] = mv ? x : 0.f;
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        f32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = lane + 64 * j;
          v[j] = *reinterpret_cast<const f32x4*>(scr + (c >> 3) * 32 + 4 * (c & 7));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = lane + 64 * j, ol = c >> 3, part = c & 7;
          float* dst = reinterpret_cast<float*>(vbase) + (long long)(32 * ni + ol) * p.ldt + m0 + 4 * part;
          *reinterpret_cast<f32x4*>(dst) = v[j];
          *reinterpret_cast<f32x4*>(dst + 64 * p.ldt) = v[j] * v[j];
        }
      }
    }
  }
}

// bf16-output form of store_tile_lds for a wave's 64-column sub-tile (TN = 2): bias and ReLU are
// applied in the accumulator layout, the values rounded to bf16 once and written to the per-wave
// scratch as a 32 x 64 bf16 block (128-B rows, 16-B chunk c of row r at slot c ^ (r & 7)), read
// back as whole 16-B chunks (lane = row 8i + (lane >> 3), chunk lane & 7) and stored 16 B per lane:
// one store instruction covers 8 rows x 128 B — half the store instructions of the 8-B form (the
// tail is store-issue bound: MI355X_MICROARCH.md "attention epilogue store tail").
template <int TM>
MHADA_DEV void store_tile_lds_bf16(const GemmP& p, const f32x16 (&acc)[TM][2], int z1, int z2, int mrow0, int ncol0,
                                   int lane, float* scr_f) {
  bf16* cbase = reinterpret_cast<bf16*>(p.c) + z1 * p.sc1 + z2 * p.sc2;
  const float* bbase = p.bias ? p.bias + z1 * p.sb1 + z2 * p.sb2 : nullptr;
  char* scr = reinterpret_cast<char*>(scr_f);
  const int h = lane >> 5, r32 = lane & 31;
  const int rr = lane >> 3, cq = lane & 7;
  f32x4 bb[2][4];
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = ncol0 + ni * 32 + 8 * g + 4 * h;
      bb[ni][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (bbase) {
        if (n + 3 < p.N) {
          bb[ni][g] = *reinterpret_cast<const f32x4*>(bbase + n);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) bb[ni][g][e] = n + e < p.N ? bbase[n + e] : 0.f;
        }
      }
    }
  const int n = ncol0 + 8 * cq;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = acc[mi][ni][4 * g + e] + bb[ni][g][e];
          if (p.relu == 1) x = fmaxf(x, 0.f);
          o[e] = (bf16)x;
        }
        const int c = 4 * ni + g;
        *reinterpret_cast<bf16x4*>(scr + r32 * 128 + 16 * (c ^ (r32 & 7)) + 8 * h) = o;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bf16x8 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 8 * i + rr;
      v[i] = *reinterpret_cast<const bf16x8*>(scr + r * 128 + 16 * (cq ^ (r & 7)));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mrow0 + mi * 32 + 8 * i + rr;
      if (m >= p.M) continue;
      bf16* crow = cbase + (long long)m * p.ldc;
      if (n + 7 < p.N && ((p.ldc & 7) == 0)) {
        *reinterpret_cast<bf16x8*>(crow + n) = v[i];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n + e < p.N) crow[n + e] = v[i][e];
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// BM x BN block tile, WM x WN waves (NT = 64*WM*WN threads); each wave owns a
// (BM/WM) x (BN/WN) sub-tile of TM x TN 32x32 MFMA blocks.
// ------------------------------------------------------------------------------------
template <typename TC, typename TA, typename TO, int AMODE, int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN) gemm_kernel(const GemmP p) {
  constexpr int NT = 64 * WM * WN, RS = NT / 8;  // RS: rows staged per pass
  constexpr int E = Cfg<TC>::E, BK = Cfg<TC>::BK, LS = Cfg<TC>::LS;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_CH = BM / RS, B_CH = BN / RS;
  static_assert(A_CH >= 1 && B_CH >= 1 && TM >= 1 && TN >= 1, "tile config");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // [nbuf][BM][LS] then [nbuf][BN][LS]: one K-step problems (the MHAda projections, K = 64) stage a
  // single buffer, half the LDS, so more workgroups share a CU
  const int nbuf = p.K > BK ? 2 : 1;
  TC* sA = reinterpret_cast<TC*>(smem);
  TC* sB = sA + nbuf * BM * LS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int z = blockIdx.y, z1 = z / p.nb2, z2 = z - z1 * p.nb2;
  const int t = xcd_remap(blockIdx.x, p.ntiles);
  const int tm = t / p.tiles_n, tn = t - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kc = tid & 7;

  const TA* abase = reinterpret_cast<const TA*>(p.a) + z1 * p.sa1 + z2 * p.sa2;
  const TC* wbase = reinterpret_cast<const TC*>(p.w) + z1 * p.sw1 + z2 * p.sw2;
  GemmP pz = p;
  if (p.a_mu) pz.a_mu = p.a_mu + z1 * p.smu1 + z2 * p.smu2;

  RowInfo ri[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = m0 + (tid >> 3) + RS * i;
    ri[i].valid = m < p.M;
    const int mm = m < p.M ? m : 0;
    if constexpr (AMODE == MHADA_A_ROWS || AMODE == kRowsCentred) {
      ri[i].b = mm; ri[i].y = 0; ri[i].x = 0;
    } else if constexpr (AMODE == MHADA_A_PATCH8) {
      const int wt = p.out_w;
      ri[i].b = 0; ri[i].y = mm / wt; ri[i].x = mm - (mm / wt) * wt;
    } else {
      const int hw = p.out_h * p.out_w;
      const int b = mm / hw, rem = mm - b * hw;
      ri[i].b = b; ri[i].y = rem / p.out_w; ri[i].x = rem - (rem / p.out_w) * p.out_w;
    }
  }
  int brow[B_CH];
  bool bval[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int n = n0 + (tid >> 3) + RS * i;
    bval[i] = n < p.N;
    brow[i] = n < p.N ? n : 0;
  }

  AStage<TA, TC, AMODE, A_CH> ast;
  typename Vec16<TC>::type bst[B_CH];
  auto issue_b = [&](int k0) {
    const int k = k0 + kc * E;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      if (bval[i] && k < p.K) {
        bst[i] = *reinterpret_cast<const typename Vec16<TC>::type*>(wbase + (long long)brow[i] * p.ldw + k);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) bst[i][e] = (TC)0.0f;
      }
    }
  };
  auto commit_b = [&](TC* dst) {
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      *reinterpret_cast<typename Vec16<TC>::type*>(dst + ((tid >> 3) + RS * i) * LS + kc * E) = bst[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int KT = (p.K + BK - 1) / BK;
  issue_a<TA, TC, AMODE, A_CH>(ast, pz, abase, ri, 0, kc);
  issue_b(0);
  commit_a<RS>(ast, sA, tid);
  commit_b(sB);
  __syncthreads();

  const int h = lane >> 5, r32 = lane & 31;
  const int arow0 = wm * (BM / WM) + r32, brow0 = wn * (BN / WN) + r32;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) {
      issue_a<TA, TC, AMODE, A_CH>(ast, pz, abase, ri, (kt + 1) * BK, kc);
      issue_b((kt + 1) * BK);
    }
    const TC* cA = sA + buf * BM * LS;
    const TC* cB = sB + buf * BN * LS;
    if constexpr (sizeof(TC) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
          af[mi] = *reinterpret_cast<const bf16x8*>(cA + (arow0 + mi * 32) * LS + ks * 16 + 8 * h);
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          bfr[ni] = *reinterpret_cast<const bf16x8*>(cB + (brow0 + ni * 32) * LS + ks * 16 + 8 * h);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
      }
    } else {
      // fp32: lane half h supplies k = 16h + s at MFMA step s (both operands agree)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        f32x4 av[TM][2], bv[TN][2];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            av[mi][q] = *reinterpret_cast<const f32x4*>(cA + (arow0 + mi * 32) * LS + 16 * h + 8 * half + 4 * q);
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            bv[ni][q] = *reinterpret_cast<const f32x4*>(cB + (brow0 + ni * 32) * LS + 16 * h + 8 * half + 4 * q);
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
          for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[ni][s >> 2][s & 3], av[mi][s >> 2][s & 3],
                                                                 acc[mi][ni], 0, 0, 0);
      }
    }
    if (kt + 1 < KT) {
      commit_a<RS>(ast, sA + (buf ^ 1) * BM * LS, tid);
      commit_b(sB + (buf ^ 1) * BN * LS);
    }
    __syncthreads();
  }

  // epilogue: through a per-wave 4-KiB LDS scratch carved from the (now idle) staging buffers —
  // whole-row stores (16 B per lane) instead of 32 rows x 8-16 B per store instruction
  if (p.vt && n0 + wn * (BN / WN) >= 64) {  // the V' half of the K|V' projection -> vt image
    if constexpr (TN == 2) {
      store_vt_tile<TO, TM>(p, acc, z1, z2, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane,
                            reinterpret_cast<float*>(smem) + wave * 1024);
    }
    return;
  }
  if (p.lds_epi) {
    float* scr = reinterpret_cast<float*>(smem) + wave * 1024;
    if constexpr (sizeof(TO) == 2 && TN == 2) {
      if (!p.r) {
        store_tile_lds_bf16<TM>(p, acc, z1, z2, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane, scr);
        return;
      }
    }
    store_tile_lds<TO, TM, TN>(p, acc, z1, z2, m0 + wm * (BM / WM), n0 + wn * (BN / WN), lane, scr);
    return;
  }
  store_tile<TO, TM, TN>(p, acc, z1, z2, m0 + arow0, n0 + brow0 - r32, h);
}

// ------------------------------------------------------------------------------------
// Ping-pong bf16 GEMM for the large dense contractions (bf16 A rows or reflect-padded 3x3
// taps, K % 64 == 0).  256x256 block tile, 8 waves in two groups of 4: group g owns output
// rows 128g..128g+127 and wave (g, wc) a 128x64 sub-tile (4x2 32x32 blocks).  Each K-tile
// (BK = 64) runs in 4 phases, each one 32-column block x 2 k-steps of the sub-tile; a phase is
// {LDS fragment reads + LDS-DMA prefetch} -> s_barrier -> {8 MFMAs} -> s_barrier, and group 1
// runs one barrier behind group 0, so on every SIMD one wave's MFMA phase pairs with the other
// wave's load phase (cdna_hip_programming.md §5 "256² 8-phase template", T3/T4/T5).
// Staging: global_load_lds (16 B per lane, lane-linear 1 KiB per wave-instruction) into a
// 2-deep ring of K-tiles, each split in 4 half-tiles [A rows 0-127 | A 128-255 | W 0-127 |
// W 128-255] of 128 rows x 128 B; rows are unpadded, chunk slot = chunk ^ ((row >> 1) & 7)
// (applied on the per-lane SOURCE address, conflict-free ds_read_b128 for the 32x32x16
// operand groups).  Waits are counted (vmcnt 4/0), never a drain inside the loop; the phase
// schedule and ring-slot reuse rules are spelled out above the main loop.
// ------------------------------------------------------------------------------------
MHADA_DEV void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

#define PP_BARRIER() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define PP_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

template <typename TO, int AMODE>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const GemmP p) {
  constexpr int BK = 64, HALF = 128 * BK, TILE = 4 * HALF;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * TILE];  // 128 KiB, the only LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wc = wave & 3;
  const int h = lane >> 5, r32 = lane & 31;
  const int z = blockIdx.y, z1 = z / p.nb2, z2 = z - z1 * p.nb2;
  const int t = xcd_remap(blockIdx.x, p.ntiles);
  const int tm = t / p.tiles_n, tn = t - tm * p.tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const bf16* abase = reinterpret_cast<const bf16*>(p.a) + z1 * p.sa1 + z2 * p.sa2;
  const bf16* wbase = reinterpret_cast<const bf16*>(p.w) + z1 * p.sw1 + z2 * p.sw2;

  // ---- staging geometry: instruction i of this wave covers rows 16*wave + 8i + (lane>>3) of a
  // half tile; lane slot lane&7 receives source chunk (lane&7) ^ ((row>>1)&7).
  int cofs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) cofs[i] = 8 * ((lane & 7) ^ (4 * i + (lane >> 4)));
  unsigned aoff[2][2], woff[2][2];  // element offsets of (half, i) rows (ROWS: incl. chunk)
  int ab[2][2], ay[2][2], ax[2][2];  // CONV: (image, y, x) of the output pixel
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = 16 * wave + 8 * i + (lane >> 3);
      const int m = min(m0 + 128 * hh + rr, p.M - 1);
      const int n = min(n0 + 128 * hh + rr, p.N - 1);
      woff[hh][i] = (unsigned)((long long)n * p.ldw + cofs[i]);
      if constexpr (AMODE == MHADA_A_ROWS) {
        aoff[hh][i] = (unsigned)((long long)m * p.lda + cofs[i]);
      } else {
        const int hw = p.out_h * p.out_w;
        const int b = m / hw, rem = m - b * hw;
        ab[hh][i] = b; ay[hh][i] = rem / p.out_w; ax[hh][i] = rem - (rem / p.out_w) * p.out_w;
        aoff[hh][i] = 0;
      }
    }
  auto stage_a = [&](int hh, int kt) {
    bf16* dst = smem + (kt & 1) * TILE + hh * HALF + wave * 1024;
    const int k0 = kt * BK;
    if constexpr (AMODE == MHADA_A_ROWS) {
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(abase + aoff[hh][i] + k0, dst + 512 * i);
    } else {
      const int cin_n = p.img_c;
      const int tap = k0 / cin_n, cin0 = k0 - tap * cin_n;
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int Y = reflect1(ay[hh][i] + dy, p.out_h), X = reflect1(ax[hh][i] + dx, p.out_w);
        const unsigned off = (unsigned)(((ab[hh][i] * p.img_h + Y) * p.img_w + X) * cin_n + cin0 + cofs[i]);
        glds16(abase + off, dst + 512 * i);
      }
    }
  };
  auto stage_w = [&](int hh, int kt) {
    bf16* dst = smem + (kt & 1) * TILE + (2 + hh) * HALF + wave * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(wbase + woff[hh][i] + kt * BK, dst + 512 * i);
  };

  // ---- fragment reads: row r32 of a 32-row block, 16-B chunk 2ks+h, swizzled slot
  const int swz = (r32 >> 1) & 7;
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = 8 * ((2 * ks + h) ^ swz);
  const bf16* sA = smem + grp * HALF + r32 * 64;                              // + mt*2048
  const bf16* sW = smem + (2 + (wc >> 1)) * HALF + ((wc & 1) * 64 + r32) * 64;  // + nt*2048
  bf16x8 af[4][2], wf[2][2];  // [mt][k-step of the pair], [nt][k-step of the pair]
  auto read_a = [&](int kp, int cb) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        af[mt][s2] = *reinterpret_cast<const bf16x8*>(sA + cb * TILE + mt * 2048 + koff[2 * kp + s2]);
  };
  auto read_w = [&](int nt, int kp, int cb) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      wf[nt][s2] = *reinterpret_cast<const bf16x8*>(sW + cb * TILE + nt * 2048 + koff[2 * kp + s2]);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  // one phase: the 4 row blocks x one 32-column block x 2 k-steps = 8 MFMAs, 4 independent chains
  auto compute = [&](int nt) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[nt][s2], af[mt][s2], acc[mt][nt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Schedule per K-tile t (buffer t&1), phases:
  //   0: read A k-steps 0,1 + W cols 0-31   | DMA W-half 0 of t+1
  //   1: read W cols 32-63                  | DMA W-half 1 of t+1
  //   2: read A k-steps 2,3 + W cols 0-31   |
  //   3: read W cols 32-63                  | DMA A-halves of t+2; vmcnt -> tile t+1 landed
  // A (the large, HBM-streamed operand) is prefetched a whole K-tile earlier than W (L2-hot).
  // Ring: tile t's A slots are last read in phase 2 and refilled (t+2) in phase 3; its W slots
  // are last read in phase 3 and refilled (t+2) in phases 0/1 of tile t+1.
  const int KT = p.K / BK;
  stage_a(0, 0); stage_a(1, 0); stage_w(0, 0); stage_w(1, 0);
  if (KT > 1) {
    stage_a(0, 1); stage_a(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  PP_BARRIER();
  if (grp == 1) PP_BARRIER();  // group 1 runs one barrier behind

  for (int kt = 0; kt < KT; ++kt) {
    const int cb = kt & 1;
    const bool n1 = kt + 1 < KT, n2 = kt + 2 < KT;
    // phase 0
    read_a(0, cb); read_w(0, 0, cb);
    if (n1) stage_w(0, kt + 1);
    PP_LGKM0(); PP_BARRIER(); compute(0); PP_BARRIER();
    // phase 1
    read_w(1, 0, cb);
    if (n1) stage_w(1, kt + 1);
    PP_LGKM0(); PP_BARRIER(); compute(1); PP_BARRIER();
    // phase 2
    read_a(1, cb); read_w(0, 1, cb);
    PP_LGKM0(); PP_BARRIER(); compute(0); PP_BARRIER();
    // phase 3
    read_w(1, 1, cb);
    if (n2) {
      stage_a(0, kt + 2); stage_a(1, kt + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    PP_LGKM0(); PP_BARRIER(); compute(1); PP_BARRIER();
  }
  if (grp == 0) PP_BARRIER();  // balance the barrier count of the two groups
  store_tile<TO, 4, 2>(p, acc, z1, z2, m0 + grp * 128 + r32, n0 + wc * 64, h);
}

// ------------------------------------------------------------------------------------
// Persistent form of the ping-pong kernel: one workgroup per CU walks work items
// w = blockIdx.x + i * gridDim.x (tile x z-batch, dealt to XCDs as a one-shot launch of
// `total` blocks would be, then xcd_remap'ed so an XCD's 32 concurrent tiles share A rows and
// W in its L2).  The K-tile stream is continuous across tiles: the ring slot is the global
// K-tile counter's parity and the lookahead stages (W one K-tile ahead, A two) reach into the
// NEXT tile's first K-tiles, so the next tile's operands are in flight while this tile's
// last phases and its epilogue run — the one-shot kernel pays the HBM latency of every
// tile's prologue and drains the CU at every epilogue (K = 512: 8 K-tiles per tile).
// Needs two K-tiles (K >= 128 bf16 / 64 fp32: the A lookahead never skips a whole tile).
// fp32 form: same 128-B rows (BK = 32), v_mfma_f32_32x32x2_f32, 32 MFMAs per phase.
// ------------------------------------------------------------------------------------
template <typename TC, typename TO, int AMODE, int BN>
__global__ void __launch_bounds__(512) gemm_ppp_kernel(const GemmP p, int total) {
  // 128-B operand rows: BK = 64 bf16 or 32 fp32; CE elements per 16-B chunk, PE per 1-KiB piece.
  // BN = 256: each wave owns 128 rows x 64 columns (TN = 2 column blocks, 4 phases per K-tile);
  // BN = 128 (N <= 128 layers): 128 rows x 32 columns (TN = 1, 2 phases), one W half per stage;
  // with only 2 phases per K-tile the lagging group still reads A(g) when the leading group
  // could stage A(g+2), so the ring has 3 slots (A two K-tiles ahead needs slot (g+2) % 3).
  constexpr int TN = BN / 128, NWH = BN / 128;
  constexpr int CE = 16 / sizeof(TC), BK = 8 * CE, PE = 1024 / sizeof(TC), HALF = 128 * BK, TILE = (2 + NWH) * HALF;
  constexpr int NSLOT = BN == 256 ? 2 : 3;
  typedef typename Vec16<TC>::type Frag;
  // BN = 256 adds 8 x 4 KiB of epilogue scratch (store_tile_lds): 160 KiB in all
  constexpr int SCR = BN == 256 ? 8 * 4096 / (int)sizeof(TC) : 0;
  __shared__ __attribute__((aligned(16))) TC smem[NSLOT * TILE + SCR];  // 160 / 144 KiB, the only LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wc = wave & 3;
  const int h = lane >> 5, r32 = lane & 31;
  const int G = gridDim.x;

  int cofs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) cofs[i] = CE * ((lane & 7) ^ (4 * i + (lane >> 4)));
  // per-tile staging state (rows 16*wave + 8i + (lane>>3) of each 128-row half)
  struct St {
    const TC* ab;
    const TC* wb;
    unsigned aoff[2][2], woff[2][2];
    int b[2][2], y[2][2], x[2][2];
    int m0, n0, z1, z2;
  };
  auto setup = [&](int w, St& s) {
    const int lg = xcd_remap(w, total);
    const int z = lg / p.ntiles, t = lg - z * p.ntiles;
    s.z1 = z / p.nb2;
    s.z2 = z - s.z1 * p.nb2;
    const int tm = t / p.tiles_n, tn = t - tm * p.tiles_n;
    s.m0 = tm * 256;
    s.n0 = tn * BN;
    s.ab = reinterpret_cast<const TC*>(p.a) + s.z1 * p.sa1 + s.z2 * p.sa2;
    s.wb = reinterpret_cast<const TC*>(p.w) + s.z1 * p.sw1 + s.z2 * p.sw2;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int rr = 16 * wave + 8 * i + (lane >> 3);
        const int m = min(s.m0 + 128 * hh + rr, p.M - 1);
        const int n = min(s.n0 + 128 * (hh % NWH) + rr, p.N - 1);
        s.woff[hh][i] = (unsigned)((long long)n * p.ldw + cofs[i]);
        if constexpr (AMODE == MHADA_A_ROWS || AMODE == kRowsSplit3) {
          s.aoff[hh][i] = (unsigned)((long long)m * p.lda + cofs[i]);
        } else {
          const int hw = p.out_h * p.out_w;
          const int b = m / hw, rem = m - b * hw;
          s.b[hh][i] = b;
          s.y[hh][i] = rem / p.out_w;
          s.x[hh][i] = rem - (rem / p.out_w) * p.out_w;
          s.aoff[hh][i] = 0;
        }
      }
  };
  auto stage_a = [&](const St& s, int hh, int kt, int slot) {
    TC* dst = smem + slot * TILE + hh * HALF + wave * 2 * PE;
    const int k0 = kt * BK;
    if constexpr (AMODE == MHADA_A_ROWS) {
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(s.ab + s.aoff[hh][i] + k0, dst + PE * i);
    } else if constexpr (AMODE == kRowsSplit3) {
      // K-tile kt of the virtual 6 K0 = term t = kt % 6 of the 64-column chunk kk = kt / 6: the six
      // terms of a chunk run back to back, so its A planes are re-read from L2 within six K-tiles
      // (term-major order re-fetched them from HBM: 3.8-5x the algorithmic A bytes)
      const int kk = kt / 6, t = kt - 6 * kk;
      const TC* src = s.ab + ((kSplitPlanes >> (4 * t)) & 15) * p.spl + kk * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16(src + s.aoff[hh][i], dst + PE * i);
    } else {
      const int cin_n = p.img_c;
      const int tap = k0 / cin_n, cin0 = k0 - tap * cin_n;
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int Y, X;
        const bool inside = conv_src<AMODE>(p, s.y[hh][i], s.x[hh][i], dy, dx, Y, X);
        const unsigned off = (unsigned)(((s.b[hh][i] * p.img_h + Y) * p.img_w + X) * cin_n + cin0 + cofs[i]);
        glds16(inside ? (const void*)(s.ab + off) : (const void*)g_zero16, dst + PE * i);
      }
    }
  };
  auto stage_w = [&](const St& s, int hh, int kt, int slot) {
    TC* dst = smem + slot * TILE + (2 + hh) * HALF + wave * 2 * PE;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(s.wb + s.woff[hh][i] + kt * BK, dst + PE * i);
  };

  // fragment reads: row r32 of a 32-row block, logical 16-B chunk j at swizzled slot j ^ swz.
  //   bf16 (32x32x16): k-step ks takes chunk 2ks + h (8 k per lane half).
  //   fp32 (32x32x2, one k per lane half per MFMA): lane half h supplies k = 16h + s at step s
  //   (A and W agree, so any such bijection is the same sum): its 16 floats are chunks 4h + q.
  const int swz = (r32 >> 1) & 7;
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = sizeof(TC) == 2 ? CE * ((2 * ks + h) ^ swz) : CE * ((4 * h + ks) ^ swz);
  const TC* sA = smem + grp * HALF + r32 * BK;
  const TC* sW = smem + (2 + (wc * TN * 32) / 128) * HALF + ((wc * TN * 32) % 128 + r32) * BK;
  Frag af[4][2], wf[TN][2];
  auto read_a = [&](int kp, int cb) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        af[mt][s2] = *reinterpret_cast<const Frag*>(sA + cb * TILE + mt * 32 * BK + koff[2 * kp + s2]);
  };
  auto read_w = [&](int nt, int kp, int cb) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      wf[nt][s2] = *reinterpret_cast<const Frag*>(sW + cb * TILE + nt * 32 * BK + koff[2 * kp + s2]);
  };
  f32x16 acc[4][TN];
  // accumulator init: zero, or (p.rinit: fp32 C, no ReLU) the tile's residual rows + bias, so the
  // MFMAs accumulate on top of them and the epilogue only stores — its R loads were 8 dependent
  // HBM round trips per tile (one per 32x32 block), now one batch issued at the tile start.
  // acc[mt][nt][4g+e] <-> C[m0 + grp*128 + 32mt + r32][n0 + wc*32TN + 32nt + 8g + 4h + e].
  auto zero_acc = [&](const St& s) {
    if constexpr (sizeof(TO) == 4) {
      if (p.rinit) {
        const float* rb = reinterpret_cast<const float*>(p.r) + s.z1 * p.sr1 + s.z2 * p.sr2;
        const float* bb = p.bias ? p.bias + s.z1 * p.sb1 + s.z2 * p.sb2 : nullptr;
#pragma unroll
        for (int nt = 0; nt < TN; ++nt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = s.n0 + wc * TN * 32 + nt * 32 + 8 * g + 4 * h;
            const bool nok = n + 3 < p.N;
            const f32x4 b4 = (bb && nok) ? *reinterpret_cast<const f32x4*>(bb + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
              const int m = s.m0 + grp * 128 + mt * 32 + r32;
              f32x4 r4 = {0.f, 0.f, 0.f, 0.f};
              if (nok && m < p.M) r4 = *reinterpret_cast<const f32x4*>(rb + (long long)m * p.ldr + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[mt][nt][4 * g + e] = r4[e] + b4[e];
            }
          }
        return;
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  };
  // the epilogue's view: with rinit the residual and bias are already in the accumulators
  GemmP pe = p;
  if (p.rinit) {
    pe.r = nullptr;
    pe.bias = nullptr;
  }
  // one phase: 4 row blocks x one 32-column block x half a K-tile (bf16: 8 MFMAs, fp32: 32)
  auto compute = [&](int nt) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (sizeof(TC) == 2) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[nt][s2], af[mt][s2], acc[mt][nt], 0, 0, 0);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[nt][s2][e], af[mt][s2][e], acc[mt][nt], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  const int KT = p.K / BK;
  int w = blockIdx.x;
  St cur, nxt;
  setup(w, cur);
  bool has_nxt = w + G < total;
  if (has_nxt) setup(w + G, nxt);
  zero_acc(cur);
  stage_a(cur, 0, 0, 0); stage_a(cur, 1, 0, 0); stage_w(cur, 0, 0, 0);
  if constexpr (NWH == 2) stage_w(cur, 1, 0, 0);
  stage_a(cur, 0, 1, 1); stage_a(cur, 1, 1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  PP_BARRIER();
  if (grp == 1) PP_BARRIER();  // group 1 runs one barrier behind

  // ring slots of K-tiles g, g+1, g+2 (global K-tile counter g, continuous across tiles)
  int sl0 = 0, sl1 = 1, sl2 = NSLOT == 2 ? 0 : 2;
  // one K-tile: W of K-tile g+1 comes from (s1, k1), A of K-tile g+2 from (s2, k2).  The three
  // call sites below bind s1 / s2 to `cur` or `nxt` at compile time: selecting the struct by a
  // runtime condition made hipcc copy the whole staging state every iteration (~280 v_mov + 50-100
  // v_readlane per K-tile in the last two K-tiles of each tile).
  // wx: the wait of this K-tile may leave EPI_MIN more operations in flight — the previous tile's
  // epilogue stores, issued after everything this wait must cover (see the tile boundary below)
  constexpr int EPI_MIN = (sizeof(TO) == 4 && TN == 2) ? 32 : 16;
  auto ktile = [&](const St& s1, const int k1, const bool w1, const St& s2, const int k2, const bool a2,
                   const bool wx) __attribute__((always_inline)) {
    const int cb = sl0;
    if constexpr (TN == 2) {
      // phase 0
      read_a(0, cb); read_w(0, 0, cb);
      if (w1) stage_w(s1, 0, k1, sl1);
      PP_LGKM0(); PP_BARRIER(); compute(0); PP_BARRIER();
      // phase 1
      read_w(1, 0, cb);
      if (w1) stage_w(s1, 1, k1, sl1);
      PP_LGKM0(); PP_BARRIER(); compute(1); PP_BARRIER();
      // phase 2
      read_a(1, cb); read_w(0, 1, cb);
      PP_LGKM0(); PP_BARRIER(); compute(0); PP_BARRIER();
      // phase 3
      read_w(1, 1, cb);
    } else {
      // phase 0: k-steps of pair 0
      read_a(0, cb); read_w(0, 0, cb);
      if (w1) stage_w(s1, 0, k1, sl1);
      PP_LGKM0(); PP_BARRIER(); compute(0); PP_BARRIER();
      // phase 1: pair 1
      read_a(1, cb); read_w(0, 1, cb);
    }
    if (a2) {
      stage_a(s2, 0, k2, sl2); stage_a(s2, 1, k2, sl2);
      if (wx) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 + EPI_MIN) : "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    PP_LGKM0(); PP_BARRIER(); compute(TN - 1); PP_BARRIER();
    if constexpr (NSLOT == 2) {
      sl0 ^= 1; sl1 ^= 1; sl2 ^= 1;
    } else {
      const int o = sl0;
      sl0 = sl1; sl1 = sl2; sl2 = o;
    }
  };
  bool pre = false;  // W of this tile's K-tile 1 was staged before the previous tile's epilogue
  while (true) {
    // KT >= 2 (checked on the host); the first K-tile skips the pre-staged W and may leave the
    // previous epilogue's stores in flight (wx)
    if constexpr (AMODE == MHADA_A_ROWS || AMODE == kRowsSplit3) {
      for (int kt = 0; kt + 2 < KT; ++kt) ktile(cur, kt + 1, kt > 0 || !pre, cur, kt + 2, true, kt == 0 && pre);
      ktile(cur, KT - 1, KT > 2 || !pre, nxt, 0, has_nxt, KT == 2 && pre);
    } else {
      for (int kt = 0; kt + 2 < KT; ++kt) ktile(cur, kt + 1, true, cur, kt + 2, true, false);
      ktile(cur, KT - 1, true, nxt, 0, has_nxt, false);
    }
    ktile(nxt, 0, has_nxt, nxt, 1, has_nxt, false);
    // tile boundary: re-align the groups so both store in the same interval (a store between
    // staggered barriers would hold the other group's compute phase), then re-stagger
    if (grp == 0) PP_BARRIER();
    // Every wave has left the last K-tile, so the ring slot of the next tile's K-tile 1 is free:
    // stage its W now, BEFORE the epilogue stores.  vmcnt is in order and counts stores, so the
    // next tile's first wait would otherwise drain this tile's whole C burst (~7 % of an fp32
    // 512-K GEMM); with everything that wait needs issued before the stores, it may leave them
    // in flight (at least EPI_MIN per wave in a full tile).  Not with rinit: the next tile's
    // residual loads follow the stores and its first MFMA needs them.
    // (ROWS only: in the implicit-GEMM conv instantiations the extra specialisation of the first
    // K-tile raised register spills and measured slower)
    pre = (AMODE == MHADA_A_ROWS || AMODE == kRowsSplit3) && has_nxt && !p.rinit && cur.m0 + 256 <= p.M &&
          cur.n0 + BN <= p.N;
    if (pre) {
      stage_w(nxt, 0, 1, sl1);
      if constexpr (NWH == 2) stage_w(nxt, 1, 1, sl1);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (SCR > 0) {
      if (p.lds_epi) {
        float* scr = reinterpret_cast<float*>(smem + NSLOT * TILE) + wave * 1024;
        if constexpr (sizeof(TO) == 2 && TN == 2) {
          store_tile_lds_bf16<4>(pe, acc, cur.z1, cur.z2, cur.m0 + grp * 128, cur.n0 + wc * TN * 32, lane, scr);
        } else {
          store_tile_lds<TO, 4, TN, AMODE == kRowsSplit3>(pe, acc, cur.z1, cur.z2, cur.m0 + grp * 128,
                                                           cur.n0 + wc * TN * 32, lane, scr);
        }
      }
      else
        store_tile<TO, 4, TN>(pe, acc, cur.z1, cur.z2, cur.m0 + grp * 128 + r32, cur.n0 + wc * TN * 32, h);
    } else {
      store_tile<TO, 4, TN>(pe, acc, cur.z1, cur.z2, cur.m0 + grp * 128 + r32, cur.n0 + wc * TN * 32, h);
    }
    if (!has_nxt) break;
    if (grp == 1) PP_BARRIER();
    zero_acc(nxt);
    cur = nxt;
    w += G;
    has_nxt = w + G < total;
    if (has_nxt) setup(w + G, nxt);
  }
}

// ------------------------------------------------------------------------------------
// fp32 GEMM for N <= 64 columns over long K (the attention backward's dQ = dS K: M = Nc, K = Ns,
// one problem per (batch, head); the grouped per-head 1x1 convs).  Streaming A is the whole
// cost: at the fp32 MFMA rate a 128x64 tile consumes 8 B/clk/CU of A, ~5 TB/s chip-wide, so the
// operands go through a 3-deep LDS-DMA ring (global_load_lds, 16 B per lane; K-tile kt + 2 in
// flight while kt is multiplied) with ONE barrier per K-tile: the barrier that publishes K-tile
// kt also proves every wave has left K-tile kt - 1, whose slot the next DMA then refills.
// 4 waves, wave w owns rows 32w..32w+31 x the 64 columns (2 accumulators); two workgroups per
// CU (72 KiB each).  Rows are 128 B (32 floats), chunk c of row r at slot c ^ ((r >> 1) & 7)
// (applied on the source address, as gemm_ppp_kernel: conflict-free ds_read_b128).
// ------------------------------------------------------------------------------------
template <int BM, int NS, int BK>
__global__ void __launch_bounds__(BM * 2) gemm_n64_kernel(const GemmP p) {
  constexpr int NWV = BM / 32, CH = BK / 4, RPI = 64 / CH;  // 16-B chunks per row, rows per DMA instruction
  constexpr int AH = BM * BK, WH = 64 * BK, STAGE = AH + WH;
  constexpr int API = 32 / RPI, WPI = 64 / RPI / NWV;  // A / W staging instructions per wave and K-tile
  static_assert(WPI >= 1 && (CH == 8 || CH == 16), "tile config");
  __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Workgroups are dealt to the 8 XCDs round-robin in launch order.  With p.xcd_z (batch count a
  // multiple of 8) all row tiles of one problem z go to ONE XCD, so its W (the dQ GEMM's K^T,
  // 1 MiB per (batch, head)) is fetched into one L2 instead of eight.
  int z, tile;
  if (p.lds_epi == 4) {
    const int L = blockIdx.y * gridDim.x + blockIdx.x, nt = gridDim.x;
    z = L % 8 + 8 * (L / (8 * nt));
    tile = (L / 8) % nt;
  } else {
    z = blockIdx.y;
    tile = xcd_remap(blockIdx.x, p.ntiles);
  }
  const int z1 = z / p.nb2, z2 = z - z1 * p.nb2;
  const int m0 = tile * BM;
  const float* ab = reinterpret_cast<const float*>(p.a) + z1 * p.sa1 + z2 * p.sa2;
  const float* wb = reinterpret_cast<const float*>(p.w) + z1 * p.sw1 + z2 * p.sw2;
  // chunk c of LDS row r sits at slot c ^ sw(r): conflict-free ds_read_b128 fragment reads
  auto sw = [](int r) { return CH == 8 ? (r >> 1) & 7 : r & 15; };
  // staging: one DMA instruction = RPI rows x 128 B (lane -> row lane / CH, slot lane % CH)
  const float* asrc[API];
  const float* wsrc[WPI];
#pragma unroll
  for (int i = 0; i < API; ++i) {
    const int r = 32 * wave + RPI * i + lane / CH;
    const int m = min(m0 + r, p.M - 1);
    asrc[i] = ab + (long long)m * p.lda + 4 * ((lane % CH) ^ sw(r));
  }
#pragma unroll
  for (int i = 0; i < WPI; ++i) {
    const int r = RPI * (WPI * wave + i) + lane / CH;
    const int n = min(r, p.N - 1);
    wsrc[i] = wb + (long long)n * p.ldw + 4 * ((lane % CH) ^ sw(r));
  }
  auto stage = [&](int kt, int slot) {
    float* dst = smem + slot * STAGE;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < API; ++i) glds16(asrc[i] + k0, dst + (32 * wave + RPI * i) * BK);
#pragma unroll
    for (int i = 0; i < WPI; ++i) glds16(wsrc[i] + k0, dst + AH + RPI * (WPI * wave + i) * BK);
  };
  const int h = lane >> 5, r32 = lane & 31;
  // lane half h supplies k = (BK / 2) h + s at MFMA step s: chunks (CH / 2) h + q of its row
  int koff[CH / 2];
#pragma unroll
  for (int q = 0; q < CH / 2; ++q) koff[q] = 4 * (((CH / 2) * h + q) ^ sw(r32));
  f32x16 acc[1][2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[0][n][e] = 0.f;
  const int KT = p.K / BK;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < KT) stage(i, i);
  for (int kt = 0; kt < KT; ++kt) {
    // own DMA of K-tile kt done: the K-tiles issued after it (kt + 1 .. kt + NS - 2) may be in flight
    const int ahead = min(KT - 1 - kt, NS - 2);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * (API + WPI)) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(API + WPI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // a bare s_barrier: __syncthreads() would also drain the DMA of the K-tiles ahead (vmcnt(0))
    PP_BARRIER();
    if (kt + NS - 1 < KT) stage(kt + NS - 1, (kt + NS - 1) % NS);
    const float* sa = smem + (kt % NS) * STAGE + (32 * wave + r32) * BK;
    const float* swp = smem + (kt % NS) * STAGE + AH + r32 * BK;
    f32x4 af[CH / 2], wf[2][CH / 2];
#pragma unroll
    for (int q = 0; q < CH / 2; ++q) af[q] = *reinterpret_cast<const f32x4*>(sa + koff[q]);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int q = 0; q < CH / 2; ++q) wf[n][q] = *reinterpret_cast<const f32x4*>(swp + n * 32 * BK + koff[q]);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[0][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[n][s >> 2][s & 3], af[s >> 2][s & 3], acc[0][n], 0, 0, 0);
  }
  store_tile<float, 1, 2>(p, acc, z1, z2, m0 + 32 * wave + r32, 0, h);
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// tuning gemm_persist = 0 selects the one-shot ping-pong kernel (A/B runs)
static bool persist_enabled() { return tuning().gemm_persist != 0; }

template <typename TC, typename TO, int AMODE, int BN = 256>
static int launch_gemm_pp(const GemmP& p0, int nz, hipStream_t stream) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.ntiles = ((p.M + 255) / 256) * p.tiles_n;
  // 1: LDS-staged epilogue (bf16 output: 16-B stores), 0: direct stores (tuning gemm_ldsepi = 0)
  p.lds_epi = tuning().gemm_ldsepi ? 1 : 0;
  // residual rows preloaded into the accumulators: fp32 output with a residual, no ReLU (the
  // reference adds the residual after the activation), 16-B aligned rows
  p.rinit = (sizeof(TO) == 4 && p.r && !p.relu && tuning().gemm_rinit && ((uintptr_t)p.r & 15) == 0 &&
             p.ldr % 4 == 0 && p.sr1 % 4 == 0 && p.sr2 % 4 == 0 && p.N % 4 == 0) ? 1 : 0;
  const long long total = (long long)p.ntiles * nz;
  if (sizeof(TC) == 4 || BN != 256 || AMODE == kRowsSplit3 || (p.K >= 128 && persist_enabled() && total < (1LL << 31))) {
    const int grid = (int)std::min<long long>(total, num_cus());
    hipLaunchKernelGGL((gemm_ppp_kernel<TC, TO, AMODE, BN>), dim3(grid), dim3(512), 0, stream, p, (int)total);
    return check_launch("mhada_gemm");
  }
  if constexpr (sizeof(TC) == 2 && BN == 256 && AMODE != kRowsSplit3) {
    hipLaunchKernelGGL((gemm_pp_kernel<TO, AMODE>), dim3(p.ntiles, nz), dim3(512), 0, stream, p);
    return check_launch("mhada_gemm");
  }
  return fail("mhada_gemm: no ping-pong form");
}

// The ping-pong kernel takes bf16 A (rows or 3x3 taps) with K % 64 == 0, N > 128 and operand
// spans addressable with 32-bit element offsets.  tuning gemm_pp = 0 disables it (A/B runs).
static bool pp_enabled() { return tuning().gemm_pp != 0; }

template <typename TC, typename TA, typename TO, int AMODE, int BM, int BN, int WM, int WN>
static int launch_gemm(const GemmP& p0, int nz, hipStream_t stream) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  // LDS-staged epilogue (tuning gemm_ldsepi = 0: direct stores); the scratch needs 4 KiB per wave
  p.lds_epi = (tuning().gemm_ldsepi &&
               (size_t)2 * (BM + BN) * Cfg<TC>::LS * sizeof(TC) >= (size_t)WM * WN * 4096) ? 1 : 0;
  const int tiles_m = (p.M + BM - 1) / BM;
  p.ntiles = tiles_m * p.tiles_n;
  const size_t lds2 = (size_t)2 * (BM + BN) * Cfg<TC>::LS * sizeof(TC);
  // one staging buffer when K fits one step (the kernel's nbuf), at least the epilogue scratch
  const size_t lds = p.K > Cfg<TC>::BK ? lds2
                                       : std::max(lds2 / 2, (size_t)(p.lds_epi || p.vt ? WM * WN * 4096 : 0));
  static std::once_flag attr_once;  // per instantiation: allow > 64 KiB dynamic LDS
  std::call_once(attr_once, [&] {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<TC, TA, TO, AMODE, BM, BN, WM, WN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
  });
  hipLaunchKernelGGL((gemm_kernel<TC, TA, TO, AMODE, BM, BN, WM, WN>), dim3(p.ntiles, nz), dim3(64 * WM * WN),
                     lds, stream, p);
  return check_launch("mhada_gemm");
}

// 32-bit element offsets inside one z-problem (the ping-pong kernel's staging addresses)
static bool pp_offsets_fit(const GemmP& p, int amode) {
  const long long lim = 1LL << 31;
  const long long wspan = (long long)(p.N - 1) * p.ldw + p.K;
  long long aspan;
  if (amode == MHADA_A_ROWS) aspan = (long long)(p.M - 1) * p.lda + p.K;
  else aspan = (long long)p.M / ((long long)p.out_h * p.out_w) * p.img_h * p.img_w * p.img_c;
  return wspan < lim && aspan < lim;
}

// Tile choice.  fp32 MFMA runs 1/16 of the bf16 rate, so 128x128 tiles (64 FLOP per staged
// byte) are far from L2-bound; bf16 needs 256-row tiles (up to 128 FLOP/B at 256x256) to stay
// under the ~34 TB/s L2 ceiling at MFMA rate.
template <typename TC, typename TA, typename TO, int AMODE>
static int dispatch_tile(const GemmP& p, int nz, hipStream_t s) {
  // the vt epilogue needs waves owning 64 columns of a 128-column tile (checked on the host:
  // N == 128, ROWS mode)
  if constexpr (AMODE == MHADA_A_ROWS || AMODE == kRowsCentred) {
    if (p.vt) {
      // (bf16: the 128x128 tile measured 5 % slower than 256x128)
      if constexpr (sizeof(TC) == 2) return launch_gemm<TC, TA, TO, AMODE, 256, 128, 4, 2>(p, nz, s);
      else return launch_gemm<TC, TA, TO, AMODE, 128, 128, 2, 2>(p, nz, s);
    }
  }
  // N <= 64: 128x64 tiles of 4 waves x (32x64), two workgroups per CU (55 KiB of LDS each), whose
  // barriers interleave: +2-10 % over one 256x64 workgroup of 8 waves (tuning gemm_n64 = 256
  // selects that form); a 4-wave 64x64-per-wave form measured 1.3-2x slower
  if (p.N <= 64) {
    if constexpr (sizeof(TC) == 4 && sizeof(TA) == 4 && sizeof(TO) == 4 && AMODE == MHADA_A_ROWS) {
      // fp32 rows, K % 32: the LDS-DMA ring kernel (the centred-A q projection stays on the
      // register-staged tile: a ring form with the centring on its fragments measured slower, round 4)
      if (p.K % 32 == 0 && p.lda % 4 == 0 && p.ldw % 4 == 0 && p.sa1 % 4 == 0 && p.sa2 % 4 == 0 &&
          p.sw1 % 4 == 0 && p.sw2 % 4 == 0 && aligned16(p.a) && aligned16(p.w)) {
        GemmP q = p;
        q.tiles_n = 1;
        // lds_epi (unused by this kernel's direct epilogue) = 4 flags the per-XCD grouping of the
        // problems
        q.lds_epi = nz % 8 == 0 ? 4 : 0;
        // long K (the dQ GEMM, K = Ns): 256 x 64 tiles of 256-B K-tiles, two stages (160 KiB);
        // short K (the grouped 1x1 convs, K = 64): 128 x 64 tiles, 2 stages of 128-B K-tiles (48 KiB,
        // three workgroups per CU; profiles/r03_opbench_n64*.log; 3-stage rings and 64-row tiles
        // measured no faster)
        if (p.K >= 1024 && p.K % 64 == 0) {
          q.ntiles = (p.M + 255) / 256;
          hipLaunchKernelGGL((gemm_n64_kernel<256, 2, 64>), dim3(q.ntiles, nz), dim3(512), 0, s, q);
        } else {
          q.ntiles = (p.M + 127) / 128;
          hipLaunchKernelGGL((gemm_n64_kernel<128, 2, 32>), dim3(q.ntiles, nz), dim3(256), 0, s, q);
        }
        return check_launch("mhada_gemm");
      }
    }
    if (tuning().gemm_n64 == 256) return launch_gemm<TC, TA, TO, AMODE, 256, 64, 8, 1>(p, nz, s);
    return launch_gemm<TC, TA, TO, AMODE, 128, 64, 4, 1>(p, nz, s);
  }
  if constexpr (sizeof(TC) == 4) {
    // persistent ping-pong (256x256 tiles) when the tiles fill at least 7/8 of the CUs (below
    // that the 128x128 kernel keeps more of the chip busy; the 1080p frame's N = 512 GEMMs have
    // 254 tiles); tuning gemm_pp / gemm_persist = 0 disable
    if constexpr (sizeof(TA) == 4 && (AMODE == MHADA_A_ROWS || AMODE == MHADA_A_CONV3X3 || AMODE == MHADA_A_CONV3X3_ZERO)) {
      const long long t256 = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256) * nz;
      if (p.N > 128 && p.K % 32 == 0 && p.K >= 64 && 8 * t256 >= 7LL * num_cus() && pp_enabled() && persist_enabled() &&
          pp_offsets_fit(p, AMODE)) {
        return launch_gemm_pp<float, TO, AMODE>(p, nz, s);
      }
      // (the 256x128 form measured 2-4 % slower than the 128x128 kernel in fp32: bf16 only)
    }
    return launch_gemm<TC, TA, TO, AMODE, 128, 128, 2, 2>(p, nz, s);
  } else {
    if constexpr (AMODE == MHADA_A_CONV3X3_UP2) {  // 4 bilinear taps staged per chunk: keep the tile small
      return launch_gemm<TC, TA, TO, AMODE, 128, 128, 2, 2>(p, nz, s);
    } else {
      if constexpr (sizeof(TA) == 2 && (AMODE == MHADA_A_ROWS || AMODE == MHADA_A_CONV3X3)) {
        if (p.N > 128 && p.K % 64 == 0 && pp_enabled() && pp_offsets_fit(p, AMODE))
          return launch_gemm_pp<bf16, TO, AMODE>(p, nz, s);
        // 65..128 columns: the 256x128 persistent ping-pong form (tuning gemm_pp128 = 0 disables)
        if (p.N > 64 && p.N <= 128 && p.K % 64 == 0 && p.K >= 128 && tuning().gemm_pp128 && pp_enabled() &&
            pp_offsets_fit(p, AMODE))
          return launch_gemm_pp<bf16, TO, AMODE, 128>(p, nz, s);
      }
      if (p.N <= 128) return launch_gemm<TC, TA, TO, AMODE, 256, 128, 4, 2>(p, nz, s);
      return launch_gemm<TC, TA, TO, AMODE, 256, 256, 2, 4>(p, nz, s);
    }
  }
}

template <typename TC, typename TA, typename TO>
static int dispatch_mode(int mode, const GemmP& p, int nz, hipStream_t s) {
  switch (mode) {
    case MHADA_A_ROWS:
      if (p.a_mu) return dispatch_tile<TC, TA, TO, kRowsCentred>(p, nz, s);
      return dispatch_tile<TC, TA, TO, MHADA_A_ROWS>(p, nz, s);
    case MHADA_A_CONV3X3: return dispatch_tile<TC, TA, TO, MHADA_A_CONV3X3>(p, nz, s);
    case MHADA_A_CONV3X3_UP2: return dispatch_tile<TC, TA, TO, MHADA_A_CONV3X3_UP2>(p, nz, s);
    case MHADA_A_CONV3X3_ZERO: return dispatch_tile<TC, TA, TO, MHADA_A_CONV3X3_ZERO>(p, nz, s);
    case MHADA_A_PATCH8:
      if constexpr (sizeof(TA) == 4) return dispatch_tile<TC, TA, TO, MHADA_A_PATCH8>(p, nz, s);
      return fail("mhada_gemm: PATCH8 needs an fp32 image");
    case MHADA_A_SPLIT3:
      // the persistent ping-pong kernel only (its K-tile walk knows the planes)
      if constexpr (sizeof(TC) == 2 && sizeof(TA) == 2) {
        if (nz != 1 || p.N <= 128 || p.K % (6 * 64) || p.K < 6 * 64 || !pp_offsets_fit(p, MHADA_A_ROWS))
          return fail("mhada_gemm: SPLIT3 needs one problem, N > 128, K0 = K / 6 a multiple of 64 and 32-bit offsets");
        return launch_gemm_pp<bf16, TO, kRowsSplit3>(p, nz, s);
      }
      return fail("mhada_gemm: SPLIT3 needs bf16 planes and bf16 compute");
  }
  return fail("mhada_gemm: bad a_mode");
}



// per-dtype dispatch entry points (gemm_d_*.hip)
int gemm_dispatch_f32(int mode, const GemmP& p, int nz, hipStream_t s);
int gemm_dispatch_bf16_a32_o32(int mode, const GemmP& p, int nz, hipStream_t s);
int gemm_dispatch_bf16_a32_o16(int mode, const GemmP& p, int nz, hipStream_t s);
int gemm_dispatch_bf16_a16_o32(int mode, const GemmP& p, int nz, hipStream_t s);
int gemm_dispatch_bf16_a16_o16(int mode, const GemmP& p, int nz, hipStream_t s);

}  // namespace mhada
