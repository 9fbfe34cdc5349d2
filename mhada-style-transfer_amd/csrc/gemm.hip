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

#include <mutex>

namespace mhada {

struct GemmP {
  int M, N, K, nb2;
  const void* a; long long lda, sa1, sa2;
  const float* a_mu; long long smu1, smu2;
  int img_c, img_h, img_w, out_h, out_w;
  const void* w; long long ldw, sw1, sw2;
  const float* bias; long long sb1, sb2;
  const void* r; long long ldr, sr1, sr2;
  void* c; long long ldc, sc1, sc2;
  int relu, tiles_n, ntiles;
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

// Internal A mode: ROWS with per-column centring (a_mu != NULL), a separate instantiation so
// the plain ROWS path stages raw chunks with no per-element work.
constexpr int kRowsCentred = 100;

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
      const int Y = reflect1(ri[i].y + dy, p.out_h);
      const int X = reflect1(ri[i].x + dx, p.out_w);
      const bool ok = ri[i].valid && kvalid;
      if constexpr (AMODE == MHADA_A_CONV3X3) {
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
        f[e] = ly0 * (lx0 * raw_get(st.raw[i][0], e) + lx1 * raw_get(st.raw[i][1], e)) +
               ly1 * (lx0 * raw_get(st.raw[i][2], e) + lx1 * raw_get(st.raw[i][3], e));
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
  TC* sA = reinterpret_cast<TC*>(smem);  // [2][BM][LS]
  TC* sB = sA + 2 * BM * LS;             // [2][BN][LS]

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

  // epilogue.  The MFMAs above take W as the A operand, so each accumulator holds C^T: the
  // lane owns ONE output row m (= lane&31 within the block) and registers 4g..4g+3 hold the 4
  // consecutive columns 8g + 4h + 0..3 — every store below moves 4 elements (8-16 B) instead of
  // one (a row-per-lane scalar-store tail is store-issue bound).
  TO* cbase = reinterpret_cast<TO*>(p.c) + z1 * p.sc1 + z2 * p.sc2;
  const TO* rbase = p.r ? reinterpret_cast<const TO*>(p.r) + z1 * p.sr1 + z2 * p.sr2 : nullptr;
  const float* bbase = p.bias ? p.bias + z1 * p.sb1 + z2 * p.sb2 : nullptr;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m = m0 + arow0 + mi * 32;
    if (m >= p.M) continue;
    TO* crow = cbase + (long long)m * p.ldc;
    const TO* rrow = rbase ? rbase + (long long)m * p.ldr : nullptr;
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + brow0 - r32 + ni * 32 + 8 * g + 4 * h;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[mi][ni][4 * g + e];
        if (n + 3 < p.N) {
          if (bbase) {
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bbase + n);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bb[e];
          }
          if (p.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if constexpr (sizeof(TO) == 4) {
            if (rrow) {
              const f32x4 rr = *reinterpret_cast<const f32x4*>(rrow + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += rr[e];
            }
            *reinterpret_cast<f32x4*>(crow + n) = f32x4{v[0], v[1], v[2], v[3]};
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
              if (p.relu) x = fmaxf(x, 0.f);
              if (rrow) x += to_f32<TO>(rrow[n + e]);
              crow[n + e] = from_f32<TO>(x);
            }
          }
        }
      }
    }
  }
}

template <typename TC, typename TA, typename TO, int AMODE, int BM, int BN, int WM, int WN>
static int launch_gemm(const GemmP& p0, int nz, hipStream_t stream) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  p.ntiles = tiles_m * p.tiles_n;
  const size_t lds = (size_t)2 * (BM + BN) * Cfg<TC>::LS * sizeof(TC);
  static std::once_flag attr_once;  // per instantiation: allow > 64 KiB dynamic LDS
  std::call_once(attr_once, [&] {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<TC, TA, TO, AMODE, BM, BN, WM, WN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  });
  hipLaunchKernelGGL((gemm_kernel<TC, TA, TO, AMODE, BM, BN, WM, WN>), dim3(p.ntiles, nz), dim3(64 * WM * WN),
                     lds, stream, p);
  return check_launch("mhada_gemm");
}

// Tile choice.  fp32 MFMA runs 1/16 of the bf16 rate, so 128x128 tiles (64 FLOP per staged
// byte) are far from L2-bound; bf16 needs 256-row tiles (up to 128 FLOP/B at 256x256) to stay
// under the ~34 TB/s L2 ceiling at MFMA rate.
template <typename TC, typename TA, typename TO, int AMODE>
static int dispatch_tile(const GemmP& p, int nz, hipStream_t s) {
  // N <= 64: 8 waves of 32x64 (one 256x64 tile keeps 8 waves per CU at 92 KiB of LDS)
  if (p.N <= 64) return launch_gemm<TC, TA, TO, AMODE, 256, 64, 8, 1>(p, nz, s);
  if constexpr (sizeof(TC) == 4) {
    return launch_gemm<TC, TA, TO, AMODE, 128, 128, 2, 2>(p, nz, s);
  } else {
    if constexpr (AMODE == MHADA_A_CONV3X3_UP2) {  // 4 bilinear taps staged per chunk: keep the tile small
      return launch_gemm<TC, TA, TO, AMODE, 128, 128, 2, 2>(p, nz, s);
    } else {
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
    case MHADA_A_PATCH8:
      if constexpr (sizeof(TA) == 4) return dispatch_tile<TC, TA, TO, MHADA_A_PATCH8>(p, nz, s);
      return fail("mhada_gemm: PATCH8 needs an fp32 image");
  }
  return fail("mhada_gemm: bad a_mode");
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_gemm(const mhada_gemm_args* a, mhada_stream_t stream_) {
  if (!a) return fail("mhada_gemm: null args");
  hipStream_t stream = (hipStream_t)stream_;
  if (a->M < 0 || a->N <= 0 || a->K <= 0 || a->nb1 <= 0 || a->nb2 <= 0)
    return fail("mhada_gemm: bad sizes");
  if (a->M == 0) return MHADA_OK;
  if (a->compute != MHADA_F32 && a->compute != MHADA_BF16) return fail("mhada_gemm: bad compute dtype");
  if (a->a_dtype != MHADA_F32 && a->a_dtype != MHADA_BF16) return fail("mhada_gemm: bad a_dtype");
  if (a->c_dtype != MHADA_F32 && a->c_dtype != MHADA_BF16) return fail("mhada_gemm: bad c_dtype");
  if (a->r && a->r_dtype != a->c_dtype) return fail("mhada_gemm: residual dtype must equal output dtype");
  if (a->compute == MHADA_F32 && (a->a_dtype != MHADA_F32 || a->c_dtype != MHADA_F32))
    return fail("mhada_gemm: fp32 compute needs fp32 A and C");
  if (!a->a || !a->w || !a->c) return fail("mhada_gemm: null operand");
  const int ec = a->compute == MHADA_F32 ? 4 : 8;      // compute elements per 16 B
  const int ea = a->a_dtype == MHADA_F32 ? 4 : 8;      // A elements per 16 B
  const int bk = a->compute == MHADA_F32 ? 32 : 64;
  if (a->K % ec) return fail("mhada_gemm: K must be a multiple of 16 bytes of compute type");
  if (!aligned16(a->w) || a->ldw % ec || a->sw1 % ec || a->sw2 % ec)
    return fail("mhada_gemm: W must be 16-byte aligned with aligned strides");
  if (!aligned16(a->a) || a->sa1 % ea || a->sa2 % ea) return fail("mhada_gemm: A must be 16-byte aligned");
  // the epilogue moves 4 consecutive output columns per access
  if (((uintptr_t)a->c & 7) || a->ldc % 4 || a->sc1 % 4 || a->sc2 % 4)
    return fail("mhada_gemm: C must be 8-byte aligned with strides that are multiples of 4");
  if (a->r && (((uintptr_t)a->r & 7) || a->ldr % 4 || a->sr1 % 4 || a->sr2 % 4))
    return fail("mhada_gemm: R must be 8-byte aligned with strides that are multiples of 4");
  if (a->bias && (!aligned16(a->bias) || a->sb1 % 4 || a->sb2 % 4))
    return fail("mhada_gemm: bias must be 16-byte aligned with strides that are multiples of 4");
  GemmP p{};
  p.M = a->M; p.N = a->N; p.K = a->K; p.nb2 = a->nb2;
  p.a = a->a; p.lda = a->lda; p.sa1 = a->sa1; p.sa2 = a->sa2;
  p.a_mu = a->a_mu; p.smu1 = a->smu1; p.smu2 = a->smu2;
  p.img_c = a->img_c; p.img_h = a->img_h; p.img_w = a->img_w;
  p.w = a->w; p.ldw = a->ldw; p.sw1 = a->sw1; p.sw2 = a->sw2;
  p.bias = a->bias; p.sb1 = a->sb1; p.sb2 = a->sb2;
  p.r = a->r; p.ldr = a->ldr; p.sr1 = a->sr1; p.sr2 = a->sr2;
  p.c = a->c; p.ldc = a->ldc; p.sc1 = a->sc1; p.sc2 = a->sc2;
  p.relu = a->relu;
  switch (a->a_mode) {
    case MHADA_A_ROWS:
      if (a->lda % ea) return fail("mhada_gemm: lda must be a multiple of 16 bytes");
      break;
    case MHADA_A_PATCH8:
      if (a->a_dtype != MHADA_F32) return fail("mhada_gemm: PATCH8 needs an fp32 image");
      if (a->img_w % 8 || a->img_h < 8) return fail("mhada_gemm: PATCH8 needs img_w % 8 == 0");
      if (a->K != a->img_c * 64) return fail("mhada_gemm: PATCH8 needs K == 64*img_c");
      p.out_h = a->img_h / 8; p.out_w = a->img_w / 8;
      if (a->M != p.out_h * p.out_w) return fail("mhada_gemm: PATCH8 needs M == (H/8)*(W/8)");
      if (a->a_mu) return fail("mhada_gemm: centring only in ROWS mode");
      break;
    case MHADA_A_CONV3X3:
    case MHADA_A_CONV3X3_UP2: {
      const int up = a->a_mode == MHADA_A_CONV3X3_UP2 ? 2 : 1;
      if (a->img_c % bk) return fail("mhada_gemm: CONV needs Cin % (128 bytes of compute type) == 0");
      if (a->K != 9 * a->img_c) return fail("mhada_gemm: CONV needs K == 9*Cin");
      p.out_h = a->img_h * up; p.out_w = a->img_w * up;
      if (p.out_h < 2 || p.out_w < 2) return fail("mhada_gemm: reflection padding needs H, W >= 2");
      if (a->M % (p.out_h * p.out_w)) return fail("mhada_gemm: CONV needs M == batch*out_h*out_w");
      if (a->nb1 * a->nb2 != 1) return fail("mhada_gemm: CONV is not z-batched (batch lives in M)");
      if (a->a_mu) return fail("mhada_gemm: centring only in ROWS mode");
      break;
    }
    default:
      return fail("mhada_gemm: bad a_mode");
  }
  const int nz = a->nb1 * a->nb2;
  if (nz > 65535) return fail("mhada_gemm: too many batch entries");
  if (a->compute == MHADA_F32) return dispatch_mode<float, float, float>(a->a_mode, p, nz, stream);
  if (a->a_dtype == MHADA_F32) {
    if (a->c_dtype == MHADA_F32) return dispatch_mode<bf16, float, float>(a->a_mode, p, nz, stream);
    return dispatch_mode<bf16, float, bf16>(a->a_mode, p, nz, stream);
  }
  if (a->c_dtype == MHADA_F32) return dispatch_mode<bf16, bf16, float>(a->a_mode, p, nz, stream);
  return dispatch_mode<bf16, bf16, bf16>(a->a_mode, p, nz, stream);
}
