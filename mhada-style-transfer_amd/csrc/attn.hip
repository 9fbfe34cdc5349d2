// Fused multi-head adaptive attention (MHAda), flash-style, one launch per block.
//
// Reference: AdaAttnMultiHead.forward (MHAdaSTr/network/adaDecoder.py:162-206).  Per head:
//   A = softmax(Q K^T)  (no 1/sqrt(d)!)     M = A V      E2 = A V^2
//   S = sqrt(max(E2 - M^2, 1e-6))           out = S * InstanceNorm(fcs) + M
// The reference materialises A (Nc x Ns fp32 per head).  Here A never leaves registers:
// each wave owns 32 query rows and streams 64-key tiles, keeping two output accumulators
// (sum p*v' and sum p*v'^2 over the centred V' = V - mean_tokens(V); the variance is
// shift-invariant, so the centring only removes E2 - M^2 cancellation) plus the running
// max / sum of an online softmax.
//
// Orientation ("swapped" products, cdna_hip_programming.md §3 accumulator-as-operand):
//   S^T (keys x queries) = K . Q^T  — the query is on the MFMA lane, so every lane holds
//       scores of ONE query: the row max/sum are lane-local plus one cross-half shuffle;
//   O^T (dv x queries)   = V'^T . P^T — P^T is the S^T accumulator itself, used as the B
//       operand with no lane movement; the dv/key index pairing follows the accumulator's
//       row permutation.
// Scores are in log2 units (the engine folds log2(e) into K), so P = exp2(s - m).
// fp32 and the cosine activation: online softmax with a deferred rescale
// (cdna_hip_programming.md T13): the running max m only moves when a tile's max exceeds it by
// more than kRescaleThr, so after the first tiles the O accumulators are touched by VALU only
// in a rare branch; P <= 2^kRescaleThr.  bf16 softmax: the fixed-shift kernel
// (attn_bf16_fs_kernel below): no in-loop max at all, an exact recompute for the rare rows
// whose scores outgrow the first tile's max by 2^64.
// Only the last, partial key tile runs the masking code.
// fp32: v_mfma_f32_32x32x2_f32 (exact fp32), K/V' streamed from kv[.][128] into LDS, V'^2
//       formed in registers.  bf16: v_mfma_f32_32x32x16_bf16, V'^T and V'^2^T streamed from
//       the pre-transposed, key-permuted vt image (mhada_transpose_v) so every operand read
//       is one 16-byte ds_read; fp32 accumulation and softmax.
// Block = NW waves = 32*NW queries of one (batch, head); blocks of one (b, h) are remapped
// onto one XCD so they share K/V in its L2.
#include "attn_common.h"

#include <type_traits>

namespace mhada {

// Scores of keys >= Ns: -inf (softmax) / -1 (cosine: p = s + 1 = 0).
template <int ACT, int NKB>
MHADA_DEV void mask_tile(f32x16 (&S)[NKB], int key0, int Ns, int h) {
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (key >= Ns) S[kb][r] = (ACT == MHADA_ACT_SOFTMAX) ? -INFINITY : -1.0f;
    }
}

// Online-softmax update of one tile: S becomes P (in place); returns true (wave-uniform)
// when the O accumulators must be multiplied by `alpha`.  m2 is the running max in log2 units.
template <int ACT, int NKB>
MHADA_DEV bool softmax_tile(f32x16 (&S)[NKB], float& m2, float& l, float& alpha) {
  float sum = 0.f;
  if constexpr (ACT == MHADA_ACT_SOFTMAX) {
    float mx = S[0][0];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const bool resc = __any(mx > m2 + kRescaleThr);
    alpha = 1.f;
    if (resc) {
      const float mn = fmaxf(m2, mx);
      alpha = fast_exp2(m2 - mn);
      l *= alpha;
      m2 = mn;
    }
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = fast_exp2(S[kb][r] - m2);
        S[kb][r] = pv;
        sum += pv;
      }
    l += sum;
    return resc;
  } else {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = S[kb][r] + 1.0f;
        S[kb][r] = pv;
        sum += pv;
      }
    l += sum;
    alpha = 1.f;
    return false;
  }
}

// Tile max of the scores in log2 units, combined over the two lane halves (same query).
template <int NKB>
MHADA_DEV float tile_max_log2(const f32x16 (&S)[NKB]) {
  float mx = S[0][0];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[kb][r]);
  return fmaxf(mx, __shfl_xor(mx, 32, 64));
}

// S -> P against the current running max (no rescale); accumulates the row sum.
template <int ACT, int NKB>
MHADA_DEV void softmax_apply(f32x16 (&S)[NKB], float m2, float& l) {
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = (ACT == MHADA_ACT_SOFTMAX) ? fast_exp2(S[kb][r] - m2) : S[kb][r] + 1.0f;
      S[kb][r] = pv;
      sum += pv;
    }
  l += sum;
}

MHADA_DEV void scale_acc(f32x16 (&O)[4], float alpha) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] *= alpha;
}


// In-kernel clock (MI355X_MICROARCH.md, DVFS give-back item 6), diagnostic builds only
// (-DATTN_CLOCK, tools/attn_clock.py): thread 0 of each workgroup stamps the shader-clock and the
// 100 MHz real-time counters before and after the key loop into a buffer of their own; no output
// is computed from them.  In the shipped build ATTN_STAMP expands to nothing.
#ifdef ATTN_CLOCK
constexpr int kClockBlocks = 65536;
__device__ unsigned long long g_attn_clock[4 * kClockBlocks];
#define ATTN_STAMP(slot)                                                                     \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < kClockBlocks) {                                     \
      const unsigned long long c_ = __builtin_amdgcn_s_memtime();                           \
      const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                       \
      g_attn_clock[4 * blockIdx.x + 2 * (slot)] = c_;                                        \
      g_attn_clock[4 * blockIdx.x + 2 * (slot) + 1] = r_;                                    \
    }                                                                                        \
  } while (0)
#else
#define ATTN_STAMP(slot) \
  do {                   \
  } while (0)
#endif

// Training epilogue (attn_train.hip's forward contract): out' = sqrt(max(E2' - M'^2, 1e-6)) x + M',
// mo = [M' | E2'], lse2 = m2 + log2(l) per query row; x = p.fcs [BH][Nc][64].
MHADA_DEV void attn_train_epilogue(const AttnP& p, const f32x16 (&O)[4], float l, float m2, long long bh, int q,
                                   int h) {
  const float lt = l + __shfl_xor(l, 32, 64);
  if (q >= p.Nc) return;
  const float inv = 1.0f / lt;
  const long long row = bh * p.Nc + q;
  const float* xr = p.fcs + row * 64;
  float* orow = reinterpret_cast<float*>(p.out) + row * 64;
  float* mrow = p.mo + row * 128;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 8 * g + 4 * h + 32 * blk;
      const f32x4 xx = *reinterpret_cast<const f32x4*>(xr + c0);
      f32x4 o, mm, ee;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[blk][4 * g + e] * inv;
        const float e2 = O[blk + 2][4 * g + e] * inv;
        o[e] = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f)) * xx[e] + m1;
        mm[e] = m1;
        ee[e] = e2;
      }
      *reinterpret_cast<f32x4*>(orow + c0) = o;
      *reinterpret_cast<f32x4*>(mrow + c0) = mm;
      *reinterpret_cast<f32x4*>(mrow + 64 + c0) = ee;
    }
  if (h == 0) p.lse[row] = m2 + __log2f(lt);
}

// fp32 V'^T | V'^2^T image [BH][128][ldt] (natural key order, zero padded) of the training v
// [BH][Ns][64] rows: the PV operand layout of attn_f32_kernel.  SQ = false: the plain transpose
// [BH][64][ldt] (mhada_transpose64: K^T, the W operand of the backward's dQ = dS K GEMM).
template <bool SQ = true>
__global__ void __launch_bounds__(256) train_vt_kernel(const float* __restrict__ v, float* __restrict__ vt, int Ns,
                                                       int ldt) {
  __shared__ float tile[64][65];
  const int bh = blockIdx.y, n0 = blockIdx.x * 64;
  const float* src = v + (long long)bh * Ns * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int n = i >> 6, o = i & 63;
    tile[n][o] = (n0 + n < Ns) ? src[(long long)(n0 + n) * 64 + o] : 0.f;
  }
  __syncthreads();
  float* dst = vt + (long long)bh * (SQ ? 128 : 64) * ldt + n0;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int o = i >> 6, n = i & 63;
    const float x = tile[n][o];
    dst[(long long)o * ldt + n] = x;
    if constexpr (SQ) dst[(long long)(64 + o) * ldt + n] = x * x;
  }
}

// ======================================================================================
// fp32 variant
// ======================================================================================
// TRAIN (mhada_attn_train_fwd_vt): the forward of the training step on the same structure —
// K rows of p.ldk = 64 floats (the training k), Q scaled by log2 e on load (the training q is in
// natural units), and the training epilogue (attn_train_epilogue: out', [M' | E2'], lse2 =
// m2 + log2 l, exact for the lazily rescaled state since l is relative to m2).
template <int ACT, int NW, bool TRAIN = false>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) attn_f32_kernel(const AttnP p) {
  constexpr int NT = 64 * NW;
  constexpr int LK = 68, LV = 68;  // padded rows (272 B): conflict-free 16-B reads down a column
  constexpr int KCH = 1024 / NT, VCH = 2048 / NT;  // 16-B chunks per thread per 64-key tile
  __shared__ __attribute__((aligned(16))) float sK[2][64 * LK];   // K rows
  __shared__ __attribute__((aligned(16))) float sV[2][128 * LV];  // V'^T | V'^2^T rows, 64 keys
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * (32 * NW) + wave * 32 + r32;
  const long long bh = (long long)b * p.H + hh;

  // Q^T operand: MFMA step s takes d = 32h + s
  float qreg[32];
  {
    const float* qp = reinterpret_cast<const float*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 32 * h;
    const float qs = TRAIN ? 1.4426950408889634f : 1.0f;  // log2 e (inference: folded into K)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(qp + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) qreg[4 * i + e] = (q < p.Nc) ? t[e] * qs : 0.f;
    }
  }
  const int ldk = TRAIN ? 64 : 128;
  const float* kvb = reinterpret_cast<const float*>(p.kv) + bh * p.Ns * ldk;
  const float* vtb = reinterpret_cast<const float*>(p.vt) + bh * 128 * (long long)p.ldt;

  // K rows from kv, V'^T | V'^2^T columns from the vt image (mhada_transpose_v, zero padded to
  // ldt): the PV operands are then one 16-B LDS read per 4 MFMAs with no VALU (reading V' rows
  // and squaring in registers cost an LDS wait and a VALU->MFMA hazard nop per 4 MFMAs)
  f32x4 sk[KCH], sv[VCH];
  auto issue = [&](int key0) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 4, col = (c & 15) * 4;
      const int key = key0 + row;
      sk[i] = key < p.Ns ? *reinterpret_cast<const f32x4*>(kvb + (long long)key * ldk + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c >> 4, col = (c & 15) * 4;
      sv[i] = *reinterpret_cast<const f32x4*>(vtb + (long long)row * p.ldt + key0 + col);
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 4, col = (c & 15) * 4;
      *reinterpret_cast<f32x4*>(&sK[buf][row * LK + col]) = sk[i];
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c >> 4, col = (c & 15) * 4;
      *reinterpret_cast<f32x4*>(&sV[buf][row * LV + col]) = sv[i];
    }
  };

  f32x16 O[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] = 0.f;
  float m2 = -INFINITY, l = 0.f;

  auto qk = [&](const float* cur, f32x16 (&S)[2]) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) S[kb][e] = 0.f;
      const float* krow = cur + (kb * 32 + r32) * LK + 32 * h;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4 kk = *reinterpret_cast<const f32x4*>(krow + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          S[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk[e], qreg[4 * i + e], S[kb], 0, 0, 0);
      }
    }
  };
  // PV step r of key block kb takes key kb*32 + (r&3) + 8(r>>2) + 4h (the accumulator row of
  // P^T): for r = 4j..4j+3 those are the 4 consecutive keys kb*32 + 8j + 4h + e of the V'^T rows
  auto pv = [&](const float* cv, const f32x16 (&P)[2]) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* vc = cv + r32 * LV + kb * 32 + 8 * j + 4 * h;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(vc);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(vc + 32 * LV);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(vc + 64 * LV);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(vc + 96 * LV);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pr = P[kb][4 * j + e];
          O[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0[e], pr, O[0], 0, 0, 0);
          O[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1[e], pr, O[1], 0, 0, 0);
          O[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[e], pr, O[2], 0, 0, 0);
          O[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[e], pr, O[3], 0, 0, 0);
        }
      }
    }
  };

  const int NTILE = (p.Ns + 63) / 64, NFULL = p.Ns / 64;
  issue(0);
  commit(0);
  __syncthreads();
  ATTN_STAMP(0);
  // Full tiles.  The rescale (P <= 2^kRescaleThr, so after the first tile it is rare) is a
  // wave-uniform branch inside the single loop: one register assignment for the O accumulators
  // (a leave-rescale-reenter loop made the compiler copy all of O between two register sets on
  // every iteration).
  for (int t = 0; t < NFULL; ++t) {
    const int cb = t & 1;
    const bool nxt = t + 1 < NTILE;
    if (nxt) issue((t + 1) * 64);
    f32x16 S[2];
    qk(sK[cb], S);
    if constexpr (ACT == MHADA_ACT_SOFTMAX) {
      const float mx = tile_max_log2<2>(S);
      if (__any(mx > m2 + kRescaleThr)) {
        const float mn = fmaxf(m2, mx);
        const float alpha = fast_exp2(m2 - mn);
        l *= alpha;
        scale_acc(O, alpha);
        m2 = mn;
      }
    }
    softmax_apply<ACT, 2>(S, m2, l);
    pv(sV[cb], S);
    if (nxt) commit(cb ^ 1);
    __syncthreads();
  }
  if (NFULL < NTILE) {  // ragged last tile: masked, full online-softmax update
    const int cb = NFULL & 1;
    f32x16 S[2];
    qk(sK[cb], S);
    mask_tile<ACT, 2>(S, NFULL * 64, p.Ns, h);
    float alpha;
    if (softmax_tile<ACT, 2>(S, m2, l, alpha)) scale_acc(O, alpha);
    pv(sV[cb], S);
  }
  ATTN_STAMP(1);
  if constexpr (TRAIN) attn_train_epilogue(p, O, l, m2, bh, q, h);
  else attn_epilogue<float>(p, O, l, b, hh, q, h);
}

// ======================================================================================
// bf16 variant
// ======================================================================================
template <int ACT, int NW, int TK>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) attn_bf16_kernel(const AttnP p) {
  constexpr int NT = 64 * NW, NKB = TK / 32;
  constexpr int LK = 72;       // K rows: 64 + 8 bf16 (144 B): conflict-free 16-B row reads
  constexpr int LV = TK + 8;   // V'^T rows: TK keys + 8 (row stride = 16 B mod 256 B): conflict-free
  constexpr int KSZ = TK * LK, VSZ = 128 * LV;
  constexpr int KCH = TK * 8 / NT, VCH = 128 * (TK / 8) / NT;  // 16-B chunks per thread per tile
  static_assert(KCH >= 1 && VCH >= 1, "tile config");
  __shared__ __attribute__((aligned(16))) bf16 sK[2][KSZ];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][VSZ];
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * (32 * NW) + wave * 32 + r32;
  const long long bh = (long long)b * p.H + hh;

  // Q^T operand: k-step s takes d = 16s + 8h + j
  bf16x8 qf[4];
  {
    const bf16* qp = reinterpret_cast<const bf16*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
      if (q >= p.Nc) {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[s][e] = (bf16)0.0f;
      }
    }
  }
  const bf16* kvb = reinterpret_cast<const bf16*>(p.kv) + bh * p.Ns * 128;
  const bf16* vtb = reinterpret_cast<const bf16*>(p.vt) + bh * 128 * (long long)p.ldt;

  bf16x8 sk[KCH], sv[VCH];
  auto issue = [&](int key0) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 3, col = (c & 7) * 8;
      const int key = key0 + row;
      if (key < p.Ns) {
        sk[i] = *reinterpret_cast<const bf16x8*>(kvb + (long long)key * 128 + col);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) sk[i][e] = (bf16)0.0f;
      }
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c / (TK / 8), col = (c % (TK / 8)) * 8;
      if (key0 + col < p.ldt) {  // the image is zero padded to ldt = ceil64(Ns)
        sv[i] = *reinterpret_cast<const bf16x8*>(vtb + (long long)row * p.ldt + key0 + col);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) sv[i][e] = (bf16)0.0f;
      }
    }
  };
  auto commit = [&](bf16* dk, bf16* dv) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<bf16x8*>(dk + row * LK + col) = sk[i];
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c / (TK / 8), col = (c % (TK / 8)) * 8;
      *reinterpret_cast<bf16x8*>(dv + row * LV + col) = sv[i];
    }
  };

  f32x16 O[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] = 0.f;
  float m2 = -INFINITY, l = 0.f;

  auto qk = [&](const bf16* ck, f32x16 (&S)[NKB]) {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) S[kb][e] = 0.f;
      const bf16* krow = ck + (kb * 32 + r32) * LK + 8 * h;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 kk = *reinterpret_cast<const bf16x8*>(krow + 16 * s);
        S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kk, qf[s], S[kb], 0, 0, 0);
      }
    }
  };
  auto pv = [&](const bf16* cv, const f32x16 (&P)[NKB]) {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // B = P^T: element j <-> key kb*32 + 16s + 8(j>>2) + 4h + (j&3) (accumulator regs 8s..8s+7);
        // the vt image stores those 8 keys contiguously at key position 16s + 8h.
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (bf16)P[kb][8 * s + j];
        const bf16* vcol = cv + r32 * LV + kb * 32 + 16 * s + 8 * h;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vcol + 32 * blk * LV);
          O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, O[blk], 0, 0, 0);
        }
      }
    }
  };

  const int NTILE = (p.Ns + TK - 1) / TK, NFULL = p.Ns / TK;
  issue(0);
  commit(sK[0], sV[0]);
  __syncthreads();
  // Full tiles.  The rescale (rare after the first tile, P <= 2^kRescaleThr) is a wave-uniform
  // branch inside the single loop so the O accumulators keep one register assignment.
  for (int t = 0; t < NFULL; ++t) {
    const int cb = t & 1;
    const bool nxt = t + 1 < NTILE;
    if (nxt) issue((t + 1) * TK);
    f32x16 S[NKB];
    qk(sK[cb], S);
    if constexpr (ACT == MHADA_ACT_SOFTMAX) {
      const float mx = tile_max_log2<NKB>(S);
      if (__any(mx > m2 + kRescaleThr)) {
        const float mn = fmaxf(m2, mx);
        const float alpha = fast_exp2(m2 - mn);
        l *= alpha;
        scale_acc(O, alpha);
        m2 = mn;
      }
    }
    softmax_apply<ACT, NKB>(S, m2, l);
    pv(sV[cb], S);
    if (nxt) commit(sK[cb ^ 1], sV[cb ^ 1]);
    __syncthreads();
  }
  if (NFULL < NTILE) {
    const int cb = NFULL & 1;
    f32x16 S[NKB];
    qk(sK[cb], S);
    mask_tile<ACT, NKB>(S, NFULL * TK, p.Ns, h);
    float alpha;
    if (softmax_tile<ACT, NKB>(S, m2, l, alpha)) scale_acc(O, alpha);
    pv(sV[cb], S);
  }
  attn_epilogue<bf16>(p, O, l, b, hh, q, h);
}

// --------------------------------------------------------------------------------------
// bf16 softmax, fixed shift ("fs"): the 8-wave kernel's structure without any in-loop max or
// rescale.  m2 = the max of each query's FIRST key tile (<= the row max, so l >= 1); every
// later tile's scores come out of the MFMA already shifted (accumulators start at -m2), so
// the per-tile softmax is exp2 + row sum + bf16 pack: no max pass, no fma, no branch (the
// 8-wave kernel spends ~45 % of its softmax VALU on the max / shift).  A row whose later scores
// rise more than 64 (log2) above m2 trips l > 2^64 and is recomputed exactly after the loop
// (attn_exact_half).  Branch-free clamped tile loads (keys past Ns re-read valid rows and are
// masked in the last tile).
// --------------------------------------------------------------------------------------
template <int NW, int TK>
__global__ void __launch_bounds__(64 * NW, 1) attn_bf16_fs_kernel(const AttnP p) {
  constexpr int NT = 64 * NW, NKB = TK / 32;
  constexpr int LK = 72, LV = TK + 8;  // padded rows: conflict-free 16-B reads
  constexpr int KSZ = TK * LK, VSZ = 128 * LV;
  constexpr int KCH = TK * 8 / NT, VCH = 128 * (TK / 8) / NT;
  static_assert(KCH >= 1 && VCH >= 1, "tile config");
  __shared__ __attribute__((aligned(16))) bf16 sK[2][KSZ];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][VSZ];
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * (32 * NW) + wave * 32 + r32;
  const long long bh = (long long)b * p.H + hh;
  const int Ns = p.Ns;
  const f32x16 zero = {};

  bf16x8 qf[4];
  {
    const bf16* qp = reinterpret_cast<const bf16*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
      if (q >= p.Nc) {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[s][e] = (bf16)0.0f;
      }
    }
  }
  const bf16* kvb = reinterpret_cast<const bf16*>(p.kv) + bh * (long long)Ns * 128;
  const bf16* vtb = reinterpret_cast<const bf16*>(p.vt) + bh * 128 * (long long)p.ldt;

  bf16x8 sk[KCH], sv[VCH];
  auto issue = [&](int key0) {  // clamped: past-the-end rows / columns re-read valid data
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 3, col = (c & 7) * 8;
      sk[i] = *reinterpret_cast<const bf16x8*>(kvb + (long long)min(key0 + row, Ns - 1) * 128 + col);
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c / (TK / 8), col = (c % (TK / 8)) * 8;
      sv[i] = *reinterpret_cast<const bf16x8*>(vtb + (long long)row * p.ldt + min(key0 + col, p.ldt - 8));
    }
  };
  auto commit = [&](bf16* dk, bf16* dv) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + NT * i, row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<bf16x8*>(dk + row * LK + col) = sk[i];
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + NT * i, row = c / (TK / 8), col = (c % (TK / 8)) * 8;
      *reinterpret_cast<bf16x8*>(dv + row * LV + col) = sv[i];
    }
  };
  auto qk = [&](const bf16* ck, f32x16 (&S)[NKB], const f32x16& init) {
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const bf16* krow = ck + (kb * 32 + r32) * LK + 8 * h;
      S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(krow), qf[0], init, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < 4; ++s)
        S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(krow + 16 * s), qf[s], S[kb], 0,
                                                        0, 0);
    }
  };
  f32x16 O[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) O[i] = zero;
  float l = 0.f;
  // exp2 of the shifted scores, row sum, PV (B = P^T: element j <-> key kb*32 + 16s + 8(j>>2) +
  // 4h + (j&3); the vt image stores those 8 keys contiguously at key position 16s + 8h)
  auto finish = [&](const bf16* cv, const f32x16 (&S)[NKB]) {
    float part[4] = {0.f, 0.f, 0.f, 0.f};  // independent add chains (a serial sum is latency bound)
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = fast_exp2(S[kb][8 * s + j]);
          part[j & 3] += e;
          pf[j] = (bf16)e;
        }
        const bf16* vcol = cv + r32 * LV + kb * 32 + 16 * s + 8 * h;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vcol + 32 * blk * LV);
          O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, O[blk], 0, 0, 0);
        }
      }
    }
    l += (part[0] + part[1]) + (part[2] + part[3]);
  };

  const int NTILE = (Ns + TK - 1) / TK, NFULL = Ns / TK;
  issue(0);
  commit(sK[0], sV[0]);
  __syncthreads();
  // tile 0: scores unshifted, m2 = their max, then shift
  f32x16 Cm;
  {
    issue(min(1, NTILE - 1) * TK);
    f32x16 S[NKB];
    qk(sK[0], S, zero);
    if (NFULL == 0) mask_tile<MHADA_ACT_SOFTMAX, NKB>(S, 0, Ns, h);
    const float m2 = tile_max_log2<NKB>(S);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) S[kb][r] -= m2;
#pragma unroll
    for (int r = 0; r < 16; ++r) Cm[r] = -m2;
    finish(sV[0], S);
    commit(sK[1], sV[1]);
    __syncthreads();
  }
  // static priority for the second-dispatched half (MI355X_MICROARCH.md "Two waves per SIMD"
  // item 4: waves 4-7 lose every arbitration otherwise); tuning attn_prio = 0 disables (A/B)
  if (p.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // full tiles 1 .. NFULL-1: no max, no branch
  for (int t = 1; t < NFULL; ++t) {
    const int cb = t & 1;
    issue(min(t + 1, NTILE - 1) * TK);
    f32x16 S[NKB];
    qk(sK[cb], S, Cm);
    finish(sV[cb], S);
    commit(sK[cb ^ 1], sV[cb ^ 1]);
    __syncthreads();
  }
  if (NFULL < NTILE && NFULL > 0) {  // ragged last tile
    const int cb = NFULL & 1;
    f32x16 S[NKB];
    qk(sK[cb], S, Cm);
    mask_tile<MHADA_ACT_SOFTMAX, NKB>(S, NFULL * TK, Ns, h);
    finish(sV[cb], S);
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  if (__any(!(lt <= kShiftSumThr))) attn_exact_half(p, kvb, vtb, qf, O, l, h, r32);
  attn_epilogue<bf16>(p, O, l, b, hh, q, h);
}

// --------------------------------------------------------------------------------------
// Fixed-shift LDS-DMA kernel on v_mfma_f32_16x16x32_bf16 ("fsq1", the bf16 softmax default when
// Ns % 128 == 0): the fixed shift of attn_bf16_fs_kernel with the K / V'^T tiles staged by
// global_load_lds into a 2-slot ring (no staging registers, no LDS write pass, the next tile's DMA
// in flight for the whole iteration), on the 16 x 16 output shape, which the chip runs at a higher
// sustained clock under load than the 32 x 32 shape at equal cycles per FLOP (MI355X_MICROARCH.md,
// DVFS give-back item 7).  LDS images are lane-linear per wave-instruction and XOR-swizzled on the
// SOURCE address: V'^T rows (256 B) keep 16-B chunk c at slot c ^ (row & 15).
// Orientation as before (swapped products, the query on the MFMA column):
//   S^T (16 keys x 16 queries) = K (16 x 32 d) . Q^T (32 d x 16 queries): lane = query r16 of a
//       16-query group qg, rows 4g..4g+3 (g = lane >> 4); a wave owns 32 queries = 2 groups, and
//       every K fragment feeds both groups' MFMAs;
//   O^T (16 dv x 16 queries) += V'^T (16 dv x 32 keys) . P^T (32 keys x 16 queries): B slot 8g+j
//       is vt position 32kg + 8g + j of the key-permuted vt image = key 32kg + 16(g>>1) +
//       8(j>>2) + 4(g&1) + (j&3).  The two score tiles t = 0 / 1 of a 32-key group are therefore
//       computed for keys 32kg + 16(r>>3) + 4((r>>2)&1) + (r&3) + 8t (r = A-operand row): lane
//       group g then holds exactly its 8 B slots (j < 4 from t = 0, j >= 4 from t = 1) — the
//       permutation costs only the K row address, no lane movement, no second vt layout.
// K image: chunk c of key row k at 16-B slot c ^ (k & 7) (conflict-free for these row sets
// under the ds_read_b128 lane groups of MI355X_MICROARCH.md's LDS table).
// Measured in round 4 (tools/attn_clock.py, profiles/r04_attn_clock.log, 1024^2 B4): the 32x32x16
// form of this loop (removed in round 5) held 1.78-1.83 GHz at 0.62-0.63 of the clock-adjusted
// peak; this shape holds 2.15-2.19 GHz at 0.54-0.55 (the 16-cycle MFMA blocks vector issue for 8
// of its 16 cycles, so the softmax VALU competes harder); net 4-6 % faster.
// The row sum l comes out of one extra MFMA per (32 keys, 16 queries) with an all-ones A operand
// (D rows = sum_k P[k][q]), removing the 64 v_add_f32 per tile and lane from the VALU stream at
// +8 MFMAs (72 instead of 64 PV MFMAs per tile and wave); l is then the sum of the bf16-rounded P
// that the PV products use.
// --------------------------------------------------------------------------------------

// Exact two-pass recompute of one wave's 2 x 16 queries (16x16x32 layout; the rare path when a row
// sum trips kShiftSumThr): true row max over all keys, then the full pass, operands from L2.
MHADA_DEV void attn_exact_q(const AttnP& p, const bf16* kvb, const bf16* vtb, const bf16x8 (&qf)[2][2],
                            f32x4 (&O)[2][8], float (&lt)[2], int g, int r16) {
  const int Ns = p.Ns;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto scores = [&](int k0, f32x4 (&S)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16* kr = kvb + (long long)(k0 + fsq_key(r16, t)) * 128 + 8 * g;
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) S[qg][t] = z4;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kr + 32 * dh);
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) S[qg][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qg][dh], S[qg][t], 0, 0, 0);
      }
    }
  };
  float m2[2] = {-INFINITY, -INFINITY};
  for (int k0 = 0; k0 < Ns; k0 += 32) {
    f32x4 S[2][2];
    scores(k0, S);
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) m2[qg] = fmaxf(m2[qg], S[qg][t][j]);
  }
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    m2[qg] = fmaxf(m2[qg], __shfl_xor(m2[qg], 16, 64));
    m2[qg] = fmaxf(m2[qg], __shfl_xor(m2[qg], 32, 64));
    lt[qg] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) O[qg][i] = z4;
  }
  for (int k0 = 0; k0 < Ns; k0 += 32) {
    f32x4 S[2][2];
    scores(k0, S);
    bf16x8 pf[2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = fast_exp2(S[qg][j >> 2][j & 3] - m2[qg]);
        lt[qg] += e;
        pf[qg][j] = (bf16)e;
      }
#pragma unroll
    for (int dvb = 0; dvb < 8; ++dvb) {
      const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vtb + (long long)(16 * dvb + r16) * p.ldt + k0 + 8 * g);
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) O[qg][dvb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qg], O[qg][dvb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    lt[qg] += __shfl_xor(lt[qg], 16, 64);
    lt[qg] += __shfl_xor(lt[qg], 32, 64);
  }
}

template <int NW>
__global__ void __launch_bounds__(64 * NW, 1) attn_bf16_fsq_kernel(const AttnP p) {
  constexpr int TK = 128, NSL = 2;
  constexpr int KSZ = TK * 64, VSZ = 128 * TK;  // bf16 elements per slot: K [128][64], V'^T [128][128]
  constexpr int KPW = TK * 128 / 1024 / NW, VPW = 128 * TK * 2 / 1024 / NW;  // 1-KiB pieces per wave
  static_assert(KPW >= 1 && VPW >= 1, "tile config");
  __shared__ __attribute__((aligned(16))) bf16 smem[NSL * (KSZ + VSZ)];  // 96 KiB
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int q0 = qb * (32 * NW) + wave * 32;
  const long long bh = (long long)b * p.H + hh;
  const int Ns = p.Ns;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  bf16x8 qf[2][2];  // Q^T fragments: query q0 + 16 qg + r16, d = 32 dh + 8 g .. + 8
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + 16 * qg + r16;
    const bf16* qp = reinterpret_cast<const bf16*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 8 * g;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      qf[qg][dh] = *reinterpret_cast<const bf16x8*>(qp + 32 * dh);
      if (q >= p.Nc) {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[qg][dh][e] = (bf16)0.0f;
      }
    }
  }
  const bf16* kvb = reinterpret_cast<const bf16*>(p.kv) + bh * (long long)Ns * 128;
  const bf16* vtb = reinterpret_cast<const bf16*>(p.vt) + bh * 128 * (long long)p.ldt;
  int ksrc[KPW], vsrc[VPW];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    const int row = 8 * (KPW * wave + i) + (lane >> 3), slot = lane & 7;
    ksrc[i] = row * 128 + 8 * (slot ^ (row & 7));
  }
#pragma unroll
  for (int i = 0; i < VPW; ++i) {
    const int row = 4 * (VPW * wave + i) + (lane >> 4), slot = lane & 15;
    vsrc[i] = row * p.ldt + 8 * (slot ^ (row & 15));
  }
  auto stage = [&](int key0, int sl) {
    bf16* kd = smem + sl * (KSZ + VSZ);
    bf16* vd = kd + KSZ;
    const bf16* ks = kvb + (long long)key0 * 128;
    const bf16* vs = vtb + key0;
#pragma unroll
    for (int i = 0; i < KPW; ++i) attn_glds16(ks + ksrc[i], kd + 512 * (KPW * wave + i));
#pragma unroll
    for (int i = 0; i < VPW; ++i) attn_glds16(vs + vsrc[i], vd + 512 * (VPW * wave + i));
  };
  // per-lane K row offsets (elements) of the two score tiles of a 32-key group
  int krow[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) krow[t] = fsq_key(r16, t) * 64;
  auto qk = [&](int sl, f32x4 (&S)[2][4][2], const f32x4 (&init)[2]) {
    const bf16* ck = smem + sl * (KSZ + VSZ);
#pragma unroll
    for (int kg = 0; kg < 4; ++kg)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16* kr = ck + kg * 32 * 64 + krow[t];
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          // key & 7 == r16 & 3 | 4 ((r16 >> 2) & 1) == r16 & 7 (fsq_key keeps the low 3 bits)
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kr + 8 * ((4 * dh + g) ^ (r16 & 7)));
#pragma unroll
          for (int qg = 0; qg < 2; ++qg)
            S[qg][kg][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qg][dh], dh == 0 ? init[qg] : S[qg][kg][t],
                                                                   0, 0, 0);
        }
      }
  };
  f32x4 O[2][8], L[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    L[qg] = z4;
#pragma unroll
    for (int i = 0; i < 8; ++i) O[qg][i] = z4;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  auto finish = [&](int sl, const f32x4 (&S)[2][4][2]) {
    const bf16* cv = smem + sl * (KSZ + VSZ) + KSZ;
#pragma unroll
    for (int kg = 0; kg < 4; ++kg) {
      bf16x8 pf[2];
#pragma unroll
      for (int qg = 0; qg < 2; ++qg)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pf[qg][j] = (bf16)fast_exp2(S[qg][kg][j >> 2][j & 3]);
        }
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qg], L[qg], 0, 0, 0);
      const int ch = (4 * kg + g) ^ r16;  // row 16 dvb + r16: row & 15 == r16
#pragma unroll
      for (int dvb = 0; dvb < 8; ++dvb) {
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(cv + (16 * dvb + r16) * TK + 8 * ch);
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) O[qg][dvb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qg], O[qg][dvb], 0, 0, 0);
      }
    }
  };

  const int NTILE = Ns / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 Sa[2][4][2], Cm[2];
  {  // tile 0: unshifted scores, m2 = their max, then shift
    const f32x4 zi[2] = {z4, z4};
    qk(0, Sa, zi);
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float m = -INFINITY;
#pragma unroll
      for (int kg = 0; kg < 4; ++kg)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) m = fmaxf(m, Sa[qg][kg][t][j]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
#pragma unroll
      for (int kg = 0; kg < 4; ++kg)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) Sa[qg][kg][t][j] -= m;
      Cm[qg] = f32x4{-m, -m, -m, -m};
    }
  }
  if (p.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  ATTN_STAMP(0);
  if (NTILE > 1) stage(TK, 1);
  finish(0, Sa);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int t = 1; t < NTILE; ++t) {
    if (t + 1 < NTILE) stage((t + 1) * TK, (t + 1) & 1);
    qk(t & 1, Sa, Cm);
    finish(t & 1, Sa);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  ATTN_STAMP(1);
  float lt[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) lt[qg] = L[qg][0];  // every D row is the full sum over the 32 keys of each MFMA
  if (__any(!(lt[0] <= kShiftSumThr) || !(lt[1] <= kShiftSumThr))) attn_exact_q(p, kvb, vtb, qf, O, lt, g, r16);
  attn_epilogue_q<bf16>(p, O, lt, b, hh, q0, g, r16);
}

// Variant selection: the fixed-shift kernels are the bf16 softmax default (fsq1 when Ns % 128 == 0,
// attn_bf16_fs_kernel for ragged Ns); the online-max kernel serves the cosine activation and, through
// tuning attn_fixed_shift = 0, tests / A-B.  Round 5 removed the measured-slower fixed-shift variants
// (the 32x32x16 LDS-DMA kernel, the half-tile pipelined and the persistent forms; their logs are
// profiles/r03_attn_variants_ab*.log and profiles/r04_attn_variants_ab*.log).
static bool attn_bf16_fixed_shift() { return tuning().attn_fixed_shift != 0; }
static int attn_tk() { return tuning().attn_tk; }

static int attn_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int NW>
static void launch_attn(const AttnP& p, int dtype, int activation, hipStream_t s) {
  const dim3 grid(p.nblk), blk(64 * NW);
  if (dtype == MHADA_F32) {
    if (activation == MHADA_ACT_SOFTMAX)
      hipLaunchKernelGGL((attn_f32_kernel<MHADA_ACT_SOFTMAX, NW>), grid, blk, 0, s, p);
    else
      hipLaunchKernelGGL((attn_f32_kernel<MHADA_ACT_COSINE, NW>), grid, blk, 0, s, p);
    return;
  }
  if (activation == MHADA_ACT_SOFTMAX && attn_bf16_fixed_shift()) {
    if (p.Ns % 128 == 0) {  // whole 128-key tiles: the LDS-DMA 16x16x32 kernel
      hipLaunchKernelGGL((attn_bf16_fsq_kernel<NW>), grid, blk, 0, s, p);
      return;
    }
    if constexpr (NW == 8) {  // ragged Ns: register-staged fixed shift (2 x 106 KiB at 4 waves does not fit)
      hipLaunchKernelGGL((attn_bf16_fs_kernel<8, 128>), grid, blk, 0, s, p);
      return;
    }
  }
  const bool t128 = NW == 8 && attn_tk() == 128;  // 2 x 106 KiB of LDS does not fit a CU
  if (activation == MHADA_ACT_SOFTMAX) {
    if (t128) hipLaunchKernelGGL((attn_bf16_kernel<MHADA_ACT_SOFTMAX, NW, (NW == 8 ? 128 : 64)>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((attn_bf16_kernel<MHADA_ACT_SOFTMAX, NW, 64>), grid, blk, 0, s, p);
  } else {
    if (t128) hipLaunchKernelGGL((attn_bf16_kernel<MHADA_ACT_COSINE, NW, (NW == 8 ? 128 : 64)>), grid, blk, 0, s, p);
    else hipLaunchKernelGGL((attn_bf16_kernel<MHADA_ACT_COSINE, NW, 64>), grid, blk, 0, s, p);
  }
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_attn(const void* q, const void* kv, const void* vt, const float* fcs, const float* fcs_mu,
                          const float* fcs_rstd, const float* v_mu, void* out, int dtype, int B, int H, int Nc,
                          int Ns, int activation, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!q || !kv || !fcs || !fcs_mu || !fcs_rstd || !v_mu || !out || B <= 0 || H <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn: bad args");
  if (!vt) return fail("mhada_attn: needs the transposed V' image (mhada_transpose_v)");
  if (activation != MHADA_ACT_SOFTMAX && activation != MHADA_ACT_COSINE) return fail("mhada_attn: bad activation");
  AttnP p;
  p.q = q; p.kv = kv; p.vt = vt; p.fcs = fcs; p.fcs_mu = fcs_mu; p.fcs_rstd = fcs_rstd; p.v_mu = v_mu;
  p.out = out; p.B = B; p.H = H; p.Nc = Nc; p.Ns = Ns;
  p.prio = tuning().attn_prio;
  p.ldk = 128;
  p.ldt = (Ns + 63) / 64 * 64;
  // tuning attn_waves: 4 or 8 waves per block as set; 0 (default) = 8, except that a grid of 8-wave
  // blocks smaller than the CU count (B = 1 at 512^2: 128 blocks) leaves CUs idle, so it runs 4-wave
  // blocks there (one wave per SIMD instead of two, twice as many CUs covered)
  int nw = tuning().attn_waves;
  if (nw == 0) nw = (long long)B * H * ((Nc + 255) / 256) < attn_num_cus() ? 4 : 8;
  p.nqb = (Nc + 32 * nw - 1) / (32 * nw);
  const long long nblk = (long long)B * H * p.nqb;
  if (nblk > (1LL << 31) - 1) return fail("mhada_attn: grid too large");
  p.nblk = (int)nblk;
  if (nw == 8) {
    launch_attn<8>(p, dtype, activation, s);
  } else {
    launch_attn<4>(p, dtype, activation, s);
  }
  return check_launch("mhada_attn");
}

#ifdef ATTN_CLOCK
// Diagnostic builds: copy the first n stamps (4 per workgroup) of the last launch to host memory.
extern "C" int mhada_dbg_attn_clock(unsigned long long* host, int n) {
  if (!host || n <= 0 || n > 4 * kClockBlocks) return fail("mhada_dbg_attn_clock: bad args");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_clock), sizeof(unsigned long long) * n) != hipSuccess)
    return fail("mhada_dbg_attn_clock: copy failed");
  return MHADA_OK;
}
#endif

// Training forward on the inference fp32 attention structure (64-key tiles, lazy rescale, the PV
// operands as one 16-B LDS read per 4 MFMAs from the V'^T | V'^2^T image): replaces
// mhada_attn_train_fwd (attn_train.hip), same outputs.  vt: caller-provided workspace
// [BH][128][ceil64(Ns)] fp32, filled here from v.
extern "C" int mhada_attn_train_fwd_vt(const float* q, const float* k, const float* v, float* vt, const float* x,
                                       float* out, float* mo, float* lse, int BH, int Nc, int Ns,
                                       mhada_stream_t s_) {
  if (!q || !k || !v || !vt || !x || !out || !mo || !lse || BH <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_train_fwd_vt: bad args");
  if (BH > 65535) return fail("mhada_attn_train_fwd_vt: BH > 65535");
  const hipStream_t s = (hipStream_t)s_;
  AttnP p = {};
  p.q = q; p.kv = k; p.vt = vt; p.fcs = x; p.out = out; p.mo = mo; p.lse = lse;
  p.B = BH; p.H = 1; p.Nc = Nc; p.Ns = Ns; p.ldk = 64;
  p.ldt = (Ns + 63) / 64 * 64;
  p.nqb = (Nc + 255) / 256;
  const long long nblk = (long long)BH * p.nqb;
  if (nblk > (1LL << 31) - 1) return fail("mhada_attn_train_fwd_vt: grid too large");
  p.nblk = (int)nblk;
  hipLaunchKernelGGL(train_vt_kernel<true>, dim3(p.ldt / 64, BH), dim3(256), 0, s, v, vt, Ns, p.ldt);
  hipLaunchKernelGGL((attn_f32_kernel<MHADA_ACT_SOFTMAX, 8, true>), dim3(p.nblk), dim3(512), 0, s, p);
  return check_launch("mhada_attn_train_fwd_vt");
}

// dst [BH][64][ldt] = src [BH][N][64] transposed per problem, columns N .. ldt - 1 zero: K^T for the
// training backward's dQ = dS K GEMM (replaces aten's strided k.transpose(1, 2).contiguous()).
extern "C" int mhada_transpose64(const float* src, float* dst, int BH, int N, int ldt, mhada_stream_t s_) {
  if (!src || !dst || BH <= 0 || N <= 0 || ldt < N || ldt % 64) return fail("mhada_transpose64: bad args (ldt % 64 == 0, >= N)");
  if (BH > 65535) return fail("mhada_transpose64: BH > 65535");
  hipLaunchKernelGGL(train_vt_kernel<false>, dim3(ldt / 64, BH), dim3(256), 0, (hipStream_t)s_, src, dst, N, ldt);
  return check_launch("mhada_transpose64");
}
