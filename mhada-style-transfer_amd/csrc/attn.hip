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
// Online softmax with a deferred rescale (cdna_hip_programming.md T13): the running max m
// only moves when a tile's max exceeds it by more than kRescaleThr (log2 units), so after the
// first tiles the O accumulators are touched by VALU only in a rare branch; P <= 2^kRescaleThr.
// Only the last, partial key tile runs the masking code.
// fp32: v_mfma_f32_32x32x2_f32 (exact fp32), K/V' streamed from kv[.][128] into LDS, V'^2
//       formed in registers.  bf16: v_mfma_f32_32x32x16_bf16, V'^T and V'^2^T streamed from
//       the pre-transposed, key-permuted vt image (mhada_transpose_v) so every operand read
//       is one 16-byte ds_read; fp32 accumulation and softmax.
// Block = NW waves = 32*NW queries of one (batch, head); blocks of one (b, h) are remapped
// onto one XCD so they share K/V in its L2.
#include "common.h"

#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

namespace mhada {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kRescaleThr = 32.0f;  // log2 units: P <= 2^32, sums stay far below fp32 overflow

struct AttnP {
  const void* q;    // [B][H][Nc][64]
  const void* kv;   // [B][H][Ns][128]
  const void* vt;   // bf16: [B][H][128][ldt], keys permuted within groups of 16
  const float* fcs; // [B][Nc][C]
  const float* fcs_mu;
  const float* fcs_rstd;
  const float* v_mu;
  void* out;        // [B][Nc][C]
  int B, H, Nc, Ns, ldt, nqb, nblk;
  unsigned long long* stamps;  // diagnostics only (MHADA_ATTN_STAMPS): s_memtime per barrier
  int dbg;                     // diagnostics only (MHADA_ATTN_DBG): 1 = no LDS-DMA in the loop
};

MHADA_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Epilogue shared by both variants.  O[blk] holds O^T[dv][q] for dv = (r&3)+8(r>>2)+4h+32(blk&1);
// blk 0,1: sum p v'   blk 2,3: sum p v'^2.
template <typename T>
MHADA_DEV void attn_epilogue(const AttnP& p, const f32x16 (&O)[4], float l, int b, int hh, int q, int h) {
  const int C = p.H * 64;
  const float lt = l + __shfl_xor(l, 32, 64);
  if (q >= p.Nc) return;
  const float inv = 1.0f / lt;
  const float* fr = p.fcs + ((long long)b * p.Nc + q) * C + hh * 64;
  const float* mu = p.fcs_mu + (long long)b * C + hh * 64;
  const float* rs = p.fcs_rstd + (long long)b * C + hh * 64;
  const float* vm = p.v_mu + (long long)b * C + hh * 64;
  T* orow = reinterpret_cast<T*>(p.out) + ((long long)b * p.Nc + q) * C + hh * 64;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // 4 contiguous dv per group
      const int dv0 = 8 * g + 4 * h + 32 * blk;
      const f32x4 f = *reinterpret_cast<const f32x4*>(fr + dv0);
      const f32x4 m4 = *reinterpret_cast<const f32x4*>(mu + dv0);
      const f32x4 r4 = *reinterpret_cast<const f32x4*>(rs + dv0);
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(vm + dv0);
      float res[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[blk][4 * g + e] * inv;
        const float e2 = O[blk + 2][4 * g + e] * inv;
        const float sd = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f));
        res[e] = sd * ((f[e] - m4[e]) * r4[e]) + (m1 + v4[e]);
      }
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(orow + dv0) = f32x4{res[0], res[1], res[2], res[3]};
      } else {
        *reinterpret_cast<bf16x4*>(orow + dv0) = bf16x4{(bf16)res[0], (bf16)res[1], (bf16)res[2], (bf16)res[3]};
      }
    }
  }
}

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
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * kLog2e;
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
        const float pv = fast_exp2(fmaf(S[kb][r], kLog2e, -m2));
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
  return fmaxf(mx, __shfl_xor(mx, 32, 64)) * kLog2e;
}

// S -> P against the current running max (no rescale); accumulates the row sum.
template <int ACT, int NKB>
MHADA_DEV void softmax_apply(f32x16 (&S)[NKB], float m2, float& l) {
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = (ACT == MHADA_ACT_SOFTMAX) ? fast_exp2(fmaf(S[kb][r], kLog2e, -m2)) : S[kb][r] + 1.0f;
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

MHADA_DEV void decode_block(const AttnP& p, int& b, int& hh, int& qb) {
  const int t = xcd_remap(blockIdx.x, p.nblk);
  qb = t % p.nqb;
  const int bh = t / p.nqb;
  b = bh / p.H;
  hh = bh - b * p.H;
}

// ======================================================================================
// fp32 variant
// ======================================================================================
template <int ACT, int NW>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) attn_f32_kernel(const AttnP p) {
  constexpr int NT = 64 * NW;
  constexpr int LS = 132;  // LDS row (128 + 4 floats): conflict-free b128 K reads, b32 V reads
  constexpr int CH = 2048 / NT;  // 16-B chunks per thread per tile (64 keys x 128 floats)
  __shared__ __attribute__((aligned(16))) float sKV[2][64 * LS];
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * (32 * NW) + wave * 32 + r32;
  const long long bh = (long long)b * p.H + hh;

  // Q^T operand: MFMA step s takes d = 32h + s
  float qreg[32];
  {
    const float* qp = reinterpret_cast<const float*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 32 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(qp + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) qreg[4 * i + e] = (q < p.Nc) ? t[e] : 0.f;
    }
  }
  const float* kvb = reinterpret_cast<const float*>(p.kv) + bh * p.Ns * 128;

  f32x4 stg[CH];
  auto issue = [&](int key0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + NT * i, row = c >> 5, col = (c & 31) * 4;
      const int key = key0 + row;
      stg[i] = key < p.Ns ? *reinterpret_cast<const f32x4*>(kvb + (long long)key * 128 + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto commit = [&](float* dst) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = tid + NT * i, row = c >> 5, col = (c & 31) * 4;
      *reinterpret_cast<f32x4*>(dst + row * LS + col) = stg[i];
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
      const float* krow = cur + (kb * 32 + r32) * LS + 32 * h;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x4 kk = *reinterpret_cast<const f32x4*>(krow + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          S[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk[e], qreg[4 * i + e], S[kb], 0, 0, 0);
      }
    }
  };
  auto pv = [&](const float* cur, const f32x16 (&P)[2]) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float* vrow = cur + key * LS + 64;
        const float v0 = vrow[r32], v1 = vrow[32 + r32];
        const float pr = P[kb][r];
        O[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, pr, O[0], 0, 0, 0);
        O[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, pr, O[1], 0, 0, 0);
        O[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0 * v0, pr, O[2], 0, 0, 0);
        O[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1 * v1, pr, O[3], 0, 0, 0);
      }
    }
  };

  const int NTILE = (p.Ns + 63) / 64, NFULL = p.Ns / 64;
  issue(0);
  commit(sKV[0]);
  __syncthreads();
  // Full tiles.  The rescale (P <= 2^kRescaleThr, so after the first tile it is rare) is a
  // wave-uniform branch inside the single loop: one register assignment for the O accumulators
  // (a leave-rescale-reenter loop made the compiler copy all of O between two register sets on
  // every iteration).
  for (int t = 0; t < NFULL; ++t) {
    const float* cur = sKV[t & 1];
    const bool nxt = t + 1 < NTILE;
    if (nxt) issue((t + 1) * 64);
    f32x16 S[2];
    qk(cur, S);
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
    pv(cur, S);
    if (nxt) commit(sKV[(t + 1) & 1]);
    __syncthreads();
  }
  if (NFULL < NTILE) {  // ragged last tile: masked, full online-softmax update
    const float* cur = sKV[NFULL & 1];
    f32x16 S[2];
    qk(cur, S);
    mask_tile<ACT, 2>(S, NFULL * 64, p.Ns, h);
    float alpha;
    if (softmax_tile<ACT, 2>(S, m2, l, alpha)) scale_acc(O, alpha);
    pv(cur, S);
  }
  attn_epilogue<float>(p, O, l, b, hh, q, h);
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
// bf16 ping-pong variant.  The plain kernel's per-tile __syncthreads keeps the two waves of a
// SIMD in the same phase — both issue QK^T, then both run the softmax (matrix pipe idle), then
// both issue PV (PMC: 42 % of wave time parked at waitcnt/barrier, MFMA busy 44 %).  Here each
// wave software-pipelines one tile: an MFMA segment {QK^T(u), PV(u-1)} and a VALU segment
// {softmax(u) -> P(u)}, separated by s_barrier, and waves 4-7 (group B) run one barrier behind
// waves 0-3 (group A), so on every SIMD one wave's MFMA segment pairs with the other wave's
// VALU segment (cdna_hip_programming.md T15/T16 in ping-pong form).
// K/V tiles arrive by LDS-DMA (global_load_lds, 16 B per lane) into 2-slot rings of unpadded
// 128-B rows, chunk slot = chunk ^ ((row >> 1) & 7) (applied on the source address; conflict-free
// 32x32x16 operand reads).  Each group moves its own half of every tile (A: K rows 0-31 and
// V'^T rows 0-63, B: the rest).  With A's segments at barrier intervals 2u (MFMA) / 2u+1 (VALU)
// and B's at 2u+1 / 2u+2:
//   A issues K(u+1), V(u) at the start of MFMA(u)  (slots last read in intervals 2u-2 / 2u-1),
//     waits vmcnt(0) at the end of VALU(u)         (first reader: A's MFMA(u+1), interval 2u+2);
//   B issues K(u+2), V(u+1) at the start of VALU(u) (slots last read in 2u / 2u+1),
//     waits vmcnt(0) at the end of MFMA(u+1)        (first reader: A's MFMA(u+2), interval 2u+4).
// Every LDS read retires (lgkmcnt(0)) before its segment's barrier; the DMAs stay in flight
// across one barrier (raw s_barrier: __syncthreads would drain them).
// Online-softmax rescale: decided in VALU(u) after PV(u-1) has been issued, so it scales O with
// every P at the old max included exactly once (T13's hazard), then P(u) uses the new max.
#define PPA_BARRIER()                                    \
  do {                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);                   \
    __builtin_amdgcn_s_barrier();                        \
    __builtin_amdgcn_sched_barrier(0);                   \
    asm volatile("" ::: "memory");                       \
  } while (0)

MHADA_DEV void attn_glds16(const void* src, bf16* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int ACT>
__global__ void __launch_bounds__(512) attn_bf16_pp_kernel(const AttnP p) {
  constexpr int KSZ = 64 * 64, VSZ = 128 * 64;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * KSZ + 2 * VSZ];  // the only LDS object
  bf16* const sK = smem;            // [2][64 keys][64 d]
  bf16* const sV = smem + 2 * KSZ;  // [2][128 dv][64 keys]
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wl = wave & 3;
  const int q = qb * 256 + wave * 32 + r32;
  const long long bh = (long long)b * p.H + hh;
  const int Ns = p.Ns, NTILE = (Ns + 63) / 64;

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

  // One LDS-DMA piece = 8 rows x 128 B; lane l fills row (l >> 3), slot (l & 7).
  auto k_piece = [&](int kt, int row0) {  // rows row0..row0+7 of K(kt); keys past Ns clamped
    const int row = row0 + (lane >> 3);  // (their scores are masked)
    const int key = min(kt * 64 + row, Ns - 1);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    attn_glds16(kvb + (long long)key * 128 + 8 * c, sK + (kt & 1) * KSZ + row0 * 64);
  };
  auto v_piece = [&](int vtile, int row0) {  // dv rows row0..row0+7 of the V'^T tile vtile
    const int row = row0 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    attn_glds16(vtb + (long long)row * p.ldt + vtile * 64 + 8 * c, sV + (vtile & 1) * VSZ + row0 * 64);
  };
  // this group's half of K(kt) (4 pieces) and V(vtile) (8 pieces): 3 pieces per wave
  auto dma = [&](int kt, int vtile) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int gi = wl * 3 + j;  // wave-uniform
      if (gi < 4) {
        if (kt < NTILE) k_piece(kt, 32 * grp + 8 * gi);
      } else {
        if (vtile < NTILE) v_piece(vtile, 64 * grp + 8 * (gi - 4));
      }
    }
  };

  f32x16 O[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] = 0.f;
  float m2 = -INFINITY, l = 0.f;
  f32x16 S[2];
  bf16x8 pf[2][2];

  // element offset of this lane's 16-B chunk 2j + h inside a swizzled row (rows r32 + 32k
  // share it); indexed only with compile-time j (a runtime index becomes a select chain)
  const int swz = (r32 >> 1) & 7;
  int koff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) koff[j] = 8 * ((2 * j + h) ^ swz);
  // diagnostics: lane 0 of each wave of the first block stamps s_memtime after its barriers
  int nst = 0;
  auto stamp = [&]() {
    if (p.stamps && blockIdx.x == 0 && lane == 0 && nst < 96) p.stamps[wave * 96 + nst] = __builtin_amdgcn_s_memtime();
    ++nst;
  };
  // MFMA segment body: all operand fragments are read in batches ahead of their MFMAs (with
  // one MFMA-issuing wave per SIMD nothing else hides a ds_read's latency).
  auto mfma_segment = [&](const bf16* ck, const bf16* cv, bool with_pv) {
    bf16x8 kf[2][4], vf[2][4];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        kf[kb][s2] = *reinterpret_cast<const bf16x8*>(ck + (kb * 32 + r32) * 64 + koff[s2]);
    if (with_pv) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
          vf[s2][blk] = *reinterpret_cast<const bf16x8*>(cv + (r32 + 32 * blk) * 64 + koff[s2]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every read ahead of the MFMAs (the scheduler sinks them)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) S[kb][e] = 0.f;
    // the two score chains alternate: a chain's next MFMA never waits on its previous result
    // (with one MFMA wave per SIMD nothing else fills that latency)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        S[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb][s2], qf[s2], S[kb], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA, in this order
      }
    if (p.stamps) { __builtin_amdgcn_sched_barrier(0); stamp(); __builtin_amdgcn_sched_barrier(0); }
    if (with_pv) {
      // the second key block's V fragments reuse the K fragments' registers (dead once the
      // QK^T MFMAs have issued) and are in flight while the first block's PV MFMAs run
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
          kf[s2][blk] = *reinterpret_cast<const bf16x8*>(cv + (r32 + 32 * blk) * 64 + koff[2 + s2]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
          O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[s2][blk], pf[0][s2], O[blk], 0, 0, 0);
      if (p.stamps) { __builtin_amdgcn_sched_barrier(0); stamp(); __builtin_amdgcn_sched_barrier(0); }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk)
          O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s2][blk], pf[1][s2], O[blk], 0, 0, 0);
    }
  };
  auto pv_only = [&](const bf16* cv) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
          const bf16x8 v8 = *reinterpret_cast<const bf16x8*>(cv + (r32 + 32 * blk) * 64 + koff[2 * kb + s2]);
          O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v8, pf[kb][s2], O[blk], 0, 0, 0);
        }
  };

  // prologue: K(0) whole (one piece per wave), group B's halves of K(1) and V(0)
  k_piece(0, 8 * wave);
  if (grp == 1) dma(1, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (grp == 1) PPA_BARRIER();  // group B runs one barrier behind

  stamp();
  auto tile = [&](int u, auto MASKC) {
    // ---- MFMA segment: QK^T(u), PV(u-1)
    if (grp == 0 && !(p.dbg & 1)) dma(u + 1, u);
    mfma_segment(sK + (u & 1) * KSZ, sV + ((u - 1) & 1) * VSZ, u > 0);
    if (p.stamps) { __builtin_amdgcn_sched_barrier(0); stamp(); __builtin_amdgcn_sched_barrier(0); }
    if (grp == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // B's DMA from VALU(u-1)
    PPA_BARRIER();
    stamp();
    // ---- VALU segment: softmax(u) -> P(u)
    if (grp == 1 && !(p.dbg & 1)) dma(u + 2, u + 1);
    if constexpr (decltype(MASKC)::value) mask_tile<ACT, 2>(S, u * 64, Ns, h);
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
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[kb][s2][j] = (bf16)S[kb][8 * s2 + j];
    if (p.stamps) { __builtin_amdgcn_sched_barrier(0); stamp(); __builtin_amdgcn_sched_barrier(0); }
    if (grp == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A's DMA from MFMA(u)
    PPA_BARRIER();
    stamp();
  };
  const int NFULL = Ns / 64;
  for (int u = 0; u < NFULL; ++u) tile(u, std::false_type{});
  if (NFULL < NTILE) tile(NFULL, std::true_type{});  // ragged last tile: key masks
  pv_only(sV + ((NTILE - 1) & 1) * VSZ);
  if (grp == 0) PPA_BARRIER();  // balance group B's extra barrier
  attn_epilogue<bf16>(p, O, l, b, hh, q, h);
}

// Opt-in (MHADA_ATTN_PP=1): measured 10-20 % slower than the plain 128-key kernel.
static bool attn_pp_enabled() {
  const char* e = getenv("MHADA_ATTN_PP");
  return e && e[0] == '1';
}

// Waves per workgroup (32 queries each).  Default per dtype; MHADA_ATTN_WAVES=4|8 overrides
// (read per call, for in-process A/B measurements).
static int attn_waves(int dtype) {
  const char* e = getenv("MHADA_ATTN_WAVES");
  if (e && (atoi(e) == 4 || atoi(e) == 8)) return atoi(e);
  return 8;
}

// Keys per bf16 tile (64 | 128): MHADA_ATTN_TK overrides the default (read per call).
static int attn_tk() {
  const char* e = getenv("MHADA_ATTN_TK");
  if (e && atoi(e) == 64) return 64;
  return 128;
}

template <int NW>
static void launch_attn(const AttnP& p, int dtype, int activation, hipStream_t s) {
  const dim3 grid(p.nblk), blk(64 * NW);
  if (dtype == MHADA_F32) {
    if (activation == MHADA_ACT_SOFTMAX)
      hipLaunchKernelGGL((attn_f32_kernel<MHADA_ACT_SOFTMAX, NW>), grid, blk, 0, s, p);
    else
      hipLaunchKernelGGL((attn_f32_kernel<MHADA_ACT_COSINE, NW>), grid, blk, 0, s, p);
  } else {
    if constexpr (NW == 8) {
      if (attn_pp_enabled()) {
        if (activation == MHADA_ACT_SOFTMAX)
          hipLaunchKernelGGL((attn_bf16_pp_kernel<MHADA_ACT_SOFTMAX>), grid, blk, 0, s, p);
        else
          hipLaunchKernelGGL((attn_bf16_pp_kernel<MHADA_ACT_COSINE>), grid, blk, 0, s, p);
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
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_attn(const void* q, const void* kv, const void* vt, const float* fcs, const float* fcs_mu,
                          const float* fcs_rstd, const float* v_mu, void* out, int dtype, int B, int H, int Nc,
                          int Ns, int activation, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!q || !kv || !fcs || !fcs_mu || !fcs_rstd || !v_mu || !out || B <= 0 || H <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn: bad args");
  if (dtype == MHADA_BF16 && !vt) return fail("mhada_attn: bf16 needs the transposed V image");
  if (activation != MHADA_ACT_SOFTMAX && activation != MHADA_ACT_COSINE) return fail("mhada_attn: bad activation");
  AttnP p;
  p.q = q; p.kv = kv; p.vt = vt; p.fcs = fcs; p.fcs_mu = fcs_mu; p.fcs_rstd = fcs_rstd; p.v_mu = v_mu;
  p.out = out; p.B = B; p.H = H; p.Nc = Nc; p.Ns = Ns;
  p.stamps = nullptr;
  p.dbg = getenv("MHADA_ATTN_DBG") ? atoi(getenv("MHADA_ATTN_DBG")) : 0;
  const bool stamps = getenv("MHADA_ATTN_STAMPS") != nullptr;
  if (stamps) {
    (void)hipMalloc((void**)&p.stamps, 8 * 96 * sizeof(unsigned long long));
    (void)hipMemsetAsync(p.stamps, 0, 8 * 96 * sizeof(unsigned long long), s);
  }
  p.ldt = (Ns + 63) / 64 * 64;
  const int nw = attn_waves(dtype);
  p.nqb = (Nc + 32 * nw - 1) / (32 * nw);
  const long long nblk = (long long)B * H * p.nqb;
  if (nblk > (1LL << 31) - 1) return fail("mhada_attn: grid too large");
  p.nblk = (int)nblk;
  if (nw == 8) {
    launch_attn<8>(p, dtype, activation, s);
  } else {
    launch_attn<4>(p, dtype, activation, s);
  }
  if (stamps) {  // diagnostics: per-wave cycles between consecutive barrier stamps of block 0
    unsigned long long h[8 * 96];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h, p.stamps, sizeof(h), hipMemcpyDeviceToHost);
    for (int w = 0; w < 8; ++w) {
      fprintf(stderr, "wave %d:", w);
      for (int k = 1; k < 96 && h[w * 96 + k]; ++k) fprintf(stderr, " %llu", h[w * 96 + k] - h[w * 96 + k - 1]);
      fprintf(stderr, "\n");
    }
    (void)hipFree(p.stamps);
  }
  return check_launch("mhada_attn");
}
