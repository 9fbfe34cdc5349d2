// Shared pieces of the MHAda attention kernels (attn.hip).
#pragma once
#include "common.h"

namespace mhada {

// Softmax scores arrive in log2 units: the engine folds log2(e) into K (mhada_fold_block).
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
  int prio;                    // fs kernel: s_setprio(1) for the younger wave half (MHADA_ATTN_PRIO)
  // training forward (attn_f32_kernel<.., TRAIN = true>, mhada_attn_train_fwd_vt): K rows of ldk
  // floats (64: the training k [BH][Ns][64]; inference reads K from kv rows of 128), Q unscaled
  // (log2 e applied on load), x = InstanceNorm(fcs) [BH][Nc][64]; writes out', [M' | E2'], lse2
  int ldk;
  float* mo;
  float* lse;
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

MHADA_DEV void decode_block(const AttnP& p, int& b, int& hh, int& qb) {
  const int t = xcd_remap(blockIdx.x, p.nblk);
  qb = t % p.nqb;
  const int bh = t / p.nqb;
  b = bh / p.H;
  hh = bh - b * p.H;
}

// Fixed-shift softmax (attn_bf16_fs_kernel): P = exp2(s - m2) with m2 the
// max of the query's first key block, never updated; the row sum l exceeds this bound iff some
// P exceeded 2^64 (|V'|^2 < 2^60 keeps O finite below it).
constexpr float kShiftSumThr = 18446744073709551616.0f;  // 2^64

// Exact two-pass recompute of one 32-query half for one wave (the rare path of the fixed-shift
// kernels when l trips kShiftSumThr): a QK^T pass for the true row max, then the full pass;
// K rows and V'^T columns are read straight from global memory (L2).
MHADA_DEV void attn_exact_half(const AttnP& p, const bf16* kvb, const bf16* vtb, const bf16x8 (&qf)[4],
                              f32x16 (&O)[4], float& l, int h, int r32) {
  const int Ns = p.Ns;
  const f32x16 zero = {};
  auto scores = [&](int key0) {
    f32x16 S = zero;
    const int key = min(key0 + r32, Ns - 1);
    const bf16* kr = kvb + (long long)key * 128 + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(kr + 16 * s), qf[s], S, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (key0 + (r & 3) + 8 * (r >> 2) + 4 * h >= Ns) S[r] = -INFINITY;
    return S;
  };
  float mx = -INFINITY;
  for (int k0 = 0; k0 < Ns; k0 += 32) {
    const f32x16 S = scores(k0);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[r]);
  }
  const float m2 = fmaxf(mx, __shfl_xor(mx, 32, 64));
#pragma unroll
  for (int i = 0; i < 4; ++i) O[i] = zero;
  l = 0.f;
  for (int k0 = 0; k0 < Ns; k0 += 32) {
    const f32x16 S = scores(k0);
    bf16x8 pf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = fast_exp2(S[8 * s + j] - m2);
        l += e;
        pf[s][j] = (bf16)e;
      }
    const bf16* vc = vtb + (long long)r32 * p.ldt + k0 + 8 * h;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int blk = 0; blk < 4; ++blk)
        O[blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            *reinterpret_cast<const bf16x8*>(vc + 16 * s + 32 * blk * (long long)p.ldt), pf[s], O[blk], 0, 0, 0);
  }
}


// --------------------------------------------------------------------------------------
// LDS-DMA (global_load_lds, 16 B per lane) for the K / V'^T rings of the LDS-DMA kernels.
// --------------------------------------------------------------------------------------
MHADA_DEV void attn_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Key of score row r (0..15) of tile t (0, 1) in a 32-key group of the 16x16x32 attention layout
// (attn_bf16_fsq_kernel, attn_s3_kernel): lane group g then holds the 8 keys its PV B slots need.
MHADA_DEV int fsq_key(int r, int t) { return 16 * (r >> 3) + 4 * ((r >> 2) & 1) + (r & 3) + 8 * t; }

// Epilogue of the 16x16x32 layout: O[qg][dvb] holds O^T[dv][q] for q = q0 + 16 qg + r16,
// dv = 16 dvb + 4g + e (dvb 0-3: sum p v', 4-7: sum p v'^2); lt = the full row sums.
template <typename T>
MHADA_DEV void attn_epilogue_q(const AttnP& p, const f32x4 (&O)[2][8], const float (&lt)[2], int b, int hh, int q0,
                               int g, int r16) {
  const int C = p.H * 64;
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + 16 * qg + r16;
    if (q >= p.Nc) continue;
    const float inv = 1.0f / lt[qg];
    const float* fr = p.fcs + ((long long)b * p.Nc + q) * C + hh * 64;
    const float* mu = p.fcs_mu + (long long)b * C + hh * 64;
    const float* rs = p.fcs_rstd + (long long)b * C + hh * 64;
    const float* vm = p.v_mu + (long long)b * C + hh * 64;
    T* orow = reinterpret_cast<T*>(p.out) + ((long long)b * p.Nc + q) * C + hh * 64;
#pragma unroll
    for (int dvb = 0; dvb < 4; ++dvb) {
      const int dv0 = 16 * dvb + 4 * g;
      const f32x4 f = *reinterpret_cast<const f32x4*>(fr + dv0);
      const f32x4 m4 = *reinterpret_cast<const f32x4*>(mu + dv0);
      const f32x4 r4 = *reinterpret_cast<const f32x4*>(rs + dv0);
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(vm + dv0);
      float res[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[qg][dvb][e] * inv;
        const float e2 = O[qg][dvb + 4][e] * inv;
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

}  // namespace mhada
