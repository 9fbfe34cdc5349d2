// Wide-head parameter-free AdaAttN for the local feature loss:
// AdaAttnForLoss.forward (MHAdaSTr/network/adaDecoder.py:52-81) called by local_feature_loss
// (lossfn.py:26-34) on VGG19 features: d_qk = 448 / 960 / 1472 (the channels of
// feature_down_sample, utilities.py:86-97), d_v = 256 / 512 / 512, N = (H/4)^2 .. (H/16)^2.
//
//   A = softmax(Q K^T) (no scale) or the cosine form, M = A V, E2 = A V^2,
//   S = sqrt(max(E2 - M^2, 1e-6)), out = S * InstanceNorm(c_x) + M
//
// Flash-style (A never in HBM), fp32 (v_mfma_f32_32x32x2_f32, exact fp32 products), the same
// swapped orientation as attn.hip (S^T = K Q^T so a lane owns one query; O^T = V^T P^T takes
// the S^T accumulator as its B operand with no lane movement).  One workgroup = 32 queries of
// one image; its W waves split the WORK, not the queries:
//   * the Q K^T reduction over d_qk: wave w owns d in [w*dsl, (w+1)*dsl) (its Q slice lives in
//     registers, its K slice streams from L2), and the W partial score tiles are summed through
//     LDS in a fixed order, so every wave holds the identical score tile;
//   * the P V / P V^2 products over d_v: wave w owns d_v columns [w*DVW, (w+1)*DVW).
// One barrier per 32-key tile (double-buffered partial-score slots).  The online softmax
// (log2 units, lazy rescale as attn.hip) is evaluated redundantly by every wave — its VALU
// cost is small next to the fp32 MFMAs.  Q and K arrive InstanceNorm-ed (mhada_rows_normalize).
#include "common.h"

namespace mhada {

struct LossAttnP {
  const float* q;      // [B][Nq][Dqk]  IN(c_1x)
  const float* k;      // [B][Ns][Dqk]  IN(s_1x)
  const float* v;      // [B][Ns][Dv]   s_x
  const float* x;      // [B][Nq][Dv]   c_x
  const float* x_mu;   // [B][Dv]
  const float* x_rs;   // [B][Dv]
  float* out;          // [B][Nq][Dv]
  int Nq, Ns, Dqk, Dv, dsl, nqb;
};

constexpr float kLossRescaleThr = 32.0f;  // log2 units, as attn.hip
constexpr float kLog2e = 1.4426950408889634f;

template <int ACT, int W, int DVW, int DH>
__global__ void __launch_bounds__(64 * W) loss_attn_kernel(const LossAttnP p) {
  constexpr int NB = DVW / 32;  // 32-column blocks of M (and of E2) per wave
  __shared__ __attribute__((aligned(16))) float sS[2][W][16][64];  // partial score tiles
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r32 = lane & 31;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int b = t / p.nqb, qb = t - b * p.nqb;
  const int q = qb * 32 + r32;
  const int qc = min(q, p.Nq - 1);
  // this wave's d range [wave*dsl, (wave+1)*dsl) in chunks of up to 2*DH: in chunk c, lane half h
  // takes d = base_c + h*dh_c + s (s < dh_c) at MFMA step s (Q and K agree, so any bijection works)
  const int nch = (p.dsl + 2 * DH - 1) / (2 * DH);
  const float* qrow = p.q + ((long long)b * p.Nq + qc) * p.Dqk;
  float qreg[DH];
  int dh = 0, dbase = 0;
  auto chunk = [&](int c) {
    const int len = min(2 * DH, p.dsl - c * 2 * DH);  // multiple of 8
    dh = __builtin_amdgcn_readfirstlane(len / 2);
    dbase = wave * p.dsl + c * 2 * DH + h * dh;
  };
  auto load_q = [&]() {
#pragma unroll
    for (int s = 0; s < DH; s += 4) {
      const f32x4 v4 = (s < dh && dbase + s < p.Dqk) ? *reinterpret_cast<const f32x4*>(qrow + dbase + s)
                                                     : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) qreg[s + e] = v4[e];
    }
  };
  if (nch == 1) {  // the common case: the Q slice stays in registers for the whole key loop
    chunk(0);
    load_q();
  }
  const float* kb = p.k + (long long)b * p.Ns * p.Dqk;
  const float* vb = p.v + (long long)b * p.Ns * p.Dv + wave * DVW;

  f32x16 O[2 * NB];
#pragma unroll
  for (int i = 0; i < 2 * NB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] = 0.f;
  float m2 = -INFINITY, l = 0.f;

  const int ntile = (p.Ns + 31) / 32;
  for (int tt = 0; tt < ntile; ++tt) {
    const int key0 = tt * 32;
    const int buf = tt & 1;
    // ---- partial S^T[key][q] over this wave's d slice
    f32x16 S;
#pragma unroll
    for (int e = 0; e < 16; ++e) S[e] = 0.f;
    {
      const int key = min(key0 + r32, p.Ns - 1);
      const float* kr = kb + (long long)key * p.Dqk;
      for (int c = 0; c < nch; ++c) {
        if (nch > 1) {  // wide slices (d_qk 1472): re-read the Q chunk (L2) per key tile
          chunk(c);
          load_q();
        }
#pragma unroll
        for (int s = 0; s < DH; s += 4) {
          if (s < dh) {  // wave-uniform
            const f32x4 k4 = dbase + s < p.Dqk ? *reinterpret_cast<const f32x4*>(kr + dbase + s)
                                               : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) S = __builtin_amdgcn_mfma_f32_32x32x2f32(k4[e], qreg[s + e], S, 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) sS[buf][wave][r][lane] = S[r];
    // V operands of this tile (issued before the barrier): key of step r = key0 + (r&3) + 8(r>>2) + 4h
    float vv[16][NB];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = min(key0 + (r & 3) + 8 * (r >> 2) + 4 * h, p.Ns - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) vv[r][j] = vb[(long long)key * p.Dv + 32 * j + r32];
    }
    __syncthreads();
    // ---- full scores: fixed-order sum of the W partial tiles (identical in every wave)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float a = sS[buf][0][r][lane];
#pragma unroll
      for (int w = 1; w < W; ++w) a += sS[buf][w][r][lane];
      S[r] = a;
    }
    // ---- softmax / cosine weights P (in place), online normaliser
    if constexpr (ACT == MHADA_ACT_SOFTMAX) {
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        S[r] *= kLog2e;
        if (key0 + 32 > p.Ns && key >= p.Ns) S[r] = -INFINITY;  // uniform test first: tail tile only
        mx = fmaxf(mx, S[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (mx > m2 + kLossRescaleThr || tt == 0) {  // per-lane (query) decision; O rows are per query
        const float mn = fmaxf(m2, mx);
        const float alpha = m2 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m2 - mn);
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 2 * NB; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) O[i][e] *= alpha;
        m2 = mn;
      }
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        S[r] = __builtin_amdgcn_exp2f(S[r] - m2);  // bare v_exp_f32 (no denormal range fix-up)
        sum += S[r];
      }
      l += sum;
    } else {
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // rows arrive unit-normalised: s = q.k/(|q||k|) + 1
        const int key = key0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        S[r] = key < p.Ns ? S[r] + 1.0f : 0.f;
        sum += S[r];
      }
      l += sum;
    }
    // ---- O^T[dv][q] += V^T P^T and (V^2)^T P^T over the 32 keys (MFMA step r: keys of reg r)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const float vx = vv[r][j];
        O[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vx, S[r], O[j], 0, 0, 0);
        O[NB + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vx * vx, S[r], O[NB + j], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: out[q][dv] = sqrt(max(E2 - M^2, 1e-6)) * (x - mu) * rs + M
  const float lt = l + __shfl_xor(l, 32, 64);
  if (q >= p.Nq) return;
  const float inv = 1.f / lt;
  const int dvb = wave * DVW;
  const float* xr = p.x + ((long long)b * p.Nq + q) * p.Dv + dvb;
  const float* mu = p.x_mu + (long long)b * p.Dv + dvb;
  const float* rs = p.x_rs + (long long)b * p.Dv + dvb;
  float* orow = p.out + ((long long)b * p.Nq + q) * p.Dv + dvb;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dv = 32 * j + 8 * g + 4 * h;
      const f32x4 xx = *reinterpret_cast<const f32x4*>(xr + dv);
      const f32x4 mm = *reinterpret_cast<const f32x4*>(mu + dv);
      const f32x4 rr = *reinterpret_cast<const f32x4*>(rs + dv);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[j][4 * g + e] * inv;
        const float e2 = O[NB + j][4 * g + e] * inv;
        o[e] = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f)) * ((xx[e] - mm[e]) * rr[e]) + m1;
      }
      *reinterpret_cast<f32x4*>(orow + dv) = o;
    }
}

// ---------------------------------------------------------------------------------------
// LDS-staged form for d_qk <= 448 with d_v = 256 (the relu3_1 level of the loss: d_qk 448,
// N = (H/4)^2 — 16384 tokens at 512^2, 90 % of the loss-attention time).  The kernel above reads
// K and V straight from L2 per lane (each wave instruction touches 32 key rows); here a workgroup
// of 8 waves = 2 query groups x the 4 d-slices shares one K / V tile staged through LDS by
// coalesced 16-B loads (whole 32-row tiles are contiguous in memory), issued a tile ahead into
// registers: half the L2 stream per query and none of the scattered row reads.  Per 32-key tile:
//   commit V(t) -> sV; issue loads of K(t+1), V(t+1); partial S^T from sK -> sS; barrier;
//   fixed-order sum of the 4 partials, softmax, P V / P V^2 from sV; commit K(t+1) -> sK; barrier
// (single-buffered sK / sV / sS: each buffer's last reader finishes before the barrier that
// precedes its next writer).  K rows padded to 4*dsl + 4 floats (= 4 mod 64 words: conflict-free
// ds_read_b128 down 32 rows), V rows to 260.
// ---------------------------------------------------------------------------------------
template <int ACT>
__global__ void __launch_bounds__(512) loss_attn_lds_kernel(const LossAttnP p) {
  constexpr int W = 4, DH = 56, NB = 2, VLD = 260;  // d slice <= 112 = 2 x DH
  constexpr int KLDMAX = 452;
  __shared__ __attribute__((aligned(16))) float sK[32 * KLDMAX];
  __shared__ __attribute__((aligned(16))) float sV[32 * VLD];
  __shared__ __attribute__((aligned(16))) float sS[2][W][16][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qg = wave >> 2, ws = wave & 3;
  const int h = lane >> 5, r32 = lane & 31;
  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  const int nqb = (p.Nq + 63) / 64;
  const int b = t0 / nqb, qb = t0 - b * nqb;
  const int q = qb * 64 + qg * 32 + r32;
  const int qc = min(q, p.Nq - 1);
  const int KLD = 4 * p.dsl + 4;
  const int dh = p.dsl / 2, dbase = ws * p.dsl + h * dh;
  float qreg[DH];
  {
    const float* qrow = p.q + ((long long)b * p.Nq + qc) * p.Dqk;
#pragma unroll
    for (int s = 0; s < DH; s += 4) {
      const f32x4 v4 = (s < dh && dbase + s < p.Dqk) ? *reinterpret_cast<const f32x4*>(qrow + dbase + s)
                                                     : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) qreg[s + e] = v4[e];
    }
  }
  // K columns [Dqk, 4 dsl) stay zero (never written by the tile commits)
  for (int i = tid; i < 32 * (KLD - p.Dqk); i += 512) {
    const int row = i / (KLD - p.Dqk), col = p.Dqk + i % (KLD - p.Dqk);
    sK[row * KLD + col] = 0.f;
  }
  const float* kb = p.k + (long long)b * p.Ns * p.Dqk;
  const float* vb = p.v + (long long)b * p.Ns * p.Dv;
  // tile staging: K tile = 32 rows x Dqk/4 16-B chunks, V tile = 32 x 64 chunks.  Loads through
  // buffer resources built per tile over the key rows key0 .. Ns - 1 (scalar work): every lane's
  // offset (and LDS destination) is a loop constant, so a tile's 11 loads cost no vector address
  // arithmetic (an fp32 MFMA holds the SIMD's vector issue for its whole 64 cycles,
  // profiles/r05_f32mfma_fill.log).  Rows past Ns read 0: their scores are masked, their P is 0.
  const int kcr = p.Dqk / 4, kch = 32 * kcr;
  constexpr int KR = (32 * 112 + 511) / 512;  // <= 7 chunks per thread (d_qk <= 448)
  f32x4 rk[KR], rv[4];
  int kvo[KR], klo[KR];
#pragma unroll
  for (int i = 0; i < KR; ++i) {
    const int c = min(tid + 512 * i, kch - 1), row = c / kcr, col = c - row * kcr;
    kvo[i] = (row * p.Dqk + 4 * col) * 4;
    klo[i] = (row * KLD + 4 * col) & 0xffff;
  }
  auto issue = [&](int key0) {
    const int left = max(p.Ns - key0, 0);
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(kb + (long long)min(key0, p.Ns) * p.Dqk), 0, left * p.Dqk * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(vb + (long long)min(key0, p.Ns) * p.Dv), 0, left * p.Dv * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < KR; ++i)
      rk[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(kr, kvo[i], 0, 0));
#pragma unroll
    for (int i = 0; i < 4; ++i)
      rv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vr, (tid + 512 * i) * 16, 0, 0));
  };
  auto commit_k = [&]() {
#pragma unroll
    for (int i = 0; i < KR; ++i) *reinterpret_cast<f32x4*>(sK + klo[i]) = rk[i];
  };
  auto commit_v = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 512 * i, row = c >> 6, col = c & 63;
      *reinterpret_cast<f32x4*>(sV + row * VLD + 4 * col) = rv[i];
    }
  };

  f32x16 O[2 * NB];
#pragma unroll
  for (int i = 0; i < 2 * NB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) O[i][e] = 0.f;
  float m2 = -INFINITY, l = 0.f;

  const int ntile = (p.Ns + 31) / 32;
  issue(0);
  commit_k();
  __syncthreads();
  for (int tt = 0; tt < ntile; ++tt) {
    const int key0 = tt * 32;
    commit_v();  // V(tt): sV's readers (P V of tile tt-1) passed the last barrier
    issue(min(tt + 1, ntile - 1) * 32);
    // ---- partial S^T[key][q] over this wave's d slice, K from LDS
    f32x16 S;
#pragma unroll
    for (int e = 0; e < 16; ++e) S[e] = 0.f;
    {
      const float* kr = sK + r32 * KLD + dbase;
#pragma unroll
      for (int s = 0; s < DH; s += 4) {
        if (s < dh) {  // wave-uniform
          const f32x4 k4 = *reinterpret_cast<const f32x4*>(kr + s);
#pragma unroll
          for (int e = 0; e < 4; ++e) S = __builtin_amdgcn_mfma_f32_32x32x2f32(k4[e], qreg[s + e], S, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) sS[qg][ws][r][lane] = S[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float a = sS[qg][0][r][lane];
#pragma unroll
      for (int w = 1; w < W; ++w) a += sS[qg][w][r][lane];
      S[r] = a;
    }
    if constexpr (ACT == MHADA_ACT_SOFTMAX) {
      // the tile max on the raw scores, then P = exp2(s log2 e - m2) as one fma per score (the
      // scale is monotonic, so the max commutes with it)
      if (key0 + 32 > p.Ns) {  // uniform: tail tile only
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (key0 + (r & 3) + 8 * (r >> 2) + 4 * h >= p.Ns) S[r] = -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * kLog2e;
      if (mx > m2 + kLossRescaleThr || tt == 0) {
        const float mn = fmaxf(m2, mx);
        const float alpha = m2 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m2 - mn);
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 2 * NB; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) O[i][e] *= alpha;
        m2 = mn;
      }
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        S[r] = __builtin_amdgcn_exp2f(fmaf(S[r], kLog2e, -m2));  // bare v_exp_f32 (no denormal range fix-up)
        sum += S[r];
      }
      l += sum;
    } else {
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        S[r] = key < p.Ns ? S[r] + 1.0f : 0.f;
        sum += S[r];
      }
      l += sum;
    }
    // ---- O^T[dv][q] += V^T P^T and (V^2)^T P^T, V from LDS
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* vr = sV + ((r & 3) + 8 * (r >> 2) + 4 * h) * VLD + ws * 64 + r32;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const float vx = vr[32 * j];
        O[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vx, S[r], O[j], 0, 0, 0);
        O[NB + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vx * vx, S[r], O[NB + j], 0, 0, 0);
      }
    }
    commit_k();  // K(tt+1): every wave's S^T reads of sK ended before the barrier above
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  if (q >= p.Nq) return;
  const float inv = 1.f / lt;
  const int dvb = ws * 64;
  const float* xr = p.x + ((long long)b * p.Nq + q) * p.Dv + dvb;
  const float* mu = p.x_mu + (long long)b * p.Dv + dvb;
  const float* rs = p.x_rs + (long long)b * p.Dv + dvb;
  float* orow = p.out + ((long long)b * p.Nq + q) * p.Dv + dvb;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dv = 32 * j + 8 * g + 4 * h;
      const f32x4 xx = *reinterpret_cast<const f32x4*>(xr + dv);
      const f32x4 mm = *reinterpret_cast<const f32x4*>(mu + dv);
      const f32x4 rr = *reinterpret_cast<const f32x4*>(rs + dv);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[j][4 * g + e] * inv;
        const float e2 = O[NB + j][4 * g + e] * inv;
        o[e] = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f)) * ((xx[e] - mm[e]) * rr[e]) + m1;
      }
      *reinterpret_cast<f32x4*>(orow + dv) = o;
    }
}

// InstanceNorm applied to token rows: out[b][n][c] = (x - mu[b][c]) * rs[b][c]; with unit != 0
// each normalised row is further divided by its L2 norm (the cosine activation's q/|q|, k/|k|:
// adaDecoder.py:30-32).  One wave per row.
__global__ void __launch_bounds__(256) rows_normalize_kernel(const float* __restrict__ x, const float* __restrict__ mu,
                                                             const float* __restrict__ rs, float* __restrict__ out,
                                                             int unit, int B, int N, int C) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= (long long)B * N) return;
  const long long b = row / N;
  const float* xr = x + row * C;
  float* orow = out + row * C;
  float ss = 0.f;
  for (int c = 4 * lane; c < C; c += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
    const f32x4 m = *reinterpret_cast<const f32x4*>(mu + b * C + c);
    const f32x4 r = *reinterpret_cast<const f32x4*>(rs + b * C + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = (v[e] - m[e]) * r[e];
      ss += o[e] * o[e];
    }
    *reinterpret_cast<f32x4*>(orow + c) = o;
  }
  if (unit) {
    ss = wave_sum(ss);
    const float inv = 1.0f / sqrtf(ss);
    for (int c = 4 * lane; c < C; c += 256) {  // this lane's own stores: no barrier needed
      f32x4 o = *reinterpret_cast<const f32x4*>(orow + c);
      o *= inv;
      *reinterpret_cast<f32x4*>(orow + c) = o;
    }
  }
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_rows_normalize(const float* x, const float* mu, const float* rs, float* out, int unit, int B,
                                    int N, int C, mhada_stream_t s_) {
  if (!x || !mu || !rs || !out || B <= 0 || N <= 0 || C <= 0 || C % 4) return fail("mhada_rows_normalize: bad args");
  const long long rows = (long long)B * N;
  hipLaunchKernelGGL(rows_normalize_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)s_, x, mu, rs,
                     out, unit, B, N, C);
  return check_launch("mhada_rows_normalize");
}

extern "C" int mhada_loss_attn(const float* q, const float* k, const float* v, const float* x, const float* x_mu,
                               const float* x_rs, float* out, int B, int Nq, int Ns, int Dqk, int Dv, int activation,
                               mhada_stream_t s_) {
  if (!q || !k || !v || !x || !x_mu || !x_rs || !out || B <= 0 || Nq <= 0 || Ns <= 0 || Dqk <= 0 || Dv <= 0)
    return fail("mhada_loss_attn: bad args");
  if (activation != MHADA_ACT_SOFTMAX && activation != MHADA_ACT_COSINE) return fail("mhada_loss_attn: bad activation");
  if (Dqk % 4) return fail("mhada_loss_attn: d_qk % 4 == 0");
  LossAttnP p;
  p.q = q; p.k = k; p.v = v; p.x = x; p.x_mu = x_mu; p.x_rs = x_rs; p.out = out;
  p.Nq = Nq; p.Ns = Ns; p.Dqk = Dqk; p.Dv = Dv;
  p.nqb = (Nq + 31) / 32;
  const long long nblk = (long long)B * p.nqb;
  if (nblk >= (1LL << 31)) return fail("mhada_loss_attn: grid too large");
  const hipStream_t s = (hipStream_t)s_;
  // work split: d_v in 64-column slices, one per wave (W <= 8: 256 registers per lane); the d_qk
  // reduction split evenly over the W waves in slices of a multiple of 8 (each lane half then
  // loads whole float4s), processed in chunks of up to 128 per wave
  if (Dv % 64 || Dv / 64 > 8) return fail("mhada_loss_attn: d_v must be 64, 128, 256 or 512 (x 64 <= 8)");
  const int W = Dv / 64;
  if (W & (W - 1)) return fail("mhada_loss_attn: d_v / 64 must be 1, 2, 4 or 8");
  p.dsl = (Dqk + W * 8 - 1) / (W * 8) * 8;
  if (W == 4 && p.dsl <= 112) {  // d_v 256, d_qk <= 448: the LDS-staged form, 64 queries per workgroup
    const long long nb64 = (long long)B * ((Nq + 63) / 64);
    if (activation == MHADA_ACT_SOFTMAX)
      hipLaunchKernelGGL(loss_attn_lds_kernel<MHADA_ACT_SOFTMAX>, dim3((unsigned)nb64), dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL(loss_attn_lds_kernel<MHADA_ACT_COSINE>, dim3((unsigned)nb64), dim3(512), 0, s, p);
    return check_launch("mhada_loss_attn");
  }
  const dim3 grid((unsigned)nblk);
#define LA(ACT, WW) hipLaunchKernelGGL((loss_attn_kernel<ACT, WW, 64, 64>), grid, dim3(64 * WW), 0, s, p)
  if (activation == MHADA_ACT_SOFTMAX) {
    if (W == 1) LA(MHADA_ACT_SOFTMAX, 1); else if (W == 2) LA(MHADA_ACT_SOFTMAX, 2);
    else if (W == 4) LA(MHADA_ACT_SOFTMAX, 4); else LA(MHADA_ACT_SOFTMAX, 8);
  } else {
    if (W == 1) LA(MHADA_ACT_COSINE, 1); else if (W == 2) LA(MHADA_ACT_COSINE, 2);
    else if (W == 4) LA(MHADA_ACT_COSINE, 4); else LA(MHADA_ACT_COSINE, 8);
  }
#undef LA
  return check_launch("mhada_loss_attn");
}
