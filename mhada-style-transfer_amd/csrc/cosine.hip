// Cosine activation of the MHAda attention in its linear form (adaDecoder.py:20-34, used by
// AdaAttnMultiHead with activation="cosine", adaDecoder.py:164-168,186-191).
//
// With unit rows q^ (Q) and k^ (K) the reference's A[i][j] = (q^_i . k^_j + 1) / l_i, where
// l_i = sum_j (q^_i . k^_j + 1) = q^_i . sum_j k^_j + Ns.  So
//   M'  = A V'   = (q^_i (K^T V')   + sum_j v'_j)   / l_i
//   E2' = A V'^2 = (q^_i (K^T V'^2) + sum_j v'^2_j) / l_i
// and the Nc x Ns matrix never needs forming: a style-side reduction over the keys (64 x 128
// moments + column sums, once per style — cached with the style by the video path) and a
// query-side 64 x 129 product per (query, head) with mhada_attn's epilogue.  O(N d^2) instead of
// the flash loop's O(Nc Ns d).  V' is the centred V of mhada_attn (v_mu added back to M), read
// from its V'^T | V'^2^T image vt (mhada_transpose_v / the K|V' GEMM's vt epilogue), so the
// E2' - M'^2 cancellation is the flash kernel's.
//
// Moment image mom [BH][65][132] fp32 (row stride 132: the query kernel's LDS image):
//   mom[d][o]   = sum_n k^[n][d] vt[o][n]    d < 64, o < 128 (V' for o < 64, V'^2 for o >= 64)
//   mom[d][128] = sum_n k^[n][d]             (the l_i term)
//   mom[64][o]  = sum_n vt[o][n]             o < 128
//   mom[64][128] = Ns; every other column 0.
#include "common.h"

namespace mhada {
namespace {

constexpr int kMomRows = 65, kMomLd = 132, kMomSize = kMomRows * kMomLd;

// bf16 vt stores key n at column pos(n) (bits 2 and 3 swapped, mhada_transpose_v); fp32 in order.
template <typename T>
MHADA_DEV int vt_key(int p) {
  if constexpr (sizeof(T) == 2) return (p & ~12) | ((p & 4) << 1) | ((p & 8) >> 1);
  return p;
}

// One (split, bh) per workgroup: keys [split * cps, min(Ns, (split + 1) * cps)) in 64-key tiles.
// Thread (og, dg) = (t >> 4, t & 15) accumulates mom[4dg .. 4dg+3][8og .. 8og+7]; threads < 64 also
// sum k^ column t, threads 64 .. 191 the vt row t - 64.  Writes the split's full [65][132] partial.
template <typename T>
__global__ void __launch_bounds__(256) cosine_mom_kernel(const T* __restrict__ kv, const T* __restrict__ vt,
                                                         float* __restrict__ part, int Ns, int ldt, int cps,
                                                         int splits) {
  __shared__ float ks[64][64];        // [key][d]
  __shared__ float vs[64][128 + 4];   // [key][o]
  const int t = threadIdx.x;
  const int split = blockIdx.x, bh = blockIdx.y;
  const int n_begin = split * cps, n_end = min(Ns, n_begin + cps);
  const int og = t >> 4, dg = t & 15;
  const T* kb = kv + (long long)bh * Ns * 128;
  const T* vb = vt + (long long)bh * 128 * ldt;
  float acc[4][8] = {};
  float ssum = 0.f;
  for (int n0 = n_begin; n0 < n_end; n0 += 64) {
    // K^ tile: 64 keys x 64 d, 16 consecutive elements per thread (zero past Ns)
    {
      const int key = t >> 2, d0 = (t & 3) * 16;
      const int n = n0 + key;
#pragma unroll
      for (int e = 0; e < 16; ++e) ks[key][d0 + e] = n < n_end ? to_f32<T>(kb[(long long)n * 128 + d0 + e]) : 0.f;
    }
    // vt tile: 128 rows x 64 key columns (ldt is a multiple of 64 and vt is zero padded)
    {
      const int o = t >> 1, p0 = (t & 1) * 32;
      const T* vr = vb + (long long)o * ldt + n0;
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const int p = p0 + e;
        // columns of the last tile past this split's end belong to no key of this split
        vs[vt_key<T>(p)][o] = n0 + vt_key<T>(p) < n_end ? to_f32<T>(vr[p]) : 0.f;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < 64; ++k) {
      const f32x4 kd = *reinterpret_cast<const f32x4*>(&ks[k][4 * dg]);
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(&vs[k][8 * og]);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(&vs[k][8 * og + 4]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = fmaf(kd[i], v0[j], acc[i][j]);
          acc[i][4 + j] = fmaf(kd[i], v1[j], acc[i][4 + j]);
        }
      }
    }
    if (t < 64) {
      for (int k = 0; k < 64; ++k) ssum += ks[k][t];
    } else if (t < 192) {
      for (int k = 0; k < 64; ++k) ssum += vs[k][t - 64];
    }
    __syncthreads();
  }
  float* dst = part + ((long long)bh * splits + split) * kMomSize;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* r = dst + (4 * dg + i) * kMomLd + 8 * og;
    *reinterpret_cast<f32x4*>(r) = f32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
    *reinterpret_cast<f32x4*>(r + 4) = f32x4{acc[i][4], acc[i][5], acc[i][6], acc[i][7]};
  }
  if (t < 64) {
    float* r = dst + t * kMomLd + 128;
    *reinterpret_cast<f32x4*>(r) = f32x4{ssum, 0.f, 0.f, 0.f};
  } else if (t < 192) {
    dst[64 * kMomLd + t - 64] = ssum;
  } else if (t == 192) {
    *reinterpret_cast<f32x4*>(dst + 64 * kMomLd + 128) = f32x4{(float)max(0, n_end - n_begin), 0.f, 0.f, 0.f};
  }
}

// Fixed-order sum of the splits' partials (deterministic): mom[bh] = sum_s part[bh][s].
__global__ void __launch_bounds__(256) cosine_mom_finish_kernel(const float* __restrict__ part,
                                                                float* __restrict__ mom, int splits) {
  const int bh = blockIdx.x;
  const float* src = part + (long long)bh * splits * kMomSize;
  for (int i = threadIdx.x; i < kMomSize; i += 256) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += src[(long long)k * kMomSize + i];
    mom[(long long)bh * kMomSize + i] = s;
  }
}

// 64 queries of one (b, h) per workgroup; thread (qg, cg) = (t >> 4, t & 15) owns queries
// 4qg .. 4qg+3 x channels 4cg .. 4cg+3 (M' and E2' of the same channel in the same thread, for the
// variance).  mhada_attn's epilogue: out = sqrt(max(E2' - M'^2, 1e-6)) * IN(fcs) + (M' + v_mu).
template <typename T>
__global__ void __launch_bounds__(256) cosine_attn_kernel(const T* __restrict__ q, const float* __restrict__ mom,
                                                          const float* __restrict__ fcs,
                                                          const float* __restrict__ fcs_mu,
                                                          const float* __restrict__ fcs_rstd,
                                                          const float* __restrict__ v_mu, T* __restrict__ out,
                                                          int H, int Nc) {
  __shared__ float ms[kMomSize];
  __shared__ float qs[64][64 + 4];  // [d][query]
  const int t = threadIdx.x;
  const int q0 = blockIdx.x * 64, h = blockIdx.y, b = blockIdx.z;
  const long long bh = (long long)b * H + h;
  const int C = 64 * H;
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(mom + bh * kMomSize);
    for (int i = t; i < kMomSize / 4; i += 256) reinterpret_cast<f32x4*>(ms)[i] = src[i];
  }
  {
    const int qi = t >> 2, d0 = (t & 3) * 16;
    const int qq = q0 + qi;
    const T* qr = q + (bh * Nc + qq) * 64 + d0;
#pragma unroll
    for (int e = 0; e < 16; ++e) qs[d0 + e][qi] = qq < Nc ? to_f32<T>(qr[e]) : 0.f;
  }
  __syncthreads();
  const int qg = t >> 4, cg = t & 15;
  float am[4][4] = {}, ae[4][4] = {}, al[4] = {};
#pragma unroll 4
  for (int d = 0; d < 64; ++d) {
    const f32x4 qv = *reinterpret_cast<const f32x4*>(&qs[d][4 * qg]);
    const f32x4 mv = *reinterpret_cast<const f32x4*>(&ms[d * kMomLd + 4 * cg]);
    const f32x4 ev = *reinterpret_cast<const f32x4*>(&ms[d * kMomLd + 64 + 4 * cg]);
    const float kd = ms[d * kMomLd + 128];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      al[i] = fmaf(qv[i], kd, al[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        am[i][j] = fmaf(qv[i], mv[j], am[i][j]);
        ae[i][j] = fmaf(qv[i], ev[j], ae[i][j]);
      }
    }
  }
  const float ns = ms[64 * kMomLd + 128];
  const int c0 = 4 * cg;
  const f32x4 vsum = *reinterpret_cast<const f32x4*>(&ms[64 * kMomLd + c0]);
  const f32x4 v2sum = *reinterpret_cast<const f32x4*>(&ms[64 * kMomLd + 64 + c0]);
  const int col = h * 64 + c0;
  const f32x4 m4 = *reinterpret_cast<const f32x4*>(fcs_mu + (long long)b * C + col);
  const f32x4 r4 = *reinterpret_cast<const f32x4*>(fcs_rstd + (long long)b * C + col);
  const f32x4 v4 = *reinterpret_cast<const f32x4*>(v_mu + (long long)b * C + col);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qq = q0 + 4 * qg + i;
    if (qq >= Nc) continue;
    const float inv = 1.0f / (al[i] + ns);
    const long long row = (long long)b * Nc + qq;
    const f32x4 f = *reinterpret_cast<const f32x4*>(fcs + row * C + col);
    float res[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float m1 = (am[i][j] + vsum[j]) * inv;
      const float e2 = (ae[i][j] + v2sum[j]) * inv;
      const float sd = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f));
      res[j] = sd * ((f[j] - m4[j]) * r4[j]) + (m1 + v4[j]);
    }
    T* orow = out + row * C + col;
    if constexpr (sizeof(T) == 4) {
      *reinterpret_cast<f32x4*>(orow) = f32x4{res[0], res[1], res[2], res[3]};
    } else {
      *reinterpret_cast<bf16x4*>(orow) = bf16x4{(bf16)res[0], (bf16)res[1], (bf16)res[2], (bf16)res[3]};
    }
  }
}

}  // namespace
}  // namespace mhada

using namespace mhada;

extern "C" int mhada_cosine_moments(const void* kv, const void* vt, int dtype, int B, int H, int Ns, float* mom,
                                    float* work, int splits, mhada_stream_t s_) {
  const hipStream_t s = (hipStream_t)s_;
  if (!kv || !vt || !mom || B <= 0 || H <= 0 || Ns <= 0 || splits <= 0 || (splits > 1 && !work))
    return fail("mhada_cosine_moments: bad args");
  if (dtype != MHADA_F32 && dtype != MHADA_BF16) return fail("mhada_cosine_moments: bad dtype");
  if ((long long)B * H > 65535) return fail("mhada_cosine_moments: B * H > 65535");
  const int ldt = (Ns + 63) / 64 * 64;
  const int cps = ((Ns + splits - 1) / splits + 63) / 64 * 64;  // keys per split, whole 64-key tiles
  float* part = splits == 1 ? mom : work;
  const dim3 grid(splits, B * H);
  if (dtype == MHADA_F32)
    hipLaunchKernelGGL((cosine_mom_kernel<float>), grid, dim3(256), 0, s, (const float*)kv, (const float*)vt, part,
                       Ns, ldt, cps, splits);
  else
    hipLaunchKernelGGL((cosine_mom_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)kv, (const bf16*)vt, part, Ns,
                       ldt, cps, splits);
  if (splits > 1) hipLaunchKernelGGL(cosine_mom_finish_kernel, dim3(B * H), dim3(256), 0, s, work, mom, splits);
  return check_launch("mhada_cosine_moments");
}

extern "C" int mhada_cosine_attn(const void* q, const float* mom, const float* fcs, const float* fcs_mu,
                                 const float* fcs_rstd, const float* v_mu, void* out, int dtype, int B, int H, int Nc,
                                 mhada_stream_t s_) {
  const hipStream_t s = (hipStream_t)s_;
  if (!q || !mom || !fcs || !fcs_mu || !fcs_rstd || !v_mu || !out || B <= 0 || H <= 0 || Nc <= 0)
    return fail("mhada_cosine_attn: bad args");
  if (dtype != MHADA_F32 && dtype != MHADA_BF16) return fail("mhada_cosine_attn: bad dtype");
  if (B > 65535 || H > 65535) return fail("mhada_cosine_attn: B or H > 65535");
  const dim3 grid((Nc + 63) / 64, H, B);
  if (dtype == MHADA_F32)
    hipLaunchKernelGGL((cosine_attn_kernel<float>), grid, dim3(256), 0, s, (const float*)q, mom, fcs, fcs_mu,
                       fcs_rstd, v_mu, (float*)out, H, Nc);
  else
    hipLaunchKernelGGL((cosine_attn_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)q, mom, fcs, fcs_mu, fcs_rstd,
                       v_mu, (bf16*)out, H, Nc);
  return check_launch("mhada_cosine_attn");
}
