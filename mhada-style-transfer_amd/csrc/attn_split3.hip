// fp32 MHAda attention as fp32-accurate SPLIT3 products on the bf16 MFMA (round 6).
//
// Reference: AdaAttnMultiHead.forward, adaDecoder.py:186-198 (A = softmax(Q K^T), M = A V,
// E2 = A V^2, out = sqrt(max(E2 - M^2, 1e-6)) * IN(fcs) + M), the fp32 arithmetic of the reference
// (BASELINE configs[1]).  attn_f32_kernel (attn.hip) computes it on v_mfma_f32_32x32x2_f32 and sits at
// that pipe's ceiling (0.83-0.87 of 157.3 TF/s, HBM traffic 1.02x the algorithmic bytes); the bf16
// pipe has 16x the MACs per cycle.  Here every fp32 operand x travels as three bf16 planes
// x = x0 + x1 + x2 (round-to-nearest split: x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1);
// exact for normal fp32 values, |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|), and each fp32 product
// x * y is the sum of the six cross products x_i y_j with i + j <= 2, accumulated in fp32 by
// v_mfma_f32_16x16x32_bf16; the three dropped terms are below 2^-24 |x y| (x1 y2, x2 y1) and 2^-32
// (x2 y2).  Both products of the loop are split this way:
//   S = Q K^T       Q split in registers on load, K from the pre-split K planes;
//   O = P [V' | V'^2]   P = exp2(S - m) computed in fp32 and split in registers after the exp,
//                   V'^T | V'^2^T from the pre-split planes of the fp32 vt image;
//   l = sum P       three all-ones MFMAs per 32 keys (one per P plane) — the exact sum of the planes.
// Against fp64 the result is at or below attn_f32_kernel's error (tests/test_gpu_kernels.py).
//
// Structure: attn_bf16_fsq_kernel's (attn.hip) — swapped products with the query on the MFMA column,
// two 16-query groups per wave sharing every K / V'^T fragment, the fsq_key score-row choice that
// leaves each lane group holding exactly its PV B-operand keys, fixed-shift softmax (the shift is the
// max of each query's first key tile; the accumulators start at -m; a row whose later scores outgrow
// it by 2^64 is recomputed exactly after the loop, attn_exact_q3) — with 64-key tiles: one ring slot
// holds the three K planes (3 x 8 KiB) and the three V'^T | V'^2^T planes (3 x 16 KiB), two slots
// = 144 KiB of LDS, filled by LDS-DMA.  Per tile and wave: 96 QK + 192 PV + 12 row-sum MFMAs for
// 64 keys x 32 queries, 24 + 48 ds_read_b128, and 32 v_exp_f32 plus ~4.5 VALU per score for the
// split of P.
//
// LDS images (per 128-B row of 64 bf16): K planes [3][64 keys][64 d], chunk c of key row k at 16-B
// slot c ^ (k & 7) (attn_bf16_fsq_kernel's K swizzle); V'^T planes [3][128 rows][64 key positions],
// chunk c of row r at slot c ^ ((r >> 1) & 7) — conflict-free for the ds_read_b128 lane groups of
// MI355X_MICROARCH.md's LDS table (rows 16 dvb + r16, chunk 4 kg + g: the 16 lanes of a group cover
// every (row parity, slot) pair once).
//
// Plane image in HBM (mhada_split3_kv), per (b, h), ldt = ceil64(Ns):
//   K planes  [3][ldt][64]   rows >= Ns zero;
//   V planes  [3][128][ldt]  V'^T (rows 0..63) | V'^2^T (64..127), key positions permuted inside
//             groups of 16 (bits 2 and 3 swapped, the bf16 vt image's order), zero padded.
#include "attn_common.h"

namespace mhada {

constexpr int kS3Tk = 64;  // keys per tile

// bf16 elements of one (b, h)'s plane image: K 3 * 64 * ldt, V 3 * 128 * ldt
__host__ __device__ constexpr long long s3_image(int ldt) { return 576LL * ldt; }

// Round-to-nearest three-way split (the split of mhada_layernorm BF16X3 and ops.split3_weight).
struct Bf3 { bf16 a, b, c; };
MHADA_DEV Bf3 split3(float x) {
  const bf16 a = (bf16)x;
  const float r = x - (float)a;
  const bf16 b = (bf16)r;
  return Bf3{a, b, (bf16)(r - (float)b)};
}
template <typename V>
MHADA_DEV void split3_into(float x, V& a, V& b, V& c, int e) {
  const Bf3 s = split3(x);
  a[e] = s.a;
  b[e] = s.b;
  c[e] = s.c;
}

// kv fp32 [BH][Ns][128] (K in columns 0..63; V' is read from vt) and the fp32 vt image [BH][128][ldt]
// (natural key order, zero padded) -> the plane image.  One workgroup per (64-key chunk, b h).
__global__ void __launch_bounds__(256) split3_kv_kernel(const float* __restrict__ kv, const float* __restrict__ vt,
                                                        bf16* __restrict__ img, int Ns, int ldt) {
  const int bh = blockIdx.y, n0 = blockIdx.x * 64, tid = threadIdx.x;
  bf16* kp = img + (long long)bh * s3_image(ldt);
  bf16* vp = kp + 192LL * ldt;
  const float* kvb = kv + (long long)bh * Ns * 128;
  const float* vtb = vt + (long long)bh * 128 * ldt;
  const long long kps = 64LL * ldt, vps = 128LL * ldt;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // K: 64 keys x 16 groups of 4 d
    const int idx = tid + 256 * i, key = n0 + (idx >> 4), d = (idx & 15) * 4;
    const f32x4 x = key < Ns ? *reinterpret_cast<const f32x4*>(kvb + (long long)key * 128 + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x4 a, b, c;
#pragma unroll
    for (int e = 0; e < 4; ++e) split3_into(x[e], a, b, c, e);
    bf16* dst = kp + (long long)key * 64 + d;
    *reinterpret_cast<bf16x4*>(dst) = a;
    *reinterpret_cast<bf16x4*>(dst + kps) = b;
    *reinterpret_cast<bf16x4*>(dst + 2 * kps) = c;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // V'^T | V'^2^T: 128 rows x 8 runs of 8 key positions
    const int idx = tid + 256 * i, row = idx >> 3, a8 = idx & 7;
    // positions 8 a8 + j hold keys 16 (a8 >> 1) + 8 (j >> 2) + 4 (a8 & 1) + (j & 3)
    const float* src = vtb + (long long)row * ldt + n0 + 16 * (a8 >> 1) + 4 * (a8 & 1);
    const f32x4 lo = *reinterpret_cast<const f32x4*>(src), hi = *reinterpret_cast<const f32x4*>(src + 8);
    bf16x8 a, b, c;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_into(j < 4 ? lo[j] : hi[j - 4], a, b, c, j);
    bf16* dst = vp + (long long)row * ldt + n0 + 8 * a8;
    *reinterpret_cast<bf16x8*>(dst) = a;
    *reinterpret_cast<bf16x8*>(dst + vps) = b;
    *reinterpret_cast<bf16x8*>(dst + 2 * vps) = c;
  }
}

// The K|V' projection of one MHAda block (adaDecoder.py:178,182 after the fold of mhada_fold_block)
// written straight as the plane image (replaces the fp32 projection GEMM with its vt epilogue plus
// split3_kv_kernel, and their fp32 kv / vt round trip through HBM):
//   Y[n][o] = sum_c (fs[b][n][64h + c] - mu[b][64h + c]) wkv[b][h][o][c] + bkv[h][o]
// K = Y[:, 0:64] -> K planes, V' = Y[:, 64:128] -> V'^T and V'^2^T (the fp32 square of the fp32 V')
// planes.  One workgroup per (64 keys, b h): X (centred on load) and W staged in LDS, the 64 x 128
// product on v_mfma_f32_32x32x2_f32 (4 waves, two 32 x 32 blocks each, K = 64), Y through LDS (over
// the operand images), then 16-B plane stores.  Keys >= Ns are written as zeros.
__global__ void __launch_bounds__(256) kv_proj_s3_kernel(const float* __restrict__ fs, const float* __restrict__ mu,
                                                         const float* __restrict__ wkv, const float* __restrict__ bkv,
                                                         bf16* __restrict__ img, int H, int Ns, int ldt) {
  constexpr int LX = 65, LY = 65;  // padded rows: the MFMA operand reads and the transposed Y reads
  __shared__ float sm[192 * LX];   // X [key][c] (centred) | W [o][c]; then Y [o][key] (50 KiB: 3 workgroups per CU)
  float* sX = sm;
  float* sW = sm + 64 * LX;
  float* sY = sm;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H, n0 = blockIdx.x * 64, tid = threadIdx.x;
  const int C = 64 * H;
  const float* xb = fs + (long long)b * Ns * C + 64 * h;
  const float* mb = mu + (long long)b * C + 64 * h;
  const float* wb = wkv + (long long)bh * 128 * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i, n = idx >> 4, c = (idx & 15) * 4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (n0 + n < Ns) {
      x = *reinterpret_cast<const f32x4*>(xb + (long long)(n0 + n) * C + c);
      const f32x4 m = *reinterpret_cast<const f32x4*>(mb + c);
      x = x - m;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) sX[n * LX + c + e] = x[e];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = tid + 256 * i, o = idx >> 4, c = (idx & 15) * 4;
    const f32x4 w = *reinterpret_cast<const f32x4*>(wb + o * 64 + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) sW[o * LX + c + e] = w[e];
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, r32 = lane & 31, hh = lane >> 5;
  const int nb = wave & 1, ob = wave >> 1;  // keys 32 nb .., outputs 64 ob ..
  f32x16 acc[2] = {};
#pragma unroll 8
  for (int k = 0; k < 64; k += 2) {
    const float bv = sX[(32 * nb + r32) * LX + k + hh];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      acc[ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(sW[(64 * ob + 32 * ni + r32) * LX + k + hh], bv, acc[ni], 0, 0, 0);
  }
  const float* bb = bkv + h * 128;
  __syncthreads();  // every wave's operand reads are done before Y overwrites them
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 64 * ob + 32 * ni + (r & 3) + 8 * (r >> 2) + 4 * hh;
      sY[o * LY + 32 * nb + r32] = acc[ni][r] + bb[o];
    }
  __syncthreads();
  bf16* kp = img + (long long)bh * s3_image(ldt);
  bf16* vp = kp + 192LL * ldt;
  const long long kps = 64LL * ldt, vps = 128LL * ldt;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // K planes: 64 keys x 8 runs of 8 outputs
    const int idx = tid + 256 * i, n = idx >> 3, o0 = (idx & 7) * 8;
    const bool valid = n0 + n < Ns;
    bf16x8 a, c1, c2;
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_into(valid ? sY[(o0 + j) * LY + n] : 0.f, a, c1, c2, j);
    bf16* dst = kp + (long long)(n0 + n) * 64 + o0;
    *reinterpret_cast<bf16x8*>(dst) = a;
    *reinterpret_cast<bf16x8*>(dst + kps) = c1;
    *reinterpret_cast<bf16x8*>(dst + 2 * kps) = c2;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // V'^T | V'^2^T planes: 64 rows x 8 runs of 8 key positions
    const int idx = tid + 256 * i, vo = idx >> 3, a8 = idx & 7;
    bf16x8 a, c1, c2, s0, s1, s2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = 16 * (a8 >> 1) + 8 * (j >> 2) + 4 * (a8 & 1) + (j & 3);  // position 8 a8 + j
      const float v = n0 + n < Ns ? sY[(64 + vo) * LY + n] : 0.f;
      split3_into(v, a, c1, c2, j);
      split3_into(v * v, s0, s1, s2, j);
    }
    bf16* dst = vp + (long long)vo * ldt + n0 + 8 * a8;
    *reinterpret_cast<bf16x8*>(dst) = a;
    *reinterpret_cast<bf16x8*>(dst + vps) = c1;
    *reinterpret_cast<bf16x8*>(dst + 2 * vps) = c2;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt) = s0;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt + vps) = s1;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt + 2 * vps) = s2;
  }
}

// x_i y_j, i + j <= 2, small terms first: acc + x2y0 + x1y1 + x0y2 + x1y0 + x0y1 + x0y0 (A = x, B = y)
MHADA_DEV f32x4 mfma6(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0, const bf16x8& b1,
                      const bf16x8& b2, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
}

// Exact two-pass recompute of one wave's 2 x 16 queries (the rare path when a row sum trips
// kShiftSumThr): the true row max over all keys, then the full pass, planes read from L2.
template <bool QK32>
MHADA_DEV void attn_exact_q3(const AttnP& p, const bf16* kp, const bf16* vp, const bf16x8 (&qf)[3][2][2],
                             const float (&qreg)[2][16], f32x4 (&O)[2][8], float (&lt)[2], float (&mx)[2], int g,
                             int r16) {
  const int Ns = p.Ns;
  const long long kps = 64LL * p.ldt, vps = 128LL * p.ldt;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto scores = [&](int k0, f32x4 (&S)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bf16* kr = kp + (long long)(k0 + fsq_key(r16, t)) * 64 + 8 * g;  // k0 + 31 < ldt
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) S[qg][t] = z4;
      if constexpr (QK32) {  // fp32 K rows, d permuted to 16 g + s
        const float* kf = reinterpret_cast<const float*>(kp) + (long long)(k0 + fsq_key(r16, t)) * 64 + 16 * g;
#pragma unroll
        for (int st = 0; st < 16; ++st)
#pragma unroll
          for (int qg = 0; qg < 2; ++qg) S[qg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[st], qreg[qg][st], S[qg][t], 0, 0, 0);
      }
#pragma unroll
      for (int dh = 0; dh < (QK32 ? 0 : 2); ++dh) {
        const bf16x8 k0f = *reinterpret_cast<const bf16x8*>(kr + 32 * dh);
        const bf16x8 k1f = *reinterpret_cast<const bf16x8*>(kr + kps + 32 * dh);
        const bf16x8 k2f = *reinterpret_cast<const bf16x8*>(kr + 2 * kps + 32 * dh);
#pragma unroll
        for (int qg = 0; qg < 2; ++qg)
          S[qg][t] = mfma6(k0f, k1f, k2f, qf[0][qg][dh], qf[1][qg][dh], qf[2][qg][dh], S[qg][t]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (k0 + fsq_key(4 * g + j, t) >= Ns) S[0][t][j] = S[1][t][j] = -INFINITY;
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
    bf16x8 pf[3][2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = fast_exp2(S[qg][j >> 2][j & 3] - m2[qg]);
        lt[qg] += e;
        split3_into(e, pf[0][qg], pf[1][qg], pf[2][qg], j);
      }
#pragma unroll
    for (int dvb = 0; dvb < 8; ++dvb) {
      const bf16* vr = vp + (long long)(16 * dvb + r16) * p.ldt + k0 + 8 * g;
      const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(vr);
      const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(vr + vps);
      const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(vr + 2 * vps);
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) O[qg][dvb] += mfma6(v0, v1, v2, pf[0][qg], pf[1][qg], pf[2][qg], z4);
    }
  }
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    lt[qg] += __shfl_xor(lt[qg], 16, 64);
    lt[qg] += __shfl_xor(lt[qg], 32, 64);
    mx[qg] = m2[qg];
  }
}

// Scores of keys >= Ns (the ragged last tile): -inf.  S[qg][kg][t][j] is key key0 + 32 kg + fsq_key(4 g + j, t).
MHADA_DEV void s3_mask(f32x4 (&S)[2][2][2], int key0, int Ns, int g) {
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (key0 + 32 * kg + fsq_key(4 * g + j, t) >= Ns) S[0][kg][t][j] = S[1][kg][t][j] = -INFINITY;
}

// Training forward (mhada_attn_train_fwd_split3): k [BH][Ns][64] and the centred v [BH][Ns][64] rows
// of the training attention -> the QK32 image: fp32 K rows [ldt][64] (d = 4 s + g at 16 g + s; in the
// K-plane region) and the V'^T | V'^2^T planes from v (its fp32 square, key positions permuted as
// split3_kv_kernel's).  One workgroup per (64 keys, b h).
__global__ void __launch_bounds__(256) train_s3_prep_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                            bf16* __restrict__ img, int Ns, int ldt) {
  __shared__ float sv[64 * 65];  // [key][o]
  const int bh = blockIdx.y, n0 = blockIdx.x * 64, tid = threadIdx.x;
  bf16* kp = img + (long long)bh * s3_image(ldt);
  bf16* vp = kp + 192LL * ldt;
  const float* kb = k + (long long)bh * Ns * 64;
  const float* vb = v + (long long)bh * Ns * 64;
  const long long vps = 128LL * ldt;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i, n = idx >> 4, d = (idx & 15) * 4;
    const bool ok = n0 + n < Ns;
    const f32x4 x = ok ? *reinterpret_cast<const f32x4*>(kb + (long long)(n0 + n) * 64 + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 y = ok ? *reinterpret_cast<const f32x4*>(vb + (long long)(n0 + n) * 64 + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    // fp32 K rows for the QK32 kernel: d = 4 s + g stored at 16 g + s
    float* kf = reinterpret_cast<float*>(kp) + (long long)(n0 + n) * 64 + d / 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) kf[16 * e] = x[e];
#pragma unroll
    for (int e = 0; e < 4; ++e) sv[n * 65 + d + e] = y[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 64 rows o x 8 runs of 8 key positions
    const int idx = tid + 256 * i, o = idx >> 3, a8 = idx & 7;
    bf16x8 a, c1, c2, s0, s1, s2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = 16 * (a8 >> 1) + 8 * (j >> 2) + 4 * (a8 & 1) + (j & 3);  // position 8 a8 + j
      const float x = sv[n * 65 + o];
      split3_into(x, a, c1, c2, j);
      split3_into(x * x, s0, s1, s2, j);
    }
    bf16* dst = vp + (long long)o * ldt + n0 + 8 * a8;
    *reinterpret_cast<bf16x8*>(dst) = a;
    *reinterpret_cast<bf16x8*>(dst + vps) = c1;
    *reinterpret_cast<bf16x8*>(dst + 2 * vps) = c2;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt) = s0;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt + vps) = s1;
    *reinterpret_cast<bf16x8*>(dst + 64LL * ldt + 2 * vps) = s2;
  }
}

// Training epilogue in the 16x16x32 layout (attn_train_epilogue's contract, attn.hip): per query row
// out' = sqrt(max(E2' - M'^2, 1e-6)) x + M', mo = [M' | E2'], lse2 = m2 + log2(l); x = p.fcs
// [BH][Nc][64].  O[qg][dvb] holds O^T[dv][q] for dv = 16 dvb + 4 g + e (dvb 0-3: M', 4-7: E2').
MHADA_DEV void attn_train_epilogue_q(const AttnP& p, const f32x4 (&O)[2][8], const float (&lt)[2],
                                     const float (&m2)[2], long long bh, int q0, int g, int r16) {
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + 16 * qg + r16;
    if (q >= p.Nc) continue;
    const float inv = 1.0f / lt[qg];
    const long long row = bh * p.Nc + q;
    const float* xr = p.fcs + row * 64;
    float* orow = reinterpret_cast<float*>(p.out) + row * 64;
    float* mrow = p.mo + row * 128;
#pragma unroll
    for (int dvb = 0; dvb < 4; ++dvb) {
      const int dv0 = 16 * dvb + 4 * g;
      const f32x4 xx = *reinterpret_cast<const f32x4*>(xr + dv0);
      f32x4 o, mm, ee;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[qg][dvb][e] * inv;
        const float e2 = O[qg][dvb + 4][e] * inv;
        o[e] = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f)) * xx[e] + m1;
        mm[e] = m1;
        ee[e] = e2;
      }
      *reinterpret_cast<f32x4*>(orow + dv0) = o;
      *reinterpret_cast<f32x4*>(mrow + dv0) = mm;
      *reinterpret_cast<f32x4*>(mrow + 64 + dv0) = ee;
    }
    if (g == 0) p.lse[row] = m2[qg] + __log2f(lt[qg]);
  }
}

// TRAIN: the training forward — Q in natural units (log2 e applied in fp32 on load, as attn_f32_kernel's
// TRAIN form), the training epilogue (out', [M' | E2'], lse2).
// QK32 (the training forward): S = Q K^T on the fp32 MFMA (v_mfma_f32_16x16x4f32, the S^T tile layout of
// the bf16 16x16x32 MFMA) from fp32 K rows, P V' / P V'^2 SPLIT3 as above.  The backward recomputes S
// on the fp32 MFMA against this kernel's lse2, so lse2 and the backward's P come from the same fp32
// products: a SPLIT3 S (the bf16 MFMA's truncating sums, ~1e-5 |S| at large logits) needs neither fp32
// pipe nor K rows and is 2 % faster per training step (424.6 vs 433.1 ms), but with ACC 1 it leaves the
// 64^2 video golden's AdaFormer gradient norm at 5.8e-3 — both changes are needed
// (profiles/r06_train_fwd_s3_acc_ab.log).
// ACC 1 (the training forward): P V' / P V'^2 and the row sums of each 32-key group from zero, added to
// the running totals by fp32 VALU adds (round to nearest).  Accumulated in the MFMA instead (ACC 0, the
// inference kernel) the bf16 MFMA's truncating partial sums bias M' and E2' low by a few 1e-7 — 3x the
// error of ACC 1 on the bench data (profiles/r06_attn_s3_acc_ab.log) — and through sqrt's gradient at
// near-degenerate variance rows that moved the 64^2 video-training golden's AdaFormer gradient norm by
// 5.9e-3 (ACC 1: 3.3e-4; the fp32-MFMA forward: 4.9e-4; profiles/r06_train_fwd_s3_acc_ab.log).  ACC 1
// costs 7 % at inference (and 10 spilled registers in the 8-wave inference kernel): not used there.
// K image: fp32 rows [ldt][64] with d permuted to 16 g + s (= d 4 s + g: lane
// group g's 16 MFMA steps are 64 contiguous bytes) in the K-plane region of the plane image; in LDS the
// 16-B chunk c of key row k at slot c ^ f(k & 7), f(k) = (k & 3) | (k >> 2) << 3 (the 16 lanes of a
// ds_read_b128 group then hit 16 distinct slots).
// IL 1 (the inference kernel, ACC 0): key group 1's exp / split interleaved with key group 0's P V
// MFMAs — bit-identical, 1.6-3.4 % faster at the bench shapes than the two groups in sequence
// (tools/attn_s3_variants_interleaved.py, profiles/r06_attn_s3_interleave_ab.log; a full-tile
// interleave with the Q K^T of group 1 beside the split of group 0 measured no better).
template <int NW, bool TRAIN = false, bool QK32 = false, int ACC = 0, int IL = 0>
__global__ void __launch_bounds__(64 * NW, 1) attn_s3_kernel(const AttnP p) {
  constexpr int TK = kS3Tk;
  constexpr int KPL = TK * 64, VPL = 128 * TK;                // bf16 elements per plane
  constexpr int KREG = QK32 ? 2 * TK * 64 : 3 * KPL;          // bf16 elements of the slot's K region
  constexpr int SLOT = KREG + 3 * VPL;
  constexpr int KPC = KREG / 512, VPC = 3 * VPL / 512;        // 1-KiB DMA pieces per slot: 24 (16) + 48
  static_assert(KPC % NW == 0 && VPC % NW == 0, "tile config");
  constexpr int KPW = KPC / NW, VPW = VPC / NW;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * SLOT];  // 144 KiB (QK32: 128 KiB)
  int b, hh, qb;
  decode_block(p, b, hh, qb);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int q0 = qb * (32 * NW) + wave * 32;
  const long long bh = (long long)b * p.H + hh;
  const int Ns = p.Ns, ldt = p.ldt;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  bf16x8 qf[3][2][2];  // Q^T planes: query q0 + 16 qg + r16, d = 32 dh + 8 g .. + 8
  float qreg[2][16];   // QK32: Q[q][4 s + g] (x log2 e) for MFMA step s
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q0 + 16 * qg + r16;
    if constexpr (QK32) {
      const float* qr = reinterpret_cast<const float*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + g;
#pragma unroll
      for (int st = 0; st < 16; ++st) qreg[qg][st] = q < p.Nc ? qr[4 * st] * 1.4426950408889634f : 0.f;
      continue;
    }
    const float* qp = reinterpret_cast<const float*>(p.q) + (bh * p.Nc + (q < p.Nc ? q : 0)) * 64 + 8 * g;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(qp + 32 * dh);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(qp + 32 * dh + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = q < p.Nc ? (e < 4 ? lo[e] : hi[e - 4]) * (TRAIN ? 1.4426950408889634f : 1.0f) : 0.f;
        split3_into(x, qf[0][qg][dh], qf[1][qg][dh], qf[2][qg][dh], e);
      }
    }
  }
  const bf16* kp = reinterpret_cast<const bf16*>(p.kv) + bh * s3_image(ldt);
  const bf16* vp = kp + 192LL * ldt;
  // per-lane DMA sources: piece NW i + wave; K pieces hold 8 key rows of one plane, V pieces 8 rows
  int ksrc[KPW], vsrc[VPW];
#pragma unroll
  for (int i = 0; i < KPW; ++i) {
    if constexpr (QK32) {  // 4 fp32 rows of 256 B per piece; bf16-element offsets
      const int pc = NW * i + wave, row = 4 * pc + (lane >> 4), slot = lane & 15;
      const int f = (row & 3) | (((row >> 2) & 1) << 3);
      ksrc[i] = 2 * (row * 64 + 4 * (slot ^ f));
    } else {
      const int pc = NW * i + wave, pl = pc >> 3, row = 8 * (pc & 7) + (lane >> 3), slot = lane & 7;
      ksrc[i] = pl * 64 * ldt + row * 64 + 8 * (slot ^ (row & 7));
    }
  }
#pragma unroll
  for (int i = 0; i < VPW; ++i) {
    const int pc = NW * i + wave, pl = pc >> 4, row = 8 * (pc & 15) + (lane >> 3), slot = lane & 7;
    vsrc[i] = pl * 128 * ldt + row * ldt + 8 * (slot ^ ((row >> 1) & 7));
  }
  auto stage = [&](int key0, int sl) {
    bf16* kd = smem + sl * SLOT;
    bf16* vd = kd + KREG;
    const bf16* ks = kp + (long long)key0 * (QK32 ? 128 : 64);
    const bf16* vs = vp + key0;
#pragma unroll
    for (int i = 0; i < KPW; ++i) attn_glds16(ks + ksrc[i], kd + 512 * (NW * i + wave));
#pragma unroll
    for (int i = 0; i < VPW; ++i) attn_glds16(vs + vsrc[i], vd + 512 * (NW * i + wave));
  };
  int krow[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) krow[t] = fsq_key(r16, t) * 64;
  auto qk = [&](int sl, f32x4 (&S)[2][2][2], const f32x4 (&init)[2]) {
    if constexpr (QK32) {
      const float* ck = reinterpret_cast<const float*>(smem + sl * SLOT);
      const int f = (r16 & 3) | (((r16 >> 2) & 1) << 3);  // f(key & 7), key & 7 == r16 & 7
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float* kr = ck + (kg * 32 + fsq_key(r16, t)) * 64;
          f32x4 kf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) kf[j] = *reinterpret_cast<const f32x4*>(kr + 4 * ((4 * g + j) ^ f));
#pragma unroll
          for (int st = 0; st < 16; ++st)
#pragma unroll
            for (int qg = 0; qg < 2; ++qg)
              S[qg][kg][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[st >> 2][st & 3], qreg[qg][st],
                                                                  st == 0 ? init[qg] : S[qg][kg][t], 0, 0, 0);
        }
      return;
    }
    const bf16* ck = smem + sl * SLOT;
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16* kr = ck + kg * 32 * 64 + krow[t];
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const int off = 8 * ((4 * dh + g) ^ (r16 & 7));  // key & 7 == r16 & 7
          const bf16x8 k0f = *reinterpret_cast<const bf16x8*>(kr + off);
          const bf16x8 k1f = *reinterpret_cast<const bf16x8*>(kr + KPL + off);
          const bf16x8 k2f = *reinterpret_cast<const bf16x8*>(kr + 2 * KPL + off);
#pragma unroll
          for (int qg = 0; qg < 2; ++qg)
            S[qg][kg][t] = mfma6(k0f, k1f, k2f, qf[0][qg][dh], qf[1][qg][dh], qf[2][qg][dh],
                                 dh == 0 ? init[qg] : S[qg][kg][t]);
        }
      }
  };
  f32x4 O[2][8], L[2];
  float lsum[2] = {0.f, 0.f};  // ACC 1: the row sums, summed per 32-key group in fp32
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    L[qg] = z4;
#pragma unroll
    for (int i = 0; i < 8; ++i) O[qg][i] = z4;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;
  // ACC 0 building blocks of the interleaved forms (IL): P V' / P V'^2 of one key group and row block,
  // and one key group's row sums
  auto pv = [&](int sl, int kg, int dvb, const bf16x8 (&pf)[3][2]) {
    const int off = 8 * ((4 * kg + g) ^ ((r16 >> 1) & 7));
    const bf16* vr = smem + sl * SLOT + KREG + (16 * dvb + r16) * TK + off;
    const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(vr);
    const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(vr + VPL);
    const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(vr + 2 * VPL);
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) O[qg][dvb] = mfma6(v0, v1, v2, pf[0][qg], pf[1][qg], pf[2][qg], O[qg][dvb]);
  };
  auto rowsum = [&](const bf16x8 (&pf)[3][2]) {
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[2][qg], L[qg], 0, 0, 0);
      L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[1][qg], L[qg], 0, 0, 0);
      L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[0][qg], L[qg], 0, 0, 0);
    }
  };
  auto finish = [&](int sl, const f32x4 (&S)[2][2][2]) {
    const bf16* cv = smem + sl * SLOT + KREG;
    if constexpr (IL != 0 && ACC == 0) {
      // the exp / split of key group 1 interleaved with key group 0's P V MFMAs (two scores per row
      // block), so this wave's VALU burst no longer runs beside an idle matrix pipe
      bf16x8 pa[3][2], pb[3][2];
#pragma unroll
      for (int qg = 0; qg < 2; ++qg)
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_into(fast_exp2(S[qg][0][j >> 2][j & 3]), pa[0][qg], pa[1][qg], pa[2][qg], j);
      rowsum(pa);
#pragma unroll
      for (int dvb = 0; dvb < 8; ++dvb) {
        pv(sl, 0, dvb, pa);
        const int qg = dvb >> 2, j = 2 * (dvb & 3);
        split3_into(fast_exp2(S[qg][1][j >> 2][j & 3]), pb[0][qg], pb[1][qg], pb[2][qg], j);
        split3_into(fast_exp2(S[qg][1][(j + 1) >> 2][(j + 1) & 3]), pb[0][qg], pb[1][qg], pb[2][qg], j + 1);
      }
      rowsum(pb);
#pragma unroll
      for (int dvb = 0; dvb < 8; ++dvb) pv(sl, 1, dvb, pb);
      return;
    }
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      bf16x8 pf[3][2];
#pragma unroll
      for (int qg = 0; qg < 2; ++qg)
#pragma unroll
        for (int j = 0; j < 8; ++j) split3_into(fast_exp2(S[qg][kg][j >> 2][j & 3]), pf[0][qg], pf[1][qg], pf[2][qg], j);
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) {
        if constexpr (ACC == 0) {
          L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[2][qg], L[qg], 0, 0, 0);
          L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[1][qg], L[qg], 0, 0, 0);
          L[qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[0][qg], L[qg], 0, 0, 0);
        } else {  // the group's sum from zero, added to the total in fp32 (round to nearest)
          f32x4 t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[2][qg], z4, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[1][qg], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[0][qg], t, 0, 0, 0);
          lsum[qg] += t[0];
        }
      }
      const int off = 8 * ((4 * kg + g) ^ ((r16 >> 1) & 7));  // row 16 dvb + r16
      f32x4 tp[2];  // ACC 1: the previous dvb's group sums, added one step later (no MFMA -> VALU wait)
#pragma unroll
      for (int dvb = 0; dvb < 8; ++dvb) {
        const bf16* vr = cv + (16 * dvb + r16) * TK + off;
        const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(vr);
        const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(vr + VPL);
        const bf16x8 v2 = *reinterpret_cast<const bf16x8*>(vr + 2 * VPL);
        if constexpr (ACC == 0) {
#pragma unroll
          for (int qg = 0; qg < 2; ++qg) O[qg][dvb] = mfma6(v0, v1, v2, pf[0][qg], pf[1][qg], pf[2][qg], O[qg][dvb]);
        } else {
          f32x4 tn[2];
#pragma unroll
          for (int qg = 0; qg < 2; ++qg) tn[qg] = mfma6(v0, v1, v2, pf[0][qg], pf[1][qg], pf[2][qg], z4);
          if (dvb > 0) {
#pragma unroll
            for (int qg = 0; qg < 2; ++qg) O[qg][dvb - 1] += tp[qg];
          }
#pragma unroll
          for (int qg = 0; qg < 2; ++qg) tp[qg] = tn[qg];
        }
      }
      if constexpr (ACC != 0) {
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) O[qg][7] += tp[qg];
      }
    }
  };

  const int NTILE = (Ns + TK - 1) / TK, NFULL = Ns / TK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 Sa[2][2][2], Cm[2];
  {  // tile 0: unshifted scores, m2 = their max, then shift
    const f32x4 zi[2] = {z4, z4};
    qk(0, Sa, zi);
    if (NFULL == 0) s3_mask(Sa, 0, Ns, g);
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float m = -INFINITY;
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) m = fmaxf(m, Sa[qg][kg][t][j]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) Sa[qg][kg][t][j] -= m;
      Cm[qg] = f32x4{-m, -m, -m, -m};
    }
  }
  if (NTILE > 1) stage(TK, 1);
  finish(0, Sa);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // Measured and not kept (profiles/r06_attn_s3_order_prio_ab.log): Q K^T and P V interleaved per
  // 32-key group (all waves or the younger half, so that the softmax VALU bursts of the two waves of a
  // SIMD fall apart) within +-1 %; s_setprio(1) for the younger half 1.5-4 % slower than none.
  for (int t = 1; t < NFULL; ++t) {
    if (t + 1 < NTILE) stage((t + 1) * TK, (t + 1) & 1);
    qk(t & 1, Sa, Cm);
    finish(t & 1, Sa);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if (NFULL < NTILE && NFULL > 0) {  // ragged last tile (its DMA was issued by the previous iteration)
    qk(NFULL & 1, Sa, Cm);
    s3_mask(Sa, NFULL * TK, Ns, g);
    finish(NFULL & 1, Sa);
  }
  float lt[2], mx[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    lt[qg] = ACC ? lsum[qg] : L[qg][0];  // every D row is the full sum over the 32 keys of each MFMA
    mx[qg] = -Cm[qg][0];
  }
  if (__any(!(lt[0] <= kShiftSumThr) || !(lt[1] <= kShiftSumThr))) attn_exact_q3<QK32>(p, kp, vp, qf, qreg, O, lt, mx, g, r16);
  if constexpr (TRAIN) attn_train_epilogue_q(p, O, lt, mx, bh, q0, g, r16);
  else attn_epilogue_q<float>(p, O, lt, b, hh, q0, g, r16);
}

static int s3_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_split3_kv(const float* kv, const float* vt, void* img, int B, int H, int Ns, mhada_stream_t s_) {
  if (!kv || !vt || !img || B <= 0 || H <= 0 || Ns <= 0) return fail("mhada_split3_kv: bad args");
  const long long bhn = (long long)B * H;
  if (bhn > 65535) return fail("mhada_split3_kv: B * H > 65535");
  const int ldt = (Ns + 63) / 64 * 64;
  hipLaunchKernelGGL(split3_kv_kernel, dim3(ldt / 64, (unsigned)bhn), dim3(256), 0, (hipStream_t)s_, kv, vt,
                     reinterpret_cast<bf16*>(img), Ns, ldt);
  return check_launch("mhada_split3_kv");
}

extern "C" int mhada_kv_proj_split3(const float* fs, const float* mu_s, const float* wkv, const float* bkv, void* img,
                                    int B, int H, int Ns, mhada_stream_t s_) {
  if (!fs || !mu_s || !wkv || !bkv || !img || B <= 0 || H <= 0 || Ns <= 0) return fail("mhada_kv_proj_split3: bad args");
  const long long bhn = (long long)B * H;
  if (bhn > 65535) return fail("mhada_kv_proj_split3: B * H > 65535");
  const int ldt = (Ns + 63) / 64 * 64;
  hipLaunchKernelGGL(kv_proj_s3_kernel, dim3(ldt / 64, (unsigned)bhn), dim3(256), 0, (hipStream_t)s_, fs, mu_s, wkv, bkv,
                     reinterpret_cast<bf16*>(img), H, Ns, ldt);
  return check_launch("mhada_kv_proj_split3");
}

extern "C" int mhada_attn_split3(const float* q, const void* img, const float* fcs, const float* fcs_mu,
                                 const float* fcs_rstd, const float* v_mu, float* out, int B, int H, int Nc, int Ns,
                                 mhada_stream_t s_) {
  if (!q || !img || !fcs || !fcs_mu || !fcs_rstd || !v_mu || !out || B <= 0 || H <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_split3: bad args");
  AttnP p = {};
  p.q = q; p.kv = img; p.vt = img; p.fcs = fcs; p.fcs_mu = fcs_mu; p.fcs_rstd = fcs_rstd; p.v_mu = v_mu;
  p.out = out; p.B = B; p.H = H; p.Nc = Nc; p.Ns = Ns;
  p.ldt = (Ns + 63) / 64 * 64;
  if (384LL * p.ldt >= (1LL << 31)) return fail("mhada_attn_split3: Ns too large for 32-bit plane offsets");
  // waves per block as mhada_attn: tuning attn_waves, 0 = 8, or 4 when the 8-wave grid has fewer
  // blocks than CUs
  int nw = tuning().attn_waves;
  if (nw == 0) nw = (long long)B * H * ((Nc + 255) / 256) < s3_num_cus() ? 4 : 8;
  p.nqb = (Nc + 32 * nw - 1) / (32 * nw);
  const long long nblk = (long long)B * H * p.nqb;
  if (nblk > (1LL << 31) - 1) return fail("mhada_attn_split3: grid too large");
  p.nblk = (int)nblk;
  const hipStream_t s = (hipStream_t)s_;
  if (nw == 8) hipLaunchKernelGGL((attn_s3_kernel<8, false, false, 0, 1>), dim3(p.nblk), dim3(512), 0, s, p);
  else hipLaunchKernelGGL((attn_s3_kernel<4, false, false, 0, 1>), dim3(p.nblk), dim3(256), 0, s, p);
  return check_launch("mhada_attn_split3");
}

// Training forward as SPLIT3 products (the contract of mhada_attn_train_fwd_vt, attn.hip): q, x
// [BH][Nc][64]; k, v [BH][Ns][64] (v centred) -> out' [BH][Nc][64], mo = [M' | E2'] [BH][Nc][128],
// lse2 [BH][Nc]; img: caller-provided workspace of BH * 576 * ceil64(Ns) bf16, filled here from k, v.
extern "C" int mhada_attn_train_fwd_split3(const float* q, const float* k, const float* v, void* img, const float* x,
                                           float* out, float* mo, float* lse, int BH, int Nc, int Ns,
                                           mhada_stream_t s_) {
  if (!q || !k || !v || !img || !x || !out || !mo || !lse || BH <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_train_fwd_split3: bad args");
  if (BH > 65535) return fail("mhada_attn_train_fwd_split3: BH > 65535");
  const hipStream_t s = (hipStream_t)s_;
  AttnP p = {};
  p.q = q; p.kv = img; p.vt = img; p.fcs = x; p.out = out; p.mo = mo; p.lse = lse;
  p.B = BH; p.H = 1; p.Nc = Nc; p.Ns = Ns; p.ldk = 64;
  p.ldt = (Ns + 63) / 64 * 64;
  if (384LL * p.ldt >= (1LL << 31)) return fail("mhada_attn_train_fwd_split3: Ns too large for 32-bit plane offsets");
  int nw = tuning().attn_waves;
  if (nw == 0) nw = (long long)BH * ((Nc + 255) / 256) < s3_num_cus() ? 4 : 8;
  p.nqb = (Nc + 32 * nw - 1) / (32 * nw);
  const long long nblk = (long long)BH * p.nqb;
  if (nblk > (1LL << 31) - 1) return fail("mhada_attn_train_fwd_split3: grid too large");
  p.nblk = (int)nblk;
  hipLaunchKernelGGL(train_s3_prep_kernel, dim3(p.ldt / 64, BH), dim3(256), 0, s, k, v, reinterpret_cast<bf16*>(img),
                     Ns, p.ldt);
  if (nw == 8) hipLaunchKernelGGL((attn_s3_kernel<8, true, true, 1>), dim3(p.nblk), dim3(512), 0, s, p);
  else hipLaunchKernelGGL((attn_s3_kernel<4, true, true, 1>), dim3(p.nblk), dim3(256), 0, s, p);
  return check_launch("mhada_attn_train_fwd_split3");
}
