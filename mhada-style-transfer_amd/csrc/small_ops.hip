// Bandwidth-bound kernels of the forward path: LayerNorm, the ViT's batch-axis attention,
// the positional-embedding resize, InstanceNorm (AdaIN) statistics, the per-block weight
// fold, the V transpose for the bf16 attention, the cosine row normalisation and the last
// (Cin -> 3) decoder convolution.  All activations are token-major.
#include "common.h"

#include <stdlib.h>

namespace mhada {

// ---------------------------------------------------------------------------------------
// LayerNorm (vit.py:54-55): one wave per row, VPL = cols/64 values per lane, two-pass in
// registers (mean, then centred sum of squares) — biased variance as nn.LayerNorm.
// ---------------------------------------------------------------------------------------
template <typename TO, int VPL, bool SPLIT = false>
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, TO* __restrict__ y,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ b, int rows, float eps) {
  constexpr int COLS = VPL * 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long long)row * COLS;
  float v[VPL];
#pragma unroll
  for (int i = 0; i < VPL / 4; ++i) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(xr + (i * 64 + lane) * 4);
    v[4 * i] = t[0]; v[4 * i + 1] = t[1]; v[4 * i + 2] = t[2]; v[4 * i + 3] = t[3];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.0f / COLS);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const float d = v[i] - mean;
    ss += d * d;
  }
  const float rstd = rsqrtf(wave_sum(ss) * (1.0f / COLS) + eps);
  TO* yr = y + (long long)row * COLS;
  const long long plane = (long long)rows * COLS;
#pragma unroll
  for (int i = 0; i < VPL / 4; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = (i * 64 + lane) * 4 + e;
      const float val = (v[4 * i + e] - mean) * rstd * g[c] + b[c];
      if constexpr (SPLIT) {  // three bf16 planes: val = p0 + p1 + p2 to 2^-25 (the SPLIT3 GEMM operand)
        const bf16 p0 = (bf16)val;
        const float r1 = val - (float)p0;
        const bf16 p1 = (bf16)r1;
        yr[c] = p0;
        yr[plane + c] = p1;
        yr[2 * plane + c] = (bf16)(r1 - (float)p1);
      } else {
        yr[c] = from_f32<TO>(val);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Batch-axis multi-head attention of the ViT (vit.py:48,59; batch_first=False on (B,N,C)):
// one wave per (token, head); lane = feature d (head_dim 64).  L = batch size is small.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) vit_batch_attn_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                             int L, int ntok, int heads) {
  constexpr int D = 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long pair = (long long)blockIdx.x * 4 + wv;
  const int C = heads * D;
  if (pair >= (long long)ntok * heads) return;
  const int n = (int)(pair / heads), hh = (int)(pair - (long long)n * heads);
  const float scale = 0.125f;                            // 1/sqrt(64)
  const long long row_stride = (long long)ntok * 3 * C;  // between sequence (= batch) positions
  const T* base = qkv + (long long)n * 3 * C + hh * D + lane;
  for (int i = 0; i < L; ++i) {
    const float qi = to_f32<T>(base[i * row_stride]) * scale;
    float m = -INFINITY, l = 0.f, o = 0.f;  // online softmax over the L keys
    for (int j = 0; j < L; ++j) {
      const float sj = wave_sum(qi * to_f32<T>(base[j * row_stride + C]));
      const float mn = fmaxf(m, sj);
      const float a = __expf(m - mn), p = __expf(sj - mn);
      l = l * a + p;
      o = o * a + p * to_f32<T>(base[j * row_stride + 2 * C]);
      m = mn;
    }
    out[((long long)i * ntok + n) * C + hh * D + lane] = from_f32<T>(o / l);
  }
}

// Vectorised small-batch form (L <= 8): a group of 8 lanes owns one (token, head), lane = 8
// consecutive features (one 16-B bf16 / two 16-B fp32 loads per q/k/v row instead of 2-4-byte
// per-lane loads); the L x L dot products are 8-lane shuffle reductions, the softmax and PV
// are lane-local.
// LMAX (4 | 8) sizes the per-lane q / k / v rows: at L <= 4 (1024^2 batch 4) the kernel keeps
// 96 instead of 192 of them live, so twice the waves hide the loads.
template <typename T, int LMAX>
__global__ void __launch_bounds__(256) vit_batch_attn_vec_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                                 int L, int ntok, int heads) {
  constexpr int D = 64, E = 8;
  const int g8 = threadIdx.x & 7;
  const long long pair = (long long)blockIdx.x * 32 + (threadIdx.x >> 3);
  const bool valid = pair < (long long)ntok * heads;
  const long long pp = valid ? pair : 0;
  const int C = heads * D;
  const int n = (int)(pp / heads), hh = (int)(pp - (long long)n * heads);
  const long long row_stride = (long long)ntok * 3 * C;
  const T* base = qkv + (long long)n * 3 * C + hh * D + g8 * E;
  auto load8 = [&](const T* p, float (&f)[E]) {
    if constexpr (sizeof(T) == 2) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
      for (int e = 0; e < E; ++e) f[e] = (float)v[e];
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = a[e];
        f[4 + e] = b[e];
      }
    }
  };
  float q[LMAX][E], k[LMAX][E], v[LMAX][E];
#pragma unroll
  for (int i = 0; i < LMAX; ++i) {
    if (i < L) {
      load8(base + i * row_stride, q[i]);
      load8(base + i * row_stride + C, k[i]);
      load8(base + i * row_stride + 2 * C, v[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < LMAX; ++i) {
    if (i >= L) break;
    float sc[LMAX];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < LMAX; ++j) {
      if (j < L) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) d = fmaf(q[i][e], k[j][e], d);
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) d += __shfl_xor(d, o, 64);
        sc[j] = d * 0.125f;  // 1/sqrt(64)
        m = fmaxf(m, sc[j]);
      }
    }
    float l = 0.f, o8[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o8[e] = 0.f;
#pragma unroll
    for (int j = 0; j < LMAX; ++j) {
      if (j < L) {
        const float p = __expf(sc[j] - m);
        l += p;
#pragma unroll
        for (int e = 0; e < E; ++e) o8[e] = fmaf(p, v[j][e], o8[e]);
      }
    }
    const float inv = 1.f / l;
    if (valid) {
      T* dst = out + ((long long)i * ntok + n) * C + hh * D + g8 * E;
      if constexpr (sizeof(T) == 2) {
        bf16x8 r;
#pragma unroll
        for (int e = 0; e < E; ++e) r[e] = (bf16)(o8[e] * inv);
        *reinterpret_cast<bf16x8*>(dst) = r;
      } else {
        *reinterpret_cast<f32x4*>(dst) = f32x4{o8[0] * inv, o8[1] * inv, o8[2] * inv, o8[3] * inv};
        *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o8[4] * inv, o8[5] * inv, o8[6] * inv, o8[7] * inv};
      }
    }
  }
}

// L = 1 (one image per call: the video path's per-frame encoder): the softmax over one key is
// exactly 1, so the attention output is V bit for bit; a strided 16-B row copy of the V slice.
__global__ void __launch_bounds__(256) vit_batch_copy_v_kernel(const uint4* __restrict__ qkv, uint4* __restrict__ out,
                                                               int ntok, int row16) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)ntok * row16) return;
  const long long n = idx / row16;
  const int c = (int)(idx - n * row16);
  out[n * row16 + c] = qkv[n * 3 * row16 + 2 * row16 + c];
}

// Small-batch form (L <= 8, every bench/training config): each (token, head) reads q, k, v
// once — q/k staged in LDS, v in registers — and the L x L scores are computed in parallel with
// lane = (i, j); the softmax over j is an 8-lane group reduction.
template <typename T>
__global__ void __launch_bounds__(256) vit_batch_attn_small_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                                   int L, int ntok, int heads) {
  constexpr int D = 64;
  __shared__ float sq[4][8][D + 1];
  __shared__ float sk[4][8][D + 1];
  __shared__ float sp[4][8][8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long pair = (long long)blockIdx.x * 4 + wv;
  const bool valid = pair < (long long)ntok * heads;
  const int C = heads * D;
  const long long pp = valid ? pair : 0;
  const int n = (int)(pp / heads), hh = (int)(pp - (long long)n * heads);
  const long long row_stride = (long long)ntok * 3 * C;
  const T* base = qkv + (long long)n * 3 * C + hh * D + lane;
  float vr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < L) {
      sq[wv][i][lane] = to_f32<T>(base[i * row_stride]) * 0.125f;  // 1/sqrt(64)
      sk[wv][i][lane] = to_f32<T>(base[i * row_stride + C]);
      vr[i] = to_f32<T>(base[i * row_stride + 2 * C]);
    } else {
      vr[i] = 0.f;
    }
  }
  __syncthreads();
  const int i = lane >> 3, j = lane & 7;
  float s = -INFINITY;
  if (i < L && j < L) {
    s = 0.f;
#pragma unroll 16
    for (int d = 0; d < D; ++d) s = fmaf(sq[wv][i][d], sk[wv][j][d], s);
  }
  float m = s;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float e = (i < L && j < L) ? __expf(s - m) : 0.f;
  float sum = e;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o, 64);
  sp[wv][i][j] = e / sum;
  __syncthreads();
  if (!valid) return;
  for (int r = 0; r < L; ++r) {
    float o = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) o = fmaf(sp[wv][r][c], vr[c], o);
    out[((long long)r * ntok + n) * C + hh * D + lane] = from_f32<T>(o);
  }
}

// ---------------------------------------------------------------------------------------
// PosEmbedding resize (vit.py:91-92) to token-major [oh*ow][C]
// ---------------------------------------------------------------------------------------
__global__ void pos_embed_kernel(const float* __restrict__ pos, float* __restrict__ out, int C, int bh,
                                 int bw, int oh, int ow) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)oh * ow * C) return;
  const int c = (int)(idx % C);
  const int tkn = (int)(idx / C);
  const int oy = tkn / ow, ox = tkn - (tkn / ow) * ow;
  const float* pc = pos + (long long)c * bh * bw;
  if (oh == bh && ow == bw) {
    out[idx] = pc[oy * bw + ox];
    return;
  }
  const float shy = (float)bh / (float)oh, shx = (float)bw / (float)ow;
  const float sy = fmaxf(shy * ((float)oy + 0.5f) - 0.5f, 0.f);
  const float sx = fmaxf(shx * ((float)ox + 0.5f) - 0.5f, 0.f);
  const int y0 = min((int)sy, bh - 1), x0 = min((int)sx, bw - 1);
  const int y1 = y0 + (y0 < bh - 1 ? 1 : 0), x1 = x0 + (x0 < bw - 1 ? 1 : 0);
  const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  out[idx] = ly0 * (lx0 * pc[y0 * bw + x0] + lx1 * pc[y0 * bw + x1]) +
             ly1 * (lx0 * pc[y1 * bw + x0] + lx1 * pc[y1 * bw + x1]);
}

// ---------------------------------------------------------------------------------------
// InstanceNorm statistics: partial sums in fp64 per (split, b, c), then a finalize pass.
// grid (C/64, B, splits), 256 threads = 64 channels x 4 row phases (coalesced 256-B rows).
// ---------------------------------------------------------------------------------------
// One block = 64 channels x one split of the token range; thread (quad, ph) accumulates channels
// 4*quad..4*quad+3 of every 16th row (16-B loads: 16 threads read one row's 256-B channel block,
// a wave 4 rows), in fp64; the 16 row phases reduce through LDS in a fixed order.
__global__ void __launch_bounds__(256) in_partial_kernel(const float* __restrict__ x, double* __restrict__ work,
                                                         int B, int N, int C, int splits) {
  __shared__ double red[2][16][65];
  const int quad = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + 4 * quad;
  const int b = blockIdx.y, s = blockIdx.z;
  const int per = (N + splits - 1) / splits;
  const int r0 = s * per, r1 = min(N, r0 + per);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (c0 < C) {  // C % 4 == 0 (checked by the entry point)
    const float* xb = x + (long long)b * N * C + c0;
#pragma unroll 4
    for (int r = r0 + ph; r < r1; r += 16) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xb + (long long)r * C);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double d = (double)v[e];
        s1[e] += d;
        s2[e] += d * d;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ph][4 * quad + e] = s1[e];
    red[1][ph][4 * quad + e] = s2[e];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int t = threadIdx.x & 63, which = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + t;
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += red[which][k][t];
    if (c < C) work[(((long long)s * B + b) * C + c) * 2 + which] = a;
  }
}

// 16 outputs x 16 split phases per block: each thread sums every 16th split in order, the 16
// partials are added in a fixed order (deterministic; a split-serial loop per output was
// latency bound at B = 1, where the partial kernel uses 256 splits).
__global__ void __launch_bounds__(256) in_finalize_kernel(const double* __restrict__ work, float* __restrict__ mu,
                                                          float* __restrict__ rstd, int B, int N, int C, int splits,
                                                          float eps) {
  __shared__ double red[2][16][17];
  const int o = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int idx = blockIdx.x * 16 + o;
  double a = 0.0, q = 0.0;
  if (idx < B * C) {
    for (int s = ph; s < splits; s += 16) {
      a += work[((long long)s * B * C + idx) * 2];
      q += work[((long long)s * B * C + idx) * 2 + 1];
    }
  }
  red[0][ph][o] = a;
  red[1][ph][o] = q;
  __syncthreads();
  if (ph == 0 && idx < B * C) {
    double sa = 0.0, sq = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      sa += red[0][k][o];
      sq += red[1][k][o];
    }
    const double mean = sa / N;
    double var = sq / N - mean * mean;
    if (var < 0.0) var = 0.0;
    mu[idx] = (float)mean;
    rstd[idx] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// ---------------------------------------------------------------------------------------
// Weight fold for one AdaAttnMultiHead block, grid B*H, 256 threads.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) fold_kernel(const float* __restrict__ wf, const float* __restrict__ wg,
                                                   const float* __restrict__ wh, const float* __restrict__ bg,
                                                   const float* __restrict__ bh, const float* __restrict__ rstd_c,
                                                   const float* __restrict__ mu_s, const float* __restrict__ rstd_s,
                                                   T* __restrict__ wq, T* __restrict__ wkv, float* __restrict__ bkv,
                                                   float* __restrict__ v_mu, float kscale, int H) {
  constexpr int D = 64;
  const int b = blockIdx.x / H, hh = blockIdx.x - (blockIdx.x / H) * H;
  const int C = H * D;
  const float* rc = rstd_c + (long long)b * C + hh * D;
  const float* rs = rstd_s + (long long)b * C + hh * D;
  const float* ms = mu_s + (long long)b * C + hh * D;
  const float* Wf = wf + (long long)hh * D * D;
  const float* Wg = wg + (long long)hh * D * D;
  const float* Wh = wh + (long long)hh * D * D;
  T* oq = wq + (long long)blockIdx.x * D * D;
  T* okv = wkv + (long long)blockIdx.x * 2 * D * D;
  for (int i = threadIdx.x; i < D * D; i += 256) {
    const int c = i & (D - 1);
    oq[i] = from_f32<T>(Wf[i] * rc[c]);
    okv[i] = from_f32<T>(Wg[i] * rs[c] * kscale);
    okv[D * D + i] = from_f32<T>(Wh[i]);
  }
  if (threadIdx.x < D) {
    const int o = threadIdx.x;
    float acc = bh[hh * D + o];
    for (int c = 0; c < D; ++c) acc += Wh[o * D + c] * ms[c];
    v_mu[(long long)b * C + hh * D + o] = acc;
    if (b == 0) {
      bkv[hh * 2 * D + o] = bg[hh * D + o] * kscale;
      bkv[hh * 2 * D + D + o] = 0.f;
    }
  }
}

// ---------------------------------------------------------------------------------------
// V transpose for the bf16 attention: vt[bh][o][pos(n)] = V'[n][o], vt[bh][64+o][pos(n)] = V'[n][o]^2
// (row stride ldt = Ns rounded up to 64, padding zero-filled).  64x64 tiles through LDS.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) transpose_v_kernel(const T* __restrict__ kv, T* __restrict__ vt, int Ns,
                                                          int ldt) {
  __shared__ float tile[64][65];
  const int bh = blockIdx.y, n0 = blockIdx.x * 64;
  const T* src = kv + (long long)bh * Ns * 128 + 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int n = i >> 6, o = i & 63;
    tile[n][o] = (n0 + n < Ns) ? to_f32<T>(src[(long long)(n0 + n) * 128 + o]) : 0.f;
  }
  __syncthreads();
  T* dst = vt + (long long)bh * 128 * ldt + n0;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int o = i >> 6, pos = i & 63;
    // bf16: key stored at position pos = swap bits 2 and 3 inside each group of 16 (an
    // involution), so the 8 keys {4h..4h+3, 8+4h..8+4h+3} one 32x32x16 lane half needs are
    // contiguous.  fp32 (32x32x2, one key per MFMA): natural order — a lane's keys 8q+4h..+3
    // are already contiguous (one 16-B read per 4 MFMAs).
    const int n = sizeof(T) == 2 ? ((pos & ~12) | ((pos & 4) << 1) | ((pos & 8) >> 1)) : pos;
    const float v = tile[n][o];
    dst[(long long)o * ldt + pos] = from_f32<T>(v);
    dst[(long long)(64 + o) * ldt + pos] = from_f32<T>(v * v);
  }
}

// ---------------------------------------------------------------------------------------
// Cosine activation prep (adaDecoder.py:30-32): L2-normalise 64-wide rows in place.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) rownorm_kernel(T* __restrict__ x, long long rows, int ld) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  T* r = x + row * ld;
  const float v = to_f32<T>(r[lane]);
  const float n = sqrtf(wave_sum(v * v));
  r[lane] = from_f32<T>(v / n);
}

// ---------------------------------------------------------------------------------------
// Last decoder layer: ReflectionPad(1) + conv3x3 Cin->3 + bias + ReLU, NHWC in, NCHW fp32 out.
// One thread per output pixel (adjacent lanes = adjacent pixels, each reading its own
// contiguous Cin-vector).  Weights are indexed only by loop counters and kernel arguments,
// so they are wave-uniform: the compiler fetches them with scalar loads into SGPRs and the
// FMAs take them as scalar operands (no LDS broadcast traffic).
// ---------------------------------------------------------------------------------------
template <typename T, int CIN>
__global__ void __launch_bounds__(256) conv_out3_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        int B, int H, int W, int clamp255) {
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (long long)B * H * W) return;
  const int b = (int)(pix / ((long long)H * W));
  const int rem = (int)(pix - (long long)b * H * W);
  const int yy = rem / W, xx = rem - (rem / W) * W;
  float a0 = bias[0], a1 = bias[1], a2 = bias[2];
  constexpr int EV = 16 / sizeof(T);
#pragma unroll 1
  for (int tap = 0; tap < 9; ++tap) {
    int Y = yy + tap / 3 - 1, X = xx + tap % 3 - 1;
    Y = Y < 0 ? -Y : (Y >= H ? 2 * H - 2 - Y : Y);
    X = X < 0 ? -X : (X >= W ? 2 * W - 2 - X : X);
    const T* px = x + (((long long)b * H + Y) * W + X) * CIN;
    const float* wt = w + tap * CIN * 3;  // [tap][cin][out]
#pragma unroll
    for (int c = 0; c < CIN; c += EV) {
      const typename Vec16<T>::type v = *reinterpret_cast<const typename Vec16<T>::type*>(px + c);
#pragma unroll
      for (int e = 0; e < EV; ++e) {
        const float f = (float)v[e];
        a0 = fmaf(f, wt[(c + e) * 3 + 0], a0);
        a1 = fmaf(f, wt[(c + e) * 3 + 1], a1);
        a2 = fmaf(f, wt[(c + e) * 3 + 2], a2);
      }
    }
  }
  a0 = fmaxf(a0, 0.f); a1 = fmaxf(a1, 0.f); a2 = fmaxf(a2, 0.f);
  if (clamp255) { a0 = fminf(a0, 255.f); a1 = fminf(a1, 255.f); a2 = fminf(a2, 255.f); }
  const long long plane = (long long)H * W;
  float* yb = y + (long long)b * 3 * plane + (long long)yy * W + xx;
  yb[0] = a0;
  yb[plane] = a1;
  yb[2 * plane] = a2;
}

// ---------------------------------------------------------------------------------------
// bf16 form of the last decoder layer on MFMA (v_mfma_f32_16x16x32_bf16).  A workgroup walks a
// strip of kOut3Rows 4-row x 64-pixel output tiles (the weight fragments are loaded once per
// strip); per tile the reflect-padded 6 x 66-pixel input halo is staged in LDS (double
// buffered, the next halo in flight in registers during the MFMAs) (pixel rows padded to CIN+8 elements: the 16-lane groups' 16-B reads hit distinct bank
// slots) and read 9x (one per tap) from there.  Per 16 output pixels the wave accumulates
// D^T (16 out-channels x 16 pixels) = W^T (16 x 32 cin) . X^T (32 cin x 16 pixels) over the 9
// taps x CIN/32 channel chunks; out-channels 3..15 are zero rows of W^T, so lanes 0-15 end
// up holding channels 0-2 of pixel (lane) and store 16 consecutive floats per channel plane.
// (The per-pixel VALU kernel above re-reads each input pixel 9x from L1/L2 and spends 1728
// FMAs + 576 conversions per pixel: ~8x slower at 1024^2.)
// ---------------------------------------------------------------------------------------
constexpr int kOut3Rows = 8;    // row tiles per workgroup strip (fp32 kernel)
constexpr int kOut3RowsM = 16;  // bf16 MFMA kernel: longer strips amortise its weight-fragment prologue

template <int CIN, int CC>
__global__ void __launch_bounds__(256, 2) conv_out3_mfma_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ bias, float* __restrict__ y,
                                                             int H, int W, int tiles_x, int strips_y, int clamp255) {
  // the halo is staged in CC-channel chunks (CC = 32: 31 KiB per buffer, two workgroups per CU;
  // the whole 64-channel halo double-buffered took 114 KiB, one workgroup per CU)
  constexpr int TR = 4, TC = 64, HR = TR + 2, HC = TC + 2, LP = CC + 8, NH = CIN / 32, NCK = CIN / CC;
  constexpr int HPC = CC / 32;  // 32-channel MFMA steps per chunk
  constexpr int CH = CC / 8, NCH = HR * HC * CH, PER = (NCH + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16 tile[2][HR * HC * LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bt = blockIdx.x, tx = bt % tiles_x, sy = (bt / tiles_x) % strips_y, b = bt / (tiles_x * strips_y);
  const int x0 = tx * TC, ys = sy * TR * kOut3RowsM;
  const bf16* xb = x + (long long)b * H * W * CIN;
  // A = W^T fragments (loaded once per block, amortised over the strip's kOut3RowsM tiles):
  // row n = lane & 15 (out channel; rows 3..15 zero), k = 32*hc + 8*(lane >> 4) + j
  // the 9 x CIN x 3 weights pass through LDS (coalesced loads into the second halo buffer, free
  // until step 0's commit): per lane 144 scattered 4-B loads with 13 of 16 lanes idle were a
  // measurable share of each strip
  bf16x8 wa[9][NH];
  const int n = lane & 15, kg = lane >> 4;
  {
    static_assert(9 * CIN * 3 * 4 <= (int)sizeof(tile[1]), "weights fit the halo buffer");
    float* sw = reinterpret_cast<float*>(tile[1]);
    for (int i = tid; i < 9 * CIN * 3; i += 256) sw[i] = w[i];
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int hc = 0; hc < NH; ++hc)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          wa[tap][hc][j] = (bf16)(n < 3 ? sw[(tap * CIN + 32 * hc + 8 * kg + j) * 3 + n] : 0.f);
  }
  const float bo[3] = {bias[0], bias[1], bias[2]};
  // halo chunk (rows y0-1 .. y0+4, channels ck*CC ..; reflect-padded, clamped past the image
  // edge) into registers; written to LDS after the current chunk's MFMAs
  // two register sets: the loads of step s + 2 are issued at step s (set s & 1), so every chunk has
  // two steps of MFMA work to arrive in (one step did not cover the load latency: 2.7 TB/s)
  bf16x8 sts[2][PER];
  auto fetch = [&](bf16x8 (&st)[PER], int y0, int ck) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = min(tid + 256 * i, NCH - 1);
      const int pix = c / CH, ch = c - pix * CH;
      const int r = pix / HC, cc = pix - r * HC;
      int Y = y0 - 1 + r, X = x0 - 1 + cc;
      Y = Y < 0 ? -Y : (Y >= H ? 2 * H - 2 - Y : Y);
      X = X < 0 ? -X : (X >= W ? 2 * W - 2 - X : X);
      Y = min(max(Y, 0), H - 1);
      X = min(max(X, 0), W - 1);
      st[i] = *reinterpret_cast<const bf16x8*>(xb + ((long long)Y * W + X) * CIN + ck * CC + ch * 8);
    }
  };
  auto commit = [&](const bf16x8 (&st)[PER], bf16* t) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + 256 * i;
      if (c < NCH) {
        const int pix = c / CH, ch = c - pix * CH;
        *reinterpret_cast<bf16x8*>(t + pix * LP + ch * 8) = st[i];
      }
    }
  };
  const int nt = min(kOut3RowsM, (H - ys + TR - 1) / TR);
  // step s = (tile r, chunk ck), s = NCK r + ck; rows of step s: ys + (s / NCK) TR, clamped past
  // the strip.  NCK == 2: the register set alternates with the chunk index (compile-time); NCK == 1
  // (CIN = 32): one set, loaded one step ahead
  constexpr bool TWO = NCK == 2;
  auto step_y = [&](int s2) { return ys + min(s2 / NCK, nt - 1) * TR; };
  fetch(sts[0], ys, 0);
  commit(sts[0], tile[0]);
  if constexpr (TWO) fetch(sts[1], step_y(1), 1);
  __syncthreads();
  int buf = 0;
  for (int r = 0; r < nt; ++r) {
    const int yy = ys + r * TR + wave;
    f32x4 acc[TC / 16];
#pragma unroll
    for (int g = 0; g < TC / 16; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ck = 0; ck < NCK; ++ck) {
      const bf16* t = tile[buf];
      const int s2 = r * NCK + ck;
      const bool more = s2 + 1 < nt * NCK;
      if constexpr (TWO) {
        if (s2 + 2 < nt * NCK) fetch(sts[ck], step_y(s2 + 2), ck);  // step s + 2 has this step's chunk index
      } else {
        if (more) fetch(sts[0], step_y(s2 + 1), 0);
      }
#pragma unroll
      for (int g = 0; g < TC / 16; ++g) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const bf16* px = t + ((wave + tap / 3) * HC + 16 * g + (lane & 15) + tap % 3) * LP + 8 * kg;
#pragma unroll
          for (int hc = 0; hc < HPC; ++hc)
            acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[tap][ck * HPC + hc],
                                                             *reinterpret_cast<const bf16x8*>(px + 32 * hc), acc[g],
                                                             0, 0, 0);
        }
      }
      if (ck == NCK - 1) {
#pragma unroll
        for (int g = 0; g < TC / 16; ++g) {
          const int xx = x0 + 16 * g + lane;
          if (lane < 16 && yy < H && xx < W) {
#pragma unroll
            for (int o = 0; o < 3; ++o) {
              float v = fmaxf(acc[g][o] + bo[o], 0.f);
              if (clamp255) v = fminf(v, 255.f);
              y[(((long long)b * 3 + o) * H + yy) * W + xx] = v;
            }
          }
        }
      }
      if (more) commit(sts[TWO ? ck ^ 1 : 0], tile[buf ^ 1]);
      __syncthreads();
      buf ^= 1;
    }
  }
}

// ---------------------------------------------------------------------------------------
// fp32 form of the last decoder layer: the same strip of 4-row x 64-pixel tiles, but VALU
// (fp32 MFMA would spend 16/3 of the FLOPs on zero weight rows at 1/16 of the bf16 rate): the
// reflect-padded 6 x 66-pixel halo is staged in LDS in CC-channel chunks (double buffered, the
// next chunk in flight in registers during this chunk's FMAs); lane = output pixel, wave =
// output row, weights wave-uniform (scalar operands).  The per-pixel kernel above reads every
// input pixel 9x as lane-strided 16-B loads (one cache line per lane per load) and is
// load-issue bound: 744 -> 219 us at 512^2 B8 with CC = 16 (63 KiB of LDS, two workgroups per
// CU; CC = 32: 306 us at one workgroup per CU, CC = 8: 329 us).
// ---------------------------------------------------------------------------------------
template <int CIN, int CC>
__global__ void __launch_bounds__(256) conv_out3_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float* __restrict__ y,
                                                            int H, int W, int tiles_x, int strips_y, int clamp255) {
  constexpr int TR = 4, TC = 64, HR = TR + 2, HC = TC + 2, LP = CC + 4, NCK = CIN / CC;
  constexpr int Q = CC / 4, NQ = HR * HC * Q, PER = (NQ + 255) / 256;
  __shared__ __attribute__((aligned(16))) float tile[2][HR * HC * LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bt = blockIdx.x, tx = bt % tiles_x, sy = (bt / tiles_x) % strips_y, b = bt / (tiles_x * strips_y);
  const int x0 = tx * TC, ys = sy * TR * kOut3Rows;
  const float* xb = x + (long long)b * H * W * CIN;
  f32x4 st[PER];
  // halo chunk (rows y0-1 .. y0+4, channels ck*CC ..), reflect-padded, clamped past the image
  auto fetch = [&](int y0, int ck) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = min(tid + 256 * i, NQ - 1);
      const int pix = c / Q, q = c - pix * Q;
      const int r = pix / HC, cc = pix - r * HC;
      int Y = y0 - 1 + r, X = x0 - 1 + cc;
      Y = Y < 0 ? -Y : (Y >= H ? 2 * H - 2 - Y : Y);
      X = X < 0 ? -X : (X >= W ? 2 * W - 2 - X : X);
      Y = min(max(Y, 0), H - 1);
      X = min(max(X, 0), W - 1);
      st[i] = *reinterpret_cast<const f32x4*>(xb + ((long long)Y * W + X) * CIN + ck * CC + 4 * q);
    }
  };
  auto commit = [&](float* t) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + 256 * i;
      if (c < NQ) {
        const int pix = c / Q, q = c - pix * Q;
        *reinterpret_cast<f32x4*>(t + pix * LP + 4 * q) = st[i];
      }
    }
  };
  const int nt = min(kOut3Rows, (H - ys + TR - 1) / TR);
  const int steps = nt * NCK;
  fetch(ys, 0);
  commit(tile[0]);
  __syncthreads();
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int s = 0; s < steps; ++s) {
    const int r = s / NCK, ck = s - r * NCK;
    const float* t = tile[s & 1];
    if (s + 1 < steps) fetch(ys + ((s + 1) / NCK) * TR, (s + 1) % NCK);
    const float* wt = w + ck * CC * 3;  // [tap][cin][out]
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float* px = t + ((wave + tap / 3) * HC + lane + tap % 3) * LP;
      const float* wtap = wt + tap * CIN * 3;
#pragma unroll
      for (int c = 0; c < CC; c += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(px + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a0 = fmaf(v[e], wtap[(c + e) * 3 + 0], a0);
          a1 = fmaf(v[e], wtap[(c + e) * 3 + 1], a1);
          a2 = fmaf(v[e], wtap[(c + e) * 3 + 2], a2);
        }
      }
    }
    if (ck == NCK - 1) {
      const int yy = ys + r * TR + wave, xx = x0 + lane;
      if (yy < H && xx < W) {
        float o[3] = {fmaxf(a0 + bias[0], 0.f), fmaxf(a1 + bias[1], 0.f), fmaxf(a2 + bias[2], 0.f)};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (clamp255) o[k] = fminf(o[k], 255.f);
          y[(((long long)b * 3 + k) * H + yy) * W + xx] = o[k];
        }
      }
      a0 = a1 = a2 = 0.f;
    }
    if (s + 1 < steps) commit(tile[(s + 1) & 1]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Bilinear x2 upsample on NHWC (F.interpolate(scale_factor=2, bilinear, align_corners=False),
// conv.py:71): one thread per (output pixel, 8-channel group), fp32 blend in PyTorch's order.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) upsample2x_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H,
                                                         int W, int C) {
  const int G = C / 8;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)B * 4 * H * W * G;
  if (idx >= total) return;
  const int g = (int)(idx % G);
  long long pix = idx / G;
  const int Wo = 2 * W, Ho = 2 * H;
  const int X = (int)(pix % Wo);
  pix /= Wo;
  const int Y = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  const float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.f);
  const float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.f);
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const T* base = x + (long long)b * H * W * C + g * 8;
  const T* p00 = base + ((long long)y0 * W + x0) * C;
  const T* p01 = base + ((long long)y0 * W + x1) * C;
  const T* p10 = base + ((long long)y1 * W + x0) * C;
  const T* p11 = base + ((long long)y1 * W + x1) * C;
  T* out = y + (((long long)b * Ho + Y) * Wo + X) * C + g * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = bilerp(ly0, ly1, lx0, lx1, to_f32<T>(p00[e]), to_f32<T>(p01[e]), to_f32<T>(p10[e]),
                           to_f32<T>(p11[e]));
    out[e] = from_f32<T>(v);
  }
}

// 16-B vector form (round 5) for 16-B aligned tensors: the same thread mapping, coordinates,
// weights and blend expression as upsample2x_kernel (bit-identical), with each tap's 8 channels
// read and the output written as whole 16-B vectors.  The fp32 path and unaligned views use it;
// bf16 takes upsample2x_quad_kernel (2 x 2 output blocks, compile-time window indexing), which
// measured faster (mhada_upsample2x).  An earlier 2 x 2-block form with runtime window indexing
// measured 1.1-1.6x SLOWER than this kernel (profiles/r05_prof_bench_per_config.txt).
template <typename T>
__global__ void __launch_bounds__(256) upsample2x_vec_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H,
                                                             int W, int C, int gshift) {
  // one 16-B output vector per thread, consecutive lanes = consecutive vectors of one output row
  // (fully coalesced stores); the row (b, Y) comes from blockIdx.y, so the per-thread index math
  // is one shift (or one 32-bit division) instead of three 64-bit divisions
  typedef typename Vec16<T>::type V;
  constexpr int N = Vec16<T>::N;
  const int G = C / N;  // vectors per pixel
  const int Wo = 2 * W, Ho = 2 * H, rows = B * Ho;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Wo * G) return;
  const int X = gshift >= 0 ? i >> gshift : i / G;
  const int gv = i - X * G;
  const float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.f);
  const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
  for (int row = blockIdx.y; row < rows; row += gridDim.y) {
    const int b = row / Ho, Y = row - b * Ho;
    const float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.f);
    const int y0 = (int)sy, y1 = y0 + (y0 < H - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
    const T* base = x + (long long)b * H * W * C + gv * N;
    const V a00 = *reinterpret_cast<const V*>(base + ((long long)y0 * W + x0) * C);
    const V a01 = *reinterpret_cast<const V*>(base + ((long long)y0 * W + x1) * C);
    const V a10 = *reinterpret_cast<const V*>(base + ((long long)y1 * W + x0) * C);
    const V a11 = *reinterpret_cast<const V*>(base + ((long long)y1 * W + x1) * C);
    V o;
#pragma unroll
    for (int e = 0; e < N; ++e)
      o[e] = from_f32<T>(bilerp(ly0, ly1, lx0, lx1, to_f32<T>(a00[e]), to_f32<T>(a01[e]), to_f32<T>(a10[e]),
                                to_f32<T>(a11[e])));
    *reinterpret_cast<V*>(y + ((long long)row * Wo + X) * C + gv * N) = o;
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// fp32 [n] -> three bf16 planes [3][n] (p0 = bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 - p1), the
// SPLIT3 GEMM operand); four elements per thread, n % 4 == 0, 16-B aligned.
__global__ void __launch_bounds__(256) split3_rows_kernel(const float* __restrict__ x, bf16* __restrict__ y,
                                                          long long n) {
  const long long i = 4 * ((long long)blockIdx.x * 256 + threadIdx.x);
  if (i >= n) return;
  const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
  bf16x4 a, b, c;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = (bf16)v[e];
    const float r = v[e] - (float)a[e];
    b[e] = (bf16)r;
    c[e] = (bf16)(r - (float)b[e]);
  }
  *reinterpret_cast<bf16x4*>(y + i) = a;
  *reinterpret_cast<bf16x4*>(y + n + i) = b;
  *reinterpret_cast<bf16x4*>(y + 2 * n + i) = c;
}

// The SPLIT3 GEMM's W operand in one pass: element (n, k) of W [N][K0] (or of W^T when
// transposed, W then [K0][N]) -> its planes q0, q1, q2 at out[n][(6 (k / 64) + t) 64 + k % 64] for the
// term order t = q1, q0, q2, q0, q1, q0 (ops.split3_weight's layout).  One thread per element.
__global__ void __launch_bounds__(256) split3_weight_kernel(const float* __restrict__ w, bf16* __restrict__ out,
                                                            int N, int K0, int transposed) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * K0) return;
  const int n = (int)(i / K0), k = (int)(i - (long long)n * K0);
  const float x = transposed ? w[(long long)k * N + n] : w[i];
  const bf16 q0 = (bf16)x;
  const float r = x - (float)q0;
  const bf16 q1 = (bf16)r;
  const bf16 q2 = (bf16)(r - (float)q1);
  bf16* o = out + (long long)n * 6 * K0 + 6 * 64 * (k >> 6) + (k & 63);
  o[0] = q1;
  o[64] = q0;
  o[128] = q2;
  o[192] = q0;
  o[256] = q1;
  o[320] = q0;
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_split3_weight(const float* w, void* out, int N, int K0, int transposed, mhada_stream_t s_) {
  if (!w || !out || N <= 0 || K0 <= 0 || K0 % 64) return fail("mhada_split3_weight: bad args (K0 % 64 == 0)");
  const long long n = (long long)N * K0;
  hipLaunchKernelGGL(split3_weight_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s_, w,
                     (bf16*)out, N, K0, transposed);
  return check_launch("mhada_split3_weight");
}

extern "C" int mhada_layernorm(const float* x, void* y, int y_dtype, const float* gamma, const float* beta,
                               int rows, int cols, float eps, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!x || !y || !gamma || !beta || rows < 0 || y_dtype < MHADA_F32 || y_dtype > MHADA_BF16X3)
    return fail("mhada_layernorm: bad args");
  if (rows == 0) return MHADA_OK;
  if (!aligned16(x)) return fail("mhada_layernorm: x must be 16-byte aligned");
  const dim3 grid((rows + 3) / 4), blk(256);
#define LN_CASE(VPL)                                                                                   \
  case VPL * 64:                                                                                       \
    if (y_dtype == MHADA_F32)                                                                          \
      hipLaunchKernelGGL((layernorm_kernel<float, VPL>), grid, blk, 0, s, x, (float*)y, gamma, beta, rows, eps); \
    else if (y_dtype == MHADA_BF16X3)                                                                  \
      hipLaunchKernelGGL((layernorm_kernel<bf16, VPL, true>), grid, blk, 0, s, x, (bf16*)y, gamma, beta, rows, eps); \
    else                                                                                               \
      hipLaunchKernelGGL((layernorm_kernel<bf16, VPL>), grid, blk, 0, s, x, (bf16*)y, gamma, beta, rows, eps); \
    break;
  switch (cols) {
    LN_CASE(4)
    LN_CASE(8)
    LN_CASE(16)
    LN_CASE(32)
    default:
      return fail("mhada_layernorm: cols must be 256, 512, 1024 or 2048");
  }
#undef LN_CASE
  return check_launch("mhada_layernorm");
}

extern "C" int mhada_vit_batch_attn(const void* qkv, void* out, int dtype, int L, int ntok, int heads,
                                    int head_dim, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!qkv || !out || L <= 0 || ntok < 0 || heads <= 0) return fail("mhada_vit_batch_attn: bad args");
  if (head_dim != 64) return fail("mhada_vit_batch_attn: head_dim must be 64");
  if (ntok == 0) return MHADA_OK;
  const long long pairs = (long long)ntok * heads;
  const size_t lds = 0;
  const dim3 grid((unsigned)((pairs + 3) / 4));
  if (L == 1 && aligned16(qkv) && aligned16(out)) {
    const int row16 = heads * head_dim * (dtype == MHADA_F32 ? 4 : 2) / 16;
    const long long n16 = (long long)ntok * row16;
    hipLaunchKernelGGL(vit_batch_copy_v_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s,
                       (const uint4*)qkv, (uint4*)out, ntok, row16);
    return check_launch("mhada_vit_batch_attn");
  }
  if (L <= 8) {
    // bf16: the vectorised form (16-byte aligned rows in qkv and out; 97 -> 67 us at 1024^2 B4).
    // fp32 keeps the per-lane form: its vectorised instance needs ~214 VGPRs and measured
    // 54.8 vs 51.4 us at 512^2 B8. tuning vit_attn_vec = 0 selects the per-lane form (A/B).
    if (dtype != MHADA_F32 && tuning().vit_attn_vec && aligned16(qkv) && aligned16(out)) {
      const dim3 g32((unsigned)((pairs + 31) / 32));
      if (L <= 4)
        hipLaunchKernelGGL((vit_batch_attn_vec_kernel<bf16, 4>), g32, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, L,
                           ntok, heads);
      else
        hipLaunchKernelGGL((vit_batch_attn_vec_kernel<bf16, 8>), g32, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, L,
                           ntok, heads);
      return check_launch("mhada_vit_batch_attn");
    }
    if (dtype == MHADA_F32)
      hipLaunchKernelGGL((vit_batch_attn_small_kernel<float>), grid, dim3(256), 0, s, (const float*)qkv, (float*)out,
                         L, ntok, heads);
    else
      hipLaunchKernelGGL((vit_batch_attn_small_kernel<bf16>), grid, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out,
                         L, ntok, heads);
  } else if (dtype == MHADA_F32) {
    hipLaunchKernelGGL((vit_batch_attn_kernel<float>), grid, dim3(256), lds, s, (const float*)qkv, (float*)out, L,
                       ntok, heads);
  } else {
    hipLaunchKernelGGL((vit_batch_attn_kernel<bf16>), grid, dim3(256), lds, s, (const bf16*)qkv, (bf16*)out, L,
                       ntok, heads);
  }
  return check_launch("mhada_vit_batch_attn");
}

extern "C" int mhada_pos_embed(const float* pos, float* out, int C, int bh, int bw, int oh, int ow,
                               mhada_stream_t s_) {
  if (!pos || !out || C <= 0 || bh <= 0 || bw <= 0 || oh <= 0 || ow <= 0) return fail("mhada_pos_embed: bad args");
  const long long n = (long long)oh * ow * C;
  hipLaunchKernelGGL(pos_embed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)s_, pos, out,
                     C, bh, bw, oh, ow);
  return check_launch("mhada_pos_embed");
}

extern "C" int mhada_instnorm_stats(const float* x, float* mu, float* rstd, double* work, int B, int N, int C,
                                    int splits, float eps, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!x || !mu || !rstd || !work || B <= 0 || N <= 0 || C <= 0 || splits <= 0)
    return fail("mhada_instnorm_stats: bad args");
  if (splits > 65535) return fail("mhada_instnorm_stats: too many splits");
  if (C % 4 || ((uintptr_t)x & 15)) return fail("mhada_instnorm_stats: needs C % 4 == 0 and a 16-byte aligned x");
  hipLaunchKernelGGL(in_partial_kernel, dim3((C + 63) / 64, B, splits), dim3(256), 0, s, x, work, B, N, C, splits);
  int rc = check_launch("mhada_instnorm_stats/partial");
  if (rc) return rc;
  hipLaunchKernelGGL(in_finalize_kernel, dim3((B * C + 15) / 16), dim3(256), 0, s, work, mu, rstd, B, N, C, splits,
                     eps);
  return check_launch("mhada_instnorm_stats/finalize");
}

extern "C" int mhada_fold_block(const float* wf, const float* wg, const float* wh, const float* bg, const float* bh,
                                const float* rstd_c, const float* mu_s, const float* rstd_s, void* wq, void* wkv,
                                float* bkv, float* v_mu, float kscale, int dtype, int B, int H, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  if (!wf || !wg || !wh || !bg || !bh || !rstd_c || !mu_s || !rstd_s || !wq || !wkv || !bkv || !v_mu || B <= 0 ||
      H <= 0)
    return fail("mhada_fold_block: bad args");
  if (dtype == MHADA_F32)
    hipLaunchKernelGGL((fold_kernel<float>), dim3(B * H), dim3(256), 0, s, wf, wg, wh, bg, bh, rstd_c, mu_s, rstd_s,
                       (float*)wq, (float*)wkv, bkv, v_mu, kscale, H);
  else
    hipLaunchKernelGGL((fold_kernel<bf16>), dim3(B * H), dim3(256), 0, s, wf, wg, wh, bg, bh, rstd_c, mu_s, rstd_s,
                       (bf16*)wq, (bf16*)wkv, bkv, v_mu, kscale, H);
  return check_launch("mhada_fold_block");
}

extern "C" int mhada_transpose_v(const void* kv, void* vt, int dtype, int B, int H, int Ns, mhada_stream_t s_) {
  if (!kv || !vt || B <= 0 || H <= 0 || Ns <= 0) return fail("mhada_transpose_v: bad args");
  if (dtype != MHADA_F32 && dtype != MHADA_BF16) return fail("mhada_transpose_v: bad dtype");
  const int ldt = (Ns + 63) / 64 * 64;
  const dim3 grid(ldt / 64, B * H);
  if (dtype == MHADA_F32)
    hipLaunchKernelGGL((transpose_v_kernel<float>), grid, dim3(256), 0, (hipStream_t)s_, (const float*)kv, (float*)vt,
                       Ns, ldt);
  else
    hipLaunchKernelGGL((transpose_v_kernel<bf16>), grid, dim3(256), 0, (hipStream_t)s_, (const bf16*)kv, (bf16*)vt,
                       Ns, ldt);
  return check_launch("mhada_transpose_v");
}

extern "C" int mhada_cosine_prep(void* q, void* kv, int dtype, int B, int H, int Nc, int Ns, mhada_stream_t s_) {
  hipStream_t s = (hipStream_t)s_;
  // Nc == 0 (q unused) or Ns == 0 (kv unused) normalises one side only: a cached style's K is
  // normalised once, each new frame's Q per call.
  if (B <= 0 || H <= 0 || Nc < 0 || Ns < 0 || (Nc == 0 && Ns == 0) || (Nc > 0 && !q) || (Ns > 0 && !kv))
    return fail("mhada_cosine_prep: bad args");
  if (dtype != MHADA_F32 && dtype != MHADA_BF16) return fail("mhada_cosine_prep: bad dtype");
  const long long rq = (long long)B * H * Nc, rk = (long long)B * H * Ns;
  if (rq > 0) {
    if (dtype == MHADA_F32)
      hipLaunchKernelGGL((rownorm_kernel<float>), dim3((unsigned)((rq + 3) / 4)), dim3(256), 0, s, (float*)q, rq, 64);
    else
      hipLaunchKernelGGL((rownorm_kernel<bf16>), dim3((unsigned)((rq + 3) / 4)), dim3(256), 0, s, (bf16*)q, rq, 64);
  }
  if (rk > 0) {
    if (dtype == MHADA_F32)
      hipLaunchKernelGGL((rownorm_kernel<float>), dim3((unsigned)((rk + 3) / 4)), dim3(256), 0, s, (float*)kv, rk, 128);
    else
      hipLaunchKernelGGL((rownorm_kernel<bf16>), dim3((unsigned)((rk + 3) / 4)), dim3(256), 0, s, (bf16*)kv, rk, 128);
  }
  return check_launch("mhada_cosine_prep");
}

extern "C" int mhada_conv3x3_out3(const void* x, int dtype, const float* w, const float* b, float* y, int B, int H,
                                  int W, int Cin, int clamp255, mhada_stream_t s_) {
  if (!x || !w || !b || !y || B <= 0 || H < 2 || W < 2) return fail("mhada_conv3x3_out3: bad args");
  if (!aligned16(x)) return fail("mhada_conv3x3_out3: x must be 16-byte aligned");
  const long long pix = (long long)B * H * W;
  const dim3 grid((unsigned)((pix + 255) / 256));
  hipStream_t s = (hipStream_t)s_;
  // bf16, Cin 32/64: the MFMA tile kernel (tuning out3_mfma = 0 selects the per-pixel VALU kernel)
  if (dtype == MHADA_BF16 && tuning().out3_mfma && (Cin == 32 || Cin == 64)) {
    const int tiles_x = (W + 63) / 64, strips_y = (H + 4 * kOut3RowsM - 1) / (4 * kOut3RowsM);
    const long long nb = (long long)B * strips_y * tiles_x;
    if (nb >= (1LL << 31)) return fail("mhada_conv3x3_out3: grid too large");
    const dim3 g((unsigned)nb);
    if (Cin == 64)
      hipLaunchKernelGGL((conv_out3_mfma_kernel<64, 32>), g, dim3(256), 0, s, (const bf16*)x, w, b, y, H, W, tiles_x, strips_y, clamp255);
    else
      hipLaunchKernelGGL((conv_out3_mfma_kernel<32, 32>), g, dim3(256), 0, s, (const bf16*)x, w, b, y, H, W, tiles_x, strips_y, clamp255);
    return check_launch("mhada_conv3x3_out3");
  }
  // fp32, Cin 32/64: the LDS-tiled kernel (tuning out3_tile = 0 selects the per-pixel kernel)
  if (dtype == MHADA_F32 && tuning().out3_tile && (Cin == 32 || Cin == 64)) {
    const int tiles_x = (W + 63) / 64, strips_y = (H + 4 * kOut3Rows - 1) / (4 * kOut3Rows);
    const long long nb = (long long)B * strips_y * tiles_x;
    if (nb >= (1LL << 31)) return fail("mhada_conv3x3_out3: grid too large");
    const dim3 g((unsigned)nb);
    if (Cin == 64)
      hipLaunchKernelGGL((conv_out3_f32_kernel<64, 16>), g, dim3(256), 0, s, (const float*)x, w, b, y, H, W, tiles_x,
                         strips_y, clamp255);
    else
      hipLaunchKernelGGL((conv_out3_f32_kernel<32, 16>), g, dim3(256), 0, s, (const float*)x, w, b, y, H, W, tiles_x,
                         strips_y, clamp255);
    return check_launch("mhada_conv3x3_out3");
  }
#define OUT3_CASE(CI)                                                                                          \
  case CI:                                                                                                     \
    if (dtype == MHADA_F32)                                                                                    \
      hipLaunchKernelGGL((conv_out3_kernel<float, CI>), grid, dim3(256), 0, s, (const float*)x, w, b, y, B, H, W, \
                         clamp255);                                                                            \
    else                                                                                                       \
      hipLaunchKernelGGL((conv_out3_kernel<bf16, CI>), grid, dim3(256), 0, s, (const bf16*)x, w, b, y, B, H, W,   \
                         clamp255);                                                                            \
    break;
  switch (Cin) {
    OUT3_CASE(64)
    OUT3_CASE(32)
    OUT3_CASE(128)
    default:
      return fail("mhada_conv3x3_out3: Cin must be 32, 64 or 128");
  }
#undef OUT3_CASE
  return check_launch("mhada_conv3x3_out3");
}

// 2 x 2 output blocks for 16-B aligned tensors (round 5): one thread per (source pixel, 8-channel
// group) writes the four outputs above source pixel (i, j).  Interior pixels (1 <= i <= H-2,
// 1 <= j <= W-2) take their taps from the 3 x 3 source window with compile-time indices and the
// weights the formula gives there exactly (1/4, 3/4: the coordinates are exact in fp32), so each
// output is the same bilerp expression on the same operands as upsample2x_kernel (bit-identical);
// border pixels evaluate the formula per output.  9 vector loads per 4 outputs instead of 16.
template <typename T>
__global__ void __launch_bounds__(256) upsample2x_quad_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H,
                                                              int W, int C) {
  typedef typename Vec16<T>::type V;
  constexpr int N = Vec16<T>::N, NV = 8 / N;
  const int G = C / 8;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)B * H * W * G;
  if (idx >= total) return;
  const int g = (int)(idx % G);
  long long pix = idx / G;
  const int j = (int)(pix % W);
  pix /= W;
  const int i = (int)(pix % H);
  const int b = (int)(pix / H);
  const T* base = x + (long long)b * H * W * C + g * 8;
  const int Wo = 2 * W, Ho = 2 * H;
  T* obase = y + (long long)b * Ho * Wo * C + g * 8;
  if (i >= 1 && i <= H - 2 && j >= 1 && j <= W - 2) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      V w[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          w[r][c] = reinterpret_cast<const V*>(base + ((long long)(i - 1 + r) * W + (j - 1 + c)) * C)[v];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const float ly0 = a ? 0.75f : 0.25f, ly1 = a ? 0.25f : 0.75f;  // rows (i-1+a, i+a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const float lx0 = bb ? 0.75f : 0.25f, lx1 = bb ? 0.25f : 0.75f;  // cols (j-1+bb, j+bb)
          V o;
#pragma unroll
          for (int e = 0; e < N; ++e)
            o[e] = from_f32<T>(bilerp(ly0, ly1, lx0, lx1, to_f32<T>(w[a][bb][e]), to_f32<T>(w[a][bb + 1][e]),
                                      to_f32<T>(w[a + 1][bb][e]), to_f32<T>(w[a + 1][bb + 1][e])));
          reinterpret_cast<V*>(obase + ((long long)(2 * i + a) * Wo + (2 * j + bb)) * C)[v] = o;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int Y = 2 * i + a;
    const float sy = fmaxf(((float)Y + 0.5f) * 0.5f - 0.5f, 0.f);
    const int y0 = (int)sy, y1 = y0 + (y0 < H - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int X = 2 * j + bb;
      const float sx = fmaxf(((float)X + 0.5f) * 0.5f - 0.5f, 0.f);
      const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
      const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
      const V* p00 = reinterpret_cast<const V*>(base + ((long long)y0 * W + x0) * C);
      const V* p01 = reinterpret_cast<const V*>(base + ((long long)y0 * W + x1) * C);
      const V* p10 = reinterpret_cast<const V*>(base + ((long long)y1 * W + x0) * C);
      const V* p11 = reinterpret_cast<const V*>(base + ((long long)y1 * W + x1) * C);
      V* out = reinterpret_cast<V*>(obase + ((long long)Y * Wo + X) * C);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const V a00 = p00[v], a01 = p01[v], a10 = p10[v], a11 = p11[v];
        V o;
#pragma unroll
        for (int e = 0; e < N; ++e)
          o[e] = from_f32<T>(bilerp(ly0, ly1, lx0, lx1, to_f32<T>(a00[e]), to_f32<T>(a01[e]), to_f32<T>(a10[e]),
                                    to_f32<T>(a11[e])));
        out[v] = o;
      }
    }
  }
}

extern "C" int mhada_upsample2x(const void* x, void* y, int dtype, int B, int H, int W, int C, mhada_stream_t s_) {
  if (!x || !y || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return fail("mhada_upsample2x: bad args");
  // bf16: 2 x 2 output blocks (34 / 88 us vs 53 / 105 us for the 16-B per-pixel form at the
  // 1024^2 B4 decoder shapes, profiles/r05_opbench_conv_upsample.log); fp32 (two vectors per
  // 8-channel group): equal or slower, per-pixel.  tuning upsample_quad = 0 forces the per-pixel form (A/B)
  if (dtype != MHADA_F32 && aligned16(x) && aligned16(y) && H >= 3 && W >= 3 && tuning().upsample_quad) {
    const long long total = (long long)B * H * W * (C / 8);
    hipLaunchKernelGGL((upsample2x_quad_kernel<bf16>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)s_, (const bf16*)x, (bf16*)y, B, H, W, C);
    return check_launch("mhada_upsample2x");
  }
  if (aligned16(x) && aligned16(y) && (long long)2 * W * C < (1LL << 31)) {
    // 16-B vector loads / stores (round 5); unaligned views: element form
    const int G = dtype == MHADA_F32 ? C / 4 : C / 8;
    const int gshift = (G & (G - 1)) == 0 ? __builtin_ctz(G) : -1;
    const long long rows = (long long)B * 2 * H;
    const dim3 grid((unsigned)((2LL * W * G + 255) / 256), (unsigned)std::min<long long>(rows, 65535));
    if (rows > (1LL << 31) - 1) return fail("mhada_upsample2x: too many rows");
    if (dtype == MHADA_F32)
      hipLaunchKernelGGL((upsample2x_vec_kernel<float>), grid, dim3(256), 0, (hipStream_t)s_, (const float*)x,
                         (float*)y, B, H, W, C, gshift);
    else
      hipLaunchKernelGGL((upsample2x_vec_kernel<bf16>), grid, dim3(256), 0, (hipStream_t)s_, (const bf16*)x,
                         (bf16*)y, B, H, W, C, gshift);
    return check_launch("mhada_upsample2x");
  }
  const long long total = (long long)B * 4 * H * W * (C / 8);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == MHADA_F32)
    hipLaunchKernelGGL((upsample2x_kernel<float>), grid, dim3(256), 0, (hipStream_t)s_, (const float*)x, (float*)y, B,
                       H, W, C);
  else
    hipLaunchKernelGGL((upsample2x_kernel<bf16>), grid, dim3(256), 0, (hipStream_t)s_, (const bf16*)x, (bf16*)y, B,
                       H, W, C);
  return check_launch("mhada_upsample2x");
}

extern "C" int mhada_split3_rows(const float* x, void* planes, long long n, mhada_stream_t s_) {
  if (!x || !planes || n < 0 || n % 4) return fail("mhada_split3_rows: bad args (n % 4 == 0)");
  if (!aligned16(x) || !aligned16(planes) || (n * 2) % 16) return fail("mhada_split3_rows: 16-byte aligned operands");
  if (n == 0) return MHADA_OK;
  const long long nb = (n / 4 + 255) / 256;
  if (nb > 0x7fffffffLL) return fail("mhada_split3_rows: too large");
  hipLaunchKernelGGL(split3_rows_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)s_, x, (bf16*)planes, n);
  return check_launch("mhada_split3_rows");
}
