// Training-path kernels (train_image.py:139 loss.backward(), fp32): the pieces autograd needs
// around the forward GEMM/conv kernels of gemm.hip.
//
//   mhada_gemm_tn     C[M][N] = sum_k A[k][m] B[k][n] — the weight-gradient contraction: conv
//                     wgrad (B = im2col of the layer input, reflect or zero padding) and linear
//                     dW = dY^T X.  fp32 MFMA (v_mfma_f32_32x32x2_f32), split over K into
//                     partial slabs that a second pass sums in a FIXED order (deterministic;
//                     no float atomics).
//   mhada_colsum      bias gradients: column sums of dY rows (split rows + the same reduction).
//   mhada_relu_bwd    dY * (Y > 0) (threshold_backward on the saved ReLU output).
//   mhada_reflect_fold  the adjoint of ReflectionPad2d(1): folds the full-correlation input
//                     gradient on the padded grid (H+2)x(W+2) back onto H x W.
//   mhada_maxpool2 / mhada_maxpool2_bwd  MaxPool2d(2, 2) (vgg19.py, torchvision cfg E) forward and
//                     backward (gradient to the FIRST maximum of each window in row-major scan
//                     order, as ATen's max_pool2d keeps it).
//   mhada_upsample2x_bwd  adjoint of the bilinear x2 upsample (conv.py:71, align_corners=False).
//   mhada_layernorm_fwd / mhada_layernorm_bwd  nn.LayerNorm (vit.py:54-55,58,62; eps 1e-6) with
//                     the row statistics kept for the backward; dX per row, dGamma / dBeta as
//                     per-block column partials summed in a fixed order.
//   mhada_instnorm_bwd  InstanceNorm (no affine) adjoint on token rows: column sums of dY and dY*Y
//                     (fp64 partials, fixed order) and dX = (dY - mean dY - Y mean dY*Y) * rstd.
//   mhada_attn_train_bwd_prep  the elementwise head of the MHAda attention backward
//                     (S = sqrt(max(E2' - M'^2, 1e-6)), out' = S x + M'): dX, d[M'|E2'] and the
//                     per-row dot delta, one pass instead of ~12 aten ops.
//   mhada_pos_embed_bwd  adjoint of the PosEmbedding bilinear resize (vit.py:91-92): a gather
//                     per source pixel (fixed order) in place of ATen's atomic scatter.
//   mhada_feat_loss_bwd  the gradient of every loss term on one VGG feature map in one pass:
//                     the global-style mean / unbiased-std distances (lossfn.py:7-23) and an MSE
//                     against a target (local feature loss lossfn.py:26-34, identity loss 2
//                     lossfn.py:41-47), replacing ATen's mse_backward, std / mean backward chains
//                     and the adds that sum them.
//   mhada_vgg_input / mhada_vgg_input_bwd  imageNet1k_normalize (vgg19.py:6-12) fused with the
//                     NCHW -> NHWC layout change (channels zero padded to a multiple of 32 so the
//                     first conv runs on the implicit-GEMM kernel), and its adjoint.
// Layouts: activations NHWC fp32 (token-major, as the inference engine).
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace mhada {

// ======================================================================================
// TN GEMM with split-K partial slabs
// ======================================================================================
struct TnP {
  int M, N, K;
  const float* a; long long lda;          // A[k * lda + m]
  const float* b; long long ldb;          // ROWS: B[k * ldb + n]
  int img_c, img_h, img_w, out_h, out_w, pad;  // CONV: k = output pixel (b, oy, ox), n = tap*Cin + ci
  float* slab;                            // [splits][M][N]
  float* cslab;                           // [splits][M] column sums of A (null: none)
  int kchunk, tiles_n;
  int nb; long long sza, szb;             // batch (blockIdx.z): A / B element strides; slabs [S][nb][M][N]
  int rsrc;                               // ROWS, 16-B A rows: loads through per-stage buffer resources
};

constexpr int kTnBN = 128, kTnBK = 32;

MHADA_DEV int tn_reflect(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// BMODE: MHADA_A_ROWS, MHADA_A_CONV3X3 (reflect pad 1), MHADA_A_CONV3X3_ZERO (zero pad `pad`),
// MHADA_A_PATCH8 (k = token (b, py, px) of the 8x8 / stride-8 patch grid, n = c*64 + ky*8 + kx
// of an NCHW image [B][img_c][img_h][img_w]: the patch-embedding weight gradient).
// VEC_A: A rows are 16-B aligned with M % 4 == 0 (else element loads, e.g. the 3-channel layer).
// BM = 128 (M >= 128) or 64 (the 64-channel layers: no half-empty M tiles); waves 2 x 2, each
// (BM/2) x 64 of the output.
template <int BMODE, bool VEC_A, int BM, bool RS = false>
__global__ void __launch_bounds__(256, 2) gemm_tn_kernel(const TnP p) {
  static_assert(!RS || (BMODE == MHADA_A_ROWS && VEC_A), "buffer-resource loads: ROWS, 16-B A rows");
  constexpr int TMW = BM / 64;   // 32-row MFMA blocks per wave
  constexpr int ACH = BM / 32;   // A chunks (16 B) staged per thread per K-stage
  __shared__ __attribute__((aligned(16))) float sA[2][kTnBK][BM];
  __shared__ __attribute__((aligned(16))) float sB[2][kTnBK][kTnBN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 2 x 2 waves of 64 x 64
  const int h = lane >> 5, r32 = lane & 31;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = t / p.tiles_n, tn = t - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * kTnBN;
  const int kbeg = blockIdx.y * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
  const int zb = blockIdx.z;
  const float* __restrict__ pa = p.a + zb * p.sza;
  const float* __restrict__ pb = p.b + zb * p.szb;

  // staging: chunk c = tid + 256 i (i < 4) -> tile row c >> 5 = (tid >> 5) + 8 i, 4 columns at 4 (c & 31)
  const int col = 4 * (tid & 31), row0 = tid >> 5;
  // B gather: the column quad of this thread is fixed for the whole K loop (tap, channel)
  int tap_dy = 0, tap_dx = 0, ci = 0;
  const bool bcol_ok = n0 + col < p.N;  // N % 4 == 0 for every B mode (checked on the host)
  if constexpr (BMODE == MHADA_A_PATCH8) {
    const int n = min(n0 + col, p.N - 4);
    ci = n >> 6;                  // image channel
    tap_dy = (n >> 3) & 7;        // ky
    tap_dx = n & 7;               // kx (0 or 4: a quad stays inside one patch row)
  } else if constexpr (BMODE != MHADA_A_ROWS) {
    const int n = min(n0 + col, p.N - 4);
    const int tap = n / p.img_c;
    ci = n - tap * p.img_c;
    tap_dy = tap / 3 - 1;
    tap_dx = tap - (tap / 3) * 3 - 1;
  }
  f32x4 ra[ACH], rb[4];
  // CONV: output pixel (b, y, x) of this thread's B rows k0 + row0 + 8i, advanced by kTnBK per
  // issue() (issue runs on k0 = kbeg, kbeg + kTnBK, ...) instead of divided out of k each time
  int cbb[4] = {}, cyy[4] = {}, cxx[4] = {};
  if constexpr (BMODE == MHADA_A_CONV3X3 || BMODE == MHADA_A_CONV3X3_ZERO) {
    const int hw = p.out_h * p.out_w;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kbeg + row0 + 8 * i;
      cbb[i] = k / hw;
      const int rem = k - cbb[i] * hw;
      cyy[i] = rem / p.out_w;
      cxx[i] = rem - cyy[i] * p.out_w;
    }
  }
  // ROWS with 16-B A rows (p.rsrc, the linears' weight gradients): A and B through buffer resources
  // rebuilt per K-stage in scalar registers over the stage's rows; every lane's offset is a loop
  // constant (columns past M / N at an out-of-range offset read 0), so a stage's loads cost no
  // vector address arithmetic and no per-lane branch — an fp32 MFMA holds its SIMD's vector issue
  // for its whole 64 cycles (profiles/r05_f32mfma_fill.log), every VALU instruction adds to the loop
  int avo[ACH], bvo[4];
  if constexpr (RS) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + 256 * i, m = m0 + 4 * (c % (BM / 4));
      avo[i] = m < p.M ? (int)(((long long)(c / (BM / 4)) * p.lda + m) * 4) : 0x7ff00000;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) bvo[i] = bcol_ok ? (int)(((long long)(row0 + 8 * i) * p.ldb + n0 + col) * 4) : 0x7ff00000;
  }
  auto issue = [&](int k0) {
    if constexpr (RS) {
      {
        const int rows = min(kend - k0, kTnBK);
        const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(pa + (long long)k0 * p.lda), 0, (int)(rows * p.lda * 4), 0x00020000);
        const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(pb + (long long)k0 * p.ldb), 0, (int)(rows * p.ldb * 4), 0x00020000);
#pragma unroll
        for (int i = 0; i < ACH; ++i)
          ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, avo[i], 0, 0));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          rb[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(br, bvo[i], 0, 0));
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {  // A: chunk c = tid + 256 i -> row c / (BM/4), 4 columns at 4 (c % (BM/4))
      const int c = tid + 256 * i;
      const int k = k0 + c / (BM / 4);
      const int m = m0 + 4 * (c % (BM / 4));
      const bool kok = k < kend;
      if constexpr (VEC_A) {
        ra[i] = (kok && m < p.M) ? *reinterpret_cast<const f32x4*>(pa + (long long)k * p.lda + m) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[i][e] = (kok && m + e < p.M) ? pa[(long long)k * p.lda + m + e] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + row0 + 8 * i;
      const bool kok = k < kend;
      // B
      if constexpr (BMODE == MHADA_A_ROWS) {
        rb[i] = (kok && bcol_ok) ? *reinterpret_cast<const f32x4*>(pb + (long long)k * p.ldb + n0 + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else if constexpr (BMODE == MHADA_A_PATCH8) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (kok && bcol_ok) {
          const int gw = p.img_w / 8, gh = p.img_h / 8;
          const int bb = k / (gh * gw), rem = k - bb * (gh * gw);
          const int py = rem / gw, px = rem - py * gw;
          v = *reinterpret_cast<const f32x4*>(pb + (((long long)bb * p.img_c + ci) * p.img_h + py * 8 + tap_dy) * p.img_w +
                                             px * 8 + tap_dx);
        }
        rb[i] = v;
      } else {
        bool ok = kok && bcol_ok;
        long long src = 0;
        const int bb = cbb[i], oy = cyy[i], ox = cxx[i];
        cxx[i] += kTnBK;  // the next issue's row
        while (cxx[i] >= p.out_w) {
          cxx[i] -= p.out_w;
          if (++cyy[i] == p.out_h) {
            cyy[i] = 0;
            ++cbb[i];
          }
        }
        if (ok) {
          int Y, X;
          if constexpr (BMODE == MHADA_A_CONV3X3_ZERO) {
            Y = oy + tap_dy + 1 - p.pad;
            X = ox + tap_dx + 1 - p.pad;
            ok = Y >= 0 && Y < p.img_h && X >= 0 && X < p.img_w;
          } else {
            Y = tn_reflect(oy + tap_dy, p.img_h);
            X = tn_reflect(ox + tap_dx, p.img_w);
          }
          src = (((long long)bb * p.img_h + Y) * p.img_w + X) * p.img_c + ci;
        }
        rb[i] = ok ? *reinterpret_cast<const f32x4*>(pb + src) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<f32x4*>(&sA[buf][c / (BM / 4)][4 * (c % (BM / 4))]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(&sB[buf][row0 + 8 * i][col]) = rb[i];
  };

  f32x16 acc[TMW][2];
#pragma unroll
  for (int a = 0; a < TMW; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  // fused bias gradient (p.cslab): the column-0 tiles also sum their staged A rows; a thread's A
  // chunks all cover columns m0 + 4 (tid % (BM/4)) .. +3 (256 is a multiple of BM/4)
  const bool csum = p.cslab && tn == 0;
  f32x4 cs = {0.f, 0.f, 0.f, 0.f};
  auto add_cs = [&]() {
#pragma unroll
    for (int i = 0; i < ACH; ++i) cs += ra[i];
  };

  const int nst = (kend - kbeg + kTnBK - 1) / kTnBK;
  if (nst > 0) {
    issue(kbeg);
    if (csum) add_cs();
    commit(0);
  }
  __syncthreads();
  // one K-stage on LDS buffer BUF (a compile-time constant: the loop runs two stages per
  // iteration, so every LDS address is a per-lane base plus an immediate)
  auto stage = [&](int st, auto bufc) __attribute__((always_inline)) {
    constexpr int buf = decltype(bufc)::value;
    const bool more = st + 1 < nst;
    if (more) issue(kbeg + (st + 1) * kTnBK);
#pragma unroll
    for (int kk = 0; kk < kTnBK; kk += 2) {
      float av[TMW], bv[2];
#pragma unroll
      for (int mi = 0; mi < TMW; ++mi) av[mi] = sA[buf][kk + h][wm * (BM / 2) + mi * 32 + r32];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bv[ni] = sB[buf][kk + h][wn * 64 + ni * 32 + r32];
      // D[n][m]: B is the MFMA A operand, so the lane owns output row m = ... + r32 and the
      // registers 4g..4g+3 hold 4 consecutive columns n (16-B slab stores)
#pragma unroll
      for (int mi = 0; mi < TMW; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[ni], av[mi], acc[mi][ni], 0, 0, 0);
    }
    if (more) {
      if (csum) add_cs();  // beside the commit: the loads were waited for there anyway
      commit(buf ^ 1);
    }
    __syncthreads();
  };
  int st = 0;
  for (; st + 1 < nst; st += 2) {
    stage(st, std::integral_constant<int, 0>());
    stage(st + 1, std::integral_constant<int, 1>());
  }
  if (st < nst) stage(st, std::integral_constant<int, 0>());

  if (csum) {  // the 256 / (BM/4) threads of one column quad, summed in thread order through LDS
    f32x4* part = reinterpret_cast<f32x4*>(&sA[0][0][0]);
    part[tid] = cs;
    __syncthreads();
    if (tid < BM / 4) {
      f32x4 v = part[tid];
      for (int j = 1; j < 256 / (BM / 4); ++j) v += part[tid + j * (BM / 4)];
      const int m = m0 + 4 * tid;
      if (m < p.M) *reinterpret_cast<f32x4*>(p.cslab + ((long long)blockIdx.y * p.nb + zb) * p.M + m) = v;  // M % 4 == 0
    }
  }
  float* slab = p.slab + ((long long)blockIdx.y * p.nb + zb) * p.M * p.N;
#pragma unroll
  for (int mi = 0; mi < TMW; ++mi) {
    const int m = m0 + wm * (BM / 2) + mi * 32 + r32;
    if (m >= p.M) continue;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 64 + ni * 32 + 8 * g + 4 * h;
        if (n < p.N)  // N % 4 == 0
          *reinterpret_cast<f32x4*>(slab + (long long)m * p.N + n) =
              f32x4{acc[mi][ni][4 * g], acc[mi][ni][4 * g + 1], acc[mi][ni][4 * g + 2], acc[mi][ni][4 * g + 3]};
      }
  }
}

// out[i] = sum_{s < S} slab[s][i], fixed order; out may have a row stride (ld >= ncol)
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          long long rows, int ncol, long long ld, int S) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;  // quad index
  const long long n4 = rows * ncol / 4;
  if (q >= n4) return;
  const long long total = rows * ncol;
  // 8 slab loads in flight per batch, summed in slab order (a one-load-per-iteration loop was
  // latency bound: 64 slabs of 1 MiB reduced at ~0.5 TB/s)
  const float* sp = slab + 4 * q;
  f32x4 acc = *reinterpret_cast<const f32x4*>(sp);
  int s = 1;
  for (; s + 8 <= S; s += 8) {
    f32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const f32x4*>(sp + (long long)(s + j) * total);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  for (; s < S; ++s) acc += *reinterpret_cast<const f32x4*>(sp + (long long)s * total);
  const long long i = 4 * q, r = i / ncol, c = i - r * ncol;
  if (ld == ncol) {
    *reinterpret_cast<f32x4*>(out + i) = acc;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) out[r * ld + c + e] = acc[e];
  }
}

// M <= 4 (the 3-channel last decoder layer's weight gradient): VALU, bandwidth-bound on the B
// gather.  Block = 256 threads over (row group, column quad); each thread keeps 4 x 4 sums
// (m, 4 columns), the row groups are summed in LDS in a fixed order, one slab row per block.
template <int BMODE>
__global__ void __launch_bounds__(256) tn_skinny_kernel(const TnP p) {
  __shared__ f32x4 part[256][4];
  const int tpc = min(p.N / 4 - (int)blockIdx.y * 256, 256);
  const int groups = 256 / tpc;
  const int t = threadIdx.x, qd = t % tpc, g = t / tpc;
  const int n = 4 * ((int)blockIdx.y * 256 + qd);
  int tap_dy = 0, tap_dx = 0, ci = 0;
  if constexpr (BMODE != MHADA_A_ROWS) {
    const int tap = n / p.img_c;
    ci = n - tap * p.img_c;
    tap_dy = tap / 3 - 1;
    tap_dx = tap - (tap / 3) * 3 - 1;
  }
  const long long k0 = (long long)blockIdx.x * p.kchunk, k1 = std::min<long long>(p.K, k0 + p.kchunk);
  f32x4 acc[4] = {};
  if (g < groups) {
    for (long long k = k0 + g; k < k1; k += groups) {
      f32x4 bv;
      if constexpr (BMODE == MHADA_A_ROWS) {
        bv = *reinterpret_cast<const f32x4*>(p.b + k * p.ldb + n);
      } else {
        const int hw = p.out_h * p.out_w;
        const int bb = (int)(k / hw), rem = (int)(k - (long long)bb * hw);
        const int oy = rem / p.out_w, ox = rem - oy * p.out_w;
        int Y, X;
        bool ok = true;
        if constexpr (BMODE == MHADA_A_CONV3X3_ZERO) {
          Y = oy + tap_dy + 1 - p.pad;
          X = ox + tap_dx + 1 - p.pad;
          ok = Y >= 0 && Y < p.img_h && X >= 0 && X < p.img_w;
        } else {
          Y = tn_reflect(oy + tap_dy, p.img_h);
          X = tn_reflect(ox + tap_dx, p.img_w);
        }
        bv = ok ? *reinterpret_cast<const f32x4*>(p.b + (((long long)bb * p.img_h + Y) * p.img_w + X) * p.img_c + ci)
                : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float av = m < p.M ? p.a[k * p.lda + m] : 0.f;
        acc[m] += av * bv;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) part[t][m] = acc[m];
  __syncthreads();
  if (t < tpc) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      f32x4 s4 = part[t][m];
      for (int j = 1; j < groups; ++j) s4 += part[j * tpc + t][m];
      if (m < p.M) *reinterpret_cast<f32x4*>(p.slab + ((long long)blockIdx.x * p.M + m) * p.N + n) = s4;
    }
  }
}

// M <= 4, CONV modes, Cin % 64 == 0 (the 3-channel last decoder layer, conv.py:92, whose weight
// gradient the gather form above reads 9x from L2: one 16-B tap load per (pixel, tap, channel
// quad)).  Here a persistent block stages a 4 x 32 output-pixel tile's (4+2) x (32+2) input patch
// of 64 channels (52 KiB) and the tile's dY rows in LDS once, and each thread (channel ci = t % 64,
// tap group t / 64: taps {g, g+4, g+8} < 9) accumulates its 12 (tap, m) sums from LDS; blocks walk
// the tiles w = blockIdx.x + i * gridDim.x in a fixed order, one slab row per block.
constexpr int kSkTY = 4, kSkTX = 32, kSkPY = kSkTY + 2, kSkPX = kSkTX + 2;
template <int BMODE>
__global__ void __launch_bounds__(256) tn_skinny_lds_kernel(const TnP p, int ntiles_x, int ntiles) {
  __shared__ __attribute__((aligned(16))) float sx[kSkPY * kSkPX * 64];
  __shared__ f32x4 sdy[kSkTY * kSkTX];
  const int t = threadIdx.x, ci = t & 63, tg = t >> 6;
  const int cblk = blockIdx.y;  // 64-channel block of the input
  const int P = BMODE == MHADA_A_CONV3X3_ZERO ? p.pad : 1;
  const int tiles_img = ntiles / (p.K / (p.out_h * p.out_w));
  float acc[3][4] = {};
  for (int w = blockIdx.x; w < ntiles; w += gridDim.x) {
    const int b = w / tiles_img, r = w - b * tiles_img;
    const int y0 = (r / ntiles_x) * kSkTY, x0 = (r - (r / ntiles_x) * ntiles_x) * kSkTX;
    // input patch rows y0 - P .. y0 - P + 5, columns x0 - P .. x0 - P + 33 (16 B per thread-item)
    for (int e = t; e < kSkPY * kSkPX * 16; e += 256) {
      const int px = e >> 4, q = e & 15;
      const int py = px / kSkPX, pxx = px - py * kSkPX;
      int Y = y0 - P + py, X = x0 - P + pxx;
      bool ok = true;
      if constexpr (BMODE == MHADA_A_CONV3X3_ZERO) {
        ok = Y >= 0 && Y < p.img_h && X >= 0 && X < p.img_w;
      } else {
        Y = tn_reflect(Y, p.img_h);
        X = tn_reflect(X, p.img_w);
      }
      Y = min(max(Y, 0), p.img_h - 1);  // rows / columns past a ragged tile edge feed no pixel
      X = min(max(X, 0), p.img_w - 1);
      const f32x4 v = ok ? *reinterpret_cast<const f32x4*>(p.b + (((long long)b * p.img_h + Y) * p.img_w + X) * p.img_c +
                                                          64 * cblk + 4 * q)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&sx[px * 64 + 4 * q]) = v;
    }
    {  // dY of the tile's pixels (lda == 4): zero past the grid edge
      const int oy = y0 + t / kSkTX, ox = x0 + t % kSkTX;
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
      if (t < kSkTY * kSkTX && oy < p.out_h && ox < p.out_w) {
        d = *reinterpret_cast<const f32x4*>(p.a + (((long long)b * p.out_h + oy) * p.out_w + ox) * 4);
#pragma unroll
        for (int m = 0; m < 4; ++m) d[m] = m < p.M ? d[m] : 0.f;
      }
      if (t < kSkTY * kSkTX) sdy[t] = d;
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < kSkTY * kSkTX; ++q) {
      const f32x4 d = sdy[q];
      const int py = q / kSkTX, px = q - py * kSkTX;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int tap = tg + 4 * j;
        if (tap < 9) {
          const int dy = tap / 3, dx = tap - (tap / 3) * 3;  // patch offset of tap (dy-1, dx-1) is (dy, dx)
          const float xv = sx[((py + dy) * kSkPX + px + dx) * 64 + ci];
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[j][m] += d[m] * xv;
        }
      }
    }
    __syncthreads();
  }
  float* slab = p.slab + (long long)blockIdx.x * p.M * p.N;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int tap = tg + 4 * j;
    if (tap < 9)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (m < p.M) slab[(long long)m * p.N + tap * p.img_c + 64 * cblk + ci] = acc[j][m];
  }
}

static int tn_bm(int M) { return M <= 64 ? 64 : 128; }

int tn_splits(int M, int N, int K) {
  if (M <= 4) return std::max(1, std::min(1024, K / 2048));
  const int tiles = ((M + tn_bm(M) - 1) / tn_bm(M)) * ((N + kTnBN - 1) / kTnBN);
  const int target = 1024;  // blocks: 2 per CU resident, 2 waves of them
  int s = (target + tiles - 1) / tiles;
  const int maxs = (K + kTnBK * 8 - 1) / (kTnBK * 8);  // at least 8 K-stages per split
  return std::max(1, std::min(s, maxs));
}

// ======================================================================================
// column sums (bias gradients): slab[chunk][c] = sum of rows in the chunk
// ======================================================================================
// block = 256 threads over (row group g, column quad q): tpc = min(C/4, 256) quads per row pass,
// 256 / tpc row groups stride the chunk's rows; the groups are then summed in a fixed order in
// LDS (deterministic).  gridDim.y covers C / 1024 column blocks when C > 1024.
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ x, float* __restrict__ slab, long long rows,
                                                     int C, long long rows_per_chunk) {
  __shared__ f32x4 part[256];
  const int tpc = min(C / 4 - (int)blockIdx.y * 256, 256);  // column quads of this column block
  const int groups = 256 / tpc;
  const int t = threadIdx.x, q = t % tpc, g = t / tpc;
  const int c = 4 * ((int)blockIdx.y * 256 + q);
  const long long r0 = (long long)blockIdx.x * rows_per_chunk, r1 = std::min(rows, r0 + rows_per_chunk);
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (g < groups)
    for (long long r = r0 + g; r < r1; r += groups) a += *reinterpret_cast<const f32x4*>(x + r * C + c);
  part[t] = a;
  __syncthreads();
  if (t < tpc) {
    f32x4 s = part[t];
    for (int k = 1; k < groups; ++k) s += part[k * tpc + t];
    *reinterpret_cast<f32x4*>(slab + (long long)blockIdx.x * C + c) = s;
  }
}

// ======================================================================================
// LayerNorm for training: forward keeps (mean, rstd) per row; backward
//   xh = (x - mean) rstd,  g' = dy * gamma,
//   dx = rstd (g' - mean_c(g') - xh mean_c(g' xh)),  dgamma = sum_rows dy xh,  dbeta = sum_rows dy
// One wave per row (VPL = cols / 64 values per lane, 16-B column quads as layernorm_kernel).
// ======================================================================================
// planes (round 6, may be null): y's three bf16 planes [3][rows][cols] as well — the following SPLIT3
// linear's operand (train_fns plane hand-off).
template <int VPL>
__global__ void __launch_bounds__(256) ln_fwd_train_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           float* __restrict__ stats, const float* __restrict__ g,
                                                           const float* __restrict__ b, int rows, float eps,
                                                           bf16* __restrict__ planes) {
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
  float* yr = y + (long long)row * COLS;
#pragma unroll
  for (int i = 0; i < VPL / 4; ++i) {
    const int c = (i * 64 + lane) * 4;
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + c);
    const f32x4 bb = *reinterpret_cast<const f32x4*>(b + c);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[4 * i + e] - mean) * rstd * gg[e] + bb[e];
    *reinterpret_cast<f32x4*>(yr + c) = o;
    if (planes) {
      const long long ps = (long long)rows * COLS;
      bf16x4 p0, p1, p2;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16 a = (bf16)o[e];
        const float r = o[e] - (float)a;
        const bf16 q = (bf16)r;
        p0[e] = a;
        p1[e] = q;
        p2[e] = (bf16)(r - (float)q);
      }
      bf16* pr = planes + (long long)row * COLS + c;
      *reinterpret_cast<bf16x4*>(pr) = p0;
      *reinterpret_cast<bf16x4*>(pr + ps) = p1;
      *reinterpret_cast<bf16x4*>(pr + 2 * ps) = p2;
    }
  }
  if (lane == 0) *reinterpret_cast<float2*>(stats + 2LL * row) = make_float2(mean, rstd);
}

constexpr int kLnBwdRows = 128;  // rows per block (32 per wave)

template <int VPL>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                     const float* __restrict__ stats, const float* __restrict__ g,
                                                     float* __restrict__ dx, float* __restrict__ slab, int rows) {
  constexpr int COLS = VPL * 64;
  __shared__ f32x4 part[4][2][VPL / 4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float gg[VPL], dgp[VPL], dbp[VPL];
#pragma unroll
  for (int i = 0; i < VPL / 4; ++i) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(g + (i * 64 + lane) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gg[4 * i + e] = t[e];
      dgp[4 * i + e] = 0.f;
      dbp[4 * i + e] = 0.f;
    }
  }
  const int r0 = blockIdx.x * kLnBwdRows, r1 = min(rows, r0 + kLnBwdRows);
  for (int row = r0 + wv; row < r1; row += 4) {
    const float2 st = *reinterpret_cast<const float2*>(stats + 2LL * row);
    const float* xr = x + (long long)row * COLS;
    const float* dr = dy + (long long)row * COLS;
    float xh[VPL], gd[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL / 4; ++i) {
      const int c = (i * 64 + lane) * 4;
      const f32x4 xv = *reinterpret_cast<const f32x4*>(xr + c);
      const f32x4 dv = *reinterpret_cast<const f32x4*>(dr + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * i + e;
        xh[k] = (xv[e] - st.x) * st.y;
        gd[k] = dv[e] * gg[k];
        s1 += gd[k];
        s2 += gd[k] * xh[k];
        dgp[k] += dv[e] * xh[k];
        dbp[k] += dv[e];
      }
    }
    const float m1 = wave_sum(s1) * (1.0f / COLS), m2 = wave_sum(s2) * (1.0f / COLS);
    float* o = dx + (long long)row * COLS;
#pragma unroll
    for (int i = 0; i < VPL / 4; ++i) {
      f32x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = st.y * (gd[4 * i + e] - m1 - xh[4 * i + e] * m2);
      *reinterpret_cast<f32x4*>(o + (i * 64 + lane) * 4) = r;
    }
  }
#pragma unroll
  for (int i = 0; i < VPL / 4; ++i) {
    part[wv][0][i][lane] = f32x4{dgp[4 * i], dgp[4 * i + 1], dgp[4 * i + 2], dgp[4 * i + 3]};
    part[wv][1][i][lane] = f32x4{dbp[4 * i], dbp[4 * i + 1], dbp[4 * i + 2], dbp[4 * i + 3]};
  }
  __syncthreads();
  // waves summed in a fixed order; slab[blk] = [dgamma partial (COLS) | dbeta partial (COLS)]
  for (int q = threadIdx.x; q < 2 * (VPL / 4) * 64; q += 256) {
    const int which = q / ((VPL / 4) * 64), rem = q - which * (VPL / 4) * 64, i = rem >> 6, ln = rem & 63;
    f32x4 a = part[0][which][i][ln];
    a += part[1][which][i][ln];
    a += part[2][which][i][ln];
    a += part[3][which][i][ln];
    *reinterpret_cast<f32x4*>(slab + (long long)blockIdx.x * 2 * COLS + which * COLS + (i * 64 + ln) * 4) = a;
  }
}

// ======================================================================================
// InstanceNorm backward on token rows [B][N][C] (adaDecoder.py:147-149,188-190 under autograd):
// m1 = mean_N(dy), m2 = mean_N(dy * y) per (b, c) — fp64 partials per (split, b, c) summed in a
// fixed order — then dx = (dy - m1 - y m2) * rstd.
// ======================================================================================
__global__ void __launch_bounds__(256) inb_partial_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                          double* __restrict__ work, int B, int N, int C, int splits) {
  __shared__ double red[2][16][65];
  const int quad = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + 4 * quad;
  const int b = blockIdx.y, s = blockIdx.z;
  const int per = (N + splits - 1) / splits;
  const int r0 = s * per, r1 = min(N, r0 + per);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  if (c0 < C) {
    const long long base = (long long)b * N * C + c0;
#pragma unroll 4
    for (int r = r0 + ph; r < r1; r += 16) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(dy + base + (long long)r * C);
      const f32x4 v = *reinterpret_cast<const f32x4*>(y + base + (long long)r * C);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s1[e] += (double)g[e];
        s2[e] += (double)(g[e] * v[e]);
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

__global__ void __launch_bounds__(256) inb_finalize_kernel(const double* __restrict__ work, float* __restrict__ mm,
                                                           int BC, int N, int splits) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= BC) return;
  double a = 0.0, q = 0.0;
  for (int s = 0; s < splits; ++s) {
    a += work[((long long)s * BC + idx) * 2];
    q += work[((long long)s * BC + idx) * 2 + 1];
  }
  mm[2 * idx] = (float)(a / N);
  mm[2 * idx + 1] = (float)(q / N);
}

__global__ void __launch_bounds__(256) inb_apply_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                        const float* __restrict__ mm, const float* __restrict__ rs,
                                                        float* __restrict__ dx, int N, int C, long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const long long e0 = 4 * i;
  const int c = (int)(e0 % C);
  const int b = (int)(e0 / ((long long)N * C));
  const f32x4 g = reinterpret_cast<const f32x4*>(dy)[i];
  const f32x4 v = reinterpret_cast<const f32x4*>(y)[i];
  const f32x4 r = *reinterpret_cast<const f32x4*>(rs + (long long)b * C + c);
  const float4 m01 = *reinterpret_cast<const float4*>(mm + 2 * ((long long)b * C + c));
  const float4 m23 = *reinterpret_cast<const float4*>(mm + 2 * ((long long)b * C + c) + 4);
  const float m1[4] = {m01.x, m01.z, m23.x, m23.z}, m2[4] = {m01.y, m01.w, m23.y, m23.w};
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (g[e] - m1[e] - v[e] * m2[e]) * r[e];
  reinterpret_cast<f32x4*>(dx)[i] = o;
}

// ======================================================================================
// MHAda attention backward head: per row (bh, query) of 64 channels, with m = M', e2 = E2':
//   var = e2 - m^2, sd = sqrt(max(var, 1e-6)), dx = dout sd,
//   dvar = dout x 0.5 / sd where var >= 1e-6 (0 where the clamp is active), dm = dout - 2 m dvar,
//   dmo = [dm | dvar], dd = sum_c (dm m + dvar e2).   One wave per row, lane = channel.
// ======================================================================================
__global__ void __launch_bounds__(256) attn_bwd_prep_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                                                            const float* __restrict__ mo, float* __restrict__ dx,
                                                            float* __restrict__ dmo, float* __restrict__ dd,
                                                            long long rows) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int c = threadIdx.x & 63;
  const float m = mo[row * 128 + c], e2 = mo[row * 128 + 64 + c];
  const float g = dout[row * 64 + c], xv = x[row * 64 + c];
  const float var = e2 - m * m;
  const float sd = sqrtf(fmaxf(var, 1e-6f));
  const float dvar = var >= 1e-6f ? (g * xv) * (0.5f / sd) : 0.f;
  const float dm = g - 2.0f * m * dvar;
  dx[row * 64 + c] = g * sd;
  dmo[row * 128 + c] = dm;
  dmo[row * 128 + 64 + c] = dvar;
  const float t = wave_sum(dm * m + dvar * e2);
  if (c == 0) dd[row] = t;
}

// ======================================================================================
// PosEmbedding resize adjoint: gpos[c][sy][sx] = sum over target pixels (oy, ox) of the bilinear
// weight pos_embed_kernel gives source (sy, sx) times g[oy*ow + ox][c].  Gather per source pixel
// over a window of target rows / columns that contains every one referencing it, re-deriving the
// forward's indices and weights with its exact float operations (deterministic, no atomics).
// ======================================================================================
MHADA_DEV void pe_src(int o, float sh, int n, int& i0, int& i1, float& l0, float& l1) {
  const float sf = fmaxf(sh * ((float)o + 0.5f) - 0.5f, 0.f);
  i0 = min((int)sf, n - 1);
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = sf - (float)i0;
  l0 = 1.f - l1;
}

MHADA_DEV float pe_weight(int o, float sh, int n, int src) {
  int i0, i1;
  float l0, l1;
  pe_src(o, sh, n, i0, i1, l0, l1);
  return (i0 == src ? l0 : 0.f) + (i1 == src ? l1 : 0.f);
}

__global__ void __launch_bounds__(256) pos_embed_bwd_kernel(const float* __restrict__ g, float* __restrict__ gpos,
                                                            int C, int bh, int bw, int oh, int ow) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)C * bh * bw) return;
  const int c = (int)(idx % C);
  const int pix = (int)(idx / C);
  const int sy = pix / bw, sx = pix - (pix / bw) * bw;
  float acc = 0.f;
  if (oh == bh && ow == bw) {
    acc = g[(long long)pix * C + c];
  } else {
    const float shy = (float)bh / (float)oh, shx = (float)bw / (float)ow;
    // target o maps to source coordinate ~ (o + 0.5) sh - 0.5; sources sy-1 .. sy+1 bound the window
    const int ylo = max(0, (int)floorf(((float)sy - 1.5f) / shy) - 1);
    const int yhi = min(oh - 1, (int)ceilf(((float)sy + 1.5f) / shy) + 1);
    const int xlo = max(0, (int)floorf(((float)sx - 1.5f) / shx) - 1);
    const int xhi = min(ow - 1, (int)ceilf(((float)sx + 1.5f) / shx) + 1);
    for (int oy = ylo; oy <= yhi; ++oy) {
      const float wy = pe_weight(oy, shy, bh, sy);
      if (wy == 0.f) continue;
      float row = 0.f;
      for (int ox = xlo; ox <= xhi; ++ox) {
        const float wx = pe_weight(ox, shx, bw, sx);
        if (wx != 0.f) row += wx * g[((long long)oy * ow + ox) * C + c];
      }
      acc += wy * row;
    }
  }
  gpos[(long long)c * bh * bw + pix] = acc;
}

// ======================================================================================
// elementwise / layout kernels
// ======================================================================================
__global__ void __launch_bounds__(256) relu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                       float* __restrict__ dx, long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const f32x4 g = reinterpret_cast<const f32x4*>(dy)[i];
  const f32x4 v = reinterpret_cast<const f32x4*>(y)[i];
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = v[e] > 0.f ? g[e] : 0.f;
  reinterpret_cast<f32x4*>(dx)[i] = o;
}

// g = alpha[b][c] + beta[b][c] * (x - mu[b][c]) + ks * kp[0] * (x - t) on NHWC rows x [B][P][C]
// (either term optional: alpha == null / t == null; kp == null reads as 1); 4 channels per thread.
// kp is a device scalar (the upstream gradient of the MSE term), so no host sync is needed.
__global__ void __launch_bounds__(256) feat_loss_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                                            const float* __restrict__ mu,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ kp, float ks,
                                                            float* __restrict__ g, long long PC4, int C4,
                                                            long long n4, int relu) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float k = kp ? ks * kp[0] : ks;
  const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
  if (alpha) {
    const long long bc = (i / PC4) * C4 + i % C4;  // (b, 4-channel group)
    const f32x4 a = reinterpret_cast<const f32x4*>(alpha)[bc];
    const f32x4 be = reinterpret_cast<const f32x4*>(beta)[bc];
    const f32x4 m = reinterpret_cast<const f32x4*>(mu)[bc];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = a[e] + be[e] * (v[e] - m[e]);
  }
  if (t) {
    const f32x4 w = reinterpret_cast<const f32x4*>(t)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] += k * (v[e] - w[e]);
  }
  if (relu) {  // x is a ReLU output: its adjoint (x > 0) applied here
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = v[e] > 0.f ? o[e] : 0.f;
  }
  reinterpret_cast<f32x4*>(g)[i] = o;
}

// dX[b][y][x] = sum of dXp[b][py][px] over the padded positions whose reflection is (y, x):
// py = y + 1, plus py = 0 when y == 1 and py = H + 1 when y == H - 2 (same in x).
__global__ void __launch_bounds__(256) reflect_fold_kernel(const float* __restrict__ dxp, float* __restrict__ dx, int B,
                                                           int H, int W, int C, const float* __restrict__ mask) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  const int C4 = C / 4;
  const long long total = (long long)B * H * W * C4;
  if (q >= total) return;
  const int c4 = (int)(q % C4);
  long long pix = q / C4;
  const int x = (int)(pix % W);
  pix /= W;
  const int y = (int)(pix % H);
  const int b = (int)(pix / H);
  // padded rows folding onto y: y + 1 always; 0 (reflect(-1) = 1) when y == 1; H + 1
  // (reflect(H) = H - 2) when y == H - 2 — both extra ones at H == 3, y == 1
  int ys[3], xs[3], ny = 0, nx = 0;
  ys[ny++] = y + 1;
  if (y == 1) ys[ny++] = 0;
  if (y == H - 2) ys[ny++] = H + 1;
  xs[nx++] = x + 1;
  if (x == 1) xs[nx++] = 0;
  if (x == W - 2) xs[nx++] = W + 1;
  const int Hp = H + 2, Wp = W + 2;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < ny; ++i)
    for (int j = 0; j < nx; ++j)
      acc += *reinterpret_cast<const f32x4*>(dxp + (((long long)b * Hp + ys[i]) * Wp + xs[j]) * C + 4 * c4);
  const long long o = (((long long)b * H + y) * W + x) * C + 4 * c4;
  if (mask) {  // the ReLU adjoint of the layer that produced x (its output's only consumer is this conv)
    const f32x4 m = *reinterpret_cast<const f32x4*>(mask + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = m[e] > 0.f ? acc[e] : 0.f;
  }
  *reinterpret_cast<f32x4*>(dx + o) = acc;
}

__global__ void __launch_bounds__(256) maxpool2_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int H,
                                                       int W, int C) {
  const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long long)B * Ho * Wo * C4) return;
  const int c4 = (int)(q % C4);
  long long pix = q / C4;
  const int ox = (int)(pix % Wo);
  pix /= Wo;
  const int oy = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  const float* base = x + (((long long)b * H + 2 * oy) * W + 2 * ox) * C + 4 * c4;
  const f32x4 v00 = *reinterpret_cast<const f32x4*>(base), v01 = *reinterpret_cast<const f32x4*>(base + C);
  const f32x4 v10 = *reinterpret_cast<const f32x4*>(base + (long long)W * C),
              v11 = *reinterpret_cast<const f32x4*>(base + (long long)W * C + C);
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = fmaxf(fmaxf(v00[e], v01[e]), fmaxf(v10[e], v11[e]));
  *reinterpret_cast<f32x4*>(y + (((long long)b * Ho + oy) * Wo + ox) * C + 4 * c4) = o;
}

// one thread per output window x 4 channels: the whole window's dX (4 positions) is written,
// the gradient to the first maximum in the scan order (0,0), (0,1), (1,0), (1,1); rows / columns
// beyond 2*Ho, 2*Wo (odd sizes) are zeroed by the caller
// relu_mask: x is a ReLU output whose only consumer is this pool, so the ReLU adjoint (x > 0)
// is applied here and the producing conv's backward skips mhada_relu_bwd (one fewer pass)
__global__ void __launch_bounds__(256) maxpool2_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                           float* __restrict__ dx, int B, int H, int W, int C,
                                                           int relu_mask) {
  const int Ho = H / 2, Wo = W / 2, C4 = C / 4;
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long long)B * Ho * Wo * C4) return;
  const int c4 = (int)(q % C4);
  long long pix = q / C4;
  const int ox = (int)(pix % Wo);
  pix /= Wo;
  const int oy = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  const long long o00 = (((long long)b * H + 2 * oy) * W + 2 * ox) * C + 4 * c4;
  const long long offs[4] = {o00, o00 + C, o00 + (long long)W * C, o00 + (long long)W * C + C};
  f32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const f32x4*>(x + offs[j]);
  const f32x4 g = *reinterpret_cast<const f32x4*>(dy + (((long long)b * Ho + oy) * Wo + ox) * C + 4 * c4);
  f32x4 out[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int arg = 0;
    float mx = v[0][e];
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (v[j][e] > mx || (v[j][e] != v[j][e] && mx == mx)) {  // first max; a NaN wins (ATen)
        mx = v[j][e];
        arg = j;
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j][e] = (j == arg && (!relu_mask || v[j][e] > 0.f)) ? g[e] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(dx + offs[j]) = out[j];
}

// adjoint of upsample2x (bilinear, align_corners=False, scale 2): input row y receives from
// output rows 2y-1 .. 2y+2 with the forward's own weights (recomputed, so border clamps agree)
MHADA_DEV float up2_weight(int o, int i, int n) {
  const float s = fmaxf(((float)o + 0.5f) * 0.5f - 0.5f, 0.f);
  const int i0 = (int)s;
  const int i1 = i0 + (i0 < n - 1 ? 1 : 0);
  const float l1 = s - (float)i0, l0 = 1.f - l1;
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}

// relu_x (nullable): the upsample input when it is a ReLU output consumed only by the upsample —
// its ReLU adjoint (x > 0) is applied to dx here and the producing conv skips mhada_relu_bwd
__global__ void __launch_bounds__(256) upsample2x_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ relu_x,
                                                             float* __restrict__ dx, int B, int H, int W, int C) {
  const int C4 = C / 4;
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= (long long)B * H * W * C4) return;
  const int c4 = (int)(q % C4);
  long long pix = q / C4;
  const int x = (int)(pix % W);
  pix /= W;
  const int y = (int)(pix % H);
  const int b = (int)(pix / H);
  const int Ho = 2 * H, Wo = 2 * W;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int oy = max(0, 2 * y - 1); oy <= min(Ho - 1, 2 * y + 2); ++oy) {
    const float wy = up2_weight(oy, y, H);
    if (wy == 0.f) continue;
    for (int ox = max(0, 2 * x - 1); ox <= min(Wo - 1, 2 * x + 2); ++ox) {
      const float wx = up2_weight(ox, x, W);
      if (wx == 0.f) continue;
      const f32x4 g = *reinterpret_cast<const f32x4*>(dy + (((long long)b * Ho + oy) * Wo + ox) * C + 4 * c4);
      acc += (wy * wx) * g;
    }
  }
  const long long o = (((long long)b * H + y) * W + x) * C + 4 * c4;
  if (relu_x) {
    const f32x4 xv = *reinterpret_cast<const f32x4*>(relu_x + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = xv[e] > 0.f ? acc[e] : 0.f;
  }
  *reinterpret_cast<f32x4*>(dx + o) = acc;
}

__constant__ float c_in_mean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float c_in_std[3] = {0.229f, 0.224f, 0.225f};

// (x / 255 - mean) / std, three fp32 roundings as vgg19.py:11; NCHW [B][3][H][W] -> NHWC [B][H][W][Cp]
__global__ void __launch_bounds__(256) vgg_input_kernel(const float* __restrict__ img, float* __restrict__ out, int B,
                                                        int H, int W, int Cp) {
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long plane = (long long)H * W;
  if (pix >= (long long)B * plane) return;
  const long long b = pix / plane, r = pix - b * plane;
  float* o = out + pix * Cp;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float v = img[(b * 3 + c) * plane + r];
    v = v / 255.0f;
    v = v - c_in_mean[c];
    o[c] = v / c_in_std[c];
  }
  for (int c = 3; c < Cp; c += 1) o[c] = 0.f;
}

// adjoint: d img[b][c][y][x] = d out[b][y][x][c] / std_c / 255 (the chain of the three ops)
__global__ void __launch_bounds__(256) vgg_input_bwd_kernel(const float* __restrict__ dout, float* __restrict__ dimg,
                                                            int B, int H, int W, int Cp) {
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long plane = (long long)H * W;
  if (pix >= (long long)B * plane) return;
  const long long b = pix / plane, r = pix - b * plane;
#pragma unroll
  for (int c = 0; c < 3; ++c) dimg[(b * 3 + c) * plane + r] = dout[pix * Cp + c] / c_in_std[c] / 255.0f;
}

// Backward of nn.MultiheadAttention over the BATCH axis (vit.py:48,59, batch_first=False on
// (B, N, C): each token n and head h attends over the L = B images).  One wave per (token, head),
// lane = head dim (64); L <= 8 so the score / probability tiles are 8 x 8 (one lane each):
//   S = (q/8) k^T, P = softmax_j(S), dP = dO v^T, dS = P (dP - rowsum(P dP)),
//   dq = dS k / 8, dk = dS^T (q/8), dv = P^T dO.   fp32; writes dqkv [L][ntok][3C] (q|k|v).
// planes (round 6, may be null): dqkv's three bf16 planes as well, plane stride pstride elements from
// the dqkv base of this call — the QKV input-gradient GEMM's SPLIT3 operand (train_fns plane hand-off).
MHADA_DEV void store_split3(bf16* p, long long ps, float x) {
  const bf16 a = (bf16)x;
  const float r = x - (float)a;
  const bf16 b = (bf16)r;
  p[0] = a;
  p[ps] = b;
  p[2 * ps] = (bf16)(r - (float)b);
}

__global__ void __launch_bounds__(256) vit_batch_attn_bwd_kernel(const float* __restrict__ qkv,
                                                                 const float* __restrict__ dout,
                                                                 float* __restrict__ dqkv, int L, int ntok,
                                                                 int heads, bf16* __restrict__ planes,
                                                                 long long pstride) {
  constexpr int D = 64;
  __shared__ float sq[4][8][D + 1];
  __shared__ float sk[4][8][D + 1];
  __shared__ float sv[4][8][D + 1];
  __shared__ float sg[4][8][D + 1];
  __shared__ float sp[4][8][8];
  __shared__ float sds[4][8][8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long long pair = (long long)blockIdx.x * 4 + wv;
  const bool valid = pair < (long long)ntok * heads;
  const int C = heads * D;
  const long long pp = valid ? pair : 0;
  const int n = (int)(pp / heads), hh = (int)(pp - (long long)n * heads);
  const long long row3 = (long long)ntok * 3 * C, row1 = (long long)ntok * C;
  const float* base = qkv + (long long)n * 3 * C + hh * D + lane;
  const float* gbase = dout + (long long)n * C + hh * D + lane;
  float qr[8], kr[8], vr[8], gr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool in = i < L;
    qr[i] = in ? base[i * row3] * 0.125f : 0.f;  // 1/sqrt(64)
    kr[i] = in ? base[i * row3 + C] : 0.f;
    vr[i] = in ? base[i * row3 + 2 * C] : 0.f;
    gr[i] = in ? gbase[i * row1] : 0.f;
    sq[wv][i][lane] = qr[i];
    sk[wv][i][lane] = kr[i];
    sv[wv][i][lane] = vr[i];
    sg[wv][i][lane] = gr[i];
  }
  __syncthreads();
  const int i = lane >> 3, j = lane & 7;
  const bool ij = i < L && j < L;
  float s = -INFINITY, dp = 0.f;
  if (ij) {
    s = 0.f;
#pragma unroll 16
    for (int d = 0; d < D; ++d) {
      s = fmaf(sq[wv][i][d], sk[wv][j][d], s);
      dp = fmaf(sg[wv][i][d], sv[wv][j][d], dp);
    }
  }
  float m = s;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float e = ij ? __expf(s - m) : 0.f;
  float sum = e;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o, 64);
  const float pr = ij ? e / sum : 0.f;  // rows i >= L have sum 0 (and must stay out of dv)
  float pdp = pr * dp;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) pdp += __shfl_xor(pdp, o, 64);
  sp[wv][i][j] = pr;
  sds[wv][i][j] = ij ? pr * (dp - pdp) : 0.f;
  __syncthreads();
  if (!valid) return;
  float* obase = dqkv + (long long)n * 3 * C + hh * D + lane;
  for (int r = 0; r < L; ++r) {
    float dq = 0.f, dk = 0.f, dv = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      dq = fmaf(sds[wv][r][c], kr[c], dq);   // sum_j dS[r][j] k_j
      dk = fmaf(sds[wv][c][r], qr[c], dk);   // sum_i dS[i][r] (q_i / 8)
      dv = fmaf(sp[wv][c][r], gr[c], dv);    // sum_i P[i][r] dO_i
    }
    obase[r * row3] = dq * 0.125f;
    obase[r * row3 + C] = dk;
    obase[r * row3 + 2 * C] = dv;
    if (planes) {
      bf16* pb = planes + (obase - dqkv) + r * row3;
      store_split3(pb, pstride, dq * 0.125f);
      store_split3(pb + C, pstride, dk);
      store_split3(pb + 2 * C, pstride, dv);
    }
  }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static dim3 grid1(long long n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_gemm_tn_splits(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  return tn_splits(M, N, K);
}

extern "C" int mhada_gemm_tn(const mhada_gemm_tn_args* a, float* work, long long work_floats, mhada_stream_t s_) {
  if (!a || !a->a || !a->b || !a->c || !work) return fail("mhada_gemm_tn: null argument");
  const hipStream_t s = (hipStream_t)s_;
  if (a->M <= 0 || a->N <= 0 || a->K <= 0) return fail("mhada_gemm_tn: bad sizes");
  if (a->N % 4) return fail("mhada_gemm_tn: N must be a multiple of 4");
  if (!al16(work) || !al16(a->b)) return fail("mhada_gemm_tn: B and the workspace must be 16-byte aligned");
  if (a->ldc < a->N) return fail("mhada_gemm_tn: ldc < N");
  TnP p{};
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.a = a->a; p.lda = a->lda; p.b = a->b; p.ldb = a->ldb;
  // batch of nb independent problems (blockIdx.z; A / B advance by sza / szb elements, C and the
  // column sums are [nb][M][N] / [nb][M] contiguous): the MFMA kernel, ROWS mode
  p.nb = a->nb > 1 ? a->nb : 1;
  p.sza = a->sza; p.szb = a->szb;
  if (p.nb > 1 && (a->b_mode != MHADA_A_ROWS || a->M <= 4 || a->ldc != a->N || (a->sza | a->szb) % 4))
    return fail("mhada_gemm_tn: batched form needs ROWS mode, M > 4, ldc == N, 16-B batch strides");
  if (p.nb > 65535) return fail("mhada_gemm_tn: batch too large");
  const bool vec_a = al16(a->a) && a->lda % 4 == 0 && a->M % 4 == 0;
  // per-stage buffer resources: 32 rows of A / B and the out-of-range offset must stay below 2^31 bytes
  p.rsrc = vec_a && a->b_mode == MHADA_A_ROWS && (long long)kTnBK * std::max(a->lda, a->ldb) * 4 < 0x7ff00000LL &&
           (long long)kTnBK * std::max(a->lda, a->ldb) * 4 <= 0x7fffffffLL;
  switch (a->b_mode) {
    case MHADA_A_ROWS:
      if (a->ldb % 4) return fail("mhada_gemm_tn: ldb must be a multiple of 4");
      break;
    case MHADA_A_PATCH8:
      if (a->img_w % 8 || a->img_h % 8 || a->N != 64 * a->img_c) return fail("mhada_gemm_tn: PATCH8 needs H, W % 8 == 0, N == 64*C");
      if (a->K % ((a->img_h / 8) * (a->img_w / 8))) return fail("mhada_gemm_tn: PATCH8 needs K == batch*(H/8)*(W/8)");
      p.img_c = a->img_c; p.img_h = a->img_h; p.img_w = a->img_w;
      break;
    case MHADA_A_CONV3X3:
    case MHADA_A_CONV3X3_ZERO: {
      const int pad = a->b_mode == MHADA_A_CONV3X3 ? 1 : (a->pad ? a->pad : 1);
      if (pad < 1 || pad > 2) return fail("mhada_gemm_tn: pad 1 or 2");
      if (a->img_c % 4 || a->N != 9 * a->img_c) return fail("mhada_gemm_tn: CONV needs N == 9*Cin, Cin % 4 == 0");
      p.img_c = a->img_c; p.img_h = a->img_h; p.img_w = a->img_w; p.pad = pad;
      p.out_h = a->img_h + 2 * (pad - 1); p.out_w = a->img_w + 2 * (pad - 1);
      if (a->b_mode == MHADA_A_CONV3X3 && (a->img_h < 2 || a->img_w < 2)) return fail("mhada_gemm_tn: reflect needs H, W >= 2");
      if (a->K % (p.out_h * p.out_w)) return fail("mhada_gemm_tn: CONV needs K == batch*out_h*out_w");
      break;
    }
    default:
      return fail("mhada_gemm_tn: bad b_mode");
  }
  // fused bias gradient (colsum of A) on the MFMA kernel's vector A path; otherwise mhada_colsum's
  // kernel after the GEMM (the 3-channel layer, unaligned A)
  const bool fuse_cs = a->colsum && vec_a && p.M > 4;
  int S = std::max(1, tn_splits(p.M, p.N, p.K) / p.nb);
  const long long per = ((long long)p.M * p.N + (fuse_cs ? p.M : 0)) * p.nb;
  if (work_floats < per) return fail("mhada_gemm_tn: workspace smaller than nb*(M*N (+M)) floats");
  S = (int)std::min<long long>(S, work_floats / per);
  p.kchunk = ((p.K + S - 1) / S + kTnBK - 1) / kTnBK * kTnBK;
  S = (p.K + p.kchunk - 1) / p.kchunk;
  p.tiles_n = (p.N + kTnBN - 1) / kTnBN;
  const int bm = tn_bm(p.M);
  const int tiles = ((p.M + bm - 1) / bm) * p.tiles_n;
  p.slab = work;
  p.cslab = fuse_cs ? work + (long long)S * p.nb * p.M * p.N : nullptr;
  if (S > 65535) return fail("mhada_gemm_tn: too many splits");
  const dim3 grid((unsigned)tiles, (unsigned)S, (unsigned)p.nb);
  const dim3 gsk((unsigned)S, (unsigned)((p.N / 4 + 255) / 256));
  // the 3-channel layer (M <= 4, 3x3 conv, Cin % 64 == 0, dY rows of 4 floats): LDS-tiled kernel
  if (p.M <= 4 && (a->b_mode == MHADA_A_CONV3X3 || a->b_mode == MHADA_A_CONV3X3_ZERO) && p.img_c % 64 == 0 &&
      a->lda == 4 && al16(a->a) && tuning().tn_skinny_lds) {
    const int ntx = (p.out_w + kSkTX - 1) / kSkTX, nty = (p.out_h + kSkTY - 1) / kSkTY;
    const long long nt = (long long)(p.K / (p.out_h * p.out_w)) * ntx * nty;
    if (nt < (1LL << 31)) {
      const int G = (int)std::min<long long>(nt, std::min<long long>(1024, work_floats / per));
      p.slab = work;
      const dim3 gl((unsigned)G, (unsigned)(p.img_c / 64));
      if (a->b_mode == MHADA_A_CONV3X3)
        hipLaunchKernelGGL(tn_skinny_lds_kernel<MHADA_A_CONV3X3>, gl, dim3(256), 0, s, p, ntx, (int)nt);
      else
        hipLaunchKernelGGL(tn_skinny_lds_kernel<MHADA_A_CONV3X3_ZERO>, gl, dim3(256), 0, s, p, ntx, (int)nt);
      if (int rc = check_launch("mhada_gemm_tn(skinny lds)")) return rc;
      hipLaunchKernelGGL(slab_reduce_kernel, grid1((long long)p.M * p.N / 4), dim3(256), 0, s, work, a->c,
                         (long long)p.M, p.N, a->ldc, G);
      if (int rc = check_launch("mhada_gemm_tn(reduce)")) return rc;
      if (!a->colsum) return 0;
      return mhada_colsum(a->a, a->colsum, p.K, p.M, work, work_floats, s_);
    }
  }
#define TN_LAUNCH(MODE)                                                                             \
  do {                                                                                              \
    if (p.M <= 4) hipLaunchKernelGGL((tn_skinny_kernel<MODE>), gsk, dim3(256), 0, s, p);           \
    else if (MODE == MHADA_A_ROWS && p.rsrc && bm == 64)                                            \
      hipLaunchKernelGGL((gemm_tn_kernel<MHADA_A_ROWS, true, 64, true>), grid, dim3(256), 0, s, p); \
    else if (MODE == MHADA_A_ROWS && p.rsrc)                                                        \
      hipLaunchKernelGGL((gemm_tn_kernel<MHADA_A_ROWS, true, 128, true>), grid, dim3(256), 0, s, p); \
    else if (bm == 64 && vec_a) hipLaunchKernelGGL((gemm_tn_kernel<MODE, true, 64>), grid, dim3(256), 0, s, p); \
    else if (bm == 64) hipLaunchKernelGGL((gemm_tn_kernel<MODE, false, 64>), grid, dim3(256), 0, s, p); \
    else if (vec_a) hipLaunchKernelGGL((gemm_tn_kernel<MODE, true, 128>), grid, dim3(256), 0, s, p); \
    else hipLaunchKernelGGL((gemm_tn_kernel<MODE, false, 128>), grid, dim3(256), 0, s, p);         \
  } while (0)
  if (a->b_mode == MHADA_A_ROWS) TN_LAUNCH(MHADA_A_ROWS);
  else if (a->b_mode == MHADA_A_CONV3X3) TN_LAUNCH(MHADA_A_CONV3X3);
  else if (a->b_mode == MHADA_A_PATCH8) {
    if (p.M <= 4) return fail("mhada_gemm_tn: PATCH8 needs M > 4");
    TN_LAUNCH(MHADA_A_PATCH8);
  }
  else TN_LAUNCH(MHADA_A_CONV3X3_ZERO);
#undef TN_LAUNCH
  if (int rc = check_launch("mhada_gemm_tn")) return rc;
  const long long mn = (long long)p.nb * p.M * p.N;
  hipLaunchKernelGGL(slab_reduce_kernel, grid1(mn / 4), dim3(256), 0, s, work, a->c, (long long)p.nb * p.M, p.N,
                     a->ldc, S);
  if (int rc = check_launch("mhada_gemm_tn(reduce)")) return rc;
  if (!a->colsum) return 0;
  if (fuse_cs) {
    hipLaunchKernelGGL(slab_reduce_kernel, grid1((long long)p.nb * p.M / 4), dim3(256), 0, s, p.cslab, a->colsum, 1LL,
                       p.nb * p.M, (long long)p.nb * p.M, S);
    return check_launch("mhada_gemm_tn(colsum reduce)");
  }
  if (p.nb > 1) return fail("mhada_gemm_tn: batched column sums need 16-B aligned A with M % 4 == 0");
  // unfused: the column sums of A [K][lda] over its first M columns (the workspace is free again)
  if (a->lda != p.M || p.M % 4 || !al16(a->a)) return fail("mhada_gemm_tn: colsum needs a dense, aligned A");
  return mhada_colsum(a->a, a->colsum, p.K, p.M, work, work_floats, s_);
}

extern "C" int mhada_colsum(const float* x, float* out, long long rows, int C, float* work, long long work_floats,
                            mhada_stream_t s_) {
  if (!x || !out || !work || rows <= 0 || C <= 0) return fail("mhada_colsum: bad args");
  if (C % 4 || !al16(x) || !al16(work)) return fail("mhada_colsum: C % 4 == 0 and 16-byte aligned x, work");
  // up to 128 blocks of at least 64 rows (the fixed-order reduction pass loops over the chunks)
  long long chunks = std::min<long long>(std::max<long long>(1, rows / 64), 128);
  chunks = std::min<long long>(chunks, work_floats / C);
  if (chunks < 1) return fail("mhada_colsum: workspace smaller than C floats");
  const long long rpc = (rows + chunks - 1) / chunks;
  chunks = (rows + rpc - 1) / rpc;
  const dim3 grid((unsigned)chunks, (unsigned)((C / 4 + 255) / 256));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, (hipStream_t)s_, x, work, rows, C, rpc);
  if (int rc = check_launch("mhada_colsum")) return rc;
  hipLaunchKernelGGL(slab_reduce_kernel, grid1(C / 4), dim3(256), 0, (hipStream_t)s_, work, out, 1LL, C, (long long)C,
                     (int)chunks);
  return check_launch("mhada_colsum(reduce)");
}

static int layernorm_fwd_launch(const float* x, float* y, void* planes, float* stats, const float* gamma,
                                const float* beta, int rows, int cols, float eps, hipStream_t s) {
  if (!x || !y || !stats || !gamma || !beta || rows <= 0) return fail("mhada_layernorm_fwd: bad args");
  if (!al16(x) || !al16(y) || !al16(gamma) || !al16(beta) || ((uintptr_t)stats & 7) || ((uintptr_t)planes & 7))
    return fail("mhada_layernorm_fwd: x, y, gamma, beta 16-byte aligned, stats and planes 8-byte aligned");
  const dim3 grid((unsigned)((rows + 3) / 4));
  bf16* pl = reinterpret_cast<bf16*>(planes);
  switch (cols) {
    case 256: hipLaunchKernelGGL(ln_fwd_train_kernel<4>, grid, dim3(256), 0, s, x, y, stats, gamma, beta, rows, eps, pl); break;
    case 512: hipLaunchKernelGGL(ln_fwd_train_kernel<8>, grid, dim3(256), 0, s, x, y, stats, gamma, beta, rows, eps, pl); break;
    case 1024: hipLaunchKernelGGL(ln_fwd_train_kernel<16>, grid, dim3(256), 0, s, x, y, stats, gamma, beta, rows, eps, pl); break;
    default: return fail("mhada_layernorm_fwd: cols must be 256, 512 or 1024");
  }
  return check_launch("mhada_layernorm_fwd");
}

extern "C" int mhada_layernorm_fwd(const float* x, float* y, float* stats, const float* gamma, const float* beta,
                                   int rows, int cols, float eps, mhada_stream_t s_) {
  return layernorm_fwd_launch(x, y, nullptr, stats, gamma, beta, rows, cols, eps, (hipStream_t)s_);
}

extern "C" int mhada_layernorm_fwd_split3(const float* x, float* y, void* planes, float* stats, const float* gamma,
                                          const float* beta, int rows, int cols, float eps, mhada_stream_t s_) {
  if (!planes) return fail("mhada_layernorm_fwd_split3: null planes");
  return layernorm_fwd_launch(x, y, planes, stats, gamma, beta, rows, cols, eps, (hipStream_t)s_);
}

extern "C" int mhada_layernorm_bwd(const float* x, const float* dy, const float* stats, const float* gamma, float* dx,
                                   float* dgamma, float* dbeta, float* work, long long work_floats, int rows, int cols,
                                   mhada_stream_t s_) {
  if (!x || !dy || !stats || !gamma || !dx || !dgamma || !dbeta || !work || rows <= 0)
    return fail("mhada_layernorm_bwd: bad args");
  if (!al16(x) || !al16(dy) || !al16(gamma) || !al16(dx) || !al16(work) || ((uintptr_t)stats & 7))
    return fail("mhada_layernorm_bwd: 16-byte aligned operands");
  const int nblk = (rows + kLnBwdRows - 1) / kLnBwdRows;
  if (work_floats < (long long)nblk * 2 * cols + 2LL * cols) return fail("mhada_layernorm_bwd: workspace too small");
  hipStream_t s = (hipStream_t)s_;
  switch (cols) {
    case 256: hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(nblk), dim3(256), 0, s, x, dy, stats, gamma, dx, work, rows); break;
    case 512: hipLaunchKernelGGL(ln_bwd_kernel<8>, dim3(nblk), dim3(256), 0, s, x, dy, stats, gamma, dx, work, rows); break;
    case 1024: hipLaunchKernelGGL(ln_bwd_kernel<16>, dim3(nblk), dim3(256), 0, s, x, dy, stats, gamma, dx, work, rows); break;
    default: return fail("mhada_layernorm_bwd: cols must be 256, 512 or 1024");
  }
  if (int rc = check_launch("mhada_layernorm_bwd")) return rc;
  float* red = work + (long long)nblk * 2 * cols;  // [dgamma | dbeta]
  hipLaunchKernelGGL(slab_reduce_kernel, grid1(2 * cols / 4), dim3(256), 0, s, work, red, 1LL, 2 * cols,
                     (long long)(2 * cols), nblk);
  if (int rc = check_launch("mhada_layernorm_bwd(reduce)")) return rc;
  if (hipMemcpyAsync(dgamma, red, sizeof(float) * cols, hipMemcpyDeviceToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dbeta, red + cols, sizeof(float) * cols, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return fail("mhada_layernorm_bwd: copy");
  return 0;
}

extern "C" int mhada_instnorm_bwd(const float* dy, const float* y, const float* rstd, float* dx, double* work,
                                  int B, int N, int C, int splits, mhada_stream_t s_) {
  if (!dy || !y || !rstd || !dx || !work || B <= 0 || N <= 0 || C <= 0 || splits <= 0 || splits > 65535)
    return fail("mhada_instnorm_bwd: bad args");
  if (C % 4 || !al16(dy) || !al16(y) || !al16(rstd) || !al16(dx) || !al16(work))
    return fail("mhada_instnorm_bwd: C % 4 == 0 and 16-byte aligned operands");
  hipStream_t s = (hipStream_t)s_;
  hipLaunchKernelGGL(inb_partial_kernel, dim3((C + 63) / 64, B, splits), dim3(256), 0, s, dy, y, work, B, N, C, splits);
  if (int rc = check_launch("mhada_instnorm_bwd/partial")) return rc;
  float* mm = reinterpret_cast<float*>(work + (long long)splits * B * C * 2);  // [B][C][2] means
  hipLaunchKernelGGL(inb_finalize_kernel, grid1((long long)B * C), dim3(256), 0, s, work, mm, B * C, N, splits);
  if (int rc = check_launch("mhada_instnorm_bwd/finalize")) return rc;
  const long long n4 = (long long)B * N * C / 4;
  hipLaunchKernelGGL(inb_apply_kernel, grid1(n4), dim3(256), 0, s, dy, y, mm, rstd, dx, N, C, n4);
  return check_launch("mhada_instnorm_bwd/apply");
}

extern "C" int mhada_attn_train_bwd_prep(const float* dout, const float* x, const float* mo, float* dx, float* dmo,
                                         float* dd, long long rows, mhada_stream_t s_) {
  if (!dout || !x || !mo || !dx || !dmo || !dd || rows <= 0) return fail("mhada_attn_train_bwd_prep: bad args");
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)s_, dout, x,
                     mo, dx, dmo, dd, rows);
  return check_launch("mhada_attn_train_bwd_prep");
}

extern "C" int mhada_pos_embed_bwd(const float* g, float* gpos, int C, int bh, int bw, int oh, int ow,
                                   mhada_stream_t s_) {
  if (!g || !gpos || C <= 0 || bh <= 0 || bw <= 0 || oh <= 0 || ow <= 0) return fail("mhada_pos_embed_bwd: bad args");
  hipLaunchKernelGGL(pos_embed_bwd_kernel, grid1((long long)C * bh * bw), dim3(256), 0, (hipStream_t)s_, g, gpos, C, bh,
                     bw, oh, ow);
  return check_launch("mhada_pos_embed_bwd");
}

extern "C" int mhada_relu_bwd(const float* dy, const float* y, float* dx, long long n, mhada_stream_t s_) {
  if (!dy || !y || !dx || n <= 0 || n % 4 || !al16(dy) || !al16(y) || !al16(dx))
    return fail("mhada_relu_bwd: bad args (n % 4 == 0, 16-byte aligned)");
  hipLaunchKernelGGL(relu_bwd_kernel, grid1(n / 4), dim3(256), 0, (hipStream_t)s_, dy, y, dx, n / 4);
  return check_launch("mhada_relu_bwd");
}

namespace mhada {
// ---------------------------------------------------------------------------------------
// Forward statistics of one VGG feature map for the losses (lossfn.py:7-47): per (b, c) the mean
// and the UNBIASED std over the P pixels (x.mean / x.std(dim=(2,3))) and, with a target t, the
// sum of (x - t)^2 (F.mse_loss numerator) — ONE read of x (and t) in place of aten's mean,
// Welford-std and mse passes.  NHWC storage [B][P][C]; fp64 partial sums per (split, b, c) and
// per (split, b, channel block), reduced in a fixed order (deterministic).
// grid (C/64, B, splits), 256 threads = 64 channels x 4 row phases (in_partial_kernel's layout).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) feat_stats_partial_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ t,
                                                                 double* __restrict__ work, double* __restrict__ sse,
                                                                 int B, long long P, int C, int splits, int stats) {
  __shared__ double red[3][16][65];
  const int quad = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 64 + 4 * quad;
  const int b = blockIdx.y, s = blockIdx.z;
  const long long per = (P + splits - 1) / splits;
  const long long r0 = s * per, r1 = min(P, r0 + per);
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0}, se = 0.0;
  if (c0 < C) {  // C % 4 == 0 (checked by the entry point)
    const float* xb = x + (long long)b * P * C + c0;
    const float* tb = t ? t + (long long)b * P * C + c0 : nullptr;
#pragma unroll 4
    for (long long r = r0 + ph; r < r1; r += 16) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xb + r * C);
      if (stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double d = (double)v[e];
          s1[e] += d;
          s2[e] += d * d;
        }
      }
      if (tb) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(tb + r * C);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double d = (double)v[e] - (double)w[e];
          se += d * d;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][ph][4 * quad + e] = s1[e];
    red[1][ph][4 * quad + e] = s2[e];
  }
  red[2][ph][quad] = se;
  __syncthreads();
  if (threadIdx.x < 128 && stats) {
    const int tt = threadIdx.x & 63, which = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + tt;
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += red[which][k][tt];
    if (c < C) work[(((long long)s * B + b) * C + c) * 2 + which] = a;
  }
  if (threadIdx.x == 128 && t) {
    double a = 0.0;
    for (int k = 0; k < 16; ++k)
      for (int q = 0; q < 16; ++q) a += red[2][k][q];
    sse[((long long)s * B + b) * gridDim.x + blockIdx.x] = a;
  }
}

// mean / unbiased std per (b, c) from the partials (16 outputs x 16 split phases per block, as
// in_finalize_kernel); block 0 also sums the sse partials in index order into mse = sse / n.
__global__ void __launch_bounds__(256) feat_stats_finalize_kernel(const double* __restrict__ work,
                                                                  const double* __restrict__ sse, float* __restrict__ mu,
                                                                  float* __restrict__ sd, float* __restrict__ mse, int B,
                                                                  long long P, int C, int splits, int nsse,
                                                                  double inv_n, int stats) {
  __shared__ double red[2][16][17];
  const int o = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int idx = blockIdx.x * 16 + o;
  if (stats) {
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
      const double mean = sa / (double)P;
      // unbiased (torch.std): a single-pixel map has no variance estimate, NaN as in the reference
      double var = P > 1 ? (sq - mean * sa) / (double)(P - 1) : (double)NAN;
      if (var < 0.0) var = 0.0;
      mu[idx] = (float)mean;
      sd[idx] = (float)sqrt(var);
    }
  }
  if (mse && blockIdx.x == 0) {  // fixed-order block reduction of the per-block sse partials
    __shared__ double rs[256];
    double a = 0.0;
    for (int i = threadIdx.x; i < nsse; i += 256) a += sse[i];
    rs[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) rs[threadIdx.x] += rs[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) mse[0] = (float)(rs[0] * inv_n);
  }
}

}  // namespace mhada

extern "C" int mhada_feat_stats(const float* x, const float* t, float* mu, float* sd, float* mse, double* work,
                                long long work_doubles, int B, long long P, int C, mhada_stream_t s_) {
  const bool stats = mu && sd;
  if (!x || B <= 0 || P <= 0 || C <= 0 || C % 4 || !al16(x) || (t && !al16(t)) || (!stats && !(t && mse)) ||
      (bool)t != (bool)mse || !work)
    return fail("mhada_feat_stats: bad args (C % 4 == 0, 16-byte aligned; mean + std and / or t + mse)");
  const int cb = (C + 63) / 64;
  int splits = (int)std::min<long long>(std::max<long long>(1, (4 * 256 + (long long)B * cb - 1) / ((long long)B * cb)),
                                        std::max<long long>(1, P / 64));
  splits = std::min(splits, 65535);
  const long long need = (long long)splits * B * C * 2 + (long long)splits * B * cb;
  if (work_doubles < need) return fail("mhada_feat_stats: workspace too small (mhada_feat_stats_work)");
  double* sse = work + (long long)splits * B * C * 2;
  const hipStream_t s = (hipStream_t)s_;
  hipLaunchKernelGGL(feat_stats_partial_kernel, dim3(cb, B, splits), dim3(256), 0, s, x, t, work, sse, B, P, C, splits,
                     stats ? 1 : 0);
  if (int rc = check_launch("mhada_feat_stats/partial")) return rc;
  hipLaunchKernelGGL(feat_stats_finalize_kernel, dim3(stats ? (B * C + 15) / 16 : 1), dim3(256), 0, s, work, sse, mu, sd,
                     mse, B, P, C, splits, splits * B * cb, 1.0 / ((double)B * P * C), stats ? 1 : 0);
  return check_launch("mhada_feat_stats/finalize");
}

extern "C" long long mhada_feat_stats_work(int B, long long P, int C) {
  if (B <= 0 || P <= 0 || C <= 0) return 0;
  const int cb = (C + 63) / 64;
  long long splits = std::min<long long>(std::max<long long>(1, (4 * 256 + (long long)B * cb - 1) / ((long long)B * cb)),
                                         std::max<long long>(1, P / 64));
  splits = std::min<long long>(splits, 65535);
  return splits * B * C * 2 + splits * B * cb;
}

extern "C" int mhada_feat_loss_bwd(const float* x, const float* t, const float* mu, const float* alpha,
                                   const float* beta, const float* kp, float ks, float* g, int B, long long P,
                                   int C, int relu, mhada_stream_t s_) {
  if (!x || !g || B <= 0 || P <= 0 || C <= 0 || C % 4 || !al16(x) || !al16(g) || (t && !al16(t)))
    return fail("mhada_feat_loss_bwd: bad args (C % 4 == 0, 16-byte aligned)");
  if (alpha && (!beta || !mu || !al16(alpha) || !al16(beta) || !al16(mu)))
    return fail("mhada_feat_loss_bwd: alpha needs beta and mu (16-byte aligned)");
  const long long n4 = (long long)B * P * (C / 4);
  hipLaunchKernelGGL(feat_loss_bwd_kernel, grid1(n4), dim3(256), 0, (hipStream_t)s_, x, t, mu, alpha, beta, kp, ks,
                     g, P * (C / 4), C / 4, n4, relu);
  return check_launch("mhada_feat_loss_bwd");
}

extern "C" int mhada_reflect_fold(const float* dxp, float* dx, int B, int H, int W, int C, const float* relu_mask,
                                  mhada_stream_t s_) {
  if (!dxp || !dx || B <= 0 || H < 2 || W < 2 || C % 4 || !al16(dxp) || !al16(dx) || (relu_mask && !al16(relu_mask)))
    return fail("mhada_reflect_fold: bad args");
  hipLaunchKernelGGL(reflect_fold_kernel, grid1((long long)B * H * W * (C / 4)), dim3(256), 0, (hipStream_t)s_, dxp, dx,
                     B, H, W, C, relu_mask);
  return check_launch("mhada_reflect_fold");
}

extern "C" int mhada_maxpool2(const float* x, float* y, int B, int H, int W, int C, mhada_stream_t s_) {
  if (!x || !y || B <= 0 || H < 2 || W < 2 || C % 4 || !al16(x) || !al16(y)) return fail("mhada_maxpool2: bad args");
  hipLaunchKernelGGL(maxpool2_kernel, grid1((long long)B * (H / 2) * (W / 2) * (C / 4)), dim3(256), 0, (hipStream_t)s_,
                     x, y, B, H, W, C);
  return check_launch("mhada_maxpool2");
}

extern "C" int mhada_maxpool2_bwd(const float* x, const float* dy, float* dx, int B, int H, int W, int C,
                                  int relu_mask, mhada_stream_t s_) {
  if (!x || !dy || !dx || B <= 0 || H < 2 || W < 2 || C % 4 || !al16(x) || !al16(dy) || !al16(dx))
    return fail("mhada_maxpool2_bwd: bad args");
  if (H % 2 || W % 2) (void)hipMemsetAsync(dx, 0, (size_t)B * H * W * C * sizeof(float), (hipStream_t)s_);
  hipLaunchKernelGGL(maxpool2_bwd_kernel, grid1((long long)B * (H / 2) * (W / 2) * (C / 4)), dim3(256), 0,
                     (hipStream_t)s_, x, dy, dx, B, H, W, C, relu_mask);
  return check_launch("mhada_maxpool2_bwd");
}

extern "C" int mhada_upsample2x_bwd(const float* dy, const float* relu_x, float* dx, int B, int H, int W, int C,
                                    mhada_stream_t s_) {
  if (!dy || !dx || B <= 0 || H <= 0 || W <= 0 || C % 4 || !al16(dy) || !al16(dx) || !al16(relu_x))
    return fail("mhada_upsample2x_bwd: bad args");
  hipLaunchKernelGGL(upsample2x_bwd_kernel, grid1((long long)B * H * W * (C / 4)), dim3(256), 0, (hipStream_t)s_, dy,
                     relu_x, dx, B, H, W, C);
  return check_launch("mhada_upsample2x_bwd");
}

extern "C" int mhada_vgg_input(const float* img, float* out, int B, int H, int W, int Cp, mhada_stream_t s_) {
  if (!img || !out || B <= 0 || H <= 0 || W <= 0 || Cp < 3) return fail("mhada_vgg_input: bad args");
  hipLaunchKernelGGL(vgg_input_kernel, grid1((long long)B * H * W), dim3(256), 0, (hipStream_t)s_, img, out, B, H, W, Cp);
  return check_launch("mhada_vgg_input");
}

extern "C" int mhada_vgg_input_bwd(const float* dout, float* dimg, int B, int H, int W, int Cp, mhada_stream_t s_) {
  if (!dout || !dimg || B <= 0 || H <= 0 || W <= 0 || Cp < 3) return fail("mhada_vgg_input_bwd: bad args");
  hipLaunchKernelGGL(vgg_input_bwd_kernel, grid1((long long)B * H * W), dim3(256), 0, (hipStream_t)s_, dout, dimg, B, H,
                     W, Cp);
  return check_launch("mhada_vgg_input_bwd");
}

extern "C" int mhada_vit_batch_attn_bwd(const float* qkv, const float* dout, float* dqkv, int L, int ntok, int heads,
                                        int head_dim, mhada_stream_t s_) {
  if (!qkv || !dout || !dqkv || L <= 0 || L > 8 || ntok <= 0 || heads <= 0)
    return fail("mhada_vit_batch_attn_bwd: bad args (1 <= L <= 8)");
  if (head_dim != 64) return fail("mhada_vit_batch_attn_bwd: head_dim must be 64");
  const long long pairs = (long long)ntok * heads;
  hipLaunchKernelGGL(vit_batch_attn_bwd_kernel, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, (hipStream_t)s_, qkv,
                     dout, dqkv, L, ntok, heads, nullptr, 0LL);
  return check_launch("mhada_vit_batch_attn_bwd");
}

extern "C" int mhada_vit_batch_attn_bwd_split3(const float* qkv, const float* dout, float* dqkv, void* planes,
                                               long long pstride, int L, int ntok, int heads, int head_dim,
                                               mhada_stream_t s_) {
  if (!qkv || !dout || !dqkv || !planes || L <= 0 || L > 8 || ntok <= 0 || heads <= 0)
    return fail("mhada_vit_batch_attn_bwd_split3: bad args (1 <= L <= 8)");
  if (head_dim != 64) return fail("mhada_vit_batch_attn_bwd_split3: head_dim must be 64");
  if (pstride < (long long)L * ntok * 3 * heads * head_dim)
    return fail("mhada_vit_batch_attn_bwd_split3: plane stride smaller than this call's dqkv");
  const long long pairs = (long long)ntok * heads;
  hipLaunchKernelGGL(vit_batch_attn_bwd_kernel, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, (hipStream_t)s_, qkv,
                     dout, dqkv, L, ntok, heads, reinterpret_cast<bf16*>(planes), pstride);
  return check_launch("mhada_vit_batch_attn_bwd_split3");
}
