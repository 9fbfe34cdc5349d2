// The 3-channel ends of the two training conv stacks (fp32, train_image.py:139 backward):
//
//   mhada_vgg_stem_dgrad  input gradient of VGG19's first layer (vgg19.py:10-11,25-26:
//                     imageNet1k_normalize -> Conv2d(3, 64, 3, padding=1) -> ReLU) with respect
//                     to the RGB image: the ReLU adjoint, the zero-padded 3x3 transposed conv
//                     64 -> 3 and the normalisation adjoint in one pass, NCHW image gradient out.
//   mhada_out3_dgrad  input gradient of the decoder's last layer (conv.py:39-45,94: ReflectionPad2d(1)
//                     -> Conv2d(64, 3, 3) -> ReLU): ReLU adjoint, transposed conv 3 -> 64 and the
//                     ReflectionPad2d adjoint (border pixels collect the mirrored taps) in one pass.
//   mhada_out3_wgrad  that layer's weight and bias gradients: per-workgroup partial sums over
//                     pixels, then a fixed-order reduction (deterministic, no float atomics).
//
// On the general conv kernels these layers pad their 3 channels to 32 (dgrad) or run 64-column
// GEMM tiles for 3 live columns; as dedicated kernels they are HBM / VALU streams over the 64-
// channel side.  The forward of the decoder layer is mhada_conv3x3_out3 (small_ops.hip).
// Layouts: 64-channel activations NHWC, 3-channel tensors NCHW (the image-side layout).
#include "common.h"

namespace mhada {
namespace {

// ---------------------------------------------------------------------------------------
// VGG stem input gradient.  dimg[b][c][p] = (sum_{tap, co} g[p + d_tap][co] W[co][c][8 - tap])
// / std_c / 255 with g = dy * (y > 0) (zero outside the image); wd[tap][co][c] = W[co][c][8-tap].
// Workgroup = a strip of kStemRows tiles of 4 rows x 64 pixels (wave = row, lane = pixel); the
// masked 6 x 66-pixel halo of g is staged in LDS in CC-channel chunks, double buffered, the next
// chunk in flight in registers while this one's FMAs run; weights are wave-uniform (scalar
// operands).
// ---------------------------------------------------------------------------------------
constexpr int kStemRows = 8;

template <int CC>
__global__ void __launch_bounds__(256) vgg_stem_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                             const float* __restrict__ wd, float* __restrict__ dimg,
                                                             int H, int W, int tiles_x, int strips_y) {
  constexpr int CIN = 64, TR = 4, TC = 64, HR = TR + 2, HC = TC + 2, LP = CC + 4, NCK = CIN / CC;
  constexpr int Q = CC / 4, NQ = HR * HC * Q, PER = (NQ + 255) / 256;
  __shared__ __attribute__((aligned(16))) float tile[2][HR * HC * LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bt = blockIdx.x, tx = bt % tiles_x, sy = (bt / tiles_x) % strips_y, b = bt / (tiles_x * strips_y);
  const int x0 = tx * TC, ys = sy * TR * kStemRows;
  const long long img = (long long)b * H * W * CIN;
  f32x4 st[PER];
  auto fetch = [&](int y0, int ck) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = min(tid + 256 * i, NQ - 1);
      const int pix = c / Q, q = c - pix * Q;
      const int r = pix / HC, cc = pix - r * HC;
      const int Y = y0 - 1 + r, X = x0 - 1 + cc;
      const bool in = Y >= 0 && Y < H && X >= 0 && X < W;
      const long long off = img + ((long long)min(max(Y, 0), H - 1) * W + min(max(X, 0), W - 1)) * CIN + ck * CC + 4 * q;
      const f32x4 g = *reinterpret_cast<const f32x4*>(dy + off);
      const f32x4 v = *reinterpret_cast<const f32x4*>(y + off);
#pragma unroll
      for (int e = 0; e < 4; ++e) st[i][e] = (in && v[e] > 0.f) ? g[e] : 0.f;
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
  const int nt = min(kStemRows, (H - ys + TR - 1) / TR);
  const int steps = nt * NCK;
  fetch(ys, 0);
  commit(tile[0]);
  __syncthreads();
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int s = 0; s < steps; ++s) {
    const int r = s / NCK, ck = s - r * NCK;
    const float* t = tile[s & 1];
    if (s + 1 < steps) fetch(ys + ((s + 1) / NCK) * TR, (s + 1) % NCK);
    const float* wc = wd + ck * CC * 3;  // [tap][co][c]
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float* px = t + ((wave + tap / 3) * HC + lane + tap % 3) * LP;
      const float* wt = wc + tap * CIN * 3;
#pragma unroll
      for (int c = 0; c < CC; c += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(px + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a0 = fmaf(v[e], wt[(c + e) * 3 + 0], a0);
          a1 = fmaf(v[e], wt[(c + e) * 3 + 1], a1);
          a2 = fmaf(v[e], wt[(c + e) * 3 + 2], a2);
        }
      }
    }
    if (ck == NCK - 1) {
      const int yy = ys + r * TR + wave, xx = x0 + lane;
      if (yy < H && xx < W) {
        // the adjoint of (x / 255 - mean) / std (vgg19.py:11), as mhada_vgg_input_bwd
        const long long plane = (long long)H * W, o = (long long)b * 3 * plane + (long long)yy * W + xx;
        dimg[o] = a0 / 0.229f / 255.0f;
        dimg[o + plane] = a1 / 0.224f / 255.0f;
        dimg[o + 2 * plane] = a2 / 0.225f / 255.0f;
      }
      a0 = a1 = a2 = 0.f;
    }
    if (s + 1 < steps) commit(tile[(s + 1) & 1]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Decoder last layer, input gradient.  Forward: out[q] = relu(b + sum_tap W[tap] x[R(q + d_tap)])
// with R the reflection into the image.  With g = dy * (out > 0) and the full correlation on the
// padded grid T(u) = sum_tap [q = u - d_tap inside] W[tap]^T g[q] (u in [-1, H] x [-1, W]),
// dx[p] = sum of T(u) over the padded positions u that R maps to p: u = p, plus u = -1 when
// p = 1 and u = H when p = H - 2 (per axis).  Workgroup = 4 rows x 64 pixels (wave = row, lane =
// pixel); g's masked 6 x 66 halo (zero outside the image, 3 channels + pad = one float4) in
// LDS; 64 accumulators per lane, weights wd[tap][co][ci] wave-uniform; the 64 x 64 result of a
// wave goes out through LDS as whole 1-KiB row slices.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) out3_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                         const float* __restrict__ wd, const float* __restrict__ relu_x,
                                                         float* __restrict__ dx, int H, int W, int tiles_x,
                                                         int tiles_y) {
  constexpr int C = 64, TR = 4, TC = 64, HR = TR + 2, HC = TC + 2, OS = C + 4;
  __shared__ __attribute__((aligned(16))) f32x4 halo[HR * HC];
  __shared__ __attribute__((aligned(16))) float sout[TR][TC * OS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bt = blockIdx.x, tx = bt % tiles_x, ty = (bt / tiles_x) % tiles_y, b = bt / (tiles_x * tiles_y);
  const int x0 = tx * TC, y0 = ty * TR;
  const long long plane = (long long)H * W;
  const float* gb = dy + (long long)b * 3 * plane;
  const float* yb = y + (long long)b * 3 * plane;
  for (int i = tid; i < HR * HC; i += 256) {
    const int r = i / HC, cc = i - r * HC;
    const int Y = y0 - 1 + r, X = x0 - 1 + cc;
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    if (Y >= 0 && Y < H && X >= 0 && X < W) {
      const long long o = (long long)Y * W + X;
#pragma unroll
      for (int c = 0; c < 3; ++c) g[c] = yb[o + c * plane] > 0.f ? gb[o + c * plane] : 0.f;
    }
    halo[i] = g;
  }
  __syncthreads();
  const int py = y0 + wave, px = x0 + lane;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  // one tap: acc += W[tap]^T g[q], q = (qy, qx) in image coordinates (inside the halo)
  auto tap_add = [&](int tap, int qy, int qx) __attribute__((always_inline)) {
    const f32x4 g = halo[(qy - y0 + 1) * HC + (qx - x0 + 1)];
    const float* wt = wd + tap * 3 * C;
#pragma unroll
    for (int co = 0; co < 3; ++co)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = fmaf(g[co], wt[co * C + c], acc[c]);
  };
  // T(u) at a mirrored position: only taps whose source is inside the image
  auto t_mirror = [&](int uy, int ux) {
    for (int tap = 0; tap < 9; ++tap) {
      const int qy = uy - (tap / 3 - 1), qx = ux - (tap % 3 - 1);
      if (qy >= 0 && qy < H && qx >= 0 && qx < W) tap_add(tap, qy, qx);
    }
  };
  if (py < H) {
    // T(p): the halo is zero outside the image, so all 9 taps read it unconditionally
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) tap_add(tap, py - (tap / 3 - 1), px - (tap % 3 - 1));
    if (px < W) {
      const bool ey0 = py == 1, ey1 = py == H - 2, ex0 = px == 1, ex1 = px == W - 2;
      if (ey0) t_mirror(-1, px);
      if (ey1) t_mirror(H, px);
      if (ex0) {
        t_mirror(py, -1);
        if (ey0) t_mirror(-1, -1);
        if (ey1) t_mirror(H, -1);
      }
      if (ex1) {
        t_mirror(py, W);
        if (ey0) t_mirror(-1, W);
        if (ey1) t_mirror(H, W);
      }
    }
  }
  float* so = sout[wave];
#pragma unroll
  for (int c = 0; c < C; c += 4)
    *reinterpret_cast<f32x4*>(so + lane * OS + c) = f32x4{acc[c], acc[c + 1], acc[c + 2], acc[c + 3]};
  __syncthreads();
  if (py < H) {
    const long long row = (((long long)b * H + py) * W + x0) * C;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int ch = lane + 64 * j, pix = ch >> 4, c4 = ch & 15;
      if (x0 + pix < W) {
        const long long o = row + (long long)pix * C + 4 * c4;
        f32x4 v = *reinterpret_cast<const f32x4*>(so + pix * OS + 4 * c4);
        if (relu_x) {  // the ReLU adjoint of the layer that produced x (its only consumer is this one)
          const f32x4 xv = *reinterpret_cast<const f32x4*>(relu_x + o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = xv[e] > 0.f ? v[e] : 0.f;
        }
        *reinterpret_cast<f32x4*>(dx + o) = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Decoder last layer, weight / bias gradients.  dW[co][ci][tap] = sum_{b,q} g[b][q][co]
// x[b][R(q + d_tap)][ci], db[co] = sum g.  Workgroup = 8 waves, wave = kWgRowsPerWave image rows,
// lane = input channel ci; a wave walks its row left to right keeping the 3 x 3 reflected
// neighbourhood of x in registers (3 new 256-B loads per pixel, the next group's columns in
// flight during this group's FMAs); the masked g of a 64-pixel row segment is one value per lane,
// read back per pixel with v_readlane.
// The 8 waves' sums are added in LDS in a fixed order and written as the workgroup's partial;
// out3_wgrad_finish sums the partials in a fixed order.
// ---------------------------------------------------------------------------------------
constexpr int kWgRowsPerWave = 2, kWgWaves = 8, kWgRows = kWgRowsPerWave * kWgWaves;
constexpr int kWgOut = 27 * 64 + 3;  // partial: [co][ci][tap] then db[co]
constexpr int kGrp = 4;              // pixels per register group

__global__ void __launch_bounds__(512) out3_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                         const float* __restrict__ y, float* __restrict__ part, int H,
                                                         int W, int strips) {
  constexpr int C = 64;
  __shared__ float red[kWgWaves][30][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.x / strips, strip = blockIdx.x - b * strips;
  const long long plane = (long long)H * W;
  const float* xb = x + (long long)b * plane * C + lane;
  const float* gb = dy + (long long)b * 3 * plane;
  const float* yb = y + (long long)b * 3 * plane;
  auto refl = [](int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); };
  float acc[27], ab[3];
#pragma unroll
  for (int i = 0; i < 27; ++i) acc[i] = 0.f;
  ab[0] = ab[1] = ab[2] = 0.f;
  for (int rr = 0; rr < kWgRowsPerWave; ++rr) {
    const int row = strip * kWgRows + rr * kWgWaves + wave;
    if (row >= H) break;
    const long long rofs[3] = {(long long)refl(row - 1, H) * W, (long long)row * W, (long long)refl(row + 1, H) * W};
    // window columns c-1, c, ..., c+kGrp: win[j][r] = x[rows r][refl(c - 1 + j)]
    float win[kGrp + 2][3], nxt[kGrp][3];
    auto ld = [&](int col, float (&v)[3]) {
      const long long cc = refl(min(col, W), W);  // columns past W + 1 are never used (clamped)
#pragma unroll
      for (int r = 0; r < 3; ++r) v[r] = xb[(rofs[r] + cc) * C];
    };
#pragma unroll
    for (int j = 0; j < kGrp + 2; ++j) ld(j - 1, win[j]);
    for (int s0 = 0; s0 < W; s0 += 64) {
      // masked g of pixel s0 + lane of this row; pixel s0 + i's values are read back with
      // v_readlane (wave-uniform index) as scalar FMA operands
      float gl[3] = {0.f, 0.f, 0.f};
      {
        const int xx = s0 + lane;
        if (xx < W) {
          const long long o = (long long)row * W + xx;
#pragma unroll
          for (int c = 0; c < 3; ++c) gl[c] = yb[o + c * plane] > 0.f ? gb[o + c * plane] : 0.f;
        }
      }
      const int n = min(64, W - s0);
      for (int i0 = 0; i0 < n; i0 += kGrp) {
        const int c = s0 + i0;
        // next group's new columns c + kGrp + 1 .. c + 2 kGrp
#pragma unroll
        for (int j = 0; j < kGrp; ++j) ld(c + kGrp + 1 + j, nxt[j]);
#pragma unroll
        for (int k = 0; k < kGrp; ++k) {
          if (i0 + k < n) {
#pragma unroll
            for (int co = 0; co < 3; ++co) {
              const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl[co]), i0 + k));
              ab[co] += g;
#pragma unroll
              for (int tap = 0; tap < 9; ++tap) acc[co * 9 + tap] = fmaf(g, win[k + tap % 3][tap / 3], acc[co * 9 + tap]);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 3; ++r) win[j][r] = win[kGrp + j][r];
#pragma unroll
        for (int j = 0; j < kGrp; ++j)
#pragma unroll
          for (int r = 0; r < 3; ++r) win[2 + j][r] = nxt[j][r];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 27; ++i) red[wave][i][lane] = acc[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) red[wave][27 + i][lane] = ab[i];
  __syncthreads();
  float* pb = part + (long long)blockIdx.x * kWgOut;
  for (int o = tid; o < 30 * 64; o += 512) {
    const int i = o >> 6, ci = o & 63;
    float s = red[0][i][ci];
#pragma unroll
    for (int w = 1; w < kWgWaves; ++w) s += red[w][i][ci];
    if (i < 27) {
      const int co = i / 9, tap = i - co * 9;
      pb[(co * C + ci) * 9 + tap] = s;
    } else if (ci == 0) {
      pb[27 * 64 + (i - 27)] = s;  // every lane holds the same bias sum
    }
  }
}

// out[o] = sum_blk part[blk][o] in blk order: 16 waves per workgroup each sum a contiguous
// range of partials for 64 outputs, then wave 0 adds the 16 range sums in order.
__global__ void __launch_bounds__(1024) out3_wgrad_finish_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                                 float* __restrict__ db, int nblk) {
  __shared__ float red[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int o = blockIdx.x * 64 + lane;
  const int per = (nblk + 15) / 16, s0 = wave * per, s1 = min(nblk, s0 + per);
  float s = 0.f;
  if (o < kWgOut) {
    int k = s0;
    for (; k + 8 <= s1; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long long)(k + j) * kWgOut + o];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < s1; ++k) s += part[(long long)k * kWgOut + o];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && o < kWgOut) {
    float t = red[0][lane];
#pragma unroll
    for (int w = 1; w < 16; ++w) t += red[w][lane];
    if (o < 27 * 64) dw[o] = t;
    else if (db) db[o - 27 * 64] = t;
  }
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int mhada_vgg_stem_dgrad(const float* dy, const float* y, const float* wd, float* dimg, int B, int H, int W,
                                    mhada_stream_t s_) {
  if (!dy || !y || !wd || !dimg || B <= 0 || H <= 0 || W <= 0) return fail("mhada_vgg_stem_dgrad: bad args");
  if (!al16(dy) || !al16(y)) return fail("mhada_vgg_stem_dgrad: dy / y must be 16-byte aligned");
  if ((long long)B * H * W * 64 >= (1LL << 40)) return fail("mhada_vgg_stem_dgrad: too large");
  const int tiles_x = (W + 63) / 64, strips_y = (H + 4 * kStemRows - 1) / (4 * kStemRows);
  const long long nb = (long long)B * strips_y * tiles_x;
  if (nb >= (1LL << 31)) return fail("mhada_vgg_stem_dgrad: grid too large");
  hipLaunchKernelGGL((vgg_stem_dgrad_kernel<16>), dim3((unsigned)nb), dim3(256), 0, (hipStream_t)s_, dy, y, wd, dimg, H,
                     W, tiles_x, strips_y);
  return check_launch("mhada_vgg_stem_dgrad");
}

extern "C" int mhada_out3_dgrad(const float* dy, const float* y, const float* wd, const float* relu_x, float* dx, int B,
                                int H, int W, mhada_stream_t s_) {
  if (!dy || !y || !wd || !dx || B <= 0 || H < 2 || W < 2) return fail("mhada_out3_dgrad: bad args (H, W >= 2)");
  if (!al16(dx) || !al16(relu_x)) return fail("mhada_out3_dgrad: dx / relu_x must be 16-byte aligned");
  const int tiles_x = (W + 63) / 64, tiles_y = (H + 3) / 4;
  const long long nb = (long long)B * tiles_x * tiles_y;
  if (nb >= (1LL << 31)) return fail("mhada_out3_dgrad: grid too large");
  hipLaunchKernelGGL(out3_dgrad_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)s_, dy, y, wd, relu_x, dx, H, W,
                     tiles_x, tiles_y);
  return check_launch("mhada_out3_dgrad");
}

extern "C" long long mhada_out3_wgrad_work(int B, int H, int W) {
  if (B <= 0 || H < 2 || W < 2) return -1;
  return (long long)B * ((H + kWgRows - 1) / kWgRows) * kWgOut;
}

extern "C" int mhada_out3_wgrad(const float* x, const float* dy, const float* y, float* dw, float* db, float* work,
                                long long work_floats, int B, int H, int W, mhada_stream_t s_) {
  if (!x || !dy || !y || !dw || !work || B <= 0 || H < 2 || W < 2) return fail("mhada_out3_wgrad: bad args (H, W >= 2)");
  const int strips = (H + kWgRows - 1) / kWgRows;
  const long long nblk = (long long)B * strips;
  if (nblk >= (1LL << 31) || work_floats < nblk * kWgOut) return fail("mhada_out3_wgrad: work buffer too small");
  hipStream_t s = (hipStream_t)s_;
  hipLaunchKernelGGL(out3_wgrad_kernel, dim3((unsigned)nblk), dim3(512), 0, s, x, dy, y, work, H, W, strips);
  if (int rc = check_launch("mhada_out3_wgrad")) return rc;
  hipLaunchKernelGGL(out3_wgrad_finish_kernel, dim3((kWgOut + 63) / 64), dim3(1024), 0, s, work, dw, db, (int)nblk);
  return check_launch("mhada_out3_wgrad(finish)");
}

}  // namespace mhada
