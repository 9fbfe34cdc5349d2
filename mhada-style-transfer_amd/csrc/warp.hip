// Optical-flow warping for the video path: HBM-bound gather kernels.
//
// warp (utilities.py:100-118): vgrid = grid + flow, normalised with (W-1) / (H-1), then
// F.grid_sample(bilinear, align_corners=False) — the two conventions do not cancel, so the
// sample position is ((2(x+fx)/(W-1) - 1) + 1) * W / 2 - 1/2, reproduced here with the same
// fp32 operation order as the reference's tensor ops and ATen's grid_sampler (unnormalise,
// floor, the four corner weights, taps accumulated nw, ne, sw, se; zero padding skips
// out-of-range taps, border padding clamps the coordinate first).
// warp_bwd: the adjoint w.r.t. the warped image, for the temporal losses of train_video.py.
// flow_warp_mask (utilities.py:121-151): forward-backward consistency of two flows.
// warp_l1 (exps_sintel.py:101-109): sum(mask * |cs2 - warp(cs1, flow)|) per image, the
// warping-error metric, fused so the warped frame never reaches HBM; fixed-order fp64
// partial sums (deterministic).
// Layouts are the reference's: NCHW fp32 images/features, flow [B][2][H][W] (x then y).
#include "common.h"

namespace mhada {

struct Tap {
  int x0, y0;
  float wnw, wne, wsw, wse;
  bool inw, ine, isw, ise;
};

// Sample position of output pixel (x, y) displaced by (fx, fy); padding 0 zeros, 1 border.
MHADA_DEV Tap warp_tap(int x, int y, float fx, float fy, int H, int W, int padding) {
  const float dx = (float)(W - 1 > 1 ? W - 1 : 1), dy = (float)(H - 1 > 1 ? H - 1 : 1);
  // vgrid normalisation (utilities.py:112-113), one rounding per tensor op
  float gx = 2.0f * ((float)x + fx);
  gx = gx / dx;
  gx = gx - 1.0f;
  float gy = 2.0f * ((float)y + fy);
  gy = gy / dy;
  gy = gy - 1.0f;
  // grid_sampler_unnormalize, align_corners=False
  float ix = ((gx + 1.f) * (float)W - 1.f) / 2.f;
  float iy = ((gy + 1.f) * (float)H - 1.f) / 2.f;
  if (padding == 1) {  // border: clip_coordinates
    ix = fminf(fmaxf(ix, 0.f), (float)(W - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(H - 1));
  }
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  Tap t;
  t.x0 = (int)fx0;
  t.y0 = (int)fy0;
  const float ix_se = fx0 + 1.f, iy_se = fy0 + 1.f;
  t.wnw = (ix_se - ix) * (iy_se - iy);
  t.wne = (ix - fx0) * (iy_se - iy);
  t.wsw = (ix_se - ix) * (iy - fy0);
  t.wse = (ix - fx0) * (iy - fy0);
  const bool x0in = t.x0 >= 0 && t.x0 < W, x1in = t.x0 + 1 >= 0 && t.x0 + 1 < W;
  const bool y0in = t.y0 >= 0 && t.y0 < H, y1in = t.y0 + 1 >= 0 && t.y0 + 1 < H;
  t.inw = x0in && y0in;
  t.ine = x1in && y0in;
  t.isw = x0in && y1in;
  t.ise = x1in && y1in;
  return t;
}

MHADA_DEV float sample(const float* plane, const Tap& t, int W) {
  float acc = 0.f;
  const long long o = (long long)t.y0 * W + t.x0;
  if (t.inw) acc += plane[o] * t.wnw;
  if (t.ine) acc += plane[o + 1] * t.wne;
  if (t.isw) acc += plane[o + W] * t.wsw;
  if (t.ise) acc += plane[o + W + 1] * t.wse;
  return acc;
}

__global__ void __launch_bounds__(256) warp_kernel(const float* __restrict__ x, const float* __restrict__ flow,
                                                   float* __restrict__ y, int C, int H, int W, int padding) {
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= HW) return;
  const int py = (int)(pix / W), px = (int)(pix - (long long)py * W);
  const float* fl = flow + (long long)b * 2 * HW;
  const Tap t = warp_tap(px, py, fl[pix], fl[HW + pix], H, W, padding);
  const float* xb = x + (long long)b * C * HW;
  float* yb = y + (long long)b * C * HW;
  for (int c = 0; c < C; ++c) yb[c * HW + pix] = sample(xb + c * HW, t, W);
}

// Adjoint of warp w.r.t. x (the temporal losses of train_video.py:147-151 under autograd):
// gx[tap] += w_tap * gy[pix] over the four taps of every output pixel — the scatter of ATen's
// grid_sampler_2d_backward (hardware fp32 atomics there too, so the summation order at a tap hit
// by several pixels is not fixed, in the reference either).  The flow is data in train_video.py
// and gets no gradient.  Grid (pixel blocks, channel groups of cpg, B); zero gradients skipped.
__global__ void __launch_bounds__(256) warp_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ flow,
                                                       float* __restrict__ gx, int C, int H, int W, int padding,
                                                       int cpg) {
  const int b = blockIdx.z;
  const long long HW = (long long)H * W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= HW) return;
  const int py = (int)(pix / W), px = (int)(pix - (long long)py * W);
  const float* fl = flow + (long long)b * 2 * HW;
  const Tap t = warp_tap(px, py, fl[pix], fl[HW + pix], H, W, padding);
  const long long o = (long long)t.y0 * W + t.x0;
  const int c0 = blockIdx.y * cpg, c1 = min(C, c0 + cpg);
  for (int c = c0; c < c1; ++c) {
    const float g = gy[((long long)b * C + c) * HW + pix];
    if (g == 0.f) continue;
    float* plane = gx + ((long long)b * C + c) * HW;
    if (t.inw) unsafeAtomicAdd(plane + o, t.wnw * g);
    if (t.ine) unsafeAtomicAdd(plane + o + 1, t.wne * g);
    if (t.isw) unsafeAtomicAdd(plane + o + W, t.wsw * g);
    if (t.ise) unsafeAtomicAdd(plane + o + W + 1, t.wse * g);
  }
}

// grid + flo01 sampled at grid + flo10 (zero padding), L1 distance to the grid < threshold.
__global__ void __launch_bounds__(256) flow_mask_kernel(const float* __restrict__ flo01, const float* __restrict__ flo10,
                                                        float* __restrict__ mask, int H, int W, float thr, int padding) {
  const long long HW = (long long)H * W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= HW) return;
  const int py = (int)(pix / W), px = (int)(pix - (long long)py * W);
  const Tap t = warp_tap(px, py, flo10[pix], flo10[HW + pix], H, W, padding);
  float e = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float* f = flo01 + c * HW;
    const long long o = (long long)t.y0 * W + t.x0;
    // the sampled field is grid_c + flo01_c (exact integer grid plus the flow, in fp32)
    auto fv = [&](long long oo, int xx, int yy) { return (float)(c == 0 ? xx : yy) + f[oo]; };
    float acc = 0.f;
    if (t.inw) acc += fv(o, t.x0, t.y0) * t.wnw;
    if (t.ine) acc += fv(o + 1, t.x0 + 1, t.y0) * t.wne;
    if (t.isw) acc += fv(o + W, t.x0, t.y0 + 1) * t.wsw;
    if (t.ise) acc += fv(o + W + 1, t.x0 + 1, t.y0 + 1) * t.wse;
    e += fabsf(acc - (float)(c == 0 ? px : py));
  }
  mask[pix] = e < thr ? 1.f : 0.f;
}

// Per-block fp64 partial of sum(mask * |cs2 - warp(cs1, flow)|) over C planes of one image.
__global__ void __launch_bounds__(256) warp_l1_kernel(const float* __restrict__ cs1, const float* __restrict__ cs2,
                                                      const float* __restrict__ flow, const float* __restrict__ mask,
                                                      double* __restrict__ part, int C, int H, int W) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const long long HW = (long long)H * W;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  if (pix < HW) {
    const float m = mask[(long long)b * HW + pix];
    if (m != 0.f) {
      const int py = (int)(pix / W), px = (int)(pix - (long long)py * W);
      const float* fl = flow + (long long)b * 2 * HW;
      const Tap t = warp_tap(px, py, fl[pix], fl[HW + pix], H, W, 0);
      const float* a = cs1 + (long long)b * C * HW;
      const float* o = cs2 + (long long)b * C * HW;
      for (int c = 0; c < C; ++c) acc += (double)(m * fabsf(o[c * HW + pix] - sample(a + c * HW, t, W)));
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)b * gridDim.x + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void __launch_bounds__(256) warp_l1_finalize(const double* __restrict__ part, float* __restrict__ out,
                                                        int nparts, double scale) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += part[(long long)b * nparts + i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[b] = (float)((((red[0] + red[1]) + red[2]) + red[3]) * scale);
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_warp(const float* x, const float* flow, float* y, int B, int C, int H, int W, int padding,
                          mhada_stream_t s_) {
  if (!x || !flow || !y || B <= 0 || C <= 0 || H <= 0 || W <= 0 || B > 65535) return fail("mhada_warp: bad args");
  if (padding != 0 && padding != 1) return fail("mhada_warp: padding must be 0 (zeros) or 1 (border)");
  const long long HW = (long long)H * W;
  hipLaunchKernelGGL(warp_kernel, dim3((unsigned)((HW + 255) / 256), B), dim3(256), 0, (hipStream_t)s_, x, flow, y, C,
                     H, W, padding);
  return check_launch("mhada_warp");
}

extern "C" int mhada_warp_bwd(const float* gy, const float* flow, float* gx, int B, int C, int H, int W, int padding,
                              mhada_stream_t s_) {
  if (!gy || !flow || !gx || B <= 0 || C <= 0 || H <= 0 || W <= 0 || B > 65535)
    return fail("mhada_warp_bwd: bad args");
  if (padding != 0 && padding != 1) return fail("mhada_warp_bwd: padding must be 0 (zeros) or 1 (border)");
  const long long HW = (long long)H * W;
  constexpr int kCpg = 16;
  const dim3 grid((unsigned)((HW + 255) / 256), (unsigned)((C + kCpg - 1) / kCpg), B);
  hipLaunchKernelGGL(warp_bwd_kernel, grid, dim3(256), 0, (hipStream_t)s_, gy, flow, gx, C, H, W, padding, kCpg);
  return check_launch("mhada_warp_bwd");
}

extern "C" int mhada_flow_warp_mask(const float* flo01, const float* flo10, float* mask, int H, int W, float threshold,
                                    int padding, mhada_stream_t s_) {
  if (!flo01 || !flo10 || !mask || H <= 0 || W <= 0) return fail("mhada_flow_warp_mask: bad args");
  if (padding != 0 && padding != 1) return fail("mhada_flow_warp_mask: padding must be 0 (zeros) or 1 (border)");
  const long long HW = (long long)H * W;
  hipLaunchKernelGGL(flow_mask_kernel, dim3((unsigned)((HW + 255) / 256)), dim3(256), 0, (hipStream_t)s_, flo01, flo10,
                     mask, H, W, threshold, padding);
  return check_launch("mhada_flow_warp_mask");
}

extern "C" int mhada_warp_l1(const float* cs1, const float* cs2, const float* flow, const float* mask, double* work,
                             float* out, int B, int C, int H, int W, mhada_stream_t s_) {
  if (!cs1 || !cs2 || !flow || !mask || !work || !out || B <= 0 || C <= 0 || H <= 0 || W <= 0 || B > 65535)
    return fail("mhada_warp_l1: bad args");
  const long long HW = (long long)H * W;
  const unsigned nb = (unsigned)((HW + 255) / 256);
  hipStream_t s = (hipStream_t)s_;
  hipLaunchKernelGGL(warp_l1_kernel, dim3(nb, B), dim3(256), 0, s, cs1, cs2, flow, mask, work, C, H, W);
  hipLaunchKernelGGL(warp_l1_finalize, dim3(B), dim3(256), 0, s, (const double*)work, out, (int)nb,
                     1.0 / ((double)C * (double)HW));
  return check_launch("mhada_warp_l1");
}
