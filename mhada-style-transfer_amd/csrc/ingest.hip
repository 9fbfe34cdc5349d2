// Video frame ingest: the per-frame input conversion of infer_video.py:80,
// utilities.cv2_to_tensor (utilities.py:43-52) on the device:
//   cv2.cvtColor(BGR -> RGB); cv2.resize(..., INTER_AREA) (box average when shrinking or same
//   size; OpenCV's area-mode 2-tap interpolation when enlarging, frame_ingest_up_kernel);
//   toTensor255 = ToTensor() (u8 HWC -> fp32 CHW / 255) then .mul(255)   (utilities.py:11-16)
// in one HBM-bound pass over a u8 HWC frame already in device memory.
//
// INTER_AREA (OpenCV cv::resize, the area-average definition): output pixel (x, y) is the mean
// of the input over the box [x*sx, (x+1)*sx) x [y*sy, (y+1)*sy), sx = W/Wo, sy = H/Ho, each input
// pixel weighted by its overlap with the box; the result is rounded to the nearest u8 (half to
// even, cvRound) because cv2.resize returns the frame's u8 type.  Same size = exact copy.  cv2
// itself is not installed here, so bit parity with cv2 is unpinned: the tests hold this kernel
// to the fp64 area-average definition (exact except at rounding ties).
// Then ToTensor's x / 255 and toTensor255's * 255, two correctly rounded fp32 operations, as torch.
//
// Layout: in [B][H][W][3] u8 rows of `row_bytes` (>= 3W: padded frames allowed); out
// [B][3][Ho][Wo] fp32 (the reference's NCHW model input).  One thread per output pixel (3
// channels): the footprint reads are L1/L2 hits, the three planar stores are coalesced.
#include "common.h"

namespace mhada {

__global__ void __launch_bounds__(256) frame_ingest_kernel(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                            int H, int W, long long row_bytes, int Ho, int Wo,
                                                            int bgr, float sx, float sy) {
  const int b = blockIdx.y;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (long long)Ho * Wo) return;
  const int oy = (int)(pix / Wo), ox = (int)(pix - (long long)oy * Wo);
  const uint8_t* frame = in + (long long)b * H * row_bytes;
  float c0, c1, c2;
  if (Ho == H && Wo == W) {
    const uint8_t* p = frame + (long long)oy * row_bytes + 3LL * ox;
    c0 = p[0]; c1 = p[1]; c2 = p[2];
  } else {
    // box [fx1, fx2) x [fy1, fy2) in input pixels, clipped to the image
    const float fx1 = ox * sx, fx2 = fminf((ox + 1) * sx, (float)W);
    const float fy1 = oy * sy, fy2 = fminf((oy + 1) * sy, (float)H);
    const int x0 = (int)floorf(fx1), x1 = min((int)ceilf(fx2), W);
    const int y0 = (int)floorf(fy1), y1 = min((int)ceilf(fy2), H);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int y = y0; y < y1; ++y) {
      const float wy = fminf((float)(y + 1), fy2) - fmaxf((float)y, fy1);
      const uint8_t* row = frame + (long long)y * row_bytes;
      float r0 = 0.f, r1 = 0.f, r2 = 0.f;
      for (int x = x0; x < x1; ++x) {
        const float wx = fminf((float)(x + 1), fx2) - fmaxf((float)x, fx1);
        const uint8_t* p = row + 3LL * x;
        r0 = fmaf(wx, (float)p[0], r0);
        r1 = fmaf(wx, (float)p[1], r1);
        r2 = fmaf(wx, (float)p[2], r2);
      }
      a0 = fmaf(wy, r0, a0);
      a1 = fmaf(wy, r1, a1);
      a2 = fmaf(wy, r2, a2);
    }
    const float inv = 1.0f / ((fx2 - fx1) * (fy2 - fy1));
    c0 = fminf(fmaxf(rintf(a0 * inv), 0.f), 255.f);
    c1 = fminf(fmaxf(rintf(a1 * inv), 0.f), 255.f);
    c2 = fminf(fmaxf(rintf(a2 * inv), 0.f), 255.f);
  }
  const float r = bgr ? c2 : c0, g = c1, bl = bgr ? c0 : c2;
  const long long plane = (long long)Ho * Wo;
  float* o = out + (long long)b * 3 * plane + pix;
  // ToTensor (/255) then .mul(255): two fp32 roundings, as the reference's tensor ops
  o[0] = (r / 255.0f) * 255.0f;
  o[plane] = (g / 255.0f) * 255.0f;
  o[2 * plane] = (bl / 255.0f) * 255.0f;
}

// INTER_AREA when the output is larger than the frame along either axis: OpenCV's cv::resize
// then takes its generic separable 2-tap path with "area-mode" coefficients (not the box average):
//   per axis, inv = out/in, scale = 1/inv (fp64); for output index d: s = floor(d*scale),
//   f = (float)((d+1) - (s+1)*inv), f = f <= 0 ? 0 : f - floor(f); taps (s, s+1) weighted
//   (1-f, f), quantised to 11-bit fixed point (saturate_cast<short>(w*2048), round half even);
//   the source index clamps at the last pixel (f = 0 there);
//   horizontal pass in int: S = a0*p[s] + a1*p[s+1] (one tap p[s]*2048 where s+1 runs off the
//   frame), vertical pass as OpenCV's vectorised 32s->8u kernel: ((S0>>4)*b0 >> 16) +
//   ((S1>>4)*b1 >> 16), then (v + 2) >> 2 saturated to u8.
// (cv2's scalar tail for the last < one-vector of a row rounds (S0*b0 + S1*b1 + 2^21) >> 22
// instead and can differ by one level; cv2 is not installed here, so this too is PARITY
// UNPINNED — the kernel is held bit-exact to oracle.resize_area_up, the numpy restatement.)
struct AreaUpTap {
  int s0, s1, w0, w1;  // source indices and 11-bit weights (w1 = 0 and s1 = s0 for one tap)
};
MHADA_DEV AreaUpTap area_up_tap(int d, int n_in, double inv) {
  const double scale = 1.0 / inv;
  int s = (int)floor(d * scale);
  float f = (float)((d + 1) - (s + 1) * inv);
  f = f <= 0.f ? 0.f : f - floorf(f);
  if (s < 0) { s = 0; f = 0.f; }
  if (s >= n_in - 1) { s = n_in - 1; f = 0.f; }
  AreaUpTap t;
  t.s0 = s;
  t.s1 = min(s + 1, n_in - 1);
  t.w0 = (int)rintf((1.f - f) * 2048.f);
  t.w1 = (int)rintf(f * 2048.f);
  return t;
}

__global__ void __launch_bounds__(256) frame_ingest_up_kernel(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                               int H, int W, long long row_bytes, int Ho, int Wo,
                                                               int bgr, double inv_x, double inv_y) {
  const int b = blockIdx.y;
  const long long pix = (long long)blockIdx.x * 256 + threadIdx.x;
  if (pix >= (long long)Ho * Wo) return;
  const int oy = (int)(pix / Wo), ox = (int)(pix - (long long)oy * Wo);
  const uint8_t* frame = in + (long long)b * H * row_bytes;
  const AreaUpTap tx = area_up_tap(ox, W, inv_x), ty = area_up_tap(oy, H, inv_y);
  // one horizontal tap where s + 1 runs off the frame (OpenCV's xmax border: p[s] * 2048)
  const bool one = (int)floor(ox * (1.0 / inv_x)) + 1 >= W;
  float c[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    int S[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint8_t* row = frame + (long long)(r ? ty.s1 : ty.s0) * row_bytes;
      S[r] = one ? (int)row[3 * tx.s0 + ch] * 2048 : (int)row[3 * tx.s0 + ch] * tx.w0 + (int)row[3 * tx.s1 + ch] * tx.w1;
    }
    const int v = (((S[0] >> 4) * ty.w0) >> 16) + (((S[1] >> 4) * ty.w1) >> 16);
    c[ch] = (float)min(max((v + 2) >> 2, 0), 255);
  }
  const float r = bgr ? c[2] : c[0], g = c[1], bl = bgr ? c[0] : c[2];
  const long long plane = (long long)Ho * Wo;
  float* o = out + (long long)b * 3 * plane + pix;
  o[0] = (r / 255.0f) * 255.0f;
  o[plane] = (g / 255.0f) * 255.0f;
  o[2 * plane] = (bl / 255.0f) * 255.0f;
}

}  // namespace mhada

using namespace mhada;

extern "C" int mhada_frame_ingest(const void* frames, int B, int H, int W, long long row_bytes, int bgr, float* out,
                                  int Ho, int Wo, mhada_stream_t s_) {
  if (!frames || !out || B <= 0 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0)
    return fail("mhada_frame_ingest: bad args");
  if (row_bytes < 3LL * W) return fail("mhada_frame_ingest: row_bytes < 3*W");
  if (B > 65535) return fail("mhada_frame_ingest: too many frames");
  const long long npix = (long long)Ho * Wo;
  const dim3 grid((unsigned)((npix + 255) / 256), (unsigned)B);
  if (Ho > H || Wo > W) {  // an upscaled axis: OpenCV's area-mode 2-tap path
    hipLaunchKernelGGL(frame_ingest_up_kernel, grid, dim3(256), 0, (hipStream_t)s_, (const uint8_t*)frames, out, H, W,
                       row_bytes, Ho, Wo, bgr, (double)Wo / W, (double)Ho / H);
    return check_launch("mhada_frame_ingest");
  }
  hipLaunchKernelGGL(frame_ingest_kernel, grid, dim3(256), 0, (hipStream_t)s_, (const uint8_t*)frames, out, H, W,
                     row_bytes, Ho, Wo, bgr, (float)W / (float)Wo, (float)H / (float)Ho);
  return check_launch("mhada_frame_ingest");
}
