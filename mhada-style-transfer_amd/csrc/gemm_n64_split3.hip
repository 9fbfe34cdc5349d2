// The training attention backward's dQ = dS K (adaDecoder.py:186-198 under train_image.py:139
// autograd; ops.attn_train_bwd after mhada_attn_train_dkv's dS spill) as fp32-accurate SPLIT3 products
// on the bf16 MFMA (round 6).
//
// C[z][m][n] = sum_k A[z][m][k] W[z][n][k] for n < 64: A = dS fp32 rows (M = Nc, K = Ns, 12.9 GB per
// launch at 512^2 B8: 24 images x 8 heads x 4096 x 4096), W = K^T (mhada_transpose64) as three bf16
// planes (mhada_split3_rows).  gemm_n64_kernel (gemm_impl.h) computes it on the fp32 MFMA at 0.73 of
// that pipe's peak while streaming A at 3.6 TB/s; here the products move to the bf16 pipe (6 cross
// products of three round-to-nearest planes, dropped terms < 2^-24 |a w|, as every SPLIT3 kernel) and
// the kernel becomes an A stream: A is split into its planes in registers from the fp32 tile in LDS,
// so HBM carries A once, as fp32.
//
// Tile: 256 rows x 64 columns per workgroup, 8 waves x (32 rows x 64 columns, two 32x32 blocks on
// v_mfma_f32_32x32x16_bf16: W fragment in the first operand slot, A in the second, so each lane ends up
// holding one output row).  K-tiles of 32: A 256 x 32 fp32 (32 KiB) + W 4 x 64 x 32 bf16 (16 KiB: the
// three planes and a duplicate of the third, which keeps every wave's DMA count at 4 A + 2 W
// instructions) per ring slot, three slots (144 KiB), filled by global_load_lds with the XOR swizzle
// applied on the source address; one barrier per K-tile (it publishes tile kt and proves tile kt - 1's
// slot free for the DMA of tile kt + 2).  Each K-tile's 12 MFMAs per column block start from zero and
// are added to the fp32 accumulators by VALU adds (round to nearest) — the bf16 MFMA's truncating sums
// then never accumulate over the 128 K-tiles of a row (the training forward's lesson, attn_split3.hip).
//
// Measured at the 512^2 B8 step's shape (tools/dq_ab.py, profiles/r06_dq_split3_ab.log): 3.23-3.29 vs
// 3.70-3.75 ms for gemm_n64_kernel, 4.0 TB/s of A, error against fp64 4.6e-7 vs 2.2e-6.  A form with A
// loaded straight into registers (four-deep register ring, W alone in a four-slot LDS ring) measured
// 3.205 vs 3.228 ms in the same run — within noise, not kept.
//
// LDS images: A row r (128 B = 8 chunks of 4 floats): chunk c at slot c ^ ((r >> 1) & 7); W plane
// row n (64 B = 4 chunks of 8 bf16): chunk c at slot c ^ ((n >> 2) & 3) — the ds_read_b128 lane
// groups (32 rows x one chunk) hit distinct (bank, slot) pairs.
#include <type_traits>

#include "common.h"

namespace mhada {
namespace {

MHADA_DEV void n64s3_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

#define N64S3_BARRIER() do { __builtin_amdgcn_sched_barrier(0); __builtin_amdgcn_s_barrier(); __builtin_amdgcn_sched_barrier(0); } while (0)

struct N64S3P {
  const float* a;    // [nz] x [M][lda] fp32, problem stride sa
  const bf16* w;     // planes [3] (stride wps) x [nz] (stride sw) x [64][ldw] bf16
  float* c;          // [nz] x [M][ldc] fp32, problem stride sc
  long long sa, sw, wps, sc;
  int M, K, lda, ldw, ldc, ntiles, xcd_group;
};

constexpr int kBM = 256, kBK = 32;  // three ring slots
constexpr int kAH = kBM * kBK;          // floats of the A image per slot
constexpr int kWH = 4 * 64 * kBK;       // bf16 of the W image per slot (4 plane images)
constexpr int kSlotBytes = kAH * 4 + kWH * 2;

MHADA_DEV void split8(const f32x4& lo, const f32x4& hi, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? lo[j] : hi[j - 4];
    const bf16 a = (bf16)x;
    const float r = x - (float)a;
    const bf16 b = (bf16)r;
    p0[j] = a;
    p1[j] = b;
    p2[j] = (bf16)(r - (float)b);
  }
}

template <int I>
using Ic = std::integral_constant<int, I>;

__global__ void __launch_bounds__(512, 1) gemm_n64_split3_kernel(const N64S3P p) {
  // three LDS objects selected at compile time: hipcc orders LDS-DMA writes before later ds_reads
  // per LDS object, so one array with a runtime slot would put a vmcnt(0) before every fragment read
  __shared__ __attribute__((aligned(16))) unsigned char slot0[kSlotBytes], slot1[kSlotBytes], slot2[kSlotBytes];
  auto slot_ptr = [&](auto I) -> unsigned char* {
    if constexpr (decltype(I)::value == 0) return slot0;
    else if constexpr (decltype(I)::value == 1) return slot1;
    else return slot2;
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // with xcd_group (problem count a multiple of 8) all row tiles of one problem go to ONE XCD
  // (workgroups are dealt to the 8 XCDs round-robin), so its W is fetched into one L2
  int z, tile;
  if (p.xcd_group) {
    const int L = blockIdx.y * gridDim.x + blockIdx.x, nt = gridDim.x;
    z = L % 8 + 8 * (L / (8 * nt));
    tile = (L / 8) % nt;
  } else {
    z = blockIdx.y;
    tile = blockIdx.x;
  }
  const int m0 = tile * kBM;
  const float* ab = p.a + z * p.sa;
  const bf16* wb = p.w + z * p.sw;
  // A staging: instruction i of wave w = rows 32 w + 8 i + lane / 8, 16-B slot lane % 8
  const float* asrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 32 * wave + 8 * i + (lane >> 3);
    const int m = min(m0 + r, p.M - 1);
    asrc[i] = ab + (long long)m * p.lda + 4 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  // W staging: instruction i of wave w = plane-image rows R = 16 (2 w + i) + lane / 4 (plane R / 64,
  // the fourth image a copy of plane 2), 16-B slot lane % 4
  const bf16* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = 16 * (2 * wave + i) + (lane >> 2), pl = min(R >> 6, 2), n = R & 63;
    wsrc[i] = wb + pl * p.wps + (long long)n * p.ldw + 8 * ((lane & 3) ^ ((n >> 2) & 3));
  }
  auto stage = [&](int kt, auto SL) {
    unsigned char* base = slot_ptr(SL);
    float* da = reinterpret_cast<float*>(base);
    bf16* dw = reinterpret_cast<bf16*>(base + kAH * 4);
    const int k0 = kt * kBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) n64s3_glds16(asrc[i] + k0, da + (32 * wave + 8 * i) * kBK);
#pragma unroll
    for (int i = 0; i < 2; ++i) n64s3_glds16(wsrc[i] + k0, dw + 16 * (2 * wave + i) * kBK);
  };
  const int h = lane >> 5, r32 = lane & 31;
  const int arow = 32 * wave + r32, asw = (arow >> 1) & 7;
  // A chunk offsets (floats) of MFMA step s: chunks 4 s + 2 h and 4 s + 2 h + 1 of row arow
  int aoff[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 2; ++e) aoff[s][e] = arow * kBK + 4 * ((4 * s + 2 * h + e) ^ asw);
  // W chunk offsets (bf16) of step s for column block nb: row 32 nb + r32, chunk 2 s + h
  int woff[2][2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int n = 32 * nb + r32;
      woff[nb][s] = n * kBK + 8 * ((2 * s + h) ^ ((n >> 2) & 3));
    }
  f32x16 acc[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[nb][e] = 0.f;
  f32x16 zero;
#pragma unroll
  for (int e = 0; e < 16; ++e) zero[e] = 0.f;
  const int KT = p.K / kBK;
  stage(0, Ic<0>{});
  if (KT > 1) stage(1, Ic<1>{});
  // K-tile kt in ring slot SL (= kt % 3, a compile-time constant)
  auto step = [&](int kt, auto SL) {
    constexpr int I = decltype(SL)::value;
    // own DMA of K-tile kt done (the 6 instructions of tile kt + 1 may still be in flight)
    if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    N64S3_BARRIER();
    if (kt + 2 < KT) stage(kt + 2, Ic<(I + 2) % 3>{});
    const unsigned char* base = slot_ptr(SL);
    const float* sa = reinterpret_cast<const float*>(base);
    const bf16* swp = reinterpret_cast<const bf16*>(base + kAH * 4);
    f32x16 t[2] = {zero, zero};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(sa + aoff[s][0]);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(sa + aoff[s][1]);
      bf16x8 a0, a1, a2;
      split8(lo, hi, a0, a1, a2);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(swp + woff[nb][s]);
        const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(swp + 64 * kBK + woff[nb][s]);
        const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(swp + 128 * kBK + woff[nb][s]);
        // smallest terms first: w2 a0, w1 a1, w0 a2, w1 a0, w0 a1, w0 a0
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, a0, t[nb], 0, 0, 0);
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, a1, t[nb], 0, 0, 0);
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a2, t[nb], 0, 0, 0);
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, a0, t[nb], 0, 0, 0);
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a1, t[nb], 0, 0, 0);
        t[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a0, t[nb], 0, 0, 0);
      }
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) acc[nb] += t[nb];
  };
  for (int kt = 0; kt < KT; kt += 3) {
    step(kt, Ic<0>{});
    if (kt + 1 < KT) step(kt + 1, Ic<1>{});
    if (kt + 2 < KT) step(kt + 2, Ic<2>{});
  }
  // lane (r32, h) holds row m0 + 32 wave + r32, columns 32 nb + 8 q + 4 h + 0..3 in acc[nb][4 q ..]
  const int m = m0 + arow;
  if (m < p.M) {
    float* crow = p.c + z * p.sc + (long long)m * p.ldc;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(crow + 32 * nb + 8 * q + 4 * h) =
            f32x4{acc[nb][4 * q], acc[nb][4 * q + 1], acc[nb][4 * q + 2], acc[nb][4 * q + 3]};
  }
}

// K [BH][N][64] fp32 -> the three bf16 planes of K^T, [3][BH][64][ldt] (plane stride BH 64 ldt; key
// columns N .. ldt - 1 zero): mhada_transpose64 and mhada_split3_rows in one pass.  One workgroup per
// (64-key chunk, problem): the 64 x 64 tile through LDS, then 16-B plane stores of 8 keys.
__global__ void __launch_bounds__(256) transpose64_split3_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                                 int N, int ldt, long long wps) {
  __shared__ float tile[64 * 65];  // [key][d]
  const int z = blockIdx.y, n0 = blockIdx.x * 64, tid = threadIdx.x;
  const float* sb = src + (long long)z * N * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 256 * i, n = idx >> 4, d = (idx & 15) * 4;
    const f32x4 x = n0 + n < N ? *reinterpret_cast<const f32x4*>(sb + (long long)(n0 + n) * 64 + d)
                               : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[n * 65 + d + e] = x[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 64 rows d x 8 runs of 8 keys
    const int idx = tid + 256 * i, d = idx >> 3, r8 = idx & 7;
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = tile[(8 * r8 + j) * 65 + d];
      const bf16 a = (bf16)x;
      const float r = x - (float)a;
      const bf16 b = (bf16)r;
      p0[j] = a;
      p1[j] = b;
      p2[j] = (bf16)(r - (float)b);
    }
    bf16* o = dst + ((long long)z * 64 + d) * ldt + n0 + 8 * r8;
    *reinterpret_cast<bf16x8*>(o) = p0;
    *reinterpret_cast<bf16x8*>(o + wps) = p1;
    *reinterpret_cast<bf16x8*>(o + 2 * wps) = p2;
  }
}

bool al16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

}  // namespace
}  // namespace mhada

using namespace mhada;

extern "C" int mhada_gemm_n64_split3(const float* a, const void* w_planes, float* c, int nz, int M, int K, int lda,
                                     long long sa, int ldw, long long sw, long long wps, int ldc, long long sc,
                                     mhada_stream_t s_) {
  if (!a || !w_planes || !c || nz <= 0 || nz > 65535 || M <= 0 || K <= 0)
    return fail("mhada_gemm_n64_split3: bad args");
  if (K % kBK || lda < K || ldw < K || ldc < 64 || lda % 4 || sa % 4 || ldw % 8 || sw % 8 || wps % 8 || ldc % 4 ||
      sc % 4 || !al16(a) || !al16(w_planes) || !al16(c))
    return fail("mhada_gemm_n64_split3: needs K % 32 == 0, 16-byte aligned rows and problems");
  if ((long long)(M - 1) * lda + K >= (1LL << 31) || 2 * wps + 63LL * ldw + K >= (1LL << 31))
    return fail("mhada_gemm_n64_split3: operand spans need 32-bit element offsets per problem");
  N64S3P p;
  p.a = a; p.w = reinterpret_cast<const bf16*>(w_planes); p.c = c;
  p.sa = sa; p.sw = sw; p.wps = wps; p.sc = sc;
  p.M = M; p.K = K; p.lda = lda; p.ldw = ldw; p.ldc = ldc;
  p.ntiles = (M + kBM - 1) / kBM;
  p.xcd_group = nz % 8 == 0 ? 1 : 0;
  hipLaunchKernelGGL(gemm_n64_split3_kernel, dim3(p.ntiles, nz), dim3(512), 0, (hipStream_t)s_, p);
  return check_launch("mhada_gemm_n64_split3");
}

extern "C" int mhada_transpose64_split3(const float* src, void* planes, int BH, int N, int ldt, mhada_stream_t s_) {
  if (!src || !planes || BH <= 0 || BH > 65535 || N <= 0 || ldt < N || ldt % 64)
    return fail("mhada_transpose64_split3: bad args (ldt % 64 == 0, ldt >= N)");
  if (!al16(src) || !al16(planes)) return fail("mhada_transpose64_split3: 16-byte aligned operands");
  const long long wps = (long long)BH * 64 * ldt;
  hipLaunchKernelGGL(transpose64_split3_kernel, dim3(ldt / 64, BH), dim3(256), 0, (hipStream_t)s_, src,
                     reinterpret_cast<bf16*>(planes), N, ldt, wps);
  return check_launch("mhada_transpose64_split3");
}
