// MHAda attention for the training path: forward that keeps the softmax statistics, and the
// backward (dual accumulator M / E2), fp32 on v_mfma_f32_32x32x2_f32.
//
// Reference: AdaAttnMultiHead.forward (MHAdaSTr/network/adaDecoder.py:186-198) under
// train_image.py:93-144 autograd.  Per (batch, head), with Q [Nc][64], K [Ns][64], V' [Ns][64]
// (V' = V - mean_tokens(V), centred by the caller under autograd: the variance is
// shift-invariant and d(out)/dV = d(out)/dV' exactly, since the rows of A sum to one) and
// X = InstanceNorm(fcs) [Nc][64]:
//   A = softmax(Q K^T)   M' = A V'   E2' = A V'^2   var = E2' - M'^2
//   out' = sqrt(max(var, 1e-6)) * X + M'            (the caller adds mean(V) back)
// The forward writes out', [M' | E2'] and the log2 row normaliser lse2 = max + log2(sum).
// The caller turns d(out') into dO = [dM' | dE2'] and D = dM'.M' + dE2'.E2' (elementwise,
// O(Nc*64)); then with P = A (recomputed from lse2) and dA = dM'.V'^T + dE2'.(V'^2)^T:
//   dS = P * (dA - D)            (gradient of the natural-unit logits)
//   dQ = dS K       dK = dS^T Q       dV' = P^T dM' + 2 V' * (P^T dE2')
// as two deterministic kernels (no atomics): key-stationary dK/dV', query-stationary dQ, each
// recomputing P — the Nc x Ns matrices never reach HBM (the reference autograd keeps A, the
// softmax output, and their gradients: 4 B x Nc x Ns per head each).
//
// MFMA 32x32x2 f32 layout (cdna_hip_programming.md §3): lane l gives A[l%32][l/32] and
// B[l/32][l%32]; accumulator register r of lane l is D[acc_row(r, l/32)][l%32].  Every
// product is arranged so that one operand is an accumulator of the previous product
// (accumulator-as-operand), so no score or probability ever moves between lanes.
#include "common.h"

#include <type_traits>

#include <stdlib.h>

namespace mhada {
namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr int TT = 32;    // keys (fwd, dQ) or queries (dK/dV') staged per LDS tile
constexpr int LP = 68;    // padded LDS row of 64 floats
constexpr int LPO = 132;  // padded LDS row of 128 floats

MHADA_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

MHADA_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
MHADA_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
MHADA_DEV f32x16 mfma(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

struct TrainP {
  const float* q;    // [BH][Nc][64]
  const float* k;    // [BH][Ns][64]
  const float* v;    // [BH][Ns][64] centred V'
  const float* x;    // [BH][Nc][64] InstanceNorm(fcs)
  float* out;        // [BH][Nc][64]
  float* mo;         // [BH][Nc][128]  M' | E2'
  float* lse;        // [BH][Nc]       log2 units
  const float* dmo;  // [BH][Nc][128]  dM' | dE2'
  const float* dd;   // [BH][Nc]       D
  float* dq;         // [BH][Nc][64]
  float* dk;         // [BH][Ns][64]
  float* dv;         // [BH][Ns][64]
  float* ds;         // [BH][Nc][Ns] dS spill (dQ = dS K as a GEMM), or null
  int Nc, Ns, nb, nblk;  // nb = row blocks per (b, h)
};

// In-kernel clock of the dK/dV' kernel, diagnostic builds only (-DATTN_CLOCK, tools/attn_clock.py
// dkv): thread 0 of each workgroup stamps the shader clock and the 100 MHz counter around the
// query loop into a buffer of its own (MI355X_MICROARCH.md, DVFS give-back item 6).
#ifdef ATTN_CLOCK
constexpr int kTrainClockBlocks = 65536;
__device__ unsigned long long g_train_clock[4 * kTrainClockBlocks];
#define TRAIN_STAMP(slot)                                                                    \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < kTrainClockBlocks) {                                \
      const unsigned long long c_ = __builtin_amdgcn_s_memtime();                           \
      const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                       \
      g_train_clock[4 * blockIdx.x + 2 * (slot)] = c_;                                       \
      g_train_clock[4 * blockIdx.x + 2 * (slot) + 1] = r_;                                   \
    }                                                                                        \
  } while (0)
#else
#define TRAIN_STAMP(slot) \
  do {                    \
  } while (0)
#endif

// Workgroup barrier for the LDS hand-off only: __syncthreads() also acts as a release fence
// that drains every outstanding global store (vmcnt counts stores on CDNA4), which would
// serialise the dS spill stores with the next tile.
MHADA_DEV void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Register-staged copy of rows [r0, r0+TT) of a [n][W] matrix (zero rows past n; with CLAMP, r0
// may lie past n) into a padded LDS tile: load() issues the global reads one tile ahead, store()
// writes them after the current tile's math (one barrier per tile, two LDS buffers).
template <int NT, int W, bool CLAMP = false>
struct Stager {
  static constexpr int CPR = W / 4;             // 16-B chunks per row
  static constexpr int N = TT * CPR / NT;       // chunks per thread
  static constexpr int LD = W == 64 ? LP : LPO;
  static_assert(N * NT == TT * CPR, "tile must divide evenly");
  f32x4 r[N];
  MHADA_DEV void load(const float* g, int r0, int n, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = tid + NT * i, row = c / CPR, col = (c % CPR) * 4, gr = r0 + row;
      if constexpr (CLAMP) {
        // unconditional load of a clamped row, zeroed afterwards: a branch around the load makes
        // the wait-count pass drain every outstanding store before the tile's LDS write
        const f32x4 x = ld4(g + (long long)min(gr, n - 1) * W + col);
        r[i] = gr < n ? x : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        r[i] = gr < n ? ld4(g + (long long)gr * W + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  MHADA_DEV void store(float* s, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = tid + NT * i, row = c / CPR, col = (c % CPR) * 4;
      st4(s + row * LD + col, r[i]);
    }
  }
};

// Per-lane row of 64 floats split by lane half: reg[s] = g[row][32h + s] * scale.
MHADA_DEV void load_half_row(float (&reg)[32], const float* g, int row, bool valid, int h, float scale) {
  const float* p = g + (long long)(valid ? row : 0) * 64 + 32 * h;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f32x4 t = ld4(p + 4 * i);
#pragma unroll
    for (int e = 0; e < 4; ++e) reg[4 * i + e] = valid ? t[e] * scale : 0.f;
  }
}

// S^T (keys x queries) in log2 units from the staged K tile and the lane's query row
// (qr pre-scaled by log2 e); keys past Ns masked to -inf.
MHADA_DEV f32x16 scores_t(const float* sK, const float (&qr)[32], int k0, int Ns, int h, int r32) {
  f32x16 S = {};
  const float* kr = sK + r32 * LP + 32 * h;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f32x4 kk = ld4(kr + 4 * i);
#pragma unroll
    for (int e = 0; e < 4; ++e) S = mfma(kk[e], qr[4 * i + e], S);
  }
  if (k0 + TT > Ns) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (k0 + acc_row(r, h) >= Ns) S[r] = -INFINITY;
  }
  return S;
}

// ---------------------------------------------------------------------------------------
// forward: wave = 32 queries (one per lane column), online softmax over 32-key tiles
// ---------------------------------------------------------------------------------------
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_train_fwd_kernel(const TrainP p) {
  constexpr int NT = 64 * NW;
  __shared__ __attribute__((aligned(16))) float sK[2][TT * LP];
  __shared__ __attribute__((aligned(16))) float sV[2][TT * LP];
  const int t = xcd_remap(blockIdx.x, p.nblk);
  const long long bh = t / p.nb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = (t % p.nb) * 32 * NW + wave * 32 + r32;
  const bool qv = q < p.Nc;
  float qr[32];
  load_half_row(qr, p.q + bh * p.Nc * 64, q, qv, h, kLog2e);
  const float* kb = p.k + bh * p.Ns * 64;
  const float* vb = p.v + bh * p.Ns * 64;

  f32x16 O[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) O[i] = f32x16{};
  float m = -INFINITY, l = 0.f;
  Stager<NT, 64> gk, gv;
  gk.load(kb, 0, p.Ns, tid);
  gv.load(vb, 0, p.Ns, tid);
  gk.store(sK[0], tid);
  gv.store(sV[0], tid);
  __syncthreads();
  const int nt = (p.Ns + TT - 1) / TT;
  for (int t = 0; t < nt; ++t) {
    const int k0 = t * TT, cb = t & 1;
    const bool nxt = t + 1 < nt;
    if (nxt) {
      gk.load(kb, k0 + TT, p.Ns, tid);
      gv.load(vb, k0 + TT, p.Ns, tid);
    }
    f32x16 S = scores_t(sK[cb], qr, k0, p.Ns, h, r32);
    float mx = S[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, S[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any(mx > m)) {  // exact online softmax: rescale whenever the running max moves
      const float mn = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) O[i][e] *= alpha;
      m = mn;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      S[r] = __builtin_amdgcn_exp2f(S[r] - m);
      l += S[r];
    }
    // O^T (c x queries) += V'^T (c x keys) . P^T (keys x queries); blocks 2,3 take V'^2
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* vr = sV[cb] + acc_row(r, h) * LP + r32;
      const float v0 = vr[0], v1 = vr[32];
      O[0] = mfma(v0, S[r], O[0]);
      O[1] = mfma(v1, S[r], O[1]);
      O[2] = mfma(v0 * v0, S[r], O[2]);
      O[3] = mfma(v1 * v1, S[r], O[3]);
    }
    if (nxt) {
      gk.store(sK[cb ^ 1], tid);
      gv.store(sV[cb ^ 1], tid);
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (!qv) return;
  const float inv = 1.0f / l;
  const long long row = bh * p.Nc + q;
  const float* xr = p.x + row * 64;
  float* orow = p.out + row * 64;
  float* mrow = p.mo + row * 128;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * cb + 8 * g + 4 * h;
      const f32x4 xx = ld4(xr + c0);
      f32x4 o, mm, ee;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float m1 = O[cb][4 * g + e] * inv;
        const float e2 = O[cb + 2][4 * g + e] * inv;
        o[e] = sqrtf(fmaxf(e2 - m1 * m1, 1e-6f)) * xx[e] + m1;
        mm[e] = m1;
        ee[e] = e2;
      }
      st4(orow + c0, o);
      st4(mrow + c0, mm);
      st4(mrow + 64 + c0, ee);
    }
  if (h == 0) p.lse[row] = m + __log2f(l);
}

// ---------------------------------------------------------------------------------------
// dQ: wave = 32 queries; streams 32-key tiles of K, V'
// ---------------------------------------------------------------------------------------
template <int NW>
__global__ void __launch_bounds__(64 * NW) attn_train_dq_kernel(const TrainP p) {
  constexpr int NT = 64 * NW;
  __shared__ __attribute__((aligned(16))) float sK[2][TT * LP];
  __shared__ __attribute__((aligned(16))) float sV[2][TT * LP];
  const int t = xcd_remap(blockIdx.x, p.nblk);
  const long long bh = t / p.nb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = (t % p.nb) * 32 * NW + wave * 32 + r32;
  const bool qv = q < p.Nc;
  const long long row = bh * p.Nc + (qv ? q : 0);
  float qr[32], dm[32], de[32];
  load_half_row(qr, p.q + bh * p.Nc * 64, q, qv, h, kLog2e);
  {
    const float* o = p.dmo + row * 128 + 32 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 a = ld4(o + 4 * i), b = ld4(o + 64 + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dm[4 * i + e] = qv ? a[e] : 0.f;
        de[4 * i + e] = qv ? b[e] : 0.f;
      }
    }
  }
  const float L = qv ? p.lse[row] : INFINITY;  // invalid query: P = 0
  const float D = qv ? p.dd[row] : 0.f;
  const float* kb = p.k + bh * p.Ns * 64;
  const float* vb = p.v + bh * p.Ns * 64;
  f32x16 dQ[2] = {f32x16{}, f32x16{}};
  Stager<NT, 64> gk, gv;
  gk.load(kb, 0, p.Ns, tid);
  gv.load(vb, 0, p.Ns, tid);
  gk.store(sK[0], tid);
  gv.store(sV[0], tid);
  __syncthreads();
  const int nt = (p.Ns + TT - 1) / TT;
  for (int t = 0; t < nt; ++t) {
    const int k0 = t * TT, cb = t & 1;
    const bool nxt = t + 1 < nt;
    if (nxt) {
      gk.load(kb, k0 + TT, p.Ns, tid);
      gv.load(vb, k0 + TT, p.Ns, tid);
    }
    const f32x16 S = scores_t(sK[cb], qr, k0, p.Ns, h, r32);
    // dA^T (keys x queries) = [V' | V'^2] (keys x 128) . [dM' | dE2']^T
    f32x16 dA = {};
    const float* vr = sV[cb] + r32 * LP + 32 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 vv = ld4(vr + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dA = mfma(vv[e], dm[4 * i + e], dA);
        dA = mfma(vv[e] * vv[e], de[4 * i + e], dA);
      }
    }
    f32x16 dS;
#pragma unroll
    for (int r = 0; r < 16; ++r) dS[r] = __builtin_amdgcn_exp2f(S[r] - L) * (dA[r] - D);
    // dQ^T (d x queries) += K^T (d x keys) . dS^T (keys x queries)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* kr = sK[cb] + acc_row(r, h) * LP + r32;
      dQ[0] = mfma(kr[0], dS[r], dQ[0]);
      dQ[1] = mfma(kr[32], dS[r], dQ[1]);
    }
    if (nxt) {
      gk.store(sK[cb ^ 1], tid);
      gv.store(sV[cb ^ 1], tid);
    }
    __syncthreads();
  }
  if (!qv) return;
  float* o = p.dq + row * 64;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      st4(o + 32 * db + 8 * g + 4 * h, f32x4{dQ[db][4 * g], dQ[db][4 * g + 1], dQ[db][4 * g + 2], dQ[db][4 * g + 3]});
}

// ---------------------------------------------------------------------------------------
// dK, dV': wave = 32 keys (one per lane column); streams 32-query tiles of Q, dO, lse2, D
// ---------------------------------------------------------------------------------------
template <int NW, int OCC, bool SPILL>
__global__ void __launch_bounds__(64 * NW, OCC) attn_train_dkv_kernel(const TrainP p) {
  constexpr int NT = 64 * NW;
  __shared__ __attribute__((aligned(16))) float sQ[2][TT * LP];
  __shared__ __attribute__((aligned(16))) float sO[2][TT * LPO];
  __shared__ float sL[2][TT], sD[2][TT];
  const int t = xcd_remap(blockIdx.x, p.nblk);
  const long long bh = t / p.nb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int key = (t % p.nb) * 32 * NW + wave * 32 + r32;
  const bool kv = key < p.Ns;
  float kr[32], vr[32], vr2[32];
  load_half_row(kr, p.k + bh * p.Ns * 64, key, kv, h, kLog2e);
  load_half_row(vr, p.v + bh * p.Ns * 64, key, kv, h, 1.0f);
#pragma unroll
  for (int s = 0; s < 32; ++s) vr2[s] = vr[s] * vr[s];  // V'^2 once (the wave's keys are fixed)
  const float* qb = p.q + bh * p.Nc * 64;
  const float* ob = p.dmo + bh * p.Nc * 128;
  const float* lb = p.lse + bh * p.Nc;
  const float* db = p.dd + bh * p.Nc;
  f32x16 G1[2] = {f32x16{}, f32x16{}}, G2[2] = {f32x16{}, f32x16{}}, dK[2] = {f32x16{}, f32x16{}};
  Stager<NT, 64, SPILL> gq;
  Stager<NT, 128, SPILL> go;
  float gl = INFINITY, gd = 0.f;
  // With SPILL the loop body is branch-free around global memory (clamped loads, the tile after
  // the last one loaded and discarded, range-checked buffer stores for dS): the wait before the
  // LDS write then counts only the tile loads, and the dS stores stay in flight across tiles
  // (a branch around any of them made the wait-count pass drain every store: 8.69 -> 8.32 ms per
  // 512^2 B8 block backward).  Without stores the plain branches are cheaper.
  auto load = [&](int q0) {
    gq.load(qb, q0, p.Nc, tid);
    go.load(ob, q0, p.Nc, tid);
    const int qi = q0 + (tid & (TT - 1));
    if constexpr (SPILL) {
      const float l0 = lb[min(qi, p.Nc - 1)], d0 = db[min(qi, p.Nc - 1)];
      gl = qi < p.Nc ? l0 : INFINITY;  // padded query: P = 0
      gd = qi < p.Nc ? d0 : 0.f;
    } else if (tid < TT && qi < p.Nc) {
      gl = lb[qi];
      gd = db[qi];
    } else {
      gl = INFINITY;
      gd = 0.f;
    }
  };
  auto store = [&](int buf) {
    gq.store(sQ[buf], tid);
    go.store(sO[buf], tid);
    if (tid < TT) {
      sL[buf][tid] = gl;
      sD[buf][tid] = gd;
    }
  };
  // dS rows of this (b, h): offsets past num_records (rows >= Nc, or a key >= Ns, whose lanes
  // add (Nc + 32) rows) are dropped; unsigned offsets < 2 (Nc + 32) Ns * 4 < 2^32 (entry check)
  const unsigned dkey = kv ? key * 4u : (unsigned)(p.Nc + TT) * p.Ns * 4;
  const __amdgpu_buffer_rsrc_t dsr =
      __builtin_amdgcn_make_buffer_rsrc(SPILL ? p.ds + bh * p.Nc * p.Ns : nullptr, 0,
                                        SPILL ? p.Nc * p.Ns * 4 : 0, 0x00020000);
  load(0);
  store(0);
  __syncthreads();
  TRAIN_STAMP(0);
  const int nt = (p.Nc + TT - 1) / TT;
  for (int t = 0; t < nt; ++t) {
    const int cb = t & 1;
    const bool nxt = t + 1 < nt;
    if (SPILL || nxt) load((t + 1) * TT);
    // S (queries x keys) = Q . K^T, dA (queries x keys) = [dM' | dE2'] . [V' | V'^2]^T
    f32x16 S = {}, dA = {};
    const float* qrow = sQ[cb] + r32 * LP + 32 * h;
    const float* orow = sO[cb] + r32 * LPO + 32 * h;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 qq = ld4(qrow + 4 * i), o1 = ld4(orow + 4 * i), o2 = ld4(orow + 64 + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = 4 * i + e;
        S = mfma(qq[e], kr[s], S);
        dA = mfma(o1[e], vr[s], dA);
        dA = mfma(o2[e], vr2[s], dA);
      }
    }
    f32x16 P, dS;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = acc_row(r, h);
      P[r] = __builtin_amdgcn_exp2f(S[r] - sL[cb][qi]);
      dS[r] = P[r] * (dA[r] - sD[cb][qi]);
    }
    if constexpr (SPILL) {  // dS [q][key]: for each register the 32 lanes of a half write 128 B
      const unsigned base = (unsigned)(t * TT + 4 * h) * p.Ns * 4 + dkey;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dS[r]), dsr,
                                              (int)(base + ((r & 3) + 8 * (r >> 2)) * p.Ns * 4u), 0, 0);
    }
    // G1^T, G2^T (c x keys) += [dM' | dE2']^T (c x queries) . P;  dK^T += Q^T . dS
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* o = sO[cb] + acc_row(r, h) * LPO + r32;
      const float* qq = sQ[cb] + acc_row(r, h) * LP + r32;
      G1[0] = mfma(o[0], P[r], G1[0]);
      G1[1] = mfma(o[32], P[r], G1[1]);
      G2[0] = mfma(o[64], P[r], G2[0]);
      G2[1] = mfma(o[96], P[r], G2[1]);
      dK[0] = mfma(qq[0], dS[r], dK[0]);
      dK[1] = mfma(qq[32], dS[r], dK[1]);
    }
    if (nxt) store(cb ^ 1);
    lds_barrier();
  }
  TRAIN_STAMP(1);
  if (!kv) return;
  const long long row = bh * p.Ns + key;
  const float* vg = p.v + row * 64;
  float* dvr = p.dv + row * 64;
  float* dkr = p.dk + row * 64;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * cb + 8 * g + 4 * h;
      const f32x4 vv = ld4(vg + c0);
      f32x4 a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = G1[cb][4 * g + e] + 2.0f * vv[e] * G2[cb][4 * g + e];
        b[e] = dK[cb][4 * g + e];
      }
      st4(dvr + c0, a);
      st4(dkr + c0, b);
    }
}

// ---------------------------------------------------------------------------------------
// dK, dV' with the dS spill, LDS-DMA + software-pipelined form (round 4; the training default):
// the same products in the same order as attn_train_dkv_kernel<.., SPILL> (bit-identical dK / dV'
// / dS).  That kernel runs one wave per SIMD (288 registers) and measured 0.76 of the
// clock-adjusted fp32 peak at 2.39 GHz (profiles/r04_train_dkv_clock.log): each tile's MFMA
// stream stops for its softmax VALU (S -> P, dA -> dS), its dS stores, its staging writes and the
// barrier.  Here:
//   * iteration t runs tile t+1's first phase (S, dA = 96 MFMAs) while tile t's softmax VALU and
//     dS stores fill the MFMA gaps, then tile t's second phase (G1, G2, dK = 96 MFMAs): the matrix
//     pipe always has independent work (two S / dA register sets, one wave per SIMD);
//   * the Q / dO / lse / D tiles arrive by LDS-DMA (global_load_lds) into a 3-slot ring — no
//     staging registers or LDS write pass, one counted vmcnt that never waits on the dS stores;
//     rows are XOR-swizzled on the source address (16-B chunk c of row r at slot c ^ (r & 15) of
//     its 256-B bank row): the phase-1 ds_read_b128 (32 rows, one chunk) and the phase-2
//     ds_read_b32 (one row, 32 consecutive floats) are conflict-free;
//   * query rows past Nc load clamped rows with lse = +inf, D = 0 (P = 0).
// 2 waves per SIMD (256 registers) was tried: 40+ spilled registers.
// ---------------------------------------------------------------------------------------
MHADA_DEV void train_glds(const float* src, float* lds, int bytes) {
  if (bytes == 16)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// padding rows of the lse | D tile (query >= Nc): P = exp2(S - inf) = 0, D = 0
__device__ float g_train_pad[2] = {INFINITY, 0.f};

__global__ void __launch_bounds__(256, 1) attn_train_dkv_dma_kernel(const TrainP p) {
  constexpr int NW = 4, NS = 3;
  constexpr int QF = TT * 64, OF = TT * 128, SLOT = QF + OF + 2 * TT;  // floats per ring slot (24.8 KiB)
  __shared__ __attribute__((aligned(16))) float smem[NS * SLOT];      // 74.5 KiB
  const int t0 = xcd_remap(blockIdx.x, p.nblk);
  const long long bh = t0 / p.nb;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int key = (t0 % p.nb) * 32 * NW + wave * 32 + r32;
  const bool kv = key < p.Ns;
  float kr[32], vr[32], vr2[32];
  load_half_row(kr, p.k + bh * p.Ns * 64, key, kv, h, kLog2e);
  load_half_row(vr, p.v + bh * p.Ns * 64, key, kv, h, 1.0f);
#pragma unroll
  for (int s2 = 0; s2 < 32; ++s2) vr2[s2] = vr[s2] * vr[s2];
  const float* qb = p.q + bh * p.Nc * 64;
  const float* ob = p.dmo + bh * p.Nc * 128;
  const float* lb = p.lse + bh * p.Nc;
  const float* db = p.dd + bh * p.Nc;
  // DMA pieces (1 KiB = 64 lanes x 16 B) of this wave: Q rows 4 per piece (pieces 2w, 2w+1), dO
  // rows 2 per piece (pieces 4w .. 4w+3); each lane fetches the global chunk its LDS slot holds.
  // Q and dO go through buffer resources built per tile (scalar work) over the rows q0 .. Nc - 1,
  // so each lane's offset is a constant and a piece costs no vector address arithmetic (an fp32
  // MFMA holds the SIMD's vector issue for its whole 64 cycles, profiles/r05_f32mfma_fill.log:
  // every VALU instruction adds to the loop).  Rows past Nc read 0 (out of range); with their
  // lse = +inf (padding piece below) P = 0 there, as with the clamped rows of the other kernel.
  typedef __attribute__((address_space(3))) void* LdsP;
  int qvo[2], ovo[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 4 * (2 * wave + i) + (lane >> 4);
    qvo[i] = (row * 64 + 4 * ((lane & 15) ^ (row & 15))) * 4;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 2 * (4 * wave + i) + (lane >> 5);
    ovo[i] = (row * 128 + 4 * (((lane >> 4) & 1) * 16 + ((lane & 15) ^ (row & 15)))) * 4;
  }
  auto stage = [&](int q0, int sl) {  // tile q0 .. q0+31 into ring slot sl
    float* d = smem + sl * SLOT;
    const int left = max(p.Nc - q0, 0);
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(qb + (long long)min(q0, p.Nc) * 64), 0, left * 64 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(ob + (long long)min(q0, p.Nc) * 128), 0, left * 128 * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (LdsP)(d + (2 * wave + i) * 256), 16, qvo[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ors, (LdsP)(d + QF + (4 * wave + i) * 256), 16, ovo[i], 0, 0, 0);
    // lse | D: lanes 0-31 / 32-63; padding queries read +inf / 0 (every wave issues the same
    // piece, so every wave's wait counts are equal)
    const int qi = q0 + r32;
    train_glds(qi < p.Nc ? (h ? db : lb) + qi : g_train_pad + h, d + QF + OF, 4);
  };
  // phase-2 reads of row R = rowb(r) + 4h: logical float r32 (chunk r32 / 4) sits at physical
  // 16-B slot (r32 / 4) ^ (R & 15) = 8 ((r >> 2) & 1) + ((r32 / 4) ^ ((r & 3) | 4h)); float 32 + r32
  // at slot 8 (1 ^ ((r >> 2) & 1)) + the same low bits.  Per lane only (r & 3) varies: 4 offsets
  // per operand (O and Q rows differ in length), the rest folds into the ds_read immediate.
  int xo[4], xq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int lo = 4 * ((r32 >> 2) ^ (j | (4 * h))) + (r32 & 3);
    xo[j] = (QF + 4 * h * 128 + lo) & 0xffff;  // the O rows' base QF folded in: immediates stay < 64 KiB
    xq[j] = (4 * h * 64 + lo) & 0xffff;
  }
  const int sw1 = r32 & 15;
  f32x16 G1[2] = {f32x16{}, f32x16{}}, G2[2] = {f32x16{}, f32x16{}}, dK[2] = {f32x16{}, f32x16{}};
  // dS spill offsets of the lane's 16 accumulator rows relative to the tile's first row (past the
  // resource for keys >= Ns)
  unsigned dvo[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) dvo[r] = kv ? (unsigned)acc_row(r, h) * p.Ns * 4 + key * 4u : 0x7ff00000u;
  // phase 1 of the tile in ring slot sl: S (queries x keys) = Q . K^T, dA = [dM' | dE2'] . [V' | V'^2]^T
  // Every LDS address below is a per-lane register plus an immediate: the ring slot is a
  // compile-time constant in each unrolled step (the loop runs six steps per iteration, two
  // register sets x three slots), and the per-lane parts are masked so their sign bit is known
  // zero (hipcc folds constants into a ds_read immediate only then).
  int qoff[8], ooff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = 4 * ((8 * h + i) ^ sw1);
    qoff[i] = (r32 * 64 + c) & 0xffff;
    ooff[i] = (QF + r32 * 128 + c) & 0xffff;
  }
  auto phase1 = [&](int sl, f32x16& S, f32x16& dA) {
    const float* sQ = smem + sl * SLOT;
    S = f32x16{};
    dA = f32x16{};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 qq = ld4(sQ + qoff[i]), o1 = ld4(sQ + ooff[i]), o2 = ld4(sQ + ooff[i] + 64);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s2 = 4 * i + e;
        S = mfma(qq[e], kr[s2], S);
        dA = mfma(o1[e], vr[s2], dA);
        dA = mfma(o2[e], vr2[s2], dA);
      }
    }
  };
  // S -> P, dA -> dS in place (tile of ring slot sl, first query q0), and dS's spill stores
  auto softmax = [&](int sl, int q0, f32x16& S, f32x16& dA) {
    const float* sLD = smem + sl * SLOT + QF + OF;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = acc_row(r, h);
      S[r] = __builtin_amdgcn_exp2f(S[r] - sLD[qi]);
      dA[r] = S[r] * (dA[r] - sLD[TT + qi]);
    }
    // dS [q][key]: 32 lanes write 128 B, through a resource over rows q0 .. Nc - 1 (rows past Nc
    // and keys past Ns are out of range: dropped) and per-lane offsets precomputed for the 16 rows
    const __amdgpu_buffer_rsrc_t dsr = __builtin_amdgcn_make_buffer_rsrc(
        p.ds + bh * p.Nc * p.Ns + (long long)min(q0, p.Nc) * p.Ns, 0, max(p.Nc - q0, 0) * p.Ns * 4, 0x00020000);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dA[r]), dsr, (int)dvo[r], 0, 0);
  };
  // phase 2: G1^T, G2^T (c x keys) += [dM' | dE2']^T (c x queries) . P;  dK^T += Q^T . dS
  auto phase2 = [&](int sl, const f32x16& P, const f32x16& dS) {
    const float* sQ = smem + sl * SLOT;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = r & 3, rowb = (r & 3) + 8 * (r >> 2), b3 = (r >> 2) & 1;
      const float* o = sQ + xo[j] + rowb * 128;
      const float* qq = sQ + xq[j] + rowb * 64;
      G1[0] = mfma(o[32 * b3], P[r], G1[0]);
      G1[1] = mfma(o[32 * (1 - b3)], P[r], G1[1]);
      G2[0] = mfma(o[64 + 32 * b3], P[r], G2[0]);
      G2[1] = mfma(o[64 + 32 * (1 - b3)], P[r], G2[1]);
      dK[0] = mfma(qq[32 * b3], dS[r], dK[0]);
      dK[1] = mfma(qq[32 * (1 - b3)], dS[r], dK[1]);
    }
  };

  const int nt = (p.Nc + TT - 1) / TT;
  stage(0, 0);
  stage(TT, 1);
  asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // tile 0 (7 pieces per tile and wave)
  lds_barrier();
  TRAIN_STAMP(0);
  f32x16 Sa, dAa, Sb, dAb;
  phase1(0, Sa, dAa);
  // iteration t: publish tile t + 1; DMA tile t + 2 into the slot tile t - 1 used; tile t + 1's
  // phase 1 beside tile t's softmax and stores; tile t's phase 2.  Two register sets, A / B,
  // alternate and the ring slot cycles 0, 1, 2: six steps per loop iteration, each with its slot
  // a compile-time constant.
  auto step = [&](int t, auto slc, f32x16& S, f32x16& dA, f32x16& Sn, f32x16& dAn) __attribute__((always_inline)) {
    constexpr int SL = decltype(slc)::value, SN = (SL + 1) % 3, S2 = (SL + 2) % 3;
    // tile t + 1 landed (younger: tile t's dS stores... issued after it in iteration t - 1: 16)
    if (t == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    lds_barrier();
    stage((t + 2) * TT, S2);  // past the end: rows read 0, never used
    softmax(SL, t * TT, S, dA);
    phase1(SN, Sn, dAn);  // tile t + 1 (past the end: result unused)
    phase2(SL, S, dA);
  };
  typedef std::integral_constant<int, 0> L0;
  typedef std::integral_constant<int, 1> L1;
  typedef std::integral_constant<int, 2> L2;
  int t = 0;
  for (; t + 5 < nt; t += 6) {
    step(t, L0(), Sa, dAa, Sb, dAb);
    step(t + 1, L1(), Sb, dAb, Sa, dAa);
    step(t + 2, L2(), Sa, dAa, Sb, dAb);
    step(t + 3, L0(), Sb, dAb, Sa, dAa);
    step(t + 4, L1(), Sa, dAa, Sb, dAb);
    step(t + 5, L2(), Sb, dAb, Sa, dAa);
  }
  if (t < nt) step(t, L0(), Sa, dAa, Sb, dAb);
  if (t + 1 < nt) step(t + 1, L1(), Sb, dAb, Sa, dAa);
  if (t + 2 < nt) step(t + 2, L2(), Sa, dAa, Sb, dAb);
  if (t + 3 < nt) step(t + 3, L0(), Sb, dAb, Sa, dAa);
  if (t + 4 < nt) step(t + 4, L1(), Sa, dAa, Sb, dAb);
  TRAIN_STAMP(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped DMA past the end has landed
  if (!kv) return;
  const long long row = bh * p.Ns + key;
  const float* vg = p.v + row * 64;
  float* dvr = p.dv + row * 64;
  float* dkr = p.dk + row * 64;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * cb + 8 * g + 4 * h;
      const f32x4 vv = ld4(vg + c0);
      f32x4 a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = G1[cb][4 * g + e] + 2.0f * vv[e] * G2[cb][4 * g + e];
        b[e] = dK[cb][4 * g + e];
      }
      st4(dvr + c0, a);
      st4(dkr + c0, b);
    }
}

constexpr int kNW = 4;
// per-(b, h) dS slice addressed by 32-bit buffer offsets, with 0x7ffffff0 free as the drop offset
constexpr long long kMaxSpillRows = (0x7fff0000LL / 4);

bool set_grid(TrainP& p, long long BH, int n) {
  p.nb = (n + 32 * kNW - 1) / (32 * kNW);
  const long long nblk = BH * p.nb;
  if (nblk > (1LL << 31) - 1) return false;
  p.nblk = (int)nblk;
  return true;
}

}  // namespace
}  // namespace mhada

using namespace mhada;

extern "C" int mhada_attn_train_fwd(const float* q, const float* k, const float* v, const float* x, float* out,
                                    float* mo, float* lse, int BH, int Nc, int Ns, mhada_stream_t s_) {
  if (!q || !k || !v || !x || !out || !mo || !lse || BH <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_train_fwd: bad args");
  TrainP p = {};
  p.q = q; p.k = k; p.v = v; p.x = x; p.out = out; p.mo = mo; p.lse = lse; p.Nc = Nc; p.Ns = Ns;
  if (!set_grid(p, BH, Nc)) return fail("mhada_attn_train_fwd: grid too large");
  hipLaunchKernelGGL(attn_train_fwd_kernel<kNW>, dim3(p.nblk), dim3(64 * kNW), 0, (hipStream_t)s_, p);
  return check_launch("mhada_attn_train_fwd");
}

extern "C" int mhada_attn_train_bwd(const float* q, const float* k, const float* v, const float* lse,
                                    const float* dmo, const float* dd, float* dq, float* dk, float* dv, int BH,
                                    int Nc, int Ns, mhada_stream_t s_) {
  if (!q || !k || !v || !lse || !dmo || !dd || !dq || !dk || !dv || BH <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_train_bwd: bad args");
  const hipStream_t s = (hipStream_t)s_;
  TrainP p = {};
  p.q = q; p.k = k; p.v = v; p.lse = const_cast<float*>(lse); p.dmo = dmo; p.dd = dd; p.dq = dq; p.dk = dk; p.dv = dv;
  p.Nc = Nc; p.Ns = Ns;
  if (!set_grid(p, BH, Nc)) return fail("mhada_attn_train_bwd: grid too large");
  hipLaunchKernelGGL(attn_train_dq_kernel<kNW>, dim3(p.nblk), dim3(64 * kNW), 0, s, p);
  if (!set_grid(p, BH, Ns)) return fail("mhada_attn_train_bwd: grid too large");
  // 288 registers, one wave per SIMD, no spills (two waves per SIMD at 256 registers spilled 18
  // and measured the same, tools/train_attn_bench.py)
  hipLaunchKernelGGL((attn_train_dkv_kernel<kNW, 1, false>), dim3(p.nblk), dim3(64 * kNW), 0, s, p);
  return check_launch("mhada_attn_train_bwd");
}

extern "C" int mhada_attn_train_dkv(const float* q, const float* k, const float* v, const float* lse,
                                    const float* dmo, const float* dd, float* dk, float* dv, float* ds, int BH,
                                    int Nc, int Ns, mhada_stream_t s_) {
  if (!q || !k || !v || !lse || !dmo || !dd || !dk || !dv || !ds || BH <= 0 || Nc <= 0 || Ns <= 0)
    return fail("mhada_attn_train_dkv: bad args");
  if ((long long)(Nc + TT) * Ns > kMaxSpillRows)
    return fail("mhada_attn_train_dkv: (Nc + 32) * Ns above 2^29 - 2^14 (32-bit dS offsets)");
  TrainP p = {};
  p.q = q; p.k = k; p.v = v; p.lse = const_cast<float*>(lse); p.dmo = dmo; p.dd = dd; p.dk = dk; p.dv = dv;
  p.ds = ds; p.Nc = Nc; p.Ns = Ns;
  if (!set_grid(p, BH, Ns)) return fail("mhada_attn_train_dkv: grid too large");
  if (tuning().train_dkv_dma)  // LDS-DMA form, two workgroups per CU (round 4)
    hipLaunchKernelGGL(attn_train_dkv_dma_kernel, dim3(p.nblk), dim3(64 * kNW), 0, (hipStream_t)s_, p);
  else
    hipLaunchKernelGGL((attn_train_dkv_kernel<kNW, 1, true>), dim3(p.nblk), dim3(64 * kNW), 0, (hipStream_t)s_, p);
  return check_launch("mhada_attn_train_dkv");
}

#ifdef ATTN_CLOCK
// Diagnostic builds: the first n stamps (4 per workgroup) of the last dK/dV' launch.
extern "C" int mhada_dbg_train_clock(unsigned long long* host, int n) {
  if (!host || n <= 0 || n > 4 * kTrainClockBlocks) return fail("mhada_dbg_train_clock: bad args");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_train_clock), sizeof(unsigned long long) * n) != hipSuccess)
    return fail("mhada_dbg_train_clock: copy failed");
  return MHADA_OK;
}
#endif
