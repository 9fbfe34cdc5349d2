// mhada_gemm: argument checks and dtype dispatch (kernels: gemm_impl.h, instantiated per dtype
// combination in gemm_d_*.hip).
#include "gemm_impl.h"



using namespace mhada;

extern "C" int mhada_gemm(const mhada_gemm_args* a, mhada_stream_t stream_) {
  if (!a) return fail("mhada_gemm: null args");
  hipStream_t stream = (hipStream_t)stream_;
  if (a->M < 0 || a->N <= 0 || a->K <= 0 || a->nb1 <= 0 || a->nb2 <= 0)
    return fail("mhada_gemm: bad sizes");
  if (a->M == 0) return MHADA_OK;
  if (a->compute != MHADA_F32 && a->compute != MHADA_BF16) return fail("mhada_gemm: bad compute dtype");
  if (a->a_dtype != MHADA_F32 && a->a_dtype != MHADA_BF16) return fail("mhada_gemm: bad a_dtype");
  if (a->c_dtype != MHADA_F32 && a->c_dtype != MHADA_BF16) return fail("mhada_gemm: bad c_dtype");
  if (a->r && a->r_dtype != a->c_dtype) return fail("mhada_gemm: residual dtype must equal output dtype");
  if (a->compute == MHADA_F32 && (a->a_dtype != MHADA_F32 || a->c_dtype != MHADA_F32))
    return fail("mhada_gemm: fp32 compute needs fp32 A and C");
  if (!a->a || !a->w || (!a->c && !a->c2_planes)) return fail("mhada_gemm: null operand");
  if (a->c2_planes && (a->a_mode != MHADA_A_SPLIT3 || !a->c2 || a->c_dtype != MHADA_F32 || a->N % 4 ||
                       !tuning().gemm_ldsepi))
    return fail("mhada_gemm: c2_planes needs SPLIT3 mode, a c2 buffer, fp32 C, N % 4 == 0 and the LDS epilogue");
  const int ec = a->compute == MHADA_F32 ? 4 : 8;      // compute elements per 16 B
  const int ea = a->a_dtype == MHADA_F32 ? 4 : 8;      // A elements per 16 B
  const int bk = a->compute == MHADA_F32 ? 32 : 64;
  if (a->K % ec) return fail("mhada_gemm: K must be a multiple of 16 bytes of compute type");
  if (!aligned16(a->w) || a->ldw % ec || a->sw1 % ec || a->sw2 % ec)
    return fail("mhada_gemm: W must be 16-byte aligned with aligned strides");
  if (!aligned16(a->a) || a->sa1 % ea || a->sa2 % ea) return fail("mhada_gemm: A must be 16-byte aligned");
  // the epilogue moves 4 consecutive output columns per access
  if (((uintptr_t)a->c & 7) || a->ldc % 4 || a->sc1 % 4 || a->sc2 % 4)
    return fail("mhada_gemm: C must be 8-byte aligned with strides that are multiples of 4");
  if (a->r && (((uintptr_t)a->r & 7) || a->ldr % 4 || a->sr1 % 4 || a->sr2 % 4))
    return fail("mhada_gemm: R must be 8-byte aligned with strides that are multiples of 4");
  if (a->bias && (!aligned16(a->bias) || a->sb1 % 4 || a->sb2 % 4))
    return fail("mhada_gemm: bias must be 16-byte aligned with strides that are multiples of 4");
  GemmP p{};
  p.M = a->M; p.N = a->N; p.K = a->K; p.nb2 = a->nb2;
  p.a = a->a; p.lda = a->lda; p.sa1 = a->sa1; p.sa2 = a->sa2;
  p.a_mu = a->a_mu; p.smu1 = a->smu1; p.smu2 = a->smu2;
  p.img_c = a->img_c; p.img_h = a->img_h; p.img_w = a->img_w;
  p.w = a->w; p.ldw = a->ldw; p.sw1 = a->sw1; p.sw2 = a->sw2;
  p.bias = a->bias; p.sb1 = a->sb1; p.sb2 = a->sb2;
  p.r = a->r; p.ldr = a->ldr; p.sr1 = a->sr1; p.sr2 = a->sr2;
  p.c = a->c; p.ldc = a->ldc; p.sc1 = a->sc1; p.sc2 = a->sc2;
  if (a->relu < 0 || a->relu > 2) return fail("mhada_gemm: relu must be 0, 1 or 2");
  // (a SPLIT3 GEMM may also write the masked result's planes: c2_planes with C, round 6)
  if (a->relu == 2 && (!a->r || a->r_dtype != MHADA_F32 || a->c_dtype != MHADA_F32 || !a->c ||
                       (a->c2 && !(a->c2_planes && a->a_mode == MHADA_A_SPLIT3)) || a->vt ||
                       (a->a_mode != MHADA_A_ROWS && a->a_mode != MHADA_A_SPLIT3)))
    return fail("mhada_gemm: relu = 2 (ReLU-adjoint mask) needs fp32 C, an fp32 mask in r, ROWS or SPLIT3 mode, "
                "no vt, c2 only as SPLIT3 planes");
  p.relu = a->relu;
  p.c2 = a->c2; p.ldc2 = a->ldc2; p.sc21 = a->sc21; p.sc22 = a->sc22;
  p.c2planes = a->c2_planes ? 1 : 0;
  p.vt = a->vt; p.ldt = a->ldt; p.svt1 = a->svt1; p.svt2 = a->svt2;
  if (a->c2 && (a->c_dtype != MHADA_F32 || ((uintptr_t)a->c2 & 7) || a->ldc2 % 4 || a->sc21 % 4 || a->sc22 % 4))
    return fail("mhada_gemm: c2 (bf16 copy) needs fp32 C, 8-byte alignment and strides that are multiples of 4");
  if (a->vt && (a->N != 128 || a->a_mode != MHADA_A_ROWS || a->relu || a->r || a->c2 || !aligned16(a->vt) ||
                a->ldt % 64 || a->ldt < a->M || a->svt1 % 8 || a->svt2 % 8))
    return fail("mhada_gemm: vt needs the K|V' projection shape (ROWS, N == 128, no ReLU/residual), a 16-byte "
                "aligned image and ldt a multiple of 64 covering M");
  switch (a->a_mode) {
    case MHADA_A_ROWS:
      if (a->lda % ea) return fail("mhada_gemm: lda must be a multiple of 16 bytes");
      break;
    case MHADA_A_PATCH8:
      if (a->a_dtype != MHADA_F32) return fail("mhada_gemm: PATCH8 needs an fp32 image");
      if (a->img_w % 8 || a->img_h < 8) return fail("mhada_gemm: PATCH8 needs img_w % 8 == 0");
      if (a->K != a->img_c * 64) return fail("mhada_gemm: PATCH8 needs K == 64*img_c");
      p.out_h = a->img_h / 8; p.out_w = a->img_w / 8;
      if (a->M != p.out_h * p.out_w) return fail("mhada_gemm: PATCH8 needs M == (H/8)*(W/8)");
      if (a->a_mu) return fail("mhada_gemm: centring only in ROWS mode");
      break;
    case MHADA_A_CONV3X3_ZERO: {
      const int pad = a->pad ? a->pad : 1;
      if (pad < 1 || pad > 2) return fail("mhada_gemm: CONV3X3_ZERO needs pad 1 or 2");
      if (a->img_c % bk) return fail("mhada_gemm: CONV needs Cin % (128 bytes of compute type) == 0");
      if (a->K != 9 * a->img_c) return fail("mhada_gemm: CONV needs K == 9*Cin");
      p.pad = pad;
      p.out_h = a->img_h + 2 * (pad - 1); p.out_w = a->img_w + 2 * (pad - 1);
      if (a->M % (p.out_h * p.out_w)) return fail("mhada_gemm: CONV needs M == batch*out_h*out_w");
      if (a->nb1 * a->nb2 != 1) return fail("mhada_gemm: CONV is not z-batched (batch lives in M)");
      if (a->a_mu) return fail("mhada_gemm: centring only in ROWS mode");
      break;
    }
    case MHADA_A_CONV3X3:
    case MHADA_A_CONV3X3_UP2: {
      const int up = a->a_mode == MHADA_A_CONV3X3_UP2 ? 2 : 1;
      if (a->img_c % bk) return fail("mhada_gemm: CONV needs Cin % (128 bytes of compute type) == 0");
      if (a->K != 9 * a->img_c) return fail("mhada_gemm: CONV needs K == 9*Cin");
      p.out_h = a->img_h * up; p.out_w = a->img_w * up;
      if (p.out_h < 2 || p.out_w < 2) return fail("mhada_gemm: reflection padding needs H, W >= 2");
      if (a->M % (p.out_h * p.out_w)) return fail("mhada_gemm: CONV needs M == batch*out_h*out_w");
      if (a->nb1 * a->nb2 != 1) return fail("mhada_gemm: CONV is not z-batched (batch lives in M)");
      if (a->a_mu) return fail("mhada_gemm: centring only in ROWS mode");
      break;
    }
    case MHADA_A_SPLIT3:
      if (a->compute != MHADA_BF16 || a->a_dtype != MHADA_BF16)
        return fail("mhada_gemm: SPLIT3 needs bf16 planes and bf16 compute");
      if (a->nb1 * a->nb2 != 1 || a->a_mu || a->vt) return fail("mhada_gemm: SPLIT3 is one problem, no centring / vt");
      if (a->K % 384) return fail("mhada_gemm: SPLIT3 needs K = 6 K0 with K0 % 64 == 0");
      if (a->lda % 8 || a->lda < a->K / 6) return fail("mhada_gemm: SPLIT3 lda must be a multiple of 8 and >= K0");
      p.spl = (long long)a->M * a->lda;
      break;
    default:
      return fail("mhada_gemm: bad a_mode");
  }
  const int nz = a->nb1 * a->nb2;
  if (nz > 65535) return fail("mhada_gemm: too many batch entries");
  // the decoder's 64 -> 64 layer (with its fused upsample): direct tile kernel (conv_tile.hip)
  if (!a->c2 && !a->vt && tuning().conv_c64 && a->compute == MHADA_BF16 && a->a_dtype == MHADA_BF16 && a->c_dtype == MHADA_BF16 &&
      (a->a_mode == MHADA_A_CONV3X3 || a->a_mode == MHADA_A_CONV3X3_UP2) && a->img_c == 64 && a->N == 64 &&
      a->ldc == 64 && a->ldw == 576 && a->bias && !a->r)
    return conv3x3_c64(a->a, a->w, a->bias, a->c, a->M / (p.out_h * p.out_w), p.out_h, p.out_w,
                       a->a_mode == MHADA_A_CONV3X3_UP2, a->relu, stream);
  // the decoder's 128-input-channel layers: direct tile kernel with a streamed weight ring
  if (!a->c2 && !a->vt && tuning().conv_dir && a->compute == MHADA_BF16 && a->a_dtype == MHADA_BF16 &&
      a->c_dtype == MHADA_BF16 && a->a_mode == MHADA_A_CONV3X3 &&
      ((a->img_c == 128 && (a->N == 64 || a->N == 128)) || (a->img_c == 256 && a->N == 128)) &&
      a->ldc == a->N && a->ldw == 9 * a->img_c && a->bias && !a->r &&
      (long long)p.out_h * p.out_w * a->img_c * 2 < 0x7ff00000LL)
    return conv3x3_dir(a->a, a->w, a->bias, a->c, a->M / (p.out_h * p.out_w), p.out_h, p.out_w, a->img_c, a->N,
                       a->relu, stream);
  if (a->compute == MHADA_F32) return gemm_dispatch_f32(a->a_mode, p, nz, stream);
  if (a->a_dtype == MHADA_F32) {
    if (a->c_dtype == MHADA_F32) return gemm_dispatch_bf16_a32_o32(a->a_mode, p, nz, stream);
    return gemm_dispatch_bf16_a32_o16(a->a_mode, p, nz, stream);
  }
  if (a->c_dtype == MHADA_F32) return gemm_dispatch_bf16_a16_o32(a->a_mode, p, nz, stream);
  return gemm_dispatch_bf16_a16_o16(a->a_mode, p, nz, stream);
}
