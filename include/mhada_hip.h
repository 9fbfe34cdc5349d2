/*
 * mhada_hip.h — C-ABI of libmhada_hip.so, the MI355X (gfx950) kernels behind the MHAdaSTr
 * style-transfer forward path.
 *
 * The reference (Maboroshi0327/MHAda-Style-Transfer, MHAdaSTr/) is pure PyTorch: its
 * "interface" for this path is the Python module API of MHAdaSTr/network/ (SURVEY.md §8b).
 * Every entry point below replaces the aten op(s) a reference module calls; the file:line of
 * that call is given per function.  The host side that mirrors the reference module API
 * (mhada-style-transfer_amd/network/) binds these symbols with ctypes.
 *
 * Conventions
 *   - Plain C: device pointers, sizes, strides (in ELEMENTS), dtype codes, an opaque stream.
 *   - The caller owns every buffer; the library never allocates device memory.
 *   - Everything is enqueued on `stream` (a hipStream_t; NULL = default stream); no call
 *     synchronises, so all entry points are hipGraph-capturable.
 *   - Return 0 on success; non-zero = bad argument (1) or launch failure (2); the message is
 *     available from mhada_last_error() (thread-local).
 *   - Internal activations are token-major ("NHWC": [batch][token][channel]).
 */
#ifndef MHADA_HIP_H
#define MHADA_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mhada_stream_t; /* hipStream_t */

enum { MHADA_OK = 0, MHADA_ERR_ARG = 1, MHADA_ERR_LAUNCH = 2 };
enum { MHADA_F32 = 0, MHADA_BF16 = 1 };
enum { MHADA_ACT_SOFTMAX = 0, MHADA_ACT_COSINE = 1 };
enum { MHADA_PAD_REFLECT = 0, MHADA_PAD_ZERO = 1 };
enum {
  MHADA_A_ROWS = 0,        /* A[m*lda + k], row-major                                     */
  MHADA_A_PATCH8 = 1,      /* A = im2col of an NCHW fp32 image, 8x8 patches, stride 8     */
  MHADA_A_CONV3X3 = 2,     /* A = im2col of NHWC input, 3x3 taps, ReflectionPad2d(1)      */
  MHADA_A_CONV3X3_UP2 = 3, /* as CONV3X3 on bilinear-x2(input) (align_corners=False)      */
  MHADA_A_CONV3X3_ZERO = 4, /* 3x3 taps with ZERO padding `pad` (1: same size, as VGG19's
                              nn.Conv2d(padding=1); 2: the full correlation, out = in + 2 —
                              the input gradient of a padded 3x3 conv)                   */
  MHADA_A_SPLIT3 = 5       /* (ABI 15) fp32-accurate products on the bf16 MFMA: A = three bf16
                              planes [3][M][lda] of an fp32 matrix (x = p0 + p1 + p2, as
                              mhada_layernorm writes with y_dtype MHADA_BF16X3); K = 6 K0 is
                              virtual — K-tile 6 kk + t reads columns 64 kk .. 64 kk + 63 of
                              plane (1, 2, 0, 1, 0, 0)[t] — and W is the matching [N][6 K0]
                              bf16 interleave: 64-column chunk kk of W's planes
                              q1, q0, q2, q0, q1, q0 in turn.  bf16 compute, nb1 = nb2 = 1,
                              N > 128, K0 % 64 == 0, no centring / vt.                  */
};
/* mhada_layernorm's y_dtype for the MHADA_A_SPLIT3 operand: three bf16 planes [3][rows][cols],
 * p0 = bf16(y), p1 = bf16(y - p0), p2 = bf16(y - p0 - p1) of the fp32 result y (ABI 15) */
enum { MHADA_BF16X3 = 2 };

int mhada_abi_version(void);  /* 16 (mhada_split3_kv / mhada_attn_split3; 15: mhada_gemm a_mode MHADA_A_SPLIT3, mhada_layernorm y_dtype MHADA_BF16X3; 14: mhada_cosine_moments / mhada_cosine_attn, mhada_warp_bwd; 13: mhada_clock_probe; tuning knobs of removed kernel variants dropped, attn_waves 0 = auto; 12: mhada_feat_stats; 11: mhada_transpose64; 10: mhada_attn_train_fwd_vt; 9: 3-channel conv adjoints mhada_vgg_stem_dgrad / mhada_out3_dgrad / mhada_out3_wgrad; 8: mhada_feat_loss_bwd; 7: gemm c2 / vt outputs, instnorm / attention backward helpers; 6: LayerNorm / pos-embed training adjoints; 5: Winograd conv; 4: training CONV3X3_ZERO, mhada_gemm_tn, backward helpers) */
const char* mhada_last_error(void);

/* Kernel-variant table.  Defaults are the measured winners; the other variants serve A/B
 * measurements and tests that force a rare path.  Initialised ONCE, at the first call into the
 * library, from MHADA_<NAME> environment variables (NAME upper-cased); afterwards only these
 * calls change it (not thread-safe against concurrent launches: set knobs between launches).
 * Knobs (value range): attn_fixed_shift (0|1), attn_waves (0|4|8; 0 = auto: 8, or 4 when the
 * 8-wave grid has fewer blocks than CUs), attn_tk (64|128), attn_prio (0|1), vit_attn_vec (0|1),
 * out3_mfma (0|1), out3_tile (0|1), gemm_pp (0|1), gemm_persist (0|1), gemm_pp128 (0|1),
 * gemm_ldsepi (0|1), gemm_n64 (128|256), conv_c64 (0|1), conv_dir (0|1), gemm_rinit (0|1), tn_skinny_lds (0|1),
 * train_dkv_dma (0|1), wino4 (0|1), upsample_quad (0|1; ABI 16), xknob (0..15, read by no shipped dispatch).
 * Returns MHADA_ERR_ARG for an unknown knob or an out-of-range value.  No reference
 * counterpart (the reference has no kernels). */
int mhada_set_tuning(const char* name, int value);
int mhada_get_tuning(const char* name, int* value);

/* Sustained shader-clock probe (ABI 13; probe.hip): nblk workgroups of 8 waves each run 4 * iters
 * v_mfma_f32_16x16x32_bf16 per wave on pseudo-random operands read from LDS; workgroup b
 * writes stamps[2b] = shader-clock ticks (s_memtime) and stamps[2b + 1] = 100 MHz ticks
 * (s_memrealtime) spent in the chain (device buffer of 2 * nblk).  clock = stamps[2b] /
 * stamps[2b + 1] * 100 MHz.  bench.py runs it after each timed region so a box's clock under dense
 * MFMA load is reported beside its throughput.  No reference counterpart (infer_time.py:64-87 is
 * the reference's only timer). */
int mhada_clock_probe(unsigned long long* stamps, int nblk, int iters, mhada_stream_t stream);

/*
 * Batched NT GEMM with fused epilogue:
 *   C[z][m][n] = act(sum_k A[z][m][k] * W[z][n][k] + bias[z][n]) + R[z][m][n]
 * z = (z1, z2) in [0,nb1) x [0,nb2); each operand has per-level strides (0 = shared).
 * A is loaded in `a_mode` (see enum) from dtype a_dtype and converted to `compute`
 * (MFMA input type: fp32 -> v_mfma_f32_32x32x2_f32, bf16 -> v_mfma_f32_32x32x16_bf16).
 * ROWS mode may centre A per column on load: A[m][k] - a_mu[z1*smu1 + z2*smu2 + k].
 * W has dtype `compute`; bias/R are optional (NULL).
 *
 * Replaces: PatchEmbedding conv 8x8/8 (vit.py:109,113) [PATCH8 + pos-embed as R];
 *   MHA in_proj/out_proj addmm + residual (vit.py:59-60); MLP Linear/ReLU/Linear + residual
 *   (vit.py:49-53,63); the per-head 1x1 convs f/g/h (adaDecoder.py:143-145,173,178,182);
 *   out_conv (adaDecoder.py:152,205); Decoder ReflectionPad2d+Conv3x3+ReLU(+bilinear x2)
 *   (conv.py:23-33,36-45,61-72) [CONV3X3 / CONV3X3_UP2].
 */
typedef struct mhada_gemm_args {
  int M, N, K;
  int nb1, nb2;
  int compute;  /* MHADA_F32 | MHADA_BF16 */
  int a_mode;   /* MHADA_A_* */
  const void* a; int a_dtype; long long lda, sa1, sa2;
  const float* a_mu; long long smu1, smu2;
  /* PATCH8: img_c/h/w of the NCHW image (a_dtype must be F32).
     CONV*: img_c = Cin, img_h/img_w = spatial size of the NHWC INPUT tensor; the output grid
     is img_h x img_w (CONV3X3), 2*img_h x 2*img_w (CONV3X3_UP2) or img + 2*(pad-1)
     (CONV3X3_ZERO); M = batch*out_h*out_w. */
  int img_c, img_h, img_w;
  const void* w; long long ldw, sw1, sw2;
  const float* bias; long long sb1, sb2;
  const void* r; int r_dtype; long long ldr, sr1, sr2;
  void* c; int c_dtype; long long ldc, sc1, sc2;
  /* 1: ReLU after the bias (before a residual).  2 (ABI 10; SPLIT3 too since ABI 16): ReLU-adjoint mask — r is not added
   * but read as a mask of C's layout: C = 0 where r <= 0 (a gradient GEMM whose input was a ReLU
   * output consumed only by the forward of this layer; fp32 C and r, ROWS mode). */
  int relu;
  int pad;      /* CONV3X3_ZERO only: 1 or 2 (0 = 1) */
  /* Optional second output (NULL = none): a bf16 copy of C (row stride ldc2, z-strides
   * sc21/sc22), fp32 C only — the last MHAda block's fcs, fp32 for the caller and bf16 for the
   * decoder's first conv. */
  void* c2; long long ldc2, sc21, sc22;
  /* Optional V' transpose (NULL = none; the MHAda K|V' projection, N = 128): columns 64..127
   * are NOT written to C but to vt[o][pos(m)] = V'[m][o] and vt[64 + o][pos(m)] = V'[m][o]^2
   * (dtype of C; row stride ldt >= M rounded up to 64, z-strides svt1/svt2; pos = the
   * mhada_transpose_v key order; positions M..ldt-1 written 0).  Replaces mhada_transpose_v. */
  void* vt; long long ldt, svt1, svt2;
  /* (ABI 15) 1: c2 receives the fp32 result as three bf16 planes [3][M][ldc2] (p0 = bf16(y),
   * p1 = bf16(y - p0), p2 = bf16(y - p0 - p1): the MHADA_A_SPLIT3 operand of the next GEMM) and
   * C may be NULL (not written).  SPLIT3 mode, fp32 C dtype, one problem. */
  int c2_planes;
} mhada_gemm_args;

int mhada_gemm(const mhada_gemm_args* args, mhada_stream_t stream);

/* Row LayerNorm over `cols` (eps 1e-6 in the ViT): y = (x-mean)/sqrt(var+eps)*gamma + beta.
 * x fp32 [rows][cols]; y dtype y_dtype (MHADA_F32, MHADA_BF16, or MHADA_BF16X3: y = three bf16
 * planes [3][rows][cols] of the fp32 result, the MHADA_A_SPLIT3 GEMM operand).  Replaces
 * nn.LayerNorm (vit.py:54-55,58,62). */
int mhada_layernorm(const float* x, void* y, int y_dtype, const float* gamma, const float* beta,
                    int rows, int cols, float eps, mhada_stream_t stream);

/* nn.MultiheadAttention(batch_first=False) applied to a (B, N, C) tensor (vit.py:48,59):
 * the SEQUENCE axis is the batch axis.  For each token n and head h:
 *   out[i][n][h] = sum_j softmax_j(q[i][n][h] . k[j][n][h] / sqrt(d)) v[j][n][h]
 * qkv [L][ntok][3C] (packed q|k|v, dtype), out [L][ntok][C] (dtype); L = batch size. */
int mhada_vit_batch_attn(const void* qkv, void* out, int dtype, int L, int ntok, int heads,
                         int head_dim, mhada_stream_t stream);

/* PosEmbedding (vit.py:81-102): bilinear (align_corners=False) resize of pos (C, bh, bw)
 * fp32 to (oh, ow), written token-major out[oh*ow][C] fp32 (copy when sizes match). */
int mhada_pos_embed(const float* pos, float* out, int C, int bh, int bw, int oh, int ow,
                    mhada_stream_t stream);

/* InstanceNorm2d(affine=False) statistics (adaDecoder.py:147-149): per (b, c) mean and
 * 1/sqrt(biased var + eps) over the N tokens of x [B][N][C] fp32.  `work` holds
 * splits*B*C*2 doubles (any splits >= 1).  C % 4 == 0, x 16-byte aligned. */
int mhada_instnorm_stats(const float* x, float* mu, float* rstd, double* work, int B, int N,
                         int C, int splits, float eps, mhada_stream_t stream);

/* Fold the InstanceNorm scale into the per-head 1x1-conv weights of one AdaAttnMultiHead
 * block (adaDecoder.py:173,178,182) and derive the style-side mean of V:
 *   wq[b][h][o][c]  = Wf[h][o][c] * rstd_c[b][64h+c]            (A is centred on load)
 *   wkv[b][h][o][c] = o<64 ? Wg[h][o][c] * rstd_s[b][64h+c] * kscale : Wh[h][o-64][c]
 *   bkv[h][o]       = o<64 ? bg[h][o] * kscale : 0               (V' = V - mean_tokens(V))
 *   v_mu[b][64h+o]  = sum_c Wh[h][o][c] * mu_s[b][64h+c] + bh[h][o]
 * kscale = log2(e) for the softmax activation (mhada_attn's K contract), 1 for cosine.
 * W* fp32 [H][64][64]; wq/wkv dtype `dtype`. */
int mhada_fold_block(const float* wf, const float* wg, const float* wh, const float* bg,
                     const float* bh, const float* rstd_c, const float* mu_s,
                     const float* rstd_s, void* wq, void* wkv, float* bkv, float* v_mu,
                     float kscale, int dtype, int B, int H, mhada_stream_t stream);

/* The transposed V' operand image the attention kernel streams, from kv [B][H][Ns][128] of
 * dtype `dtype`: VT[b][h][o][pos(n)] = V'[b][h][n][64+o] (o<64) and V'^2 (64<=o<128), row
 * stride ceil64(Ns) (zero padded).  bf16: pos() swaps bits 2 and 3 of n (keys permuted inside
 * groups of 16 to match the 32x32x16 accumulator's row order); fp32: pos(n) = n. */
int mhada_transpose_v(const void* kv, void* vt, int dtype, int B, int H, int Ns, mhada_stream_t stream);

/* L2-normalise the 64-wide rows of q [B][H][Nc][64] and the K half of kv [B][H][Ns][128]
 * in place (CosineSimilarity, adaDecoder.py:30-32).  Nc == 0 (q may be NULL) or Ns == 0 (kv
 * may be NULL) normalises one side only (a cached style's K once, each frame's Q per call). */
int mhada_cosine_prep(void* q, void* kv, int dtype, int B, int H, int Nc, int Ns,
                      mhada_stream_t stream);

/* Fused multi-head adaptive attention (adaDecoder.py:186-198), one launch per block:
 *   A = softmax(Q K^T) (no 1/sqrt(d); or the cosine form), M = A V, E2 = A V^2,
 *   S = sqrt(max(E2 - M^2, 1e-6)), out = S * IN(fcs) + M
 * computed flash-style (A never materialised) with V centred (v_mu added back to M).
 * Softmax: the K half of kv carries the factor log2(e) (mhada_fold_block kscale), so Q.K^T is
 * the logit in log2 units and P = exp2(Q.K^T - max).
 * q [B][H][Nc][64], kv [B][H][Ns][128] (K | V'), vt [B][H][128][ceil64(Ns)] (mhada_transpose_v),
 * fcs [B][Nc][64H] fp32 with its stats fcs_mu/fcs_rstd [B][64H], v_mu [B][64H];
 * out [B][Nc][64H] dtype. */
int mhada_attn(const void* q, const void* kv, const void* vt, const float* fcs,
               const float* fcs_mu, const float* fcs_rstd, const float* v_mu, void* out,
               int dtype, int B, int H, int Nc, int Ns, int activation, mhada_stream_t stream);

/* The fp32 softmax MHAda attention (adaDecoder.py:186-198, mhada_attn's contract and output) as
 * fp32-accurate SPLIT3 products on the bf16 MFMA (ABI 16; csrc/attn_split3.hip): every fp32 operand as
 * three bf16 planes x = x0 + x1 + x2 (round to nearest: x0 = bf16(x), x1 = bf16(x - x0),
 * x2 = bf16(x - x0 - x1)) and every product as the six cross products x_i y_j, i + j <= 2, summed in
 * fp32 accumulators (dropped terms < 2^-24 |x y|).  Replaces mhada_attn(dtype MHADA_F32, softmax).
 * mhada_split3_kv: the style-side operands kv fp32 [B][H][Ns][128] (K | V', only K read) and the fp32
 *   vt image [B][H][128][ldt] (mhada_transpose_v, ldt = ceil64(Ns)) -> img bf16 [B][H][576 ldt]:
 *   K planes [3][ldt][64] (rows >= Ns zero) | V'^T|V'^2^T planes [3][128][ldt] (key positions permuted
 *   in groups of 16 as the bf16 vt image).  Once per style (cacheable like kv / vt); B * H <= 65535.
 * mhada_attn_split3: q fp32 [B][H][Nc][64] (split on load) and img -> out fp32 [B][Nc][64H]; the other
 *   arguments as mhada_attn. */
int mhada_split3_kv(const float* kv, const float* vt, void* img, int B, int H, int Ns, mhada_stream_t stream);
/* x fp32 [n] -> planes bf16 [3][n]: p0 = bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 - p1) (the
 * MHADA_A_SPLIT3 operand of any fp32 matrix, e.g. the training step's activations and gradients;
 * ABI 16).  n % 4 == 0 and n * 2 % 16 == 0, 16-byte aligned pointers. */
int mhada_split3_rows(const float* x, void* planes, long long n, mhada_stream_t stream);
/* The SPLIT3 GEMM's weight operand in one launch (ABI 16): W fp32 [N][K0] (transposed = 0) or the W
 * of W^T (transposed = 1: w is [K0][N], the operand is W^T's [N][K0]) -> out bf16 [N][6 K0], per
 * 64-column chunk the planes q1 | q0 | q2 | q0 | q1 | q0 (q0 = bf16(x), q1 = bf16(x - q0),
 * q2 = bf16(x - q0 - q1)).  K0 % 64 == 0. */
int mhada_split3_weight(const float* w, void* out, int N, int K0, int transposed, mhada_stream_t stream);
/* The block's K|V' projection written straight as that plane image (the engine's fp32 softmax path:
 * replaces mhada_gemm with the vt epilogue plus mhada_split3_kv, adaDecoder.py:178,182):
 *   Y[n][o] = sum_c (fs[b][n][64h+c] - mu_s[b][64h+c]) wkv[b][h][o][c] + bkv[h][o]  (fp32 MFMA),
 * K = Y[:, :64], V' = Y[:, 64:] (V'^2 its fp32 square); fs [B][Ns][64H] fp32, mu_s [B][64H], wkv
 * [B][H][128][64] fp32 and bkv [H][128] from mhada_fold_block (dtype MHADA_F32). */
int mhada_kv_proj_split3(const float* fs, const float* mu_s, const float* wkv, const float* bkv, void* img,
                         int B, int H, int Ns, mhada_stream_t stream);
int mhada_attn_split3(const float* q, const void* img, const float* fcs, const float* fcs_mu,
                      const float* fcs_rstd, const float* v_mu, float* out, int B, int H, int Nc, int Ns,
                      mhada_stream_t stream);

/* The cosine activation (CosineSimilarity, adaDecoder.py:20-34) in its linear form (ABI 14):
 * A[i][j] = (q^_i.k^_j + 1) / l_i with l_i = q^_i.sum_j k^_j + Ns, so A V' and A V'^2 need only the
 * style-side moments — O(N d^2) instead of mhada_attn's Nc x Ns loop.  After mhada_cosine_prep:
 * mhada_cosine_moments reduces the normalised K half of kv [B][H][Ns][128] and vt
 * [B][H][128][ceil64(Ns)] (mhada_transpose_v layout) over the keys into mom [B][H][65][132] fp32:
 *   mom[d][o] = sum_n k^[n][d] vt[o][n] (d < 64, o < 128), mom[d][128] = sum_n k^[n][d],
 *   mom[64][o] = sum_n vt[o][n], mom[64][128] = Ns, other entries 0;
 * splits > 1 splits the keys over that many workgroups per (b, h) with a fixed-order sum
 * (work: splits*B*H*65*132 floats; splits == 1 may pass work = NULL).  Once per style.
 * mhada_cosine_attn: per query, M' = (q^.mom[:, o<64] + mom[64][o]) / l, E2' likewise with o + 64,
 * out = sqrt(max(E2' - M'^2, 1e-6)) * IN(fcs) + M' + v_mu — mhada_attn's arguments and output. */
int mhada_cosine_moments(const void* kv, const void* vt, int dtype, int B, int H, int Ns, float* mom,
                         float* work, int splits, mhada_stream_t stream);
int mhada_cosine_attn(const void* q, const float* mom, const float* fcs, const float* fcs_mu,
                      const float* fcs_rstd, const float* v_mu, void* out, int dtype, int B, int H,
                      int Nc, mhada_stream_t stream);

/* MHAda attention for training (adaDecoder.py:186-198 under train_image.py:139 autograd), fp32,
 * one (batch, head) per leading index, all rows of 64 (or 128) contiguous floats:
 *   fwd: q [BH][Nc][64], k [BH][Ns][64], v [BH][Ns][64] (V' = V - mean_tokens(V)),
 *        x [BH][Nc][64] (InstanceNorm(fcs)) -> out' = sqrt(max(E2'-M'^2,1e-6))*x + M' [BH][Nc][64],
 *        mo = [M' | E2'] [BH][Nc][128], lse = log2(sum exp) row normaliser [BH][Nc].
 *   bwd: dmo = [dM' | dE2'] [BH][Nc][128], dd = dM'.M' + dE2'.E2' [BH][Nc]
 *        -> dq [BH][Nc][64], dk [BH][Ns][64], dv [BH][Ns][64] (gradient w.r.t. V').
 * Replaces the autograd of adaDecoder.py:186-198 (bmm/softmax/bmm/sqrt); A is never stored. */
int mhada_attn_train_fwd(const float* q, const float* k, const float* v, const float* x, float* out,
                         float* mo, float* lse, int BH, int Nc, int Ns, mhada_stream_t stream);
/* The same forward on the inference fp32 attention structure (64-key tiles, lazy rescale, PV
 * operands from a V'^T | V'^2^T image): vt is caller-provided fp32 workspace [BH][128][ceil64(Ns)]
 * that this call fills from v.  Same outputs as mhada_attn_train_fwd (ABI 10). */
int mhada_attn_train_fwd_vt(const float* q, const float* k, const float* v, float* vt, const float* x,
                            float* out, float* mo, float* lse, int BH, int Nc, int Ns, mhada_stream_t stream);
/* The same forward with P V' / P V'^2 as fp32-accurate SPLIT3 products on the bf16 MFMA (ABI 16;
 * csrc/attn_split3.hip): S = Q K^T on the fp32 MFMA (as the backward recomputes it, so lse2 matches),
 * the PV products and row sums summed per 32-key group and added in fp32.  img is caller-provided
 * workspace of BH * 576 * ceil64(Ns) bf16 that this call fills from k (fp32 rows) and v (planes).
 * Same outputs as mhada_attn_train_fwd_vt. */
int mhada_attn_train_fwd_split3(const float* q, const float* k, const float* v, void* img, const float* x,
                                float* out, float* mo, float* lse, int BH, int Nc, int Ns, mhada_stream_t stream);
/* dst [BH][64][ldt] = src [BH][N][64] transposed per problem (columns N..ldt-1 zero; ldt % 64 == 0,
 * ldt >= N): K^T, the W operand of the dQ = dS K GEMM after mhada_attn_train_dkv's dS spill
 * (replaces the strided aten copy k.transpose(1, 2).contiguous()) (ABI 11). */
int mhada_transpose64(const float* src, float* dst, int BH, int N, int ldt, mhada_stream_t stream);
/* dQ = dS K of the dS-spill backward as fp32-accurate SPLIT3 products on the bf16 MFMA (ABI 16;
 * csrc/gemm_n64_split3.hip): c[z][m][n] = sum_k a[z][m][k] w[z][n][k], n < 64, for z < nz.  a fp32
 * rows (dS [BH][Nc][Ns]: M = Nc, K = Ns, lda, problem stride sa), split into three bf16 planes in
 * registers; w_planes = mhada_split3_rows of K^T (mhada_transpose64): three bf16 planes of stride wps
 * elements, each [nz][64][ldw] (problem stride sw); c fp32 [nz][M][ldc] (problem stride sc).
 * K % 32 == 0, 16-byte aligned rows and problems.  Replaces mhada_gemm(a = dS, w = K^T, N = 64, fp32). */
int mhada_gemm_n64_split3(const float* a, const void* w_planes, float* c, int nz, int M, int K, int lda,
                          long long sa, int ldw, long long sw, long long wps, int ldc, long long sc,
                          mhada_stream_t stream);
/* Its W operand in one pass (ABI 16): k fp32 [BH][N][64] -> planes bf16 [3][BH][64][ldt], the three
 * planes of K^T (= mhada_split3_rows(mhada_transpose64(k))), key columns >= N zero; ldt % 64 == 0. */
int mhada_transpose64_split3(const float* k, void* planes, int BH, int N, int ldt, mhada_stream_t stream);
int mhada_attn_train_bwd(const float* q, const float* k, const float* v, const float* lse,
                         const float* dmo, const float* dd, float* dq, float* dk, float* dv,
                         int BH, int Nc, int Ns, mhada_stream_t stream);
/* The dK / dV' half of mhada_attn_train_bwd, optionally spilling dS (the gradient of the
 * natural-unit logits) to ds [BH][Nc][Ns] fp32 (NULL: no spill).  With the spill, dQ = dS K is a
 * plain batched GEMM (mhada_gemm with W = K^T) instead of the query-stationary kernel that
 * recomputes S and dA: 896 instead of 1280 FLOP per (query, key, head), for 8 B of HBM traffic
 * per (query, key, head) — the trade the 288 GB / 8 TB/s part makes cheaply. */
int mhada_attn_train_dkv(const float* q, const float* k, const float* v, const float* lse, const float* dmo,
                         const float* dd, float* dk, float* dv, float* ds, int BH, int Nc, int Ns,
                         mhada_stream_t stream);

/* Last decoder layer (conv.py:96, ConvReLU(64, 3)): ReflectionPad2d(1) + conv3x3 Cin->3 +
 * bias + ReLU on NHWC x [B][H][W][Cin] (dtype), written NCHW fp32 y [B][3][H][W] — the
 * module's output layout.  clamp255 != 0 also applies the caller's clamp(0,255)
 * (infer_image.py:86). w fp32 [9][Cin][3] (tap = 3*ky+kx, cin, out); Cin in {32, 64, 128}. */
int mhada_conv3x3_out3(const void* x, int dtype, const float* w, const float* b, float* y,
                       int B, int H, int W, int Cin, int clamp255, mhada_stream_t stream);

/* Bilinear x2 upsample, align_corners=False (ConvReluInterpolate, conv.py:71) on NHWC:
 * x [B][H][W][C] -> y [B][2H][2W][C], dtype fp32|bf16, C % 8 == 0.  Used where the decoder's
 * upsample is not fused into the next conv's operand gather (the bf16 path). */
int mhada_upsample2x(const void* x, void* y, int dtype, int B, int H, int W, int C,
                     mhada_stream_t stream);

/* ---- video path: optical-flow warping, NCHW fp32 ---------------------- */

/* warp (utilities.py:100-118): y = grid_sample(x, (grid + flow) normalised by (W-1, H-1),
 * bilinear, align_corners=False).  x, y [B][C][H][W]; flow [B][2][H][W] (x then y
 * displacement, pixels); padding 0 = "zeros", 1 = "border". */
int mhada_warp(const float* x, const float* flow, float* y, int B, int C, int H, int W,
               int padding, mhada_stream_t stream);

/* Adjoint of mhada_warp w.r.t. x (ABI 14; train_video.py:147-151 temporal losses under
 * autograd): gx += W^T gy, i.e. each output pixel's gradient scattered to its four bilinear taps
 * with the forward's weights (fp32 atomics, as ATen's grid_sampler_2d_backward).  gx must be
 * initialised by the caller (zeros); the flow receives no gradient.  Shapes as mhada_warp. */
int mhada_warp_bwd(const float* gy, const float* flow, float* gx, int B, int C, int H, int W,
                   int padding, mhada_stream_t stream);

/* flow_warp_mask (utilities.py:121-151): mask [H][W] = 1 where the forward flow flo01 warped
 * back by flo10 returns within `threshold` (L1, pixels) of the start, else 0.  flo01, flo10
 * [2][H][W]; padding as mhada_warp. */
int mhada_flow_warp_mask(const float* flo01, const float* flo10, float* mask, int H, int W,
                         float threshold, int padding, mhada_stream_t stream);

/* Warping error (exps_sintel.py:101-109): out[b] = sum(mask * |cs2 - warp(cs1, flow)|) /
 * (C*H*W) per image, zero padding; cs1, cs2 [B][C][H][W], flow [B][2][H][W], mask [B][H][W].
 * work: fp64 scratch of B * ceil(H*W/256) entries (fixed-order partial sums). */
int mhada_warp_l1(const float* cs1, const float* cs2, const float* flow, const float* mask,
                  double* work, float* out, int B, int C, int H, int W, mhada_stream_t stream);

/* ---- training path (train_image.py:139 loss.backward(), fp32, NHWC activations) ---------- */

/* Weight-gradient contraction C[M][N] = sum_k A[k][m] * B[k][n] (C row stride ldc), fp32:
 *   conv wgrad: A = dY' [pixels][Cout] (lda = Cout), B = im2col of the layer input in b_mode
 *     MHADA_A_CONV3X3 (reflect pad 1) or MHADA_A_CONV3X3_ZERO (zero pad `pad`): k = output pixel,
 *     n = tap*Cin + ci (N = 9*Cin; img_* = the NHWC input), C = dW [Cout][ky][kx][Cin];
 *   linear dW = dY^T X: A = dY [rows][out], B = X [rows][in] (b_mode MHADA_A_ROWS, ldb);
 *   patch-embedding dW (vit.py:109): b_mode MHADA_A_PATCH8, B = the NCHW fp32 image (img_*),
 *     k = token, n = c*64 + ky*8 + kx (N = 64*img_c).
 * Replaces the weight-gradient half of conv2d / addmm backward (conv.py:27-32, vgg19 convs,
 * vit.py:49-63 Linear layers).  K is split into partial slabs in `work` (>= M*N floats; up to
 * mhada_gemm_tn_splits(M,N,K)*M*N are used) summed in a fixed order: deterministic.  N % 4 == 0. */
typedef struct mhada_gemm_tn_args {
  int M, N, K;
  const float* a; long long lda;
  const float* b; long long ldb;
  int b_mode;
  int img_c, img_h, img_w, pad;
  float* c; long long ldc;
  float* colsum;  /* optional [M]: sum_k A[k][m] (the bias gradient), fused into the GEMM's A staging */
  int nb;         /* batch of nb problems (0 / 1: one): A and B advance by sza / szb elements, C is
                     [nb][M][N] (ldc == N), colsum [nb][M]; ROWS mode, M > 4 */
  long long sza, szb;
} mhada_gemm_tn_args;
int mhada_gemm_tn_splits(int M, int N, int K);
int mhada_gemm_tn(const mhada_gemm_tn_args* args, float* work, long long work_floats, mhada_stream_t stream);

/* Backward of the batch-axis MHA core (vit.py:48,59; forward mhada_vit_batch_attn), fp32:
 * qkv [L][ntok][3C] (the forward input), dout [L][ntok][C] -> dqkv [L][ntok][3C]; L <= 8. */
int mhada_vit_batch_attn_bwd(const float* qkv, const float* dout, float* dqkv, int L, int ntok, int heads,
                             int head_dim, mhada_stream_t stream);
/* The same with dqkv's three bf16 planes written as well (ABI 16): plane p of element e of this call's
 * dqkv at planes[p * pstride + e] (pstride >= L * ntok * 3C; a grouped call passes its slice of the full
 * planes): the QKV input-gradient GEMM's SPLIT3 operand in training. */
int mhada_vit_batch_attn_bwd_split3(const float* qkv, const float* dout, float* dqkv, void* planes,
                                    long long pstride, int L, int ntok, int heads, int head_dim,
                                    mhada_stream_t stream);

/* Bias gradients: out[c] = sum_r x[r][c] (x [rows][C] fp32, C % 4 == 0); work >= C floats
 * (up to 1024*C used), fixed-order reduction. */
int mhada_colsum(const float* x, float* out, long long rows, int C, float* work, long long work_floats,
                 mhada_stream_t stream);

/* nn.LayerNorm for the training path (vit.py:54-55,58,62; replaces aten native_layer_norm and
 * its backward): y fp32 [rows][cols], stats [rows][2] = (mean, rstd) for the backward.
 * cols 256 / 512 / 1024; 16-byte aligned x, y, gamma, beta. */
int mhada_layernorm_fwd(const float* x, float* y, float* stats, const float* gamma, const float* beta,
                        int rows, int cols, float eps, mhada_stream_t stream);
/* The same with y's three bf16 planes [3][rows][cols] written as well (ABI 16): the next SPLIT3 linear's
 * A operand in training (replaces mhada_split3_rows of y). */
int mhada_layernorm_fwd_split3(const float* x, float* y, void* planes, float* stats, const float* gamma,
                               const float* beta, int rows, int cols, float eps, mhada_stream_t stream);

/* LayerNorm backward: dx [rows][cols], dgamma / dbeta [cols] (fixed-order sums: per-128-row block
 * partials, then the slab reduction).  work: >= (ceil(rows/128) * 2 + 2) * cols floats. */
int mhada_layernorm_bwd(const float* x, const float* dy, const float* stats, const float* gamma, float* dx,
                        float* dgamma, float* dbeta, float* work, long long work_floats, int rows, int cols,
                        mhada_stream_t stream);

/* Adjoint of mhada_pos_embed (vit.py:91-92 under autograd; replaces aten's atomic
 * upsample_bilinear2d_backward): g token-major [oh*ow][C] -> gpos [C][bh][bw], a gather per source
 * pixel in a fixed order (deterministic). */
/* InstanceNorm2d(affine=False) backward on token rows [B][N][C] (adaDecoder.py:147-149 under
 * autograd; replaces ~7 aten ops): dx = (dy - mean_N dy - y mean_N(dy y)) * rstd, y the normalised
 * forward output.  work: splits*B*C*2 doubles + B*C*2 floats; C % 4 == 0, 16-byte aligned. */
int mhada_instnorm_bwd(const float* dy, const float* y, const float* rstd, float* dx, double* work,
                       int B, int N, int C, int splits, mhada_stream_t stream);

/* Elementwise head of the MHAda attention-core backward (adaDecoder.py:189-198 under autograd):
 * rows of 64 channels; mo = [M' | E2'] (rows x 128), x = IN(fcs) head rows, dout; writes dx,
 * dmo = [dM' | dVar] (rows x 128) and dd = rowsum(dM' M' + dVar E2') for mhada_attn_train_bwd. */
int mhada_attn_train_bwd_prep(const float* dout, const float* x, const float* mo, float* dx, float* dmo,
                              float* dd, long long rows, mhada_stream_t stream);

int mhada_pos_embed_bwd(const float* g, float* gpos, int C, int bh, int bw, int oh, int ow,
                        mhada_stream_t stream);
/* Gradient of the loss terms on one VGG feature map x, NHWC rows [B][P][C] (P = H*W), in one pass
 * (replaces the ATen backward of lossfn.py:7-23 mean/std distances and lossfn.py:26-34,41-47 MSEs):
 *   g = alpha[b][c] + beta[b][c] * (x - mu[b][c]) + ks * kp[0] * (x - t)
 * alpha / beta / mu [B][C] (all null: no statistics term), t [B][P][C] (null: no MSE term), kp a
 * device scalar (null: 1); C % 4 == 0, 16-byte aligned pointers.  relu = 1 (ABI 10): x is a ReLU
 * output and g is multiplied by its adjoint (x > 0) (the producing conv then skips mhada_relu_bwd). */
/* Forward statistics of one feature map x (NHWC fp32 [B][P][C], C % 4 == 0) for the losses of
 * lossfn.py:7-47: mu / sd [B][C] = the per-channel mean and UNBIASED std over the P pixels (x.mean /
 * x.std(dim=(2,3))), and with a target t (same layout) mse[0] = mean((x - t)^2) (F.mse_loss) — one
 * read of x (and t), fp64 partial sums reduced in a fixed order.  mu / sd may be NULL (then t and
 * mse are required); work: mhada_feat_stats_work(B, P, C) doubles (ABI 12). */
long long mhada_feat_stats_work(int B, long long P, int C);
int mhada_feat_stats(const float* x, const float* t, float* mu, float* sd, float* mse, double* work,
                     long long work_doubles, int B, long long P, int C, mhada_stream_t stream);
int mhada_feat_loss_bwd(const float* x, const float* t, const float* mu, const float* alpha, const float* beta,
                        const float* kp, float ks, float* g, int B, long long P, int C, int relu, mhada_stream_t stream);
/* ReLU backward on the saved output: dx = dy * (y > 0); n % 4 == 0 (dx may alias dy). */
int mhada_relu_bwd(const float* dy, const float* y, float* dx, long long n, mhada_stream_t stream);
/* Adjoint of ReflectionPad2d(1) (conv.py:27,31): dxp [B][H+2][W+2][C] (the full-correlation
 * input gradient on the padded grid) -> dx [B][H][W][C].  relu_mask (null: none; layout of dx):
 * dx = 0 where relu_mask <= 0 — the ReLU adjoint of the layer that produced the conv's input,
 * when this conv is that output's only consumer (replaces a mhada_relu_bwd pass; ABI 10). */
int mhada_reflect_fold(const float* dxp, float* dx, int B, int H, int W, int C, const float* relu_mask,
                       mhada_stream_t stream);
/* MaxPool2d(2, 2) on NHWC (vgg19.py slices, torchvision cfg E) and its backward (the gradient
 * goes to the first maximum of each window in row-major order, as ATen keeps it).  relu_mask = 1:
 * x is a ReLU output consumed only by this pool, and the ReLU adjoint (x > 0) is applied too. */
int mhada_maxpool2(const float* x, float* y, int B, int H, int W, int C, mhada_stream_t stream);
int mhada_maxpool2_bwd(const float* x, const float* dy, float* dx, int B, int H, int W, int C, int relu_mask,
                       mhada_stream_t stream);
/* Adjoint of the bilinear x2 upsample (conv.py:71): dy [B][2H][2W][C] -> dx [B][H][W][C]. */
/* relu_x (nullable): the upsample input when it is a ReLU output consumed only by the upsample;
 * dx is then also multiplied by (x > 0). */
int mhada_upsample2x_bwd(const float* dy, const float* relu_x, float* dx, int B, int H, int W, int C,
                         mhada_stream_t stream);
/* imageNet1k_normalize (vgg19.py:6-12): img [B][3][H][W] fp32 0..255 -> NHWC [B][H][W][Cp]
 * ((x/255 - mean)/std, channels 3..Cp-1 zero), and the adjoint of that map. */
int mhada_vgg_input(const float* img, float* out, int B, int H, int W, int Cp, mhada_stream_t stream);
int mhada_vgg_input_bwd(const float* dout, float* dimg, int B, int H, int W, int Cp, mhada_stream_t stream);

/* AdaAttnForLoss (adaDecoder.py:52-81, the local-feature-loss target of lossfn.py:26-34), fp32,
 * flash-style (A never stored): out = sqrt(max(A V^2 - (A V)^2, 1e-6)) * IN(c_x) + A V with
 * A = softmax(Q K^T) or the cosine form.  q [B][Nq][Dqk] = IN(c_1x), k [B][Ns][Dqk] = IN(s_1x)
 * (mhada_rows_normalize; for cosine with unit = 1, i.e. rows divided by their L2 norm), v
 * [B][Ns][Dv] = s_x, x [B][Nq][Dv] = c_x with its IN statistics x_mu / x_rs [B][Dv].
 * Dqk % 4 == 0; Dv in {64, 128, 256, 512}. */
int mhada_loss_attn(const float* q, const float* k, const float* v, const float* x, const float* x_mu,
                    const float* x_rs, float* out, int B, int Nq, int Ns, int Dqk, int Dv, int activation,
                    mhada_stream_t stream);
/* InstanceNorm of token rows: out = (x - mu[b]) * rs[b] on x [B][N][C] (C % 4 == 0); unit != 0
 * also divides each normalised row by its L2 norm (CosineSimilarity, adaDecoder.py:30-32). */
int mhada_rows_normalize(const float* x, const float* mu, const float* rs, float* out, int unit,
                         int B, int N, int C, mhada_stream_t stream);

/* Frame ingest (utilities.py:43-52 cv2_to_tensor, used per frame at infer_video.py:80):
 * BGR->RGB (bgr != 0; bgr == 0 keeps the channel order), INTER_AREA resize to Ho x Wo (area
 * average rounded to u8; Ho <= H, Wo <= W — upscaling is rejected), then toTensor255
 * (utilities.py:11-16: /255 then *255 in fp32).  frames: [B][H][W][3] u8, rows of row_bytes;
 * out: [B][3][Ho][Wo] fp32. */
int mhada_frame_ingest(const void* frames, int B, int H, int W, long long row_bytes, int bgr, float* out,
                       int Ho, int Wo, mhada_stream_t stream);

/* fp32 3x3 convolution as Winograd F(2x2,3x3) on the fp32 MFMA (2.25x fewer products than the
 * direct correlation).  Replaces the fp32 Conv2d(k=3) of the decoder (ReflectionPad2d(1) + conv,
 * conv.py:23-33,36-45,61-72: pad_mode MHADA_PAD_REFLECT) and of VGG19 (vgg19.py:15-70, zero
 * padding 1), and the training input-gradient convs (zero pad 1, or pad 2 = the full correlation,
 * output (H+2) x (W+2); train_image.py:139).  x NHWC [B][H][W][Cin] fp32, u = the transformed
 * filters from mhada_wino_weights (w packed [Cout][3][3][Cin] fp32 -> u [Cin/8][16][Cout][8]),
 * bias [Cout] or NULL, y NHWC [B][Ho][Wo][ldc] (ldc >= Cout), optional ReLU.
 * Cin % 8 == 0, Cout % 64 == 0. */
int mhada_wino_weights(const float* w, float* u, int Cout, int Cin, mhada_stream_t stream);
/* Weight (and bias) gradient of the same 3x3 conv (pad 1: MHADA_PAD_REFLECT as the decoder's
 * ReflectionPad2d(1), or MHADA_PAD_ZERO), Winograd F(2x2,3x3) on the fp32 MFMA (replaces the
 * im2col mhada_gemm_tn for the decoder convs of train_image.py:139):
 *   dw [Cout][3][3][Cin] = sum over pixels of g[b][y][x][co] * x_pad[b][y+ky-1][x+kx-1][ci],
 *   db [Cout] = sum of g (null: not computed).
 * x NHWC [B][H][W][Cin], g NHWC [B][H][W][ldg] (ldg >= Cout, % 4).  Cin % 64 == 0, Cout % 64 == 0,
 * H even, W % 16 == 0.  Tile-split partial sums in work (>= splits * (16*Cout*Cin + Cout) floats,
 * splits = mhada_conv3x3_wgrad_wino_splits(...)), summed in a fixed order: deterministic. */
int mhada_conv3x3_wgrad_wino_splits(int B, int H, int W, int Cin, int Cout);
int mhada_conv3x3_wgrad_wino(const float* x, const float* g, float* dw, float* db, float* work, long long work_floats,
                             int B, int H, int W, int Cin, int Cout, long long ldg, int pad_mode,
                             mhada_stream_t stream);
/* relu_mask (null: none; layout of y): y = 0 where relu_mask <= 0 — a ReLU adjoint folded into a
 * dgrad's output stage (ABI 10). */
int mhada_conv3x3_wino(const float* x, const float* u, const float* bias, float* y, int B, int H, int W,
                       int Cin, int Cout, long long ldc, int pad_mode, int pad, int relu,
                       const float* relu_mask, mhada_stream_t stream);

/* The 3-channel ends of the training conv stacks (rgb_ops.hip), fp32:
 * VGG19's first layer (vgg19.py:10-11,25-26: normalise -> Conv2d(3, 64, 3, padding=1) -> ReLU),
 * input gradient w.r.t. the RGB image in one pass (replaces mhada_relu_bwd + a 64 -> 32-channel
 * zero-padded transposed conv on mhada_gemm + mhada_vgg_input_bwd):
 *   dimg [B][3][H][W] = adjoint of normalise( sum_{tap,co} g[p + d_tap][co] wd[tap][co][c] ),
 *   g = dy * (y > 0); dy, y NHWC [B][H][W][64]; wd [9][64][3] = W[co][c][8 - tap] (flipped). */
int mhada_vgg_stem_dgrad(const float* dy, const float* y, const float* wd, float* dimg, int B, int H, int W,
                         mhada_stream_t stream);
/* The decoder's last layer (conv.py:39-45,94: ReflectionPad2d(1) -> Conv2d(64, 3, 3) -> ReLU; its
 * forward is mhada_conv3x3_out3): input gradient dx NHWC [B][H][W][64] with the reflection-pad
 * adjoint folded in, from dy and the layer output y (NCHW [B][3][H][W]) and wd [9][3][64] =
 * W[co][ci][tap] (replaces relu_bwd + channel padding + a pad-2 transposed conv + mhada_reflect_fold).
 * relu_x (nullable): the layer input x when it is a ReLU output consumed only by this layer — dx is
 * then also multiplied by (x > 0), the producing layer's ReLU adjoint. */
int mhada_out3_dgrad(const float* dy, const float* y, const float* wd, const float* relu_x, float* dx, int B, int H,
                     int W, mhada_stream_t stream);
/* Its weight gradient dw [3][64][3][3] and bias gradient db [3] (null: skipped) from the layer
 * input x NHWC [B][H][W][64], dy and y as above; per-workgroup partials in work (>= mhada_out3_wgrad_work
 * floats) summed in a fixed order (replaces the M <= 4 mhada_gemm_tn + colsum). */
long long mhada_out3_wgrad_work(int B, int H, int W);
int mhada_out3_wgrad(const float* x, const float* dy, const float* y, float* dw, float* db, float* work,
                     long long work_floats, int B, int H, int W, mhada_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MHADA_HIP_H */
