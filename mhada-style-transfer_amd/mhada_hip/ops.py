"""Tensor-level wrappers over the C-ABI (one function per entry point of include/mhada_hip.h).

Every wrapper takes ROCm device tensors, validates shapes/dtypes on the host, launches on the
current stream of the operands' device (with that device made current for the call, so modules
moved with ``.to('cuda:1')`` work without ``set_device``) and allocates outputs through the
torch caching allocator (the library itself never allocates).  No wrapper has a CPU or aten
fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import A_CONV3X3, A_CONV3X3_UP2, A_CONV3X3_ZERO, A_PATCH8, A_ROWS, A_SPLIT3, BF16, BF16X3, F32, GemmArgs, GemmTnArgs

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dt_code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise ValueError(f"unsupported dtype {dtype}; the HIP path computes in float32 or bfloat16")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need_gpu(*ts: Optional[torch.Tensor]) -> None:
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("mhada_hip ops need ROCm device tensors (the MI355X path has no CPU fallback)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"mhada_hip ops need all operands on one device, got {dev} and {t.device}")


def _call(name: str, dev_tensor: torch.Tensor, *args) -> None:
    """Launch entry point ``name`` with ``dev_tensor``'s device current, on that device's current
    stream (appended as the last argument); raise on a non-zero status."""
    idx = dev_tensor.device.index
    guard = contextlib.nullcontext() if idx is None or idx == torch.cuda.current_device() \
        else torch.cuda.device(idx)
    with guard:
        rc = getattr(_lib.load(), name)(*args, torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, name)


def gemm(*, a: torch.Tensor, w: torch.Tensor, c: torch.Tensor, M: int, N: int, K: int,
         compute: torch.dtype, a_mode: int = A_ROWS, lda: int = 0, sa=(0, 0), nb=(1, 1),
         a_mu: Optional[torch.Tensor] = None, smu=(0, 0), img=(0, 0, 0),
         ldw: int = 0, sw=(0, 0), bias: Optional[torch.Tensor] = None, sb=(0, 0),
         r: Optional[torch.Tensor] = None, ldr: int = 0, sr=(0, 0),
         ldc: int = 0, sc=(0, 0), relu: bool = False, pad: int = 0,
         c2: Optional[torch.Tensor] = None, ldc2: int = 0, sc2=(0, 0),
         vt: Optional[torch.Tensor] = None, ldt: int = 0, svt=(0, 0), c2_planes: bool = False) -> torch.Tensor:
    """``mhada_gemm``: C[z] = act(A[z] W[z]^T + bias[z]) + R[z]; strides in elements.  Optional
    c2 (a bf16 copy of an fp32 C; ``c2_planes``: C's three bf16 planes [3][M][ldc2], the next
    SPLIT3 GEMM's operand, with C None = not written) and vt (the transposed V' image of the
    K|V' projection)."""
    _need_gpu(a, w, c, a_mu, bias, r, c2, vt)
    if c is None and not c2_planes:
        raise ValueError("gemm: C may be None only with c2_planes")
    if c2 is not None and (c2.dtype != torch.bfloat16 or (c is not None and c.dtype != torch.float32)):
        raise ValueError("c2 is the bf16 copy of an fp32 C")
    if c2_planes and (c2 is None or c2.shape[0] != 3 or not c2.is_contiguous()):
        raise ValueError("c2_planes needs c2 = contiguous bf16 [3][M][ldc2]")
    if vt is not None and vt.dtype != c.dtype:
        raise ValueError("vt has the dtype of C")
    if w.dtype != compute:
        raise ValueError("W must already be in the compute dtype")
    for t in (a_mu, bias):
        if t is not None and t.dtype != torch.float32:
            raise ValueError("a_mu / bias must be float32")
    if r is not None and r.dtype != (c.dtype if c is not None else torch.float32):
        raise ValueError("residual dtype must equal the output dtype (fp32 for a c2_planes-only output)")
    args = GemmArgs()
    args.M, args.N, args.K = M, N, K
    args.nb1, args.nb2 = nb
    args.compute = dt_code(compute)
    args.a_mode = a_mode
    args.a, args.a_dtype, args.lda = a.data_ptr(), dt_code(a.dtype), lda
    args.sa1, args.sa2 = sa
    args.a_mu = _ptr(a_mu)
    args.smu1, args.smu2 = smu
    args.img_c, args.img_h, args.img_w = img
    args.w, args.ldw = w.data_ptr(), ldw
    args.sw1, args.sw2 = sw
    args.bias = _ptr(bias)
    args.sb1, args.sb2 = sb
    args.r = _ptr(r)
    args.r_dtype = dt_code(r.dtype) if r is not None else 0
    args.ldr = ldr
    args.sr1, args.sr2 = sr
    args.c, args.c_dtype, args.ldc = _ptr(c), dt_code(c.dtype) if c is not None else F32, ldc
    args.sc1, args.sc2 = sc
    args.relu = int(relu)
    args.pad = int(pad)
    args.c2, args.ldc2 = _ptr(c2), ldc2
    args.sc21, args.sc22 = sc2
    args.vt, args.ldt = _ptr(vt), ldt
    args.svt1, args.svt2 = svt
    args.c2_planes = int(c2_planes)
    _call("mhada_gemm", a, ctypes.byref(args))
    return c if c is not None else c2


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], out_dtype: torch.dtype,
           residual: Optional[torch.Tensor] = None, relu: bool = False,
           relu_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [M][K] @ w[N][K]^T + bias (+relu) (+residual) -> [M][N] of out_dtype.  ``relu_mask``
    (fp32 [M][N], instead of a residual): the result is zeroed where relu_mask <= 0 (a ReLU
    adjoint folded into a gradient GEMM's epilogue, mhada_gemm relu = 2)."""
    M, K = x.shape
    N = w.shape[0]
    c = torch.empty(M, N, device=x.device, dtype=out_dtype)
    if relu_mask is not None:
        if residual is not None or relu or out_dtype != torch.float32 or relu_mask.dtype != torch.float32 \
                or relu_mask.shape != (M, N) or not relu_mask.is_contiguous():
            raise ValueError("linear: relu_mask needs fp32 output, a contiguous fp32 [M][N] mask, no residual / relu")
        return gemm(a=x, w=w, c=c, M=M, N=N, K=K, compute=w.dtype, lda=x.stride(0), ldw=w.stride(0),
                    bias=bias, r=relu_mask, ldr=N, ldc=N, relu=2)
    return gemm(a=x, w=w, c=c, M=M, N=N, K=K, compute=w.dtype, lda=x.stride(0), ldw=w.stride(0),
                bias=bias, r=residual, ldr=N if residual is not None else 0, ldc=N, relu=relu)


def patch_embed(img: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, pos: Optional[torch.Tensor],
                patch: int = 8) -> torch.Tensor:
    """img (B,3,H,W) fp32 -> tokens [B][N][C] fp32 (+ pos [N][C] broadcast over B)."""
    if patch != 8:
        raise ValueError("the HIP patch embedding implements patch_size=8 (the reference default)")
    B, Ci, H, W = img.shape
    h, wd = H // 8, W // 8
    N, C = h * wd, w.shape[0]
    out = torch.empty(B, N, C, device=img.device, dtype=torch.float32)
    return gemm(a=img, w=w, c=out, M=N, N=C, K=Ci * 64, compute=w.dtype, a_mode=A_PATCH8,
                sa=(Ci * H * W, 0), nb=(B, 1), img=(Ci, H, W), ldw=w.stride(0), bias=bias,
                r=pos, ldr=C, sr=(0, 0), ldc=C, sc=(N * C, 0))


# fp32 3x3 convs run as Winograd F(2x2,3x3) (csrc/wino.hip) where the shape allows it; False
# forces the implicit-GEMM direct product (A/B measurements, tests).
WINO = True


def wino_eligible(x: torch.Tensor, w: torch.Tensor, upsample: bool) -> bool:
    """The Winograd kernel's constraints (csrc/wino.hip): fp32, Cin % 8, Cout % 64, >= 2x2 pixels
    and 32-bit element offsets (B*H*W*Cin and the output's B*H*W*Cout < 2^31); anything else runs
    on the implicit-GEMM conv."""
    return (WINO and w.dtype == torch.float32 and x.dtype == torch.float32 and not upsample
            and x.shape[-1] % 8 == 0 and w.shape[0] % 64 == 0 and x.shape[1] >= 2 and x.shape[2] >= 2
            and x.numel() < 2 ** 31 and x.numel() // x.shape[-1] * w.shape[0] < 2 ** 31)


# Winograd weight gradients for the eligible training convs (tests flip this to compare with the TN GEMM)
WINO_WGRAD = True


def wgrad_wino_eligible(x: torch.Tensor, g: torch.Tensor, cout: int) -> bool:
    """mhada_conv3x3_wgrad_wino's constraints: fp32 NHWC x [B][H][W][Cin] and g [B][H][W][ldg],
    Cin % 64 == 0, Cout % 64 == 0, H even, W % 16 == 0, 32-bit element offsets."""
    if not (WINO_WGRAD and x.is_cuda and x.dtype == torch.float32 and g.dtype == torch.float32):
        return False
    B, H, W, ci = x.shape
    return (ci % 64 == 0 and cout % 64 == 0 and H % 2 == 0 and W % 16 == 0 and g.shape[:3] == x.shape[:3]
            and g.shape[3] >= cout and g.shape[3] % 4 == 0 and x.is_contiguous() and g.is_contiguous()
            and B * H * W * max(ci, g.shape[3]) < 2 ** 31)


def conv3x3_wgrad_wino(x: torch.Tensor, g: torch.Tensor, cout: int, pad_mode: str = "reflect",
                       bias: bool = True):
    """``mhada_conv3x3_wgrad_wino``: the weight gradient [Cout][9*Cin] (k = tap*Cin + ci, the
    gemm_tn layout) and the bias gradient [Cout] (or None) of a pad-1 3x3 conv, from its input x
    and output gradient g (NHWC fp32)."""
    _need_gpu(x, g)
    B, H, W, ci = x.shape
    lib = _lib.load()
    S = lib.mhada_conv3x3_wgrad_wino_splits(B, H, W, ci, cout)
    if S <= 0:
        raise ValueError("conv3x3_wgrad_wino: ineligible shape")
    work = torch.empty(S * (16 * cout * ci + (cout if bias else 0)), device=x.device, dtype=torch.float32)
    dw = torch.empty(cout, 9 * ci, device=x.device, dtype=torch.float32)
    db = torch.empty(cout, device=x.device, dtype=torch.float32) if bias else None
    _call("mhada_conv3x3_wgrad_wino", x, x.data_ptr(), g.data_ptr(), dw.data_ptr(),
          db.data_ptr() if bias else None, work.data_ptr(), work.numel(), B, H, W, ci, cout, g.shape[3],
          _lib.PAD_REFLECT if pad_mode == "reflect" else _lib.PAD_ZERO)
    return dw, db


def wino_weights(w: torch.Tensor) -> torch.Tensor:
    """``mhada_wino_weights``: w packed [Cout][9*Cin] fp32 -> U [Cin/8][16][Cout][8]."""
    _need_gpu(w)
    Co, K = w.shape
    Ci = K // 9
    if w.dtype != torch.float32 or K != 9 * Ci or not w.is_contiguous():
        raise ValueError("wino_weights needs a contiguous fp32 [Cout][9*Cin] weight")
    u = torch.empty(Ci // 8, 16, Co, 8, device=w.device, dtype=torch.float32)
    _call("mhada_wino_weights", w, w.data_ptr(), u.data_ptr(), Co, Ci)
    return u


def conv3x3_wino(x: torch.Tensor, u: torch.Tensor, bias: Optional[torch.Tensor], relu: bool = True,
                 pad_mode: str = "reflect", pad: int = 1, out: Optional[torch.Tensor] = None,
                 relu_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``mhada_conv3x3_wino``: fp32 NHWC conv3x3 from the transformed filters ``u``; ``relu_mask``
    (the output's layout): zero the outputs where relu_mask <= 0 (a folded ReLU adjoint)."""
    _need_gpu(x, u, bias, out, relu_mask)
    B, H, W, Ci = x.shape
    Co = u.shape[2]
    if x.dtype != torch.float32 or not x.is_contiguous() or u.shape[0] * 8 != Ci:
        raise ValueError("conv3x3_wino: contiguous fp32 NHWC input matching the filters")
    if pad_mode == "reflect":
        mode, Ho, Wo, pad = _lib.PAD_REFLECT, H, W, 1
    elif pad_mode == "zero":
        mode, Ho, Wo = _lib.PAD_ZERO, H + 2 * (pad - 1), W + 2 * (pad - 1)
    else:
        raise ValueError(f"pad_mode {pad_mode!r}")
    y = torch.empty(B, Ho, Wo, Co, device=x.device, dtype=torch.float32) if out is None else out
    if y.shape[:3] != (B, Ho, Wo) or y.dtype != torch.float32 or y.shape[-1] < Co or not y.is_contiguous():
        raise ValueError("conv3x3_wino: bad output buffer")
    if relu_mask is not None and (relu_mask.shape != y.shape or relu_mask.dtype != torch.float32
                                  or not relu_mask.is_contiguous()):
        raise ValueError("conv3x3_wino: relu_mask must be a contiguous fp32 tensor shaped like the output")
    _call("mhada_conv3x3_wino", x, x.data_ptr(), u.data_ptr(), _ptr(bias), y.data_ptr(), B, H, W, Ci, Co,
          y.shape[-1], mode, pad, int(relu), _ptr(relu_mask))
    return y


def conv3x3(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], out_dtype: torch.dtype,
            upsample: bool, relu: bool = True, pad_mode: str = "reflect", pad: int = 1,
            out: Optional[torch.Tensor] = None, wino_u: Optional[torch.Tensor] = None,
            relu_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NHWC x [B][H][W][Cin] -> NHWC [B][H'][W'][Cout]; ReflectionPad2d(1)+conv3x3(+ReLU),
    optionally on bilinear-x2(x), or (pad_mode "zero") a zero-padded conv with padding `pad`
    (1: same size, 2: the full correlation, H' = H + 2).  w packed [Cout][9*Cin] in the compute
    dtype.  ``out`` may be a preallocated [B][H'][W'][ldc >= Cout] buffer (channel padding).
    fp32 runs as Winograd F(2x2,3x3) when the shape allows (``wino_u``: cached transformed
    filters of ``w``).  ``relu_mask`` (fp32, shaped like the output): zero the outputs where
    relu_mask <= 0 — a ReLU adjoint folded into a dgrad (in the Winograd output stage; a separate
    mhada_relu_bwd pass on the implicit-GEMM path)."""
    B, H, W, Ci = x.shape
    Co = w.shape[0]
    if out_dtype == torch.float32 and wino_eligible(x, w, upsample) and x.is_contiguous():
        u = wino_u if wino_u is not None else wino_weights(w)
        return conv3x3_wino(x, u, bias, relu, pad_mode, pad, out, relu_mask)
    if relu_mask is not None:
        return relu_bwd(conv3x3(x, w, bias, out_dtype, upsample, relu, pad_mode, pad, out), relu_mask)
    if pad_mode == "zero":
        if upsample:
            raise ValueError("zero-padded conv3x3 has no fused upsample")
        Ho, Wo = H + 2 * (pad - 1), W + 2 * (pad - 1)
        mode = A_CONV3X3_ZERO
    elif pad_mode == "reflect":
        Ho, Wo = (2 * H, 2 * W) if upsample else (H, W)
        mode = A_CONV3X3_UP2 if upsample else A_CONV3X3
        pad = 0
    else:
        raise ValueError(f"pad_mode {pad_mode!r}")
    y = torch.empty(B, Ho, Wo, Co, device=x.device, dtype=out_dtype) if out is None else out
    return gemm(a=x, w=w, c=y, M=B * Ho * Wo, N=Co, K=9 * Ci, compute=w.dtype, a_mode=mode, img=(Ci, H, W),
                ldw=w.stride(0), bias=bias, ldc=y.shape[-1], relu=relu, pad=pad)


def upsample2x(x: torch.Tensor) -> torch.Tensor:
    """NHWC bilinear x2 (align_corners=False)."""
    _need_gpu(x)
    B, H, W, C = x.shape
    y = torch.empty(B, 2 * H, 2 * W, C, device=x.device, dtype=x.dtype)
    _call("mhada_upsample2x", x, x.data_ptr(), y.data_ptr(), dt_code(x.dtype), B, H, W, C)
    return y


def conv3x3_out3(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, clamp255: bool = False) -> torch.Tensor:
    B, H, W, Ci = x.shape
    _need_gpu(x, w, bias)
    y = torch.empty(B, 3, H, W, device=x.device, dtype=torch.float32)
    _call("mhada_conv3x3_out3", x, x.data_ptr(), dt_code(x.dtype), w.data_ptr(), bias.data_ptr(),
                                        y.data_ptr(), B, H, W, Ci, int(clamp255))
    return y


def layernorm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, out_dtype: torch.dtype, eps: float) -> torch.Tensor:
    _need_gpu(x, g, b)
    rows, cols = x.shape
    y = torch.empty(rows, cols, device=x.device, dtype=out_dtype)
    _call("mhada_layernorm", x, x.data_ptr(), y.data_ptr(), dt_code(out_dtype), g.data_ptr(), b.data_ptr(),
                                     rows, cols, eps)
    return y


# fp32 GEMMs whose A comes from a LayerNorm (the ViT's QKV and MLP1) run as SPLIT3 products on the
# bf16 MFMA (mhada_gemm a_mode MHADA_A_SPLIT3): fp32-accurate — against fp64 their error is below
# the fp32 MFMA path's (tools/split_bf16_probe.py) — and 1.4-1.5x faster.  False: the fp32 MFMA.
F32_SPLIT = True


def layernorm_split3(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    """``mhada_layernorm`` with y_dtype MHADA_BF16X3: the fp32 LayerNorm of x as three bf16 planes
    [3][rows][cols] (y = p0 + p1 + p2 to 2^-25 relative), the A operand of ``linear_split3``."""
    _need_gpu(x, g, b)
    rows, cols = x.shape
    y = torch.empty(3, rows, cols, device=x.device, dtype=torch.bfloat16)
    _call("mhada_layernorm", x, x.data_ptr(), y.data_ptr(), BF16X3, g.data_ptr(), b.data_ptr(), rows, cols, eps)
    return y


def split3_weight(w: torch.Tensor) -> torch.Tensor:
    """An fp32 weight [N][K0] (K0 % 64 == 0) as the SPLIT3 GEMM's W operand: its bf16 planes q0 + q1 +
    q2 (8 + 8 + 8 mantissa bits) interleaved per 64-column chunk kk as q1 | q0 | q2 | q0 | q1 | q0
    -> [N][6 K0] bf16, the GEMM's K-tile 6 kk + t (one-time weight preparation, cached with the
    module's other prepared weights)."""
    w = w.float()
    N, K0 = w.shape
    if K0 % 64:
        raise ValueError("split3_weight: K0 must be a multiple of 64")
    q0 = w.bfloat16()
    r = w - q0.float()
    q1 = r.bfloat16()
    q2 = (r - q1.float()).bfloat16()
    terms = torch.stack([t.view(N, K0 // 64, 64) for t in (q1, q0, q2, q0, q1, q0)], dim=2)
    return terms.reshape(N, 6 * K0).contiguous()


def split3_weight_dev(w: torch.Tensor, transposed: bool = False) -> torch.Tensor:
    """``mhada_split3_weight``: split3_weight(w) (or of w.t()) in one device launch, bit-identical to
    split3_weight — the training step re-splits its weights after every optimizer step."""
    _need_gpu(w)
    if w.dtype != torch.float32 or not w.is_contiguous() or w.dim() != 2:
        raise ValueError("split3_weight_dev needs a contiguous float32 matrix")
    N, K0 = (w.shape[1], w.shape[0]) if transposed else w.shape
    if K0 % 64:
        raise ValueError("split3_weight_dev: K0 must be a multiple of 64")
    out = torch.empty(N, 6 * K0, device=w.device, dtype=torch.bfloat16)
    _call("mhada_split3_weight", w, w.data_ptr(), out.data_ptr(), N, K0, int(transposed))
    return out


def split3_rows(x: torch.Tensor) -> torch.Tensor:
    """``mhada_split3_rows``: a contiguous fp32 matrix [M][K0] as its three bf16 planes [3][M][K0] (the
    ``linear_split3`` A operand of an activation or gradient that no LayerNorm produced)."""
    _need_gpu(x)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 2:
        raise ValueError("split3_rows needs a contiguous float32 [M][K0] matrix")
    y = torch.empty(3, *x.shape, device=x.device, dtype=torch.bfloat16)
    _call("mhada_split3_rows", x, x.data_ptr(), y.data_ptr(), x.numel())
    return y


def linear_split3(planes: torch.Tensor, w6: torch.Tensor, bias: Optional[torch.Tensor], out_dtype: torch.dtype,
                  residual: Optional[torch.Tensor] = None, relu: bool = False,
                  out_planes: bool = False, relu_mask: Optional[torch.Tensor] = None, both: bool = False):
    """fp32-accurate x @ w^T (+bias, relu, residual) from x's bf16 planes [3][M][K0] and
    ``split3_weight(w)`` [N][6 K0]: the six significant cross products summed in fp32 accumulators
    on the bf16 MFMA (mhada_gemm MHADA_A_SPLIT3).  ``out_planes``: return the fp32 result as its
    three bf16 planes [3][M][N] (the next SPLIT3 GEMM's operand) instead of an fp32 [M][N].
    ``relu_mask`` (fp32 [M][N], as ``linear``'s): the result zeroed where relu_mask <= 0.  ``both``: return
    (the fp32 result, its three bf16 planes) from the one epilogue — for a result that is kept in fp32
    (saved for a backward) and also feeds a SPLIT3 GEMM."""
    if planes.dim() != 3 or planes.shape[0] != 3 or planes.dtype != torch.bfloat16 or not planes.is_contiguous():
        raise ValueError("linear_split3: planes must be contiguous bf16 [3][M][K0]")
    _, M, K0 = planes.shape
    N = w6.shape[0]
    if w6.dtype != torch.bfloat16 or w6.shape[1] != 6 * K0:
        raise ValueError("linear_split3: w6 must be split3_weight(w), bf16 [N][6*K0]")
    if out_planes:
        if out_dtype != torch.float32:
            raise ValueError("linear_split3: out_planes splits an fp32 result")
        c2 = torch.empty(3, M, N, device=planes.device, dtype=torch.bfloat16)
        return gemm(a=planes, w=w6, c=None, M=M, N=N, K=6 * K0, compute=torch.bfloat16, a_mode=A_SPLIT3, lda=K0,
                    ldw=6 * K0, bias=bias, r=residual, ldr=N if residual is not None else 0, ldc=N, relu=relu,
                    c2=c2, ldc2=N, c2_planes=True)
    c = torch.empty(M, N, device=planes.device, dtype=out_dtype)
    c2 = None
    if both:
        if out_dtype != torch.float32:
            raise ValueError("linear_split3: both splits an fp32 result")
        c2 = torch.empty(3, M, N, device=planes.device, dtype=torch.bfloat16)
    if relu_mask is not None:
        if residual is not None or relu or out_dtype != torch.float32 or relu_mask.dtype != torch.float32 \
                or relu_mask.shape != (M, N) or not relu_mask.is_contiguous():
            raise ValueError("linear_split3: relu_mask needs fp32 output, a contiguous fp32 [M][N] mask, no residual / relu")
        gemm(a=planes, w=w6, c=c, M=M, N=N, K=6 * K0, compute=torch.bfloat16, a_mode=A_SPLIT3, lda=K0,
             ldw=6 * K0, bias=bias, r=relu_mask, ldr=N, ldc=N, relu=2, c2=c2, ldc2=N if both else 0, c2_planes=both)
    else:
        gemm(a=planes, w=w6, c=c, M=M, N=N, K=6 * K0, compute=torch.bfloat16, a_mode=A_SPLIT3, lda=K0,
             ldw=6 * K0, bias=bias, r=residual, ldr=N if residual is not None else 0, ldc=N, relu=relu,
             c2=c2, ldc2=N if both else 0, c2_planes=both)
    return (c, c2) if both else c


def vit_batch_attn(qkv: torch.Tensor, L: int, ntok: int, heads: int, groups: int = 1) -> torch.Tensor:
    """``mhada_vit_batch_attn`` on qkv [L][ntok][3C]; ``groups`` > 1: the L images are that many
    independent calls of L / groups images each (consecutive slices), attended separately."""
    _need_gpu(qkv)
    C = qkv.shape[-1] // 3
    if L % groups:
        raise ValueError("vit_batch_attn: L must be a multiple of groups")
    out = torch.empty(L, ntok, C, device=qkv.device, dtype=qkv.dtype)
    Lg, es = L // groups, qkv.element_size()
    for g in range(groups):
        _call("mhada_vit_batch_attn", qkv, qkv.data_ptr() + g * Lg * ntok * 3 * C * es,
              out.data_ptr() + g * Lg * ntok * C * es, dt_code(qkv.dtype), Lg, ntok, heads, C // heads)
    return out


def pos_embed(pos: torch.Tensor, oh: int, ow: int) -> torch.Tensor:
    _need_gpu(pos)
    _, C, bh, bw = pos.shape
    out = torch.empty(oh * ow, C, device=pos.device, dtype=torch.float32)
    _call("mhada_pos_embed", pos, pos.data_ptr(), out.data_ptr(), C, bh, bw, oh, ow)
    return out


def pos_embed_bwd(g: torch.Tensor, bh: int, bw: int) -> torch.Tensor:
    """``mhada_pos_embed_bwd``: token-major gradient g [oh][ow][C] -> (1, C, bh, bw)."""
    _need_gpu(g)
    oh, ow, C = g.shape
    if g.dtype != torch.float32 or not g.is_contiguous():
        raise ValueError("pos_embed_bwd needs a contiguous float32 [oh][ow][C] gradient")
    out = torch.empty(1, C, bh, bw, device=g.device, dtype=torch.float32)
    _call("mhada_pos_embed_bwd", g, g.data_ptr(), out.data_ptr(), C, bh, bw, oh, ow)
    return out


def instnorm_bwd(dy: torch.Tensor, y: torch.Tensor, rs: torch.Tensor) -> torch.Tensor:
    """``mhada_instnorm_bwd``: token rows dy, y [B][N][C], rstd [B][C] -> dx."""
    _need_gpu(dy, y, rs)
    for t in (dy, y, rs):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("instnorm_bwd needs contiguous float32 operands")
    B, N, C = y.shape
    if dy.shape != y.shape or rs.shape != (B, C):
        raise ValueError("instnorm_bwd: shape mismatch")
    splits = max(1, min(N // 32, 2048 // max(1, B * ((C + 63) // 64))))
    work = torch.empty(splits * B * C * 2 + B * C, device=y.device, dtype=torch.float64)
    dx = torch.empty_like(y)
    _call("mhada_instnorm_bwd", y, dy.data_ptr(), y.data_ptr(), rs.data_ptr(), dx.data_ptr(), work.data_ptr(), B, N, C,
          splits)
    return dx


def attn_train_bwd_prep(dout: torch.Tensor, x: torch.Tensor, mo: torch.Tensor):
    """``mhada_attn_train_bwd_prep``: (dx, dmo, dd) of the MHAda core's elementwise head."""
    _rows64(dout, x, mo)
    BH, Nc, _ = x.shape
    if dout.shape != x.shape or mo.shape != (BH, Nc, 128):
        raise ValueError("attn_train_bwd_prep: bad shapes")
    dx = torch.empty_like(x)
    dmo = torch.empty_like(mo)
    dd = torch.empty(BH, Nc, device=x.device, dtype=torch.float32)
    _call("mhada_attn_train_bwd_prep", x, dout.data_ptr(), x.data_ptr(), mo.data_ptr(), dx.data_ptr(), dmo.data_ptr(),
          dd.data_ptr(), BH * Nc)
    return dx, dmo, dd


def layernorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, planes: bool = False):
    """``mhada_layernorm_fwd``: fp32 rows [M][C] -> (y fp32, stats [M][2]); ``planes``: also y's three bf16
    planes [3][M][C] (``mhada_layernorm_fwd_split3``) -> (y, stats, planes)."""
    _need_gpu(x, gamma, beta)
    for t in (x, gamma, beta):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("layernorm_fwd needs contiguous float32 operands")
    M, C = x.shape
    y = torch.empty_like(x)
    st = torch.empty(M, 2, device=x.device, dtype=torch.float32)
    if planes:
        pl = torch.empty(3, M, C, device=x.device, dtype=torch.bfloat16)
        _call("mhada_layernorm_fwd_split3", x, x.data_ptr(), y.data_ptr(), pl.data_ptr(), st.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), M, C, float(eps))
        return y, st, pl
    _call("mhada_layernorm_fwd", x, x.data_ptr(), y.data_ptr(), st.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
          M, C, float(eps))
    return y, st


def layernorm_bwd(x: torch.Tensor, dy: torch.Tensor, st: torch.Tensor, gamma: torch.Tensor):
    """``mhada_layernorm_bwd``: -> (dx, dgamma, dbeta)."""
    _need_gpu(x, dy, st, gamma)
    for t in (x, dy, st, gamma):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("layernorm_bwd needs contiguous float32 operands")
    M, C = x.shape
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=x.device, dtype=torch.float32)
    db = torch.empty(C, device=x.device, dtype=torch.float32)
    nw = ((M + 127) // 128 * 2 + 2) * C
    work = torch.empty(nw, device=x.device, dtype=torch.float32)
    _call("mhada_layernorm_bwd", x, x.data_ptr(), dy.data_ptr(), st.data_ptr(), gamma.data_ptr(), dx.data_ptr(),
          dg.data_ptr(), db.data_ptr(), work.data_ptr(), nw, M, C)
    return dx, dg, db


def instnorm_stats(x: torch.Tensor, eps: float = 1e-5):
    """x [B][N][C] fp32 -> (mu, rstd) [B][C] fp32."""
    _need_gpu(x)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 3:
        raise ValueError(f"instnorm_stats needs contiguous float32 token rows [B][N][C], got {x.dtype} "
                         f"{tuple(x.shape)}")
    B, N, C = x.shape
    splits = max(1, min(N // 32, 2048 // max(1, B * ((C + 63) // 64))))
    mu = torch.empty(B, C, device=x.device, dtype=torch.float32)
    rstd = torch.empty(B, C, device=x.device, dtype=torch.float32)
    work = torch.empty(splits, B, C, 2, device=x.device, dtype=torch.float64)
    _call("mhada_instnorm_stats", x, x.data_ptr(), mu.data_ptr(), rstd.data_ptr(), work.data_ptr(), B, N, C,
                                          splits, eps)
    return mu, rstd


LOG2E = 1.4426950408889634


def fold_block(wf, wg, wh, bg, bh, rstd_c, mu_s, rstd_s, dtype: torch.dtype, kscale: float = LOG2E):
    """Per-call weight fold of one MHAda block (include/mhada_hip.h).  kscale = log2(e) puts K
    in the softmax attention's log2 units (mhada_attn's K contract); 1.0 for cosine."""
    B, C = rstd_c.shape
    H = wf.shape[0]
    dev = wf.device
    wq = torch.empty(B, H, 64, 64, device=dev, dtype=dtype)
    wkv = torch.empty(B, H, 128, 64, device=dev, dtype=dtype)
    bkv = torch.empty(H, 128, device=dev, dtype=torch.float32)
    v_mu = torch.empty(B, C, device=dev, dtype=torch.float32)
    _need_gpu(wf, wg, wh, bg, bh, rstd_c, mu_s, rstd_s)
    _call("mhada_fold_block", wf, wf.data_ptr(), wg.data_ptr(), wh.data_ptr(), bg.data_ptr(), bh.data_ptr(),
          rstd_c.data_ptr(), mu_s.data_ptr(), rstd_s.data_ptr(), wq.data_ptr(), wkv.data_ptr(), bkv.data_ptr(),
          v_mu.data_ptr(), kscale, dt_code(dtype), B, H)
    return wq, wkv, bkv, v_mu


def transpose_v(kv: torch.Tensor) -> torch.Tensor:
    _need_gpu(kv)
    B, H, Ns, _ = kv.shape
    ldt = (Ns + 63) // 64 * 64
    vt = torch.empty(B, H, 128, ldt, device=kv.device, dtype=kv.dtype)
    _call("mhada_transpose_v", kv, kv.data_ptr(), vt.data_ptr(), dt_code(kv.dtype), B, H, Ns)
    return vt


def cosine_prep(q: Optional[torch.Tensor], kv: Optional[torch.Tensor]) -> None:
    """L2-normalise Q rows and/or the K half of KV rows in place (either may be None)."""
    _need_gpu(q, kv)
    ref = q if q is not None else kv
    B, H = ref.shape[0], ref.shape[1]
    Nc = q.shape[2] if q is not None else 0
    Ns = kv.shape[2] if kv is not None else 0
    _call("mhada_cosine_prep", ref, _ptr(q), _ptr(kv), dt_code(ref.dtype), B, H, Nc, Ns)


def cosine_moments(kv: torch.Tensor, vt: torch.Tensor) -> torch.Tensor:
    """``mhada_cosine_moments``: the style-side moments [B][H][65][132] fp32 of the linear cosine
    activation from the normalised K half of kv and the V'^T | V'^2^T image vt.  The keys are split
    so that about 512 workgroups run (fixed-order sum of the splits: deterministic)."""
    _need_gpu(kv, vt)
    B, H, Ns, _ = kv.shape
    if vt.shape != (B, H, 128, (Ns + 63) // 64 * 64) or vt.dtype != kv.dtype:
        raise ValueError(f"cosine_moments: vt {tuple(vt.shape)} does not match kv {tuple(kv.shape)}")
    splits = max(1, min((Ns + 63) // 64, -(-512 // (B * H))))
    mom = torch.empty(B, H, 65, 132, device=kv.device, dtype=torch.float32)
    work = torch.empty(splits, B * H * 65 * 132, device=kv.device, dtype=torch.float32) if splits > 1 else None
    _call("mhada_cosine_moments", kv, kv.data_ptr(), vt.data_ptr(), dt_code(kv.dtype), B, H, Ns, mom.data_ptr(),
          _ptr(work), splits)
    return mom


def cosine_attn(q, mom, fcs, fcs_mu, fcs_rstd, v_mu) -> torch.Tensor:
    """``mhada_cosine_attn``: mhada_attn's output for the cosine activation from normalised q and
    the style moments of cosine_moments."""
    _need_gpu(q, mom, fcs, fcs_mu, fcs_rstd, v_mu)
    B, H, Nc, _ = q.shape
    if mom.shape != (B, H, 65, 132) or mom.dtype != torch.float32:
        raise ValueError(f"cosine_attn: mom {tuple(mom.shape)} does not match q {tuple(q.shape)}")
    out = torch.empty(B, Nc, H * 64, device=q.device, dtype=q.dtype)
    _call("mhada_cosine_attn", q, q.data_ptr(), mom.data_ptr(), fcs.data_ptr(), fcs_mu.data_ptr(),
          fcs_rstd.data_ptr(), v_mu.data_ptr(), out.data_ptr(), dt_code(q.dtype), B, H, Nc)
    return out


def mhada_attn(q, kv, vt, fcs, fcs_mu, fcs_rstd, v_mu, activation: int) -> torch.Tensor:
    _need_gpu(q, kv, vt, fcs, fcs_mu, fcs_rstd, v_mu)
    B, H, Nc, _ = q.shape
    Ns = kv.shape[2]
    out = torch.empty(B, Nc, H * 64, device=q.device, dtype=q.dtype)
    _call("mhada_attn", q, q.data_ptr(), kv.data_ptr(), _ptr(vt), fcs.data_ptr(), fcs_mu.data_ptr(),
                                fcs_rstd.data_ptr(), v_mu.data_ptr(), out.data_ptr(), dt_code(q.dtype), B, H, Nc,
                                Ns, activation)
    return out


# The fp32 softmax MHAda attention as SPLIT3 products on the bf16 MFMA (mhada_attn_split3): fp32-accurate
# (against fp64 at or below the fp32 MFMA kernel's error) and faster.  False: the fp32 MFMA kernel.
F32_SPLIT_ATTN = True


def split3_kv(kv: torch.Tensor, vt: torch.Tensor) -> torch.Tensor:
    """``mhada_split3_kv``: the fp32 K half of kv [B][H][Ns][128] and the fp32 V'^T | V'^2^T image vt
    [B][H][128][ceil64(Ns)] as the bf16 plane image [B][H][576 ceil64(Ns)] of ``attn_split3``."""
    _need_gpu(kv, vt)
    B, H, Ns, _ = kv.shape
    ldt = (Ns + 63) // 64 * 64
    if kv.dtype != torch.float32 or vt.dtype != torch.float32 or vt.shape != (B, H, 128, ldt) \
            or kv.shape[3] != 128 or not kv.is_contiguous() or not vt.is_contiguous():
        raise ValueError(f"split3_kv: needs contiguous fp32 kv [B][H][Ns][128] and vt [B][H][128][{ldt}], "
                         f"got {tuple(kv.shape)} / {tuple(vt.shape)}")
    img = torch.empty(B, H, 576 * ldt, device=kv.device, dtype=torch.bfloat16)
    _call("mhada_split3_kv", kv, kv.data_ptr(), vt.data_ptr(), img.data_ptr(), B, H, Ns)
    return img


def kv_proj_split3(fs: torch.Tensor, mu_s: torch.Tensor, wkv: torch.Tensor, bkv: torch.Tensor) -> torch.Tensor:
    """``mhada_kv_proj_split3``: the MHAda block's K|V' projection of the fp32 style tokens fs [B][Ns][64H]
    (centred by mu_s [B][64H], folded fp32 weights wkv [B][H][128][64] and bias bkv [H][128] of
    ``fold_block``) written straight as the ``attn_split3`` plane image [B][H][576 ceil64(Ns)]."""
    _need_gpu(fs, mu_s, wkv, bkv)
    B, Ns, C = fs.shape
    H = C // 64
    for t in (fs, mu_s, wkv, bkv):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("kv_proj_split3 needs contiguous float32 operands")
    if C % 64 or mu_s.shape != (B, C) or wkv.shape != (B, H, 128, 64) or bkv.shape != (H, 128):
        raise ValueError(f"kv_proj_split3: bad shapes fs {tuple(fs.shape)} mu {tuple(mu_s.shape)} "
                         f"wkv {tuple(wkv.shape)} bkv {tuple(bkv.shape)}")
    ldt = (Ns + 63) // 64 * 64
    img = torch.empty(B, H, 576 * ldt, device=fs.device, dtype=torch.bfloat16)
    _call("mhada_kv_proj_split3", fs, fs.data_ptr(), mu_s.data_ptr(), wkv.data_ptr(), bkv.data_ptr(), img.data_ptr(),
          B, H, Ns)
    return img


def attn_split3(q, img, Ns: int, fcs, fcs_mu, fcs_rstd, v_mu) -> torch.Tensor:
    """``mhada_attn_split3``: mhada_attn's fp32 softmax output from fp32 q [B][H][Nc][64] and the
    ``split3_kv`` plane image of Ns keys."""
    _need_gpu(q, img, fcs, fcs_mu, fcs_rstd, v_mu)
    B, H, Nc, _ = q.shape
    ldt = (Ns + 63) // 64 * 64
    if q.dtype != torch.float32 or not q.is_contiguous() or img.dtype != torch.bfloat16 \
            or img.shape != (B, H, 576 * ldt):
        raise ValueError(f"attn_split3: q must be contiguous fp32 and img bf16 [B][H][576*{ldt}], got "
                         f"{q.dtype} / {tuple(img.shape)}")
    out = torch.empty(B, Nc, H * 64, device=q.device, dtype=torch.float32)
    _call("mhada_attn_split3", q, q.data_ptr(), img.data_ptr(), fcs.data_ptr(), fcs_mu.data_ptr(),
          fcs_rstd.data_ptr(), v_mu.data_ptr(), out.data_ptr(), B, H, Nc, Ns)
    return out


def _rows64(*ts: torch.Tensor) -> None:
    _need_gpu(*ts)
    for t in ts:
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("training attention operands must be contiguous float32")


def attn_train_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, x: torch.Tensor):
    """``mhada_attn_train_fwd``: q, x (BH, Nc, 64); k, v (BH, Ns, 64) with v centred.
    Returns out' (BH, Nc, 64), [M' | E2'] (BH, Nc, 128), lse2 (BH, Nc)."""
    _rows64(q, k, v, x)
    BH, Nc, d = q.shape
    Ns = k.shape[1]
    if d != 64 or k.shape != (BH, Ns, 64) or v.shape != k.shape or x.shape != q.shape:
        raise ValueError(f"attn_train_fwd: bad shapes q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)} "
                         f"x{tuple(x.shape)}")
    out = torch.empty_like(q)
    mo = torch.empty(BH, Nc, 128, device=q.device, dtype=torch.float32)
    lse = torch.empty(BH, Nc, device=q.device, dtype=torch.float32)
    if TRAIN_FWD_S3:
        # SPLIT3 products on the bf16 MFMA (csrc/attn_split3.hip) over a bf16 plane image of k, v
        # (workspace, freed after)
        img = torch.empty(BH, 576 * ((Ns + 63) // 64 * 64), device=q.device, dtype=torch.bfloat16)
        _call("mhada_attn_train_fwd_split3", q, q.data_ptr(), k.data_ptr(), v.data_ptr(), img.data_ptr(), x.data_ptr(),
              out.data_ptr(), mo.data_ptr(), lse.data_ptr(), BH, Nc, Ns)
    elif TRAIN_FWD_VT:
        # the inference fp32 attention structure on a V'^T | V'^2^T image (workspace, freed after)
        vt = torch.empty(BH, 128, (Ns + 63) // 64 * 64, device=q.device, dtype=torch.float32)
        _call("mhada_attn_train_fwd_vt", q, q.data_ptr(), k.data_ptr(), v.data_ptr(), vt.data_ptr(), x.data_ptr(),
              out.data_ptr(), mo.data_ptr(), lse.data_ptr(), BH, Nc, Ns)
    else:
        _call("mhada_attn_train_fwd", q, q.data_ptr(), k.data_ptr(), v.data_ptr(), x.data_ptr(), out.data_ptr(),
              mo.data_ptr(), lse.data_ptr(), BH, Nc, Ns)
    return out, mo, lse


# attn_train_fwd: TRAIN_FWD_S3 = mhada_attn_train_fwd_split3 (round 6, the default): S on the fp32
# MFMA, P V' / P V'^2 as SPLIT3 products on the bf16 MFMA with per-group sums added in fp32
# (csrc/attn_split3.hip) — 450 -> 433 ms per 512^2 B8 training step; the 64^2 video-training golden's
# gradient norms within 3.3e-4 (the fp32-MFMA forward: 4.9e-4;
# tools/video_golden_ab.py, profiles/r06_train_fwd_s3_acc_ab.log).  TRAIN_FWD_VT =
# mhada_attn_train_fwd_vt (the fp32-MFMA inference structure, round 4) when TRAIN_FWD_S3 is off;
# both off = the round-1 kernel (A/B, tests).
TRAIN_FWD_S3 = True
TRAIN_FWD_VT = True


# Largest dS spill (BH * Nc * Ns fp32) the training backward takes (512^2 batch 8, the three
# AdaFormer calls batched: 12.9 GB, reused across the step's attention calls by the caching
# allocator); larger problems, or spill=False, recompute S and dA in the query-stationary dQ
# kernel instead.  The choice depends on the shapes and this budget only — never on the device's
# free memory — so a step's dQ bits are reproducible run to run (the two paths sum dQ in different
# fp32 orders).  A spill that does not fit raises the allocator's OOM instead of switching paths.
DS_SPILL_BYTES = 16 << 30
# Per-(b, h) slice bound of the kernel's 32-bit dS buffer offsets ((Nc + 32) * Ns, attn_train.hip)
DS_SPILL_MAX_ROWS = 0x7fff0000 // 4
# Which backward each attn_train_bwd call took ("spill" / "recompute"): tests and tools read it.
BWD_PATH_COUNTS = {"spill": 0, "recompute": 0}


def ds_spill_eligible(BH: int, Nc: int, Ns: int) -> bool:
    """The shape rule of attn_train_bwd's default path (see DS_SPILL_BYTES)."""
    return Ns % 4 == 0 and 4 * BH * Nc * Ns <= DS_SPILL_BYTES and (Nc + 32) * Ns <= DS_SPILL_MAX_ROWS


def transpose64(x: torch.Tensor) -> torch.Tensor:
    """``mhada_transpose64``: fp32 [BH][N][64] -> [BH][64][ceil64(N)] (columns >= N zero)."""
    _need_gpu(x)
    if x.dtype != torch.float32 or x.dim() != 3 or x.shape[-1] != 64:
        raise ValueError("transpose64: fp32 [BH][N][64]")
    x = x.contiguous()
    BH, N, _ = x.shape
    ldt = (N + 63) // 64 * 64
    out = torch.empty(BH, 64, ldt, device=x.device, dtype=torch.float32)
    _call("mhada_transpose64", x, x.data_ptr(), out.data_ptr(), BH, N, ldt)
    return out


def attn_train_bwd(q, k, v, lse, dmo, dd, spill: Optional[bool] = None):
    """``mhada_attn_train_bwd``: returns dq (BH, Nc, 64), dk, dv (BH, Ns, 64).  With the dS spill
    (default when ``ds_spill_eligible``): ``mhada_attn_train_dkv`` writes dS and dQ = dS K runs as
    one batched GEMM (896 instead of 1280 FLOP per query-key-head pair)."""
    _rows64(q, k, v, lse, dmo, dd)
    BH, Nc, _ = q.shape
    Ns = k.shape[1]
    if lse.shape != (BH, Nc) or dmo.shape != (BH, Nc, 128) or dd.shape != (BH, Nc) or k.shape != (BH, Ns, 64) \
            or v.shape != k.shape:
        raise ValueError("attn_train_bwd: bad shapes")
    auto = spill is None
    if auto:
        spill = ds_spill_eligible(BH, Nc, Ns)
    ds = None
    if spill:
        try:
            ds = torch.empty(BH, Nc, Ns, device=q.device, dtype=torch.float32)
        except torch.cuda.OutOfMemoryError:
            # the shape rule chose the spill but the device has no room for dS (a smaller card or a
            # larger batch): the recompute backward needs no workspace (same gradients to fp32 order)
            if not auto:
                raise
            spill = False
    BWD_PATH_COUNTS["spill" if spill else "recompute"] += 1
    dq = torch.empty_like(q)
    dk = torch.empty_like(k)
    dv = torch.empty_like(v)
    if not spill:
        _call("mhada_attn_train_bwd", q, q.data_ptr(), k.data_ptr(), v.data_ptr(), lse.data_ptr(), dmo.data_ptr(),
              dd.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), BH, Nc, Ns)
        return dq, dk, dv
    if Ns % 4:
        raise ValueError("attn_train_bwd: the dS spill needs Ns % 4 == 0")
    _call("mhada_attn_train_dkv", q, q.data_ptr(), k.data_ptr(), v.data_ptr(), lse.data_ptr(), dmo.data_ptr(),
          dd.data_ptr(), dk.data_ptr(), dv.data_ptr(), ds.data_ptr(), BH, Nc, Ns)
    if TRAIN_DQ_S3 and Ns % 32 == 0:
        ldt = (Ns + 63) // 64 * 64
        gemm_n64_split3(ds, transpose64_split3(k), dq, BH, Nc, Ns, ldt)
    else:
        kt = transpose64(k)  # W[n = d][k = key] of the NT GEMM, rows padded to ceil64(Ns)
        ldt = kt.shape[-1]
        gemm(a=ds, w=kt, c=dq, M=Nc, N=64, K=Ns, compute=torch.float32, lda=Ns, sa=(Nc * Ns, 0), nb=(BH, 1),
             ldw=ldt, sw=(64 * ldt, 0), ldc=64, sc=(Nc * 64, 0))
    return dq, dk, dv


# dQ = dS K of the dS-spill backward as SPLIT3 products on the bf16 MFMA (csrc/gemm_n64_split3.hip,
# round 6) where Ns % 32 == 0; False: the fp32-MFMA N <= 64 GEMM (gemm_n64_kernel)
TRAIN_DQ_S3 = True


def transpose64_split3(k: torch.Tensor) -> torch.Tensor:
    """``mhada_transpose64_split3``: fp32 [BH][N][64] -> the bf16 planes of its transpose [3][BH * 64][ldt]
    (ldt = ceil64(N), columns >= N zero) = ``split3_rows(transpose64(k))`` in one pass."""
    _need_gpu(k)
    if k.dtype != torch.float32 or k.dim() != 3 or k.shape[-1] != 64:
        raise ValueError("transpose64_split3: fp32 [BH][N][64]")
    k = k.contiguous()
    BH, N, _ = k.shape
    ldt = (N + 63) // 64 * 64
    out = torch.empty(3, BH * 64, ldt, device=k.device, dtype=torch.bfloat16)
    _call("mhada_transpose64_split3", k, k.data_ptr(), out.data_ptr(), BH, N, ldt)
    return out


def gemm_n64_split3(ds: torch.Tensor, kt_planes: torch.Tensor, dq: torch.Tensor, BH: int, Nc: int, Ns: int,
                    ldt: int):
    """``mhada_gemm_n64_split3``: dq [BH][Nc][64] = ds [BH][Nc][Ns] @ K where kt_planes = the three bf16
    planes [3][BH * 64][ldt] of K^T (``split3_rows(transpose64(k))``)."""
    if ds.dtype != torch.float32 or not ds.is_contiguous() or ds.shape != (BH, Nc, Ns):
        raise ValueError("gemm_n64_split3: ds must be contiguous float32 [BH][Nc][Ns]")
    if kt_planes.dtype != torch.bfloat16 or kt_planes.shape != (3, BH * 64, ldt) or not kt_planes.is_contiguous():
        raise ValueError("gemm_n64_split3: kt_planes must be contiguous bf16 [3][BH*64][ldt]")
    if dq.dtype != torch.float32 or not dq.is_contiguous() or dq.shape != (BH, Nc, 64):
        raise ValueError("gemm_n64_split3: dq must be contiguous float32 [BH][Nc][64]")
    _call("mhada_gemm_n64_split3", ds, ds.data_ptr(), kt_planes.data_ptr(), dq.data_ptr(), BH, Nc, Ns, Ns, Nc * Ns,
          ldt, 64 * ldt, BH * 64 * ldt, 64, Nc * 64)


# ---- video path: optical-flow warping (NCHW fp32) ---------------------------------------
_PADDING = {"zeros": 0, "border": 1}


def _padding_code(padding_mode: str) -> int:
    try:
        return _PADDING[padding_mode]
    except KeyError:
        raise ValueError(f"padding_mode {padding_mode!r}: the HIP warp implements 'zeros' and 'border'")


def _f32c(t: torch.Tensor, what: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise ValueError(f"{what} must be float32")
    return t.contiguous()


def warp(x: torch.Tensor, flow: torch.Tensor, padding_mode: str = "zeros") -> torch.Tensor:
    """``mhada_warp``: x [B][C][H][W], flow [B][2][H][W] -> warped x (utilities.py:100-118)."""
    _need_gpu(x, flow)
    x, flow = _f32c(x, "x"), _f32c(flow, "flow")
    B, C, H, W = x.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"flow must be [B,2,H,W] = {[B, 2, H, W]}, got {list(flow.shape)}")
    y = torch.empty_like(x)
    _call("mhada_warp", x, x.data_ptr(), flow.data_ptr(), y.data_ptr(), B, C, H, W,
                                _padding_code(padding_mode))
    return y


def warp_bwd(gy: torch.Tensor, flow: torch.Tensor, padding_mode: str = "zeros") -> torch.Tensor:
    """``mhada_warp_bwd``: the gradient of warp(x, flow) w.r.t. x for the output gradient gy."""
    _need_gpu(gy, flow)
    gy, flow = _f32c(gy, "gy"), _f32c(flow, "flow")
    B, C, H, W = gy.shape
    if tuple(flow.shape) != (B, 2, H, W):
        raise ValueError(f"flow must be [B,2,H,W] = {[B, 2, H, W]}, got {list(flow.shape)}")
    gx = torch.zeros_like(gy)
    _call("mhada_warp_bwd", gy, gy.data_ptr(), flow.data_ptr(), gx.data_ptr(), B, C, H, W, _padding_code(padding_mode))
    return gx


def flow_warp_mask(flo01: torch.Tensor, flo10: torch.Tensor, padding_mode: str = "zeros",
                   threshold: float = 2) -> torch.Tensor:
    """``mhada_flow_warp_mask``: flo01, flo10 [2][H][W] -> mask [H][W] (utilities.py:121-151)."""
    _need_gpu(flo01, flo10)
    flo01, flo10 = _f32c(flo01, "flo01"), _f32c(flo10, "flo10")
    if flo01.dim() != 3 or flo01.shape[0] != 2 or flo01.shape != flo10.shape:
        raise ValueError("flows must both be [2,H,W]")
    H, W = flo01.shape[1:]
    mask = torch.empty(H, W, device=flo01.device, dtype=torch.float32)
    _call("mhada_flow_warp_mask", flo01, flo01.data_ptr(), flo10.data_ptr(), mask.data_ptr(), H, W,
                                          float(threshold), _padding_code(padding_mode))
    return mask


def warp_l1(cs1: torch.Tensor, cs2: torch.Tensor, flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """``mhada_warp_l1``: per-image sum(mask * |cs2 - warp(cs1, flow)|) / (C*H*W)."""
    _need_gpu(cs1, cs2, flow, mask)
    cs1, cs2, flow, mask = (_f32c(t, n) for t, n in ((cs1, "cs1"), (cs2, "cs2"), (flow, "flow"), (mask, "mask")))
    B, C, H, W = cs1.shape
    if cs2.shape != cs1.shape or tuple(flow.shape) != (B, 2, H, W) or tuple(mask.shape) != (B, H, W):
        raise ValueError("warp_l1: cs1/cs2 [B,C,H,W], flow [B,2,H,W], mask [B,H,W]")
    work = torch.empty(B * ((H * W + 255) // 256), device=cs1.device, dtype=torch.float64)
    out = torch.empty(B, device=cs1.device, dtype=torch.float32)
    _call("mhada_warp_l1", cs1, cs1.data_ptr(), cs2.data_ptr(), flow.data_ptr(), mask.data_ptr(),
                                   work.data_ptr(), out.data_ptr(), B, C, H, W)
    return out


def frame_ingest(frames: torch.Tensor, out_hw=None, bgr: bool = True) -> torch.Tensor:
    """``mhada_frame_ingest``: u8 frames [B][H][W][3] (or one [H][W][3]; rows may be padded) ->
    fp32 [B][3][Ho][Wo] (BGR->RGB, INTER_AREA to out_hw = (Ho, Wo), toTensor255)."""
    _need_gpu(frames)
    if frames.dtype != torch.uint8:
        raise ValueError("frames must be uint8 (H, W, 3) images")
    if frames.dim() == 3:
        frames = frames.unsqueeze(0)
    if frames.dim() != 4 or frames.shape[3] != 3 or frames.stride(3) != 1 or frames.stride(2) != 3:
        raise ValueError(f"frames must be [B][H][W][3] with packed pixels, got {tuple(frames.shape)}")
    B, H, W, _ = frames.shape
    if B > 1 and frames.stride(0) != H * frames.stride(1):
        frames = frames.contiguous()
    Ho, Wo = (H, W) if out_hw is None else out_hw
    out = torch.empty(B, 3, Ho, Wo, device=frames.device, dtype=torch.float32)
    _call("mhada_frame_ingest", frames, frames.data_ptr(), B, H, W, frames.stride(1), int(bgr), out.data_ptr(), Ho, Wo)
    return out


# ---- training path (fp32, NHWC): backward helpers (include/mhada_hip.h) ------------------
def gemm_tn(a: torch.Tensor, b: torch.Tensor, M: int, N: int, K: int, lda: int, ldb: int = 0,
            b_mode: int = A_ROWS, img=(0, 0, 0), pad: int = 0, colsum: bool = False, nb: int = 1,
            sza: int = 0, szb: int = 0):
    """``mhada_gemm_tn``: C[M][N] = sum_k A[k][m] B[k][n] (fp32), deterministic split-K.  With
    ``colsum`` also the column sums of A (sum_k A[k][m], the bias gradient) from the same pass:
    returns (C, colsum).  ``nb`` > 1: a batch of problems whose A / B start sza / szb elements
    apart (ROWS mode); C is [nb][M][N] and the column sums [nb][M]."""
    _need_gpu(a, b)
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise ValueError("gemm_tn is fp32")
    lib = _lib.load()
    splits = lib.mhada_gemm_tn_splits(M, N, K)
    work = torch.empty(max(1, splits) * (M * N + (M if colsum else 0)) if nb == 1 else
                       max(1, splits // nb) * nb * (M * N + (M if colsum else 0)), device=a.device, dtype=torch.float32)
    c = torch.empty(*((nb,) if nb > 1 else ()), M, N, device=a.device, dtype=torch.float32)
    cs = torch.empty(*((nb,) if nb > 1 else ()), M, device=a.device, dtype=torch.float32) if colsum else None
    args = GemmTnArgs()
    args.M, args.N, args.K = M, N, K
    args.a, args.lda, args.b, args.ldb, args.b_mode = a.data_ptr(), lda, b.data_ptr(), ldb, b_mode
    args.img_c, args.img_h, args.img_w = img
    args.pad = pad
    args.c, args.ldc = c.data_ptr(), N
    args.colsum = cs.data_ptr() if colsum else None
    args.nb, args.sza, args.szb = nb, sza, szb
    _call("mhada_gemm_tn", a, ctypes.byref(args), work.data_ptr(), work.numel())
    return (c, cs) if colsum else c


def colsum(x: torch.Tensor) -> torch.Tensor:
    """``mhada_colsum`` over the rows of a contiguous [..., C] fp32 tensor -> [C]."""
    _need_gpu(x)
    C = x.shape[-1]
    rows = x.numel() // C
    out = torch.empty(C, device=x.device, dtype=torch.float32)
    work = torch.empty(min(128, max(1, rows // 64)) * C, device=x.device, dtype=torch.float32)
    _call("mhada_colsum", x, x.data_ptr(), out.data_ptr(), rows, C, work.data_ptr(), work.numel())
    return out


def relu_bwd(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    _need_gpu(dy, y)
    dx = torch.empty_like(y)
    _call("mhada_relu_bwd", y, dy.data_ptr(), y.data_ptr(), dx.data_ptr(), y.numel())
    return dx


def feat_stats(x: torch.Tensor, t: Optional[torch.Tensor] = None, stats: bool = True):
    """``mhada_feat_stats`` on NHWC storage x [B][H][W][C] fp32 (t the same shape, or None):
    (mean [B][C], unbiased std [B][C]) or (None, None) without ``stats``, and mean((x - t)^2) as a
    0-dim fp32 device tensor (None without t)."""
    _need_gpu(x, t)
    B, H, W, C = x.shape
    for u in (x, t):
        if u is not None and (u.dtype != torch.float32 or not u.is_contiguous()):
            raise ValueError("feat_stats: contiguous fp32 NHWC operands")
    if t is not None and t.shape != x.shape:
        raise ValueError("feat_stats: target shape")
    if not stats and t is None:
        raise ValueError("feat_stats: nothing to compute")
    P = H * W
    nwork = int(_lib.load().mhada_feat_stats_work(B, P, C))
    work = torch.empty(max(1, nwork), device=x.device, dtype=torch.float64)
    mu = torch.empty(B, C, device=x.device, dtype=torch.float32) if stats else None
    sd = torch.empty(B, C, device=x.device, dtype=torch.float32) if stats else None
    mse = torch.empty((), device=x.device, dtype=torch.float32) if t is not None else None
    ptr = lambda u: None if u is None else u.data_ptr()  # noqa: E731
    _call("mhada_feat_stats", x, x.data_ptr(), ptr(t), ptr(mu), ptr(sd), ptr(mse), work.data_ptr(), nwork, B, P, C)
    return mu, sd, mse


def feat_loss_bwd(x: torch.Tensor, mu: Optional[torch.Tensor], alpha: Optional[torch.Tensor],
                  beta: Optional[torch.Tensor], t: Optional[torch.Tensor], ks: float,
                  kp: Optional[torch.Tensor] = None, relu: bool = False) -> torch.Tensor:
    """``mhada_feat_loss_bwd`` on NHWC storage x [B][H][W][C] fp32 (t the same shape, or None;
    mu / alpha / beta [B][C] fp32, or all None; kp a one-element fp32 device tensor or None):
    alpha + beta (x - mu) + ks * kp (x - t), times (x > 0) with ``relu`` (x a ReLU output)."""
    _need_gpu(x)
    B, H, W, C = x.shape
    for u in (x, t, mu, alpha, beta, kp):
        if u is not None and (u.dtype != torch.float32 or not u.is_contiguous()):
            raise ValueError("feat_loss_bwd: contiguous fp32 operands")
    if kp is not None and kp.numel() != 1:
        raise ValueError("feat_loss_bwd: kp is one element")
    if t is not None and t.shape != x.shape:
        raise ValueError("feat_loss_bwd: target shape")
    if alpha is not None and not (alpha.shape == beta.shape == mu.shape == (B, C)):
        raise ValueError("feat_loss_bwd: statistics [B][C]")
    g = torch.empty_like(x)
    ptr = lambda u: None if u is None else u.data_ptr()  # noqa: E731
    _call("mhada_feat_loss_bwd", x, x.data_ptr(), ptr(t), ptr(mu), ptr(alpha), ptr(beta), ptr(kp), float(ks),
          g.data_ptr(), B, H * W, C, int(relu))
    return g


def reflect_fold(dxp: torch.Tensor, relu_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``mhada_reflect_fold``; ``relu_mask`` (shaped like the result): zero where relu_mask <= 0."""
    _need_gpu(dxp, relu_mask)
    B, Hp, Wp, C = dxp.shape
    dx = torch.empty(B, Hp - 2, Wp - 2, C, device=dxp.device, dtype=torch.float32)
    if relu_mask is not None and (relu_mask.shape != dx.shape or relu_mask.dtype != torch.float32
                                  or not relu_mask.is_contiguous()):
        raise ValueError("reflect_fold: relu_mask must be a contiguous fp32 tensor shaped like the result")
    _call("mhada_reflect_fold", dxp, dxp.data_ptr(), dx.data_ptr(), B, Hp - 2, Wp - 2, C, _ptr(relu_mask))
    return dx


def maxpool2(x: torch.Tensor) -> torch.Tensor:
    _need_gpu(x)
    B, H, W, C = x.shape
    y = torch.empty(B, H // 2, W // 2, C, device=x.device, dtype=torch.float32)
    _call("mhada_maxpool2", x, x.data_ptr(), y.data_ptr(), B, H, W, C)
    return y


def maxpool2_bwd(x: torch.Tensor, dy: torch.Tensor, relu_mask: bool = False) -> torch.Tensor:
    """MaxPool2d(2, 2) adjoint; relu_mask also applies the ReLU adjoint (x > 0) of a ReLU output x."""
    _need_gpu(x, dy)
    B, H, W, C = x.shape
    dx = torch.empty_like(x)
    _call("mhada_maxpool2_bwd", x, x.data_ptr(), dy.data_ptr(), dx.data_ptr(), B, H, W, C, int(relu_mask))
    return dx


def upsample2x_bwd(dy: torch.Tensor, relu_x: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Adjoint of the NHWC bilinear x2; with relu_x (the upsample input, a ReLU output) also the
    producing ReLU's adjoint."""
    _need_gpu(dy, relu_x)
    B, Ho, Wo, C = dy.shape
    dx = torch.empty(B, Ho // 2, Wo // 2, C, device=dy.device, dtype=torch.float32)
    if relu_x is not None and (relu_x.shape != dx.shape or relu_x.dtype != torch.float32 or not relu_x.is_contiguous()):
        raise ValueError("upsample2x_bwd: relu_x must be the contiguous fp32 upsample input")
    _call("mhada_upsample2x_bwd", dy, dy.data_ptr(), _ptr(relu_x), dx.data_ptr(), B, Ho // 2, Wo // 2, C)
    return dx


def vgg_input(img: torch.Tensor, cp: int = 32) -> torch.Tensor:
    _need_gpu(img)
    B, _, H, W = img.shape
    out = torch.empty(B, H, W, cp, device=img.device, dtype=torch.float32)
    _call("mhada_vgg_input", img, img.data_ptr(), out.data_ptr(), B, H, W, cp)
    return out


def vgg_input_bwd(dout: torch.Tensor) -> torch.Tensor:
    _need_gpu(dout)
    B, H, W, cp = dout.shape
    dimg = torch.empty(B, 3, H, W, device=dout.device, dtype=torch.float32)
    _call("mhada_vgg_input_bwd", dout, dout.data_ptr(), dimg.data_ptr(), B, H, W, cp)
    return dimg


def _f32_contig(*ts: torch.Tensor, what: str) -> None:
    for t in ts:
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"{what}: contiguous fp32 tensors expected")


def vgg_stem_dgrad(dy: torch.Tensor, y: torch.Tensor, wd: torch.Tensor) -> torch.Tensor:
    """``mhada_vgg_stem_dgrad``: image gradient [B][3][H][W] of normalise -> conv3x3(3 -> 64, zero
    pad) -> ReLU from dy, y NHWC [B][H][W][64] and the flipped weights wd [9][64][3]."""
    _need_gpu(dy, y, wd)
    _f32_contig(dy, y, wd, what="vgg_stem_dgrad")
    B, H, W, C = y.shape
    if C != 64 or dy.shape != y.shape or wd.shape != (9, 64, 3):
        raise ValueError("vgg_stem_dgrad: dy, y [B][H][W][64], wd [9][64][3]")
    dimg = torch.empty(B, 3, H, W, device=y.device, dtype=torch.float32)
    _call("mhada_vgg_stem_dgrad", y, dy.data_ptr(), y.data_ptr(), wd.data_ptr(), dimg.data_ptr(), B, H, W)
    return dimg


def out3_dgrad(dy: torch.Tensor, y: torch.Tensor, wd: torch.Tensor, relu_x: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``mhada_out3_dgrad``: input gradient NHWC [B][H][W][64] of ReflectionPad2d(1) -> conv3x3(64 -> 3)
    -> ReLU from dy and the output y (NCHW [B][3][H][W]) and wd [9][3][64] (W[co][ci][tap]); with
    relu_x (the layer input, a ReLU output) also the producing ReLU's adjoint."""
    _need_gpu(dy, y, wd, relu_x)
    _f32_contig(dy, y, wd, *(() if relu_x is None else (relu_x,)), what="out3_dgrad")
    B, C, H, W = y.shape
    if C != 3 or dy.shape != y.shape or wd.shape != (9, 3, 64):
        raise ValueError("out3_dgrad: dy, y [B][3][H][W], wd [9][3][64]")
    dx = torch.empty(B, H, W, 64, device=y.device, dtype=torch.float32)
    if relu_x is not None and relu_x.shape != dx.shape:
        raise ValueError("out3_dgrad: relu_x must be the [B][H][W][64] layer input")
    _call("mhada_out3_dgrad", y, dy.data_ptr(), y.data_ptr(), wd.data_ptr(), _ptr(relu_x), dx.data_ptr(), B, H, W)
    return dx


def out3_wgrad(x: torch.Tensor, dy: torch.Tensor, y: torch.Tensor, bias: bool = True):
    """``mhada_out3_wgrad``: (dw [3][64][3][3], db [3] or None) of the same layer from its input x
    NHWC [B][H][W][64], dy and y NCHW [B][3][H][W]."""
    _need_gpu(x, dy, y)
    _f32_contig(x, dy, y, what="out3_wgrad")
    B, H, W, C = x.shape
    if C != 64 or y.shape != (B, 3, H, W) or dy.shape != y.shape:
        raise ValueError("out3_wgrad: x [B][H][W][64], dy, y [B][3][H][W]")
    lib = _lib.load()
    n = lib.mhada_out3_wgrad_work(B, H, W)
    if n <= 0:
        raise ValueError("out3_wgrad: bad shape")
    work = torch.empty(n, device=x.device, dtype=torch.float32)
    dw = torch.empty(3, 64, 3, 3, device=x.device, dtype=torch.float32)
    db = torch.empty(3, device=x.device, dtype=torch.float32) if bias else None
    _call("mhada_out3_wgrad", x, x.data_ptr(), dy.data_ptr(), y.data_ptr(), dw.data_ptr(), _ptr(db),
          work.data_ptr(), n, B, H, W)
    return dw, db


def rows_normalize(x: torch.Tensor, mu: torch.Tensor, rs: torch.Tensor, unit: bool = False) -> torch.Tensor:
    """``mhada_rows_normalize``: (x - mu) * rs on token rows [B][N][C] (and / |row| if unit)."""
    _need_gpu(x, mu, rs)
    for t in (x, mu, rs):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("rows_normalize needs contiguous float32 rows and statistics")
    B, N, C = x.shape
    if mu.shape != (B, C) or rs.shape != (B, C):
        raise ValueError(f"rows_normalize: statistics {tuple(mu.shape)} do not match rows {tuple(x.shape)}")
    out = torch.empty_like(x)
    _call("mhada_rows_normalize", x, x.data_ptr(), mu.data_ptr(), rs.data_ptr(), out.data_ptr(), int(unit), B, N, C)
    return out


def loss_attn(qn: torch.Tensor, kn: torch.Tensor, v: torch.Tensor, x: torch.Tensor, x_mu: torch.Tensor,
              x_rs: torch.Tensor, activation: int) -> torch.Tensor:
    """``mhada_loss_attn``: AdaAttnForLoss on token rows; returns [B][Nq][Dv] fp32."""
    _need_gpu(qn, kn, v, x, x_mu, x_rs)
    for t in (qn, kn, v, x):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("loss_attn operands must be contiguous float32 token rows")
    B, Nq, Dqk = qn.shape
    Ns, Dv = v.shape[1], v.shape[2]
    if kn.shape != (B, Ns, Dqk) or x.shape != (B, Nq, Dv):
        raise ValueError(f"loss_attn: bad shapes q{tuple(qn.shape)} k{tuple(kn.shape)} v{tuple(v.shape)} "
                         f"x{tuple(x.shape)}")
    out = torch.empty(B, Nq, Dv, device=qn.device, dtype=torch.float32)
    _call("mhada_loss_attn", qn, qn.data_ptr(), kn.data_ptr(), v.data_ptr(), x.data_ptr(), x_mu.data_ptr(),
          x_rs.data_ptr(), out.data_ptr(), B, Nq, Ns, Dqk, Dv, activation)
    return out


def vit_batch_attn_bwd(qkv: torch.Tensor, dout: torch.Tensor, L: int, ntok: int, heads: int,
                       groups: int = 1, planes: bool = False):
    """``mhada_vit_batch_attn_bwd``: fp32 qkv [L][ntok][3C], dout [L][ntok][C] -> dqkv (``groups``
    as in vit_batch_attn); ``planes``: also dqkv's three bf16 planes [3][L * ntok][3C]
    (``mhada_vit_batch_attn_bwd_split3``) -> (dqkv, planes)."""
    _need_gpu(qkv, dout)
    C = qkv.shape[-1] // 3
    if L % groups:
        raise ValueError("vit_batch_attn_bwd: L must be a multiple of groups")
    dqkv = torch.empty_like(qkv)
    pl = torch.empty(3, L * ntok, 3 * C, device=qkv.device, dtype=torch.bfloat16) if planes else None
    Lg = L // groups
    for g in range(groups):
        o3, o1 = g * Lg * ntok * 3 * C * 4, g * Lg * ntok * C * 4
        if planes:
            _call("mhada_vit_batch_attn_bwd_split3", qkv, qkv.data_ptr() + o3, dout.data_ptr() + o1,
                  dqkv.data_ptr() + o3, pl.data_ptr() + o3 // 2, L * ntok * 3 * C, Lg, ntok, heads, C // heads)
        else:
            _call("mhada_vit_batch_attn_bwd", qkv, qkv.data_ptr() + o3, dout.data_ptr() + o1, dqkv.data_ptr() + o3,
                  Lg, ntok, heads, C // heads)
    return (dqkv, pl) if planes else dqkv
