"""Per-kernel numerics on the GPU: every C-ABI entry point against a plain-PyTorch fp64/fp32
computation of the same op (tolerances stated per test).  Runs through libmhada_hip.so."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from mhada_hip import _lib, ops
    DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def rnd(*shape, scale=1.0, seed=0, dtype=torch.float32):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV, dtype)


# fp32 compute: exact-fp32 MFMA, only summation order differs -> 1e-5; bf16 operands -> 1e-2
TOL = {torch.float32: 2e-5, torch.bfloat16: 1e-2}


def test_library_is_the_native_one():
    lib = _lib.load()
    assert lib.mhada_abi_version() == _lib.ABI_VERSION
    assert _lib.LIB_PATH.endswith("libmhada_hip.so")


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(100, 96, 64), (1024, 1536, 512), (333, 512, 2048), (4096, 64, 64), (17, 2048, 512),
                                   (32400, 512, 2048), (32400, 512, 512),
                                   (1000, 384, 576), (8192, 512, 64), (2000, 128, 512), (700, 100, 256),
                                   # several persistent tiles per CU (the next tile's W staged before the
                                   # epilogue stores), K = 2 K-tiles included, a partial last row tile
                                   (70000, 1024, 64), (70000, 1024, 128), (70000, 768, 512)])
def test_linear(cdt, M, N, K):
    x = rnd(M, K, seed=1, dtype=cdt)
    w = rnd(N, K, scale=K ** -0.5, seed=2, dtype=cdt)
    b = rnd(N, seed=3)
    r = rnd(M, N, seed=4)
    y = ops.linear(x, w, b, torch.float32, residual=r, relu=False)
    ref = x.double() @ w.double().T + b.double() + r.double()
    assert rel(y, ref) < TOL[cdt]
    y2 = ops.linear(x, w, b, cdt, relu=True)
    ref2 = torch.relu(x.double() @ w.double().T + b.double())
    assert rel(y2, ref2) < TOL[cdt] + (4e-3 if cdt == torch.bfloat16 else 0)


@pytest.mark.parametrize("cols", [512, 1024])
def test_layernorm_split3_planes(cols):
    """mhada_layernorm y_dtype MHADA_BF16X3: plane 0 is the bf16 LayerNorm bit for bit; each later
    plane is at most half a bf16 ulp of the one before (a non-overlapping expansion); the sum agrees
    with the fp32 LayerNorm to a few fp32 ulp of the affine step's O(1) terms (the two kernel
    instantiations may contract (x - mean) * rstd * g + b into FMAs differently: where y cancels to
    ~1e-5 that is a large RELATIVE difference of two equally valid fp32 evaluations)."""
    x = rnd(3001, cols, seed=11) * 3 + 0.5
    g = rnd(cols, seed=12)
    b = rnd(cols, seed=13)
    pl = ops.layernorm_split3(x, g, b, 1e-6)
    y32 = ops.layernorm(x, g, b, torch.float32, 1e-6)
    assert torch.equal(pl[0], ops.layernorm(x, g, b, torch.bfloat16, 1e-6))
    p0, p1, p2 = (pl[i].double() for i in range(3))
    assert (p1.abs() <= p0.abs() * 2.0 ** -8).all() and (p2.abs() <= p1.abs() * 2.0 ** -8).all()
    s = p0 + p1 + p2
    assert ((s - y32.double()).abs() <= 2.0 ** -20 * (y32.double().abs() + b.double().abs() + 4 * g.double().abs())).all()


@pytest.mark.parametrize("M,N,K0", [(4096, 1536, 512), (1000, 2048, 512), (70000, 768, 512), (333, 512, 2048),
                                    (300, 256, 256), (257, 2048, 1024)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (False, True)])
def test_linear_split3_fp32_accuracy(M, N, K0, relu, res):
    """SPLIT3 (fp32-accurate products on the bf16 MFMA, mhada_gemm MHADA_A_SPLIT3): against fp64 at
    an fp32-class error (< 2e-6, a tenth of the fp32 kernel tolerance) and within 2.5x of the fp32
    MFMA GEMM's error on the same operands — the products are exact to 2^-24, the accumulator sees
    6 K0 instead of K0 roundings (measured: below the fp32 path without a residual, up to 1.75x it
    with a residual preloaded into the accumulators); bias / ReLU / residual epilogues, partial row
    tiles, one to several tiles per CU, K0 = 256 .. 2048; run-to-run bit-identical."""
    x = rnd(M, K0, seed=1) * 2
    w = rnd(N, K0, scale=K0 ** -0.5, seed=2)
    b = rnd(N, seed=3)
    r = rnd(M, N, seed=4) if res else None
    g1 = torch.ones(K0, device=DEV)
    b0 = torch.zeros(K0, device=DEV)
    # the planes of x itself: LayerNorm with unit gain of an already-normalised x is x up to its
    # own rounding, so use the LayerNorm output y as THE fp32 operand of both paths
    y = ops.layernorm(x, g1, b0, torch.float32, 1e-6)
    pl = ops.layernorm_split3(x, g1, b0, 1e-6)
    w6 = ops.split3_weight(w)
    out = ops.linear_split3(pl, w6, b, torch.float32, residual=r, relu=relu)
    out2 = ops.linear_split3(pl, w6, b, torch.float32, residual=r, relu=relu)
    assert torch.equal(out, out2)
    ref = y.double() @ w.double().T + b.double()
    if relu:
        ref = torch.relu(ref)
    if res:
        ref = ref + r.double()
    f32 = ops.linear(y, w, b, torch.float32, residual=r, relu=relu)
    e_split, e_f32 = rel(out, ref), rel(f32, ref)
    assert e_split < 2e-6, (e_split, e_f32)
    assert e_split <= 2.5 * e_f32 + 1e-7, (e_split, e_f32)


@pytest.mark.parametrize("M,N,K0", [(4096, 2048, 512), (1000, 512, 256), (70000, 1024, 512)])
def test_linear_split3_plane_output_chain(M, N, K0):
    """SPLIT3 with the result written as three bf16 planes (c2_planes, C not written): the planes
    are the split of exactly the fp32 result the plain SPLIT3 call returns (plane 0 = its bf16
    rounding, the sum within 2^-26), and a MLP1 -> MLP2 chain through them (ReLU, then a residual)
    matches fp64 at an fp32-class error."""
    x = rnd(M, K0, seed=1) * 2
    w1 = rnd(N, K0, scale=K0 ** -0.5, seed=2)
    b1 = rnd(N, seed=3)
    g1, b0 = torch.ones(K0, device=DEV), torch.zeros(K0, device=DEV)
    y = ops.layernorm(x, g1, b0, torch.float32, 1e-6)
    pl = ops.layernorm_split3(x, g1, b0, 1e-6)
    w16 = ops.split3_weight(w1)
    full = ops.linear_split3(pl, w16, b1, torch.float32, relu=True)
    m1 = ops.linear_split3(pl, w16, b1, torch.float32, relu=True, out_planes=True)
    assert m1.shape == (3, M, N) and m1.dtype == torch.bfloat16
    assert torch.equal(m1[0], full.bfloat16())
    s = m1[0].double() + m1[1].double() + m1[2].double()
    assert ((s - full.double()).abs() <= full.double().abs() * 2.0 ** -26).all()
    w2 = rnd(K0, N, scale=N ** -0.5, seed=5)
    b2 = rnd(K0, seed=6)
    r = rnd(M, K0, seed=7)
    out = ops.linear_split3(m1, ops.split3_weight(w2), b2, torch.float32, residual=r)
    h = torch.relu(y.double() @ w1.double().T + b1.double())
    ref = h @ w2.double().T + b2.double() + r.double()
    assert rel(out, ref) < 2e-6
    # plane output with a residual and no ReLU (residual + bias preloaded into the accumulators, then
    # the plane epilogue): plane 0 is the bf16 rounding of the fp32 result, the sum within 2^-26
    r1 = rnd(M, N, seed=8)
    full_r = ops.linear_split3(pl, w16, b1, torch.float32, residual=r1)
    pl_r = ops.linear_split3(pl, w16, b1, torch.float32, residual=r1, out_planes=True)
    assert torch.equal(pl_r[0], full_r.bfloat16())
    s_r = pl_r[0].double() + pl_r[1].double() + pl_r[2].double()
    assert ((s_r - full_r.double()).abs() <= full_r.double().abs() * 2.0 ** -26).all()
    assert rel(s_r, y.double() @ w1.double().T + b1.double() + r1.double()) < 2e-6


def test_linear_split3_rejects_unsupported_shapes():
    """SPLIT3 runs only on the persistent ping-pong kernel: N <= 128 fails loudly in the library,
    mismatched operands in the host wrapper."""
    x = rnd(256, 512, seed=1)
    g1, b0 = torch.ones(512, device=DEV), torch.zeros(512, device=DEV)
    pl = ops.layernorm_split3(x, g1, b0, 1e-6)
    with pytest.raises(ValueError, match="SPLIT3"):
        ops.linear_split3(pl, ops.split3_weight(rnd(128, 512, seed=2)), None, torch.float32)
    with pytest.raises(ValueError):
        ops.linear_split3(pl, ops.split3_weight(rnd(256, 256, seed=2)), None, torch.float32)
    with pytest.raises(ValueError):
        ops.linear_split3(pl[:, :, :256], ops.split3_weight(rnd(256, 256, seed=2)), None, torch.float32)


@pytest.mark.parametrize("M,N,K", [(70000, 1024, 64), (70000, 768, 512), (32400, 512, 2048), (57000, 600, 96),
                                   (65536, 2048, 512)])
def test_gemm_f32_persistent_epilogues(M, N, K):
    """The fp32 persistent ping-pong GEMM: bias / ReLU / residual (preloaded into the
    accumulators) / bf16 copy outputs against fp64 on every row tile (last partial), several tiles
    per CU, 2 to 64 K-tiles, partial column tiles; a second run is bit-identical."""
    x = rnd(M, K, seed=1)
    w = rnd(N, K, scale=K ** -0.5, seed=2)
    b = rnd(N, seed=3)
    r = rnd(M, N, seed=4)

    def run():
        c2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        y0 = torch.empty(M, N, device=DEV)
        ops.gemm(a=x, w=w, c=y0, M=M, N=N, K=K, compute=torch.float32, lda=K, ldw=K, bias=b, ldc=N,
                 c2=c2, ldc2=N)
        out = (ops.linear(x, w, b, torch.float32, residual=r),
               ops.linear(x, w, b, torch.float32, relu=True),
               ops.linear(x, w, None, torch.float32), y0, c2)
        torch.cuda.synchronize()
        return out

    outs = [run(), run()]
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    res, rl, plain, y0, c2 = outs[0]
    assert rel(c2, y0) < 4e-3
    rows = torch.cat([torch.arange(0, M, 997), torch.arange(M - 300, M)]).to(DEV)
    ref = x[rows].double() @ w.double().T + b.double()
    assert rel(res[rows], ref + r[rows].double()) < TOL[torch.float32]
    assert rel(rl[rows], torch.relu(ref)) < TOL[torch.float32]
    assert rel(y0[rows], ref) < TOL[torch.float32]
    assert rel(plain[rows], ref - b.double()) < TOL[torch.float32]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
def test_linear_fp32_input_converted_on_load(cdt):
    x = rnd(300, 512, seed=5)
    w = rnd(512, 512, scale=512 ** -0.5, seed=6, dtype=cdt)
    y = ops.linear(x, w, None, torch.float32)
    ref = x.to(cdt).double() @ w.double().T
    assert rel(y, ref) < TOL[cdt]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N", [200, 4096])
def test_grouped_centred_projection(cdt, N):
    """The MHAda per-head projection pattern: z = (batch, head), A centred per column."""
    B, H, C = 2, 8, 512
    x = rnd(B, N, C, seed=7) * 3 + 1.5
    mu = x.mean(dim=1)  # [B][C]
    w = rnd(B, H, 64, 64, scale=0.125, seed=8, dtype=cdt)
    bias = rnd(H, 64, seed=9)
    q = torch.empty(B, H, N, 64, device=DEV, dtype=cdt)
    ops.gemm(a=x, w=w, c=q, M=N, N=64, K=64, compute=cdt, lda=C, sa=(N * C, 64), nb=(B, H), a_mu=mu,
             smu=(C, 64), ldw=64, sw=(H * 4096, 4096), bias=bias, sb=(0, 64), ldc=64, sc=(H * N * 64, N * 64))
    torch.cuda.synchronize()
    xc = (x - mu[:, None, :]).view(B, N, H, 64).permute(0, 2, 1, 3).to(cdt).double()
    ref = xc @ w.double().transpose(-1, -2) + bias.double()[None, :, None, :]
    assert rel(q, ref) < TOL[cdt]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Ns", [4096, 200, 1000, 64, 37])
def test_kv_projection_vt_epilogue_matches_transpose_v(cdt, Ns):
    """The K|V' projection's vt epilogue (V'^T | V'^2^T written by the GEMM, keys permuted for
    bf16, zero padding to ldt) is bit-identical to the separate mhada_transpose_v of the same
    GEMM's kv output; the K half of kv is unchanged."""
    B, H, C = 2, 8, 512
    x = rnd(B, Ns, C, seed=7) * 3 + 1.5
    mu = x.mean(dim=1)
    w = rnd(B, H, 128, 64, scale=0.125, seed=8, dtype=cdt)
    bias = rnd(H, 128, seed=9)
    args = dict(a=x, w=w, M=Ns, N=128, K=64, compute=cdt, lda=C, sa=(Ns * C, 64), nb=(B, H), a_mu=mu,
                smu=(C, 64), ldw=64, sw=(H * 128 * 64, 128 * 64), bias=bias, sb=(0, 128), ldc=128,
                sc=(H * Ns * 128, Ns * 128))
    kv = torch.empty(B, H, Ns, 128, device=DEV, dtype=cdt)
    ops.gemm(c=kv, **args)
    ref = ops.transpose_v(kv)
    ldt = ref.shape[-1]
    kv2 = torch.empty_like(kv)
    vt = torch.full((B, H, 128, ldt), float("nan"), device=DEV, dtype=cdt)
    ops.gemm(c=kv2, vt=vt, ldt=ldt, svt=(H * 128 * ldt, 128 * ldt), **args)
    assert torch.equal(vt, ref)
    assert torch.equal(kv2[..., :64], kv[..., :64])


def test_gemm_bf16_copy_output():
    """The optional bf16 copy (c2) of an fp32-output GEMM equals the fp32 result rounded once."""
    x = rnd(4096, 512, seed=1, dtype=torch.bfloat16)
    w = rnd(512, 512, scale=512 ** -0.5, seed=2, dtype=torch.bfloat16)
    b = rnd(512, seed=3)
    for M in (4096, 1000):
        c = torch.empty(M, 512, device=DEV)
        c2 = torch.empty(M, 512, device=DEV, dtype=torch.bfloat16)
        ops.gemm(a=x, w=w, c=c, M=M, N=512, K=512, compute=torch.bfloat16, lda=512, ldw=512, bias=b, ldc=512,
                 c2=c2, ldc2=512)
        assert torch.equal(c2, c.bfloat16())
        c3 = torch.empty(M, 512, device=DEV)
        ops.gemm(a=x, w=w, c=c3, M=M, N=512, K=512, compute=torch.bfloat16, lda=512, ldw=512, bias=b, ldc=512)
        assert torch.equal(c, c3)


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,W", [(64, 64), (72, 128), (16, 24)])
def test_patch_embed(cdt, H, W):
    B = 2
    img = torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(3)).to(DEV) * 255
    w = rnd(512, 3, 8, 8, scale=0.05, seed=4)
    b = rnd(512, seed=5)
    pos = rnd((H // 8) * (W // 8), 512, seed=6)
    y = ops.patch_embed(img, w.reshape(512, -1).to(cdt).contiguous(), b, pos)
    ref = F.conv2d(img.to(cdt).double(), w.to(cdt).double(), b.double(), stride=8)
    ref = ref.flatten(2).transpose(1, 2) + pos.double()
    assert rel(y, ref) < TOL[cdt]


@pytest.mark.parametrize("cdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("up", [False, True])
@pytest.mark.parametrize("Ci,Co,H,W", [(64, 64, 9, 13), (128, 64, 16, 16), (512, 256, 8, 8), (256, 128, 5, 3),
                                         (256, 256, 40, 36), (64, 320, 23, 50), (128, 128, 33, 20)])
def test_conv3x3(cdt, up, Ci, Co, H, W):
    B = 2
    x = torch.rand(B, H, W, Ci, generator=torch.Generator().manual_seed(Ci + H)).to(DEV)
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, seed=2)
    b = rnd(Co, seed=3)
    wp = w.permute(0, 2, 3, 1).reshape(Co, -1).to(cdt).contiguous()
    y = ops.conv3x3(x.to(cdt) if cdt == torch.bfloat16 and not up else x, wp, b, torch.float32, upsample=up)
    xn = x.permute(0, 3, 1, 2).double()
    if cdt == torch.bfloat16 and not up:
        xn = x.to(cdt).permute(0, 3, 1, 2).double()
    if up:
        xn = F.interpolate(xn, scale_factor=2, mode="bilinear", align_corners=False)
    ref = torch.relu(F.conv2d(F.pad(xn, (1, 1, 1, 1), mode="reflect"), w.to(cdt).double(), b.double()))
    assert rel(y.permute(0, 3, 1, 2), ref) < TOL[cdt]


@pytest.mark.parametrize("pad_mode,pad", [("reflect", 1), ("zero", 1), ("zero", 2)])
@pytest.mark.parametrize("B,H,W,Ci,Co,ldc", [(2, 8, 8, 8, 64, 64), (1, 9, 13, 32, 128, 128), (2, 33, 20, 64, 64, 68),
                                              (1, 3, 2, 16, 64, 64), (3, 17, 70, 256, 64, 64),
                                              (1, 16, 16, 512, 256, 256), (2, 2, 5, 24, 192, 196),
                                              (1, 40, 36, 96, 64, 64)])
def test_conv3x3_wino(pad_mode, pad, B, H, W, Ci, Co, ldc):
    """fp32 Winograd F(2x2,3x3) (wino.hip) against fp64 conv2d: reflect / zero padding 1 / the
    pad-2 full correlation, odd and tiny output grids (partial tiles), channel-padded outputs
    (ldc > Cout, pad columns untouched), bias + ReLU and none; and against the direct
    implicit-GEMM product (ops.WINO = False)."""
    x = torch.rand(B, H, W, Ci, generator=torch.Generator().manual_seed(H * W + Ci)).to(DEV) - 0.3
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, seed=2)
    b = rnd(Co, seed=3)
    wp = w.permute(0, 2, 3, 1).reshape(Co, -1).contiguous()
    Ho, Wo = (H, W) if pad_mode == "reflect" else (H + 2 * (pad - 1), W + 2 * (pad - 1))
    xn = x.permute(0, 3, 1, 2).double()
    xp = F.pad(xn, (1, 1, 1, 1), mode="reflect") if pad_mode == "reflect" else F.pad(xn, (pad,) * 4)
    mask = (torch.rand(B, Ho, Wo, ldc, generator=torch.Generator().manual_seed(Ci)) - 0.5).to(DEV)
    for bias, relu in ((b, True), (None, False)):
        out = torch.full((B, Ho, Wo, ldc), 7.0, device=DEV)
        y = ops.conv3x3_wino(x, ops.wino_weights(wp), bias, relu, pad_mode, pad, out=out)
        ref = F.conv2d(xp, w.double(), None if bias is None else bias.double())
        ref = torch.relu(ref) if relu else ref
        assert rel(y[..., :Co].permute(0, 3, 1, 2), ref) < 2e-6
        assert bool((y[..., Co:] == 7.0).all())
        # the folded ReLU adjoint (relu_mask): zero exactly where mask <= 0, the same values elsewhere
        outm = torch.full((B, Ho, Wo, ldc), 7.0, device=DEV)
        ym = ops.conv3x3_wino(x, ops.wino_weights(wp), bias, relu, pad_mode, pad, out=outm, relu_mask=mask)
        keep = mask[..., :Co] > 0
        assert torch.equal(ym[..., :Co], torch.where(keep, y[..., :Co], torch.zeros_like(y[..., :Co])))
        assert bool((ym[..., Co:] == 7.0).all())
        if Ci % 32:  # the fp32 implicit GEMM gathers 32-channel chunks
            continue
        ops.WINO = False
        try:
            yd = ops.conv3x3(x, wp, bias, torch.float32, upsample=False, relu=relu, pad_mode=pad_mode, pad=pad)
        finally:
            ops.WINO = True
        assert rel(y[..., :Co], yd) < 2e-6


@pytest.mark.parametrize("pad_mode,pad", [("reflect", 1), ("zero", 1), ("zero", 2)])
@pytest.mark.parametrize("B,H,W,Ci,Co,ldc", [(2, 8, 8, 8, 64, 64), (1, 9, 13, 32, 128, 128), (2, 33, 20, 64, 64, 68),
                                              (1, 3, 2, 16, 64, 64), (1, 16, 16, 512, 256, 256), (2, 2, 5, 24, 192, 196),
                                              (2, 40, 36, 96, 128, 128)])
def test_conv3x3_wino4_bit_identical(pad_mode, pad, B, H, W, Ci, Co, ldc):
    """The 4-wave Winograd kernel (tuning wino4 = 1) runs every MFMA of the 8-wave kernel in the
    same order and keeps its output-transform association: the outputs are bit-identical, with
    and without bias / ReLU / the folded ReLU mask, partial tiles and channel-padded outputs."""
    from mhada_hip import _lib
    x = torch.rand(B, H, W, Ci, generator=torch.Generator().manual_seed(H * W + Ci)).to(DEV) - 0.3
    wp = rnd(Co, 9 * Ci, scale=(9 * Ci) ** -0.5, seed=2)
    b = rnd(Co, seed=3)
    Ho, Wo = (H, W) if pad_mode == "reflect" else (H + 2 * (pad - 1), W + 2 * (pad - 1))
    mask = (torch.rand(B, Ho, Wo, ldc, generator=torch.Generator().manual_seed(Ci)) - 0.5).to(DEV)
    u = ops.wino_weights(wp)
    for bias, relu, m in ((b, True, None), (None, False, None), (b, False, mask)):
        outs = []
        for knob in (0, 1):
            with _lib.tuning(wino4=knob):
                out = torch.full((B, Ho, Wo, ldc), 7.0, device=DEV)
                outs.append(ops.conv3x3_wino(x, u, bias, relu, pad_mode, pad, out=out, relu_mask=m))
        assert torch.equal(outs[0], outs[1])


def test_conv3x3_wino_routing():
    """ops.conv3x3 takes the Winograd kernel for eligible fp32 shapes (same result as the explicit
    call) and the implicit GEMM otherwise (Cout % 64 != 0)."""
    x = torch.rand(1, 12, 10, 64, generator=torch.Generator().manual_seed(4)).to(DEV)
    w = rnd(128, 9 * 64, scale=1 / 24, seed=5)
    b = rnd(128, seed=6)
    assert ops.wino_eligible(x, w, False) and not ops.wino_eligible(x, w[:96], False)
    assert torch.equal(ops.conv3x3(x, w, b, torch.float32, upsample=False),
                       ops.conv3x3_wino(x, ops.wino_weights(w), b))


@pytest.mark.parametrize("up", [False, True])
@pytest.mark.parametrize("B,H,W", [(2, 4, 8), (1, 9, 13), (2, 33, 20), (1, 64, 128), (1, 3, 2), (3, 17, 70)])
def test_conv3x3_c64_tile(up, B, H, W):
    """The decoder's 64 -> 64 layer on the direct tile kernel (conv_tile.hip, bf16 in / out):
    against fp64 on the same bf16 input (upsampled by upsample2x_kernel for up=True), the fused
    upsample bit-identical to upsample2x + conv, and close to the implicit-GEMM path."""
    x = torch.rand(B, H, W, 64, generator=torch.Generator().manual_seed(H * W)).to(DEV).bfloat16()
    w = rnd(64, 64, 3, 3, scale=(9 * 64) ** -0.5, seed=2)
    b = rnd(64, seed=3)
    wp = w.permute(0, 2, 3, 1).reshape(64, -1).bfloat16().contiguous()
    y = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=up)
    xin = ops.upsample2x(x) if up else x
    ref = torch.relu(F.conv2d(F.pad(xin.permute(0, 3, 1, 2).double(), (1, 1, 1, 1), mode="reflect"),
                              wp.double().view(64, 3, 3, 64).permute(0, 3, 1, 2), b.double()))
    assert rel(y.permute(0, 3, 1, 2), ref) < 5e-3
    if up:
        assert torch.equal(y, ops.conv3x3(xin, wp, b, torch.bfloat16, upsample=False))
    with _lib.tuning(conv_c64=0):
        y0 = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=up)
    assert rel(y, y0) < 5e-3


@pytest.mark.parametrize("Ci,Co", [(128, 64), (128, 128), (256, 128)])
@pytest.mark.parametrize("B,H,W", [(2, 8, 32), (1, 9, 13), (2, 33, 20), (1, 64, 128), (1, 2, 2), (3, 17, 70),
                                   (1, 40, 100)])
@pytest.mark.parametrize("relu", [True, False])
def test_conv3x3_dir_tile(Ci, Co, B, H, W, relu):
    """The decoder's 128 / 256-input-channel layers on the direct tile kernel with the streamed
    weight ring (conv_tile.hip conv3x3_dir_kernel, bf16 in / out, reflect pad): against fp64 on
    the same bf16 input and close to the implicit-GEMM path (tuning conv_dir = 0); partial tiles in
    both directions, several tiles per workgroup (the ring running on across tiles), 2 x 2 images;
    a second run is bit-identical."""
    x = (torch.rand(B, H, W, Ci, generator=torch.Generator().manual_seed(H * W + Co)).to(DEV) - 0.3).bfloat16()
    w = rnd(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5, seed=2)
    b = rnd(Co, seed=3)
    wp = w.permute(0, 2, 3, 1).reshape(Co, -1).bfloat16().contiguous()
    y = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=False, relu=relu)
    assert torch.equal(y, ops.conv3x3(x, wp, b, torch.bfloat16, upsample=False, relu=relu))
    ref = F.conv2d(F.pad(x.permute(0, 3, 1, 2).double(), (1, 1, 1, 1), mode="reflect"),
                   wp.double().view(Co, 3, 3, Ci).permute(0, 3, 1, 2), b.double())
    ref = torch.relu(ref) if relu else ref
    assert rel(y.permute(0, 3, 1, 2), ref) < 5e-3
    with _lib.tuning(conv_dir=0):
        y0 = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=False, relu=relu)
    assert rel(y, y0) < 5e-3


def test_conv3x3_dir_full_size():
    """conv2.1 (128 -> 64) and conv2.0 (128 -> 128) at the 1024^2 batch-4 decoder size (512 x 512,
    16 tiles per workgroup) and conv1.4 (256 -> 128 at 256 x 256); against the implicit GEMM and
    fp64 on a row band."""
    for Ci, Co, S in ((128, 64, 512), (128, 128, 512), (256, 128, 256)):
        x = (torch.rand(4, S, S, Ci, generator=torch.Generator().manual_seed(7)).to(DEV) - 0.3).bfloat16()
        wp = rnd(Co, 9 * Ci, scale=(9 * Ci) ** -0.5, seed=Co).bfloat16()
        b = rnd(Co, seed=3)
        y = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=False)
        with _lib.tuning(conv_dir=0):
            y0 = ops.conv3x3(x, wp, b, torch.bfloat16, upsample=False)
        assert rel(y, y0) < 5e-3
        band = x[:, 200:240].permute(0, 3, 1, 2).double()  # rows 201..238 of the output, full width
        ref = torch.relu(F.conv2d(F.pad(band, (1, 1, 0, 0), mode="reflect"),
                                  wp.double().view(Co, 3, 3, Ci).permute(0, 3, 1, 2), b.double()))
        assert rel(y[:, 201:239].permute(0, 3, 1, 2), ref) < 5e-3


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,W,C", [(8, 8, 256), (5, 7, 64), (64, 32, 128), (1, 3, 8), (3, 1, 16), (3, 3, 8),
                                   (4, 9, 24)])
def test_upsample2x(dt, H, W, C):
    """The default kernel (bf16: 2 x 2 output blocks when H, W >= 3; fp32 and small maps: 16-B per
    pixel) against fp64 F.interpolate, bit-identical to the 16-B per-pixel kernel (tuning upsample_quad 0
    forces it) and to the element-wise per-pixel kernel (which a misaligned view takes)."""
    from mhada_hip import _lib
    x = rnd(2, H, W, C, seed=H).to(dt)
    y = ops.upsample2x(x)
    ref = F.interpolate(x.permute(0, 3, 1, 2).double(), scale_factor=2, mode="bilinear", align_corners=False)
    assert rel(y.permute(0, 3, 1, 2), ref) < (1e-6 if dt == torch.float32 else 5e-3)
    with _lib.tuning(upsample_quad=0):
        assert torch.equal(ops.upsample2x(x), y)
    buf = torch.empty(x.numel() + 1, device=DEV, dtype=dt)
    xm = buf[1:].view(x.shape)  # 2 or 4 bytes past a 16-B boundary
    xm.copy_(x)
    assert xm.data_ptr() % 16 != 0
    assert torch.equal(ops.upsample2x(xm), y)


@pytest.mark.parametrize("dt,mfma", [(torch.float32, "1"), (torch.float32, "0"), (torch.bfloat16, "1"),
                                     (torch.bfloat16, "0")])
@pytest.mark.parametrize("clamp", [False, True])
@pytest.mark.parametrize("B,H,W,Ci", [(2, 20, 33, 64), (1, 64, 128, 64), (1, 7, 70, 32), (1, 9, 65, 128),
                                      (3, 37, 2, 64)])
def test_conv_out3(dt, mfma, clamp, B, H, W, Ci):
    """Last decoder layer; bf16 runs the MFMA tile kernel (bf16 weights), fp32 the LDS-tiled
    VALU kernel, or, with mfma == "0", the per-pixel VALU kernel (fp32 weights)."""
    x = torch.rand(B, H, W, Ci, generator=torch.Generator().manual_seed(9)).to(DEV).to(dt)
    w = rnd(3, Ci, 3, 3, scale=0.5, seed=2)
    b = rnd(3, seed=3) * 30
    with _lib.tuning(out3_mfma=int(mfma), out3_tile=int(mfma)):
        y = ops.conv3x3_out3(x, w.permute(2, 3, 1, 0).contiguous(), b, clamp255=clamp)
    ref = torch.relu(F.conv2d(F.pad(x.permute(0, 3, 1, 2).double(), (1, 1, 1, 1), mode="reflect"),
                              w.double(), b.double()))
    if clamp:
        ref = ref.clamp(max=255)
    # fp32 / VALU: fp32 weights, summation order only; MFMA: weights rounded to bf16 (2^-9)
    assert rel(y, ref) < (4e-3 if (dt == torch.bfloat16 and mfma == "1") else 1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm(dt):
    x = rnd(1000, 512, seed=1) * 4 + 2
    g, b = rnd(512, seed=2), rnd(512, seed=3)
    y = ops.layernorm(x, g, b, dt, 1e-6)
    ref = F.layer_norm(x.double(), (512,), g.double(), b.double(), 1e-6)
    assert rel(y, ref) < (1e-6 if dt == torch.float32 else 5e-3)


@pytest.mark.parametrize("dt,vec", [(torch.float32, "1"), (torch.bfloat16, "1"), (torch.bfloat16, "0")])
@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 8, 11])
def test_vit_batch_attention_matches_nn_mha(dt, vec, L):
    N, C, heads = 300, 512, 8
    mha = torch.nn.MultiheadAttention(C, heads).to(DEV).double()
    x = rnd(L, N, C, seed=L).double()
    with torch.no_grad():
        ref, _ = mha(x, x, x, need_weights=False)  # batch_first=False on (B, N, C): attends over B
        qkv = F.linear(x, mha.in_proj_weight, mha.in_proj_bias).to(dt)
        with _lib.tuning(vit_attn_vec=int(vec)):  # bf16 L <= 8: vectorised form unless 0
            att = ops.vit_batch_attn(qkv.contiguous(), L, N, heads)
        y = F.linear(att.double(), mha.out_proj.weight, mha.out_proj.bias)
    assert rel(y, ref) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("oh,ow", [(8, 8), (64, 64), (135, 240), (32, 32), (9, 16)])
def test_pos_embed(oh, ow):
    pos = rnd(1, 512, 32, 32, scale=0.02, seed=1)
    y = ops.pos_embed(pos, oh, ow)
    ref = pos if (oh, ow) == (32, 32) else F.interpolate(pos, size=(oh, ow), mode="bilinear", align_corners=False)
    ref = ref.reshape(512, -1).T
    assert rel(y, ref) < 1e-6


@pytest.mark.parametrize("B,N,C", [(3, 4097, 512), (1, 37, 68), (2, 16384, 512), (1, 32400, 512)])
def test_instnorm_stats(B, N, C):
    x = rnd(B, N, C, seed=2) * 5 + 10
    mu, rstd = ops.instnorm_stats(x)
    xd = x.double()
    ref_mu = xd.mean(1)
    ref_rstd = 1 / torch.sqrt(xd.var(1, unbiased=False) + 1e-5)
    assert rel(mu, ref_mu) < 1e-7
    assert rel(rstd, ref_rstd) < 1e-6


# ---- the fused MHAda attention, through the AdaAttnMultiHead module --------------------------
def _block(act, dt):
    import network
    from mhada_hip.recipe import load_recipe
    blk = load_recipe(network.AdaAttnMultiHead(512, 8, act), "blk").to(DEV)
    blk.compute_dtype = dt
    return blk


def _ref_block(blk, fc, fs, fcs, act):
    import torch_ref
    sd = {k: v.double() for k, v in blk.state_dict().items()}
    with torch.no_grad():
        return torch_ref.block(fc.double(), fs.double(), fcs.double(), sd, "", activation=act)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["softmax", "cosine"])
@pytest.mark.parametrize("B,hc,wc,hs,ws", [(1, 8, 8, 8, 8), (2, 10, 13, 3, 5), (1, 16, 17, 20, 11), (2, 64, 64, 32, 32)])
def test_mhada_block(dt, act, B, hc, wc, hs, ws):
    blk = _block(act, dt)
    fc = rnd(B, 512, hc, wc, seed=1) * 2 + 0.5
    fs = rnd(B, 512, hs, ws, seed=2) * 1.5 - 0.25
    fcs = rnd(B, 512, hc, wc, seed=3)
    with torch.no_grad():
        y = blk(fc, fs, fcs)
    ref = _ref_block(blk, fc, fs, fcs, act)
    assert rel(y, ref) < (1e-5 if dt == torch.float32 else 1.5e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,Nc,Ns", [(1, 1, 5, 3), (2, 3, 100, 97), (1, 2, 130, 5000), (2, 8, 4096, 4096)])
def test_cosine_linear_form(dt, B, H, Nc, Ns):
    """mhada_cosine_moments + mhada_cosine_attn (the cosine activation's O(N d^2) form,
    adaDecoder.py:20-34) against an fp64 evaluation of the reference's quadratic expression on the
    same normalised operands, and against the flash kernel (mhada_attn ACT_COSINE).  Ragged Ns
    (97, 5000: a partial last 64-key tile, several key splits), the bf16 key permutation of vt,
    Nc not a multiple of 64.  Tolerance: fp32 2e-5 (summation order only); bf16 1e-2 (bf16 q, k,
    V', V'^2 operands and output)."""
    C = 64 * H
    q = rnd(B, H, Nc, 64, seed=1, dtype=dt)
    kv = rnd(B, H, Ns, 128, seed=2, dtype=dt)
    vt = ops.transpose_v(kv)
    ops.cosine_prep(q, kv)
    fcs = rnd(B, Nc, C, seed=3)
    mu = rnd(B, C, seed=4, scale=0.1)
    rs = rnd(B, C, seed=5).abs() + 0.5
    vmu = rnd(B, C, seed=6)
    mom = ops.cosine_moments(kv, vt)
    out = ops.cosine_attn(q, mom, fcs, mu, rs, vmu)
    flash = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, _lib.ACT_COSINE)
    torch.cuda.synchronize()
    # fp64 reference: A = (q^ k^T + 1) / rowsum, M = A V', E2 = A V'^2 (the operands as the kernels see them)
    qd, kd, vd = q.double(), kv[..., :64].double(), kv[..., 64:].double()
    a = torch.matmul(qd, kd.transpose(-1, -2)) + 1
    a = a / a.sum(-1, keepdim=True)
    m = torch.matmul(a, vd)
    e2 = torch.matmul(a, vd * vd)
    s = torch.sqrt((e2 - m * m).clamp(min=1e-6))
    x = (fcs.double().view(B, Nc, H, 64).permute(0, 2, 1, 3) - mu.double().view(B, H, 1, 64)) * \
        rs.double().view(B, H, 1, 64)
    ref = (s * x + m + vmu.double().view(B, H, 1, 64)).permute(0, 2, 1, 3).reshape(B, Nc, C)
    assert torch.isfinite(out.float()).all()
    assert rel(out, ref) < TOL[dt]
    assert rel(out, flash) < 2 * TOL[dt]
    # the style-side image: row 64 column 128 carries Ns, the padding columns are zero
    assert torch.all(mom[..., 64, 128] == Ns)
    assert torch.all(mom[..., :, 129:] == 0) and torch.all(mom[..., 64, :128].isfinite())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_mhada_online_softmax_rescale_branch(dt):
    """Force the running max to jump in a LATE key tile (cdna_hip_programming.md rule 26):
    one style token far out along the content direction dominates every query."""
    blk = _block("softmax", dt)
    B, hc, wc, hs, ws = 1, 16, 16, 16, 16
    fc = rnd(B, 512, hc, wc, seed=4)
    fs = rnd(B, 512, hs, ws, seed=5)
    fs[:, :, 15, 10] = 12.0  # token 250 of 256: in the last 64-key tile
    fcs = rnd(B, 512, hc, wc, seed=6)
    with torch.no_grad():
        y = blk(fc, fs, fcs)
    ref = _ref_block(blk, fc, fs, fcs, "softmax")
    assert torch.isfinite(y).all()
    # logits reach +-58 here: the fp32 PyTorch computation itself is 3.7e-5 off fp64, and bf16
    # Q/K carry ~0.2 absolute logit error; a wrong rescale at the jump would be O(1) off.
    import torch_ref
    sd32 = {k: v.float() for k, v in blk.state_dict().items()}
    with torch.no_grad():
        err32 = rel(torch_ref.block(fc, fs, fcs, sd32, ""), ref)
    assert rel(y, ref) < (max(1e-5, 2 * err32) if dt == torch.float32 else 5e-2)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs a second visible GPU")
def test_block_on_a_non_current_device():
    """Every launch runs under a device guard on its operands' device and that device's current
    stream (ops._call): a module moved to cuda:1 works while cuda:0 is current."""
    blk0 = _block("softmax", torch.float32)
    blk1 = _block("softmax", torch.float32).to("cuda:1")
    fc = rnd(2, 512, 9, 7, seed=21)
    fs = rnd(2, 512, 5, 6, seed=22)
    torch.cuda.set_device(0)
    with torch.no_grad():
        y0 = blk0(fc, fs, fc)
        y1 = blk1(fc.to("cuda:1"), fs.to("cuda:1"), fc.to("cuda:1"))
    assert y1.device == torch.device("cuda:1")
    assert torch.equal(y0.cpu(), y1.cpu())


def test_mhada_is_per_sample_independent():
    """Unlike the ViT (batch-axis attention), MHAda blocks are per-sample."""
    blk = _block("softmax", torch.float32)
    fc = rnd(3, 512, 12, 12, seed=7)
    fs = rnd(3, 512, 9, 9, seed=8)
    with torch.no_grad():
        y = blk(fc, fs, fc)
        y1 = blk(fc[1:2], fs[1:2], fc[1:2])
    assert rel(y[1:2], y1) < 1e-6


def _attn_ref(q, kv, fcs, mu, rstd, v_mu):
    """fp64 mhada_attn (include/mhada_hip.h): K carries log2(e), so the natural-unit logit is
    (q.k) * ln 2; out = sqrt(max(E[v'^2] - E[v']^2, 1e-6)) * (fcs - mu) * rstd + E[v'] + v_mu."""
    B, H, Nc, _ = q.shape
    qd, kd, vd = q.double(), kv[..., :64].double(), kv[..., 64:].double()
    a = torch.softmax(qd @ kd.transpose(-1, -2) * math.log(2.0), dim=-1)
    m = a @ vd
    e2 = a @ (vd * vd)
    s = torch.sqrt(torch.clamp(e2 - m * m, min=1e-6))
    out = s.permute(0, 2, 1, 3).reshape(B, Nc, H * 64)
    mm = m.permute(0, 2, 1, 3).reshape(B, Nc, H * 64)
    f = (fcs.double() - mu.double()[:, None]) * rstd.double()[:, None]
    return out * f + mm + v_mu.double()[:, None]


# bf16 softmax attention kernels (attn.hip), each pinned to its wave count (tuning attn_waves) so the
# named kernel runs whatever the grid size: "fsq1_8" / "fsq1_4" — the fixed-shift LDS-DMA kernel on
# 16x16x32 MFMAs at 8 / 4 waves (Ns % 128 == 0; ragged Ns takes the register-staged fixed-shift kernel
# "fs" at 8 waves and the online-max kernel at 4) — and the online-max kernel "w8" / "w4".
ATTN_VARIANTS = {"fsq1_8": dict(attn_fixed_shift=1, attn_waves=8), "fsq1_4": dict(attn_fixed_shift=1, attn_waves=4),
                 "w8": dict(attn_fixed_shift=0, attn_waves=8), "w4": dict(attn_fixed_shift=0, attn_waves=4)}


@pytest.mark.parametrize("kernel", list(ATTN_VARIANTS))
@pytest.mark.parametrize("Nc,Ns", [(300, 700), (256, 128), (97, 33), (256, 1024), (97, 384)])
def test_mhada_attn_late_max_jump(kernel, Nc, Ns):
    """A key far beyond the first tile's scores (> 2^64 in P against the first tile's max): the
    fixed-shift kernels must take their exact-recompute path, the online-max kernel ("w8") its
    rescale branch; all against fp64 torch on the same bf16 operands."""
    B, H = 1, 8
    q = rnd(B, H, Nc, 64, seed=11)
    q = q / q.norm(dim=-1, keepdim=True) * 4.0
    kv = rnd(B, H, Ns, 128, scale=0.1, seed=12)
    late = Ns - 5  # in the last key tile
    kv[:, :, late, :64] = 30.0 * q[:, :, : min(Nc, 1), :].mean(dim=2)  # ~120 log2 units above
    kv[:, :, late - 1, :64] = -kv[:, :, late, :64]
    q, kv = q.bfloat16(), kv.bfloat16()
    vt = ops.transpose_v(kv)
    fcs = rnd(B, Nc, 512, seed=13)
    mu, rs = ops.instnorm_stats(fcs)
    vmu = rnd(B, 512, seed=14)
    with _lib.tuning(**ATTN_VARIANTS[kernel]):
        y = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
    ref = _attn_ref(q.float(), kv.float(), fcs, mu, rs, vmu)
    assert torch.isfinite(y.float()).all()
    assert rel(y.float(), ref) < 1.5e-2


@pytest.mark.parametrize("kernel", list(ATTN_VARIANTS))
@pytest.mark.parametrize("B,Nc,Ns", [(1, 256, 64), (2, 300, 100), (1, 513, 128), (1, 97, 1000), (2, 1000, 777),
                                     (1, 64, 4096), (2, 300, 256), (1, 97, 384), (1, 520, 1024),
                                     (2, 5000, 256), (3, 3000, 128)])
def test_mhada_attn_bf16_tile_counts(kernel, B, Nc, Ns):
    """The bf16 softmax kernels (ATTN_VARIANTS) at 1..32 key tiles of 128, ragged and whole (1, 2,
    3 and 8 whole tiles exercise the pipelined kernels' prologue, odd tile counts and the 3-slot
    ring), partial query blocks, and more query blocks than CUs (the persistent kernel's block
    seams, with 1 and 2 tiles per block): against fp64 torch on the same bf16 operands (1e-2)."""
    H = 8
    q = (rnd(B, H, Nc, 64, seed=15) * 0.35).bfloat16()
    kv = (rnd(B, H, Ns, 128, seed=16) * 0.35).bfloat16()
    vt = ops.transpose_v(kv)
    fcs = rnd(B, Nc, 512, seed=17)
    mu, rs = ops.instnorm_stats(fcs)
    vmu = rnd(B, 512, seed=18)
    with _lib.tuning(**ATTN_VARIANTS[kernel]):
        y = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
    ref = _attn_ref(q.float(), kv.float(), fcs, mu, rs, vmu)
    assert rel(y.float(), ref) < 1e-2


@pytest.mark.parametrize("nz,M,N,K", [(3, 1000, 64, 4096), (2, 4096, 64, 96), (1, 333, 37, 64), (4, 77, 3, 32),
                                      (1, 98304, 64, 64), (8, 500, 64, 128), (16, 300, 61, 4096)])
def test_gemm_n64_ring_kernel(nz, M, N, K):
    """The fp32 N <= 64 LDS-DMA ring GEMM (the attention backward's dQ = dS K, the per-head 1x1
    convs): batched strided operands, bias, ReLU and residual epilogues against fp64, and against
    the register-staged tile it replaces (K % 32 != 0)."""
    a = rnd(nz, M, K + 4, seed=11)[..., :K]  # row stride K + 4 (16-B aligned, not dense)
    w = rnd(nz, N, K, scale=K ** -0.5, seed=12)
    b = rnd(N, seed=13)
    ldc = (N + 3) // 4 * 4
    r = rnd(nz, M, ldc, seed=14)
    args = dict(a=a, w=w, M=M, N=N, K=K, compute=torch.float32, lda=K + 4, sa=(M * (K + 4), 0), nb=(nz, 1),
                ldw=K, sw=(N * K, 0), ldc=ldc, sc=(M * ldc, 0))
    c = torch.zeros(nz, M, ldc, device=DEV)
    ops.gemm(c=c, bias=b, **args)
    ref = a.double() @ w.double().transpose(1, 2) + b.double()
    assert rel(c[..., :N], ref) < TOL[torch.float32]
    c2 = torch.zeros_like(c)
    ops.gemm(c=c2, bias=b, r=r, ldr=ldc, sr=(M * ldc, 0), relu=True, **args)
    assert rel(c2[..., :N], torch.relu(ref) + r[..., :N].double()) < TOL[torch.float32]
    # K % 32 != 0 (here K + 4) takes the register-staged tile the ring kernel replaces
    a1 = rnd(nz, M, K + 4, seed=11)
    w1 = rnd(nz, N, K + 4, scale=K ** -0.5, seed=15)
    c3 = torch.zeros_like(c)
    ops.gemm(c=c3, bias=b, **dict(args, a=a1, w=w1, K=K + 4, lda=K + 4, sa=(M * (K + 4), 0), ldw=K + 4,
                                  sw=(N * (K + 4), 0)))
    ref1 = a1.double() @ w1.double().transpose(1, 2) + b.double()
    assert rel(c3[..., :N], ref1) < TOL[torch.float32]


# ---- the fp32 MHAda attention as SPLIT3 products on the bf16 MFMA (attn_split3.hip, round 6) ---------
S3_WAVES = {"s3_8": dict(attn_waves=8), "s3_4": dict(attn_waves=4)}


def _f32_attn_operands(B, H, Nc, Ns, scale, seed):
    q = rnd(B, H, Nc, 64, seed=seed) * scale
    kv = rnd(B, H, Ns, 128, seed=seed + 1) * scale
    fcs = rnd(B, Nc, H * 64, seed=seed + 2)
    mu, rs = ops.instnorm_stats(fcs)
    vmu = rnd(B, H * 64, seed=seed + 3)
    return q, kv, fcs, mu, rs, vmu


@pytest.mark.parametrize("B,H,Ns", [(1, 1, 64), (2, 3, 100), (1, 2, 33), (2, 8, 1000), (1, 8, 4096)])
def test_split3_kv_planes_are_exact(B, H, Ns):
    """mhada_split3_kv: the three K planes sum to the fp32 K rows exactly (rows past Ns zero), the
    three V'^T | V'^2^T planes to the fp32 vt image exactly, with key positions permuted inside groups
    of 16 (bits 2 and 3 swapped, the bf16 vt image's order), and each plane is the round-to-nearest
    bf16 of what the planes before it leave."""
    kv = rnd(B, H, Ns, 128, seed=3) * 3
    vt = ops.transpose_v(kv)
    img = ops.split3_kv(kv, vt)
    ldt = (Ns + 63) // 64 * 64
    kp = img[..., :192 * ldt].view(B, H, 3, ldt, 64).double()
    vp = img[..., 192 * ldt:].view(B, H, 3, 128, ldt).double()
    ks = kp.sum(2)
    assert torch.equal(ks[:, :, :Ns], kv[..., :64].double())
    assert torch.all(ks[:, :, Ns:] == 0)
    assert torch.equal(kp[:, :, 0, :Ns], kv[..., :64].bfloat16().double())
    pos = torch.arange(ldt, device=DEV)
    key = (pos & ~12) | ((pos & 4) << 1) | ((pos & 8) >> 1)
    assert torch.equal(vp.sum(2), vt.double()[..., key])
    assert torch.equal(vp[:, :, 0], vt[..., key].bfloat16().double())
    r1 = vt[..., key].double() - vp[:, :, 0]
    assert torch.equal(vp[:, :, 1], r1.float().bfloat16().double())


@pytest.mark.parametrize("kernel", list(S3_WAVES))
@pytest.mark.parametrize("B,Nc,Ns,scale", [(1, 256, 64, 0.5), (2, 300, 100, 0.5), (1, 97, 33, 0.5), (1, 513, 128, 1.0),
                                           (2, 1000, 777, 0.5), (1, 64, 4096, 0.5), (1, 520, 1024, 1.0),
                                           (2, 4096, 4096, 0.35), (1, 3000, 192, 1.5)])
def test_attn_split3_fp32_accuracy(kernel, B, Nc, Ns, scale):
    """The SPLIT3 attention (mhada_attn_split3) against fp64 on the same fp32 operands, at one to 64
    key tiles of 64 (whole and ragged, Ns < 64), partial query blocks, 4- and 8-wave blocks, and logits
    from ~2 to ~18 in standard deviation: within the fp32 tolerance and at most 1.3x the fp32-MFMA
    kernel's error (mhada_attn, attn_f32_kernel) on the same operands; run-to-run bit-identical.
    Measured (profiles/r06_gpu_tests_s3.log): 0.5-0.8x the fp32 kernel's error at logit std <= 4
    (the bench shapes), up to 1.23x at std 8-18 — the bf16 MFMA sums its 32 products with truncating
    partial sums (tools/split3_mfma_emulation.py), which weighs on large cancelling logits."""
    H = 8
    q, kv, fcs, mu, rs, vmu = _f32_attn_operands(B, H, Nc, Ns, scale, seed=31)
    vt = ops.transpose_v(kv)
    img = ops.split3_kv(kv, vt)
    with _lib.tuning(**S3_WAVES[kernel]):
        y = ops.attn_split3(q, img, Ns, fcs, mu, rs, vmu)
        y2 = ops.attn_split3(q, img, Ns, fcs, mu, rs, vmu)
    assert torch.equal(y, y2)
    y32 = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
    ref = _attn_ref(q, kv, fcs, mu, rs, vmu)
    e_s3, e_32 = rel(y, ref), rel(y32, ref)
    assert e_s3 < TOL[torch.float32], (e_s3, e_32)
    assert e_s3 <= 1.3 * e_32 + 1e-8, (e_s3, e_32)


@pytest.mark.parametrize("kernel", list(S3_WAVES))
@pytest.mark.parametrize("Nc,Ns", [(300, 700), (256, 128), (97, 33), (256, 1024), (97, 384)])
def test_attn_split3_late_max_jump(kernel, Nc, Ns):
    """A key ~120 log2 units above the first tile's scores: the fixed-shift SPLIT3 kernel must take its
    exact recompute (attn_exact_q3); against fp64 within 1e-5 and 3x the fp32-MFMA kernel's error (whose
    online max handles the jump by its rescale branch).  This case is adversarial for the bf16 MFMA:
    the late key is 30x a query, so its logits (+-60 log2 units) are sums of large cancelling
    products, and the MFMA's truncating 32-product partial sums cost up to 2.6x the fp32 kernel's
    error here (measured; reproduced by tools/split3_mfma_emulation.py, whose exactly-rounded model
    of the same SPLIT3 algorithm lands below the fp32 kernel)."""
    B, H = 1, 8
    q = rnd(B, H, Nc, 64, seed=11)
    q = q / q.norm(dim=-1, keepdim=True) * 4.0
    kv = rnd(B, H, Ns, 128, scale=0.1, seed=12)
    late = Ns - 5
    kv[:, :, late, :64] = 30.0 * q[:, :, : min(Nc, 1), :].mean(dim=2)
    kv[:, :, late - 1, :64] = -kv[:, :, late, :64]
    vt = ops.transpose_v(kv)
    fcs = rnd(B, Nc, 512, seed=13)
    mu, rs = ops.instnorm_stats(fcs)
    vmu = rnd(B, 512, seed=14)
    img = ops.split3_kv(kv, vt)
    with _lib.tuning(**S3_WAVES[kernel]):
        y = ops.attn_split3(q, img, Ns, fcs, mu, rs, vmu)
    y32 = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
    ref = _attn_ref(q, kv, fcs, mu, rs, vmu)
    assert torch.isfinite(y).all()
    e_s3, e_32 = rel(y, ref), rel(y32, ref)
    assert e_s3 < 1e-5 and e_s3 <= 3.0 * e_32 + 1e-8, (e_s3, e_32)


def test_attn_split3_rejects_bad_operands():
    q, kv, fcs, mu, rs, vmu = _f32_attn_operands(1, 2, 64, 100, 0.5, seed=1)
    vt = ops.transpose_v(kv)
    img = ops.split3_kv(kv, vt)
    with pytest.raises(ValueError):
        ops.attn_split3(q, img, 200, fcs, mu, rs, vmu)  # image of another Ns
    with pytest.raises(ValueError):
        ops.attn_split3(q.bfloat16(), img, 100, fcs, mu, rs, vmu)
    with pytest.raises(ValueError):
        ops.split3_kv(kv.bfloat16(), ops.transpose_v(kv.bfloat16()))


@pytest.mark.parametrize("B,H,Ns", [(1, 8, 64), (2, 8, 100), (1, 2, 33), (2, 8, 4096), (1, 8, 1000)])
def test_kv_proj_split3_matches_projection_then_split(B, H, Ns):
    """mhada_kv_proj_split3 (the K|V' projection written straight as the SPLIT3 plane image) against
    fp64 and against the fp32 projection GEMM with its vt epilogue followed by mhada_split3_kv: the
    plane sums agree to fp32 rounding (the two fp32 MFMA reductions differ in order only), keys past Ns
    are zero in both."""
    C = 64 * H
    fs = rnd(B, Ns, C, seed=1) * 2 + 0.3
    mu = fs.mean(1)
    w = rnd(B, H, 128, 64, scale=0.125, seed=2)
    bkv = rnd(H, 128, seed=3)
    bkv[:, 64:] = 0
    img = ops.kv_proj_split3(fs, mu, w, bkv)
    ldt = (Ns + 63) // 64 * 64
    kv = torch.empty(B, H, Ns, 128, device=DEV)
    vt = torch.empty(B, H, 128, ldt, device=DEV)
    ops.gemm(a=fs, w=w, c=kv, M=Ns, N=128, K=64, compute=torch.float32, lda=C, sa=(Ns * C, 64), nb=(B, H), a_mu=mu,
             smu=(C, 64), ldw=64, sw=(H * 128 * 64, 128 * 64), bias=bkv, sb=(0, 128), ldc=128,
             sc=(H * Ns * 128, Ns * 128), vt=vt, ldt=ldt, svt=(H * 128 * ldt, 128 * ldt))
    ref = ops.split3_kv(kv, vt)

    def sums(im):
        kp = im[..., :192 * ldt].view(B, H, 3, ldt, 64).double().sum(2)
        vp = im[..., 192 * ldt:].view(B, H, 3, 128, ldt).double().sum(2)
        return kp, vp
    (k1, v1), (k2, v2) = sums(img), sums(ref)
    pos = torch.arange(ldt, device=DEV)
    key = (pos & ~12) | ((pos & 4) << 1) | ((pos & 8) >> 1)  # the key at each (permuted) position
    assert torch.all(k1[:, :, Ns:] == 0) and torch.all(v1[..., key >= Ns] == 0)
    assert rel(k1, k2) < 1e-6 and rel(v1, v2) < 1e-6
    y = torch.einsum("bnhc,bhoc->bhno", (fs.double() - mu.double()[:, None]).view(B, Ns, H, 64), w.double()) + \
        bkv.double()[None, :, None, :]
    assert rel(k1[:, :, :Ns], y[..., :64]) < 1e-6
    vref = torch.zeros(B, H, 128, ldt, device=DEV, dtype=torch.float64)
    vref[..., :Ns] = torch.cat([y[..., 64:], y[..., 64:] ** 2], -1).transpose(-1, -2)
    assert rel(v1, vref[..., key]) < 2e-6
