"""Training attention kernels (csrc/attn_train.hip) against fp64 PyTorch autograd of the
reference formula (adaDecoder.py:186-198), and the fused block against the plain-autograd block.

Tolerances: fp32 MFMA (exact fp32 products, fp32 accumulation) vs fp64 — relative max error
of outputs < 2e-4 of the tensor's max magnitude; of gradients < max(2e-4, 4x the error of the
reference's own fp32 autograd on the same inputs) — peaky softmaxes (logit std 12) lose digits
in dS = P (dA - D) in any fp32 evaluation: over four seeds of each shape both training forwards
(SPLIT3 and the fp32-MFMA one, sharing the backward) land 1-5x the yardstick at logit std >= 12,
neither systematically ahead (tools/train_attn_err.py, profiles/r06_train_attn_err.log)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

import network
from mhada_hip import autograd_path, ops
from mhada_hip.recipe import load_recipe


def _ref(q, k, v, x):
    """adaDecoder.py:186-198 on centred v (v passed already centred)."""
    a = torch.softmax(q @ k.transpose(1, 2), dim=-1)
    m = a @ v
    e2 = a @ (v * v)
    s = torch.sqrt((e2 - m * m).clamp(min=1e-6))
    return s * x + m


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-30)).item()


@pytest.mark.parametrize("dq", ["s3", "f32"])
@pytest.mark.parametrize("form", ["s3", "vt"])
@pytest.mark.parametrize("BH,Nc,Ns,scale", [(2, 128, 64, 0.4), (3, 100, 70, 0.4), (1, 37, 300, 0.6),
                                            (2, 256, 129, 1.5), (2, 200, 160, 1.0)])
def test_attn_train_fwd_bwd_vs_fp64(monkeypatch, dq, form, BH, Nc, Ns, scale):
    """Forward + backward through MHAdaAttnFn for both training forwards and both dQ GEMMs (the SPLIT3
    one takes Ns % 32 == 0: Ns = 64, 160 here; the others fall back to the fp32 GEMM either way)."""
    monkeypatch.setattr(ops, "TRAIN_FWD_S3", form == "s3")
    monkeypatch.setattr(ops, "TRAIN_FWD_VT", True)
    monkeypatch.setattr(ops, "TRAIN_DQ_S3", dq == "s3")
    g = torch.Generator().manual_seed(Nc * 7 + Ns)
    q = torch.randn(BH, Nc, 64, generator=g) * scale
    k = torch.randn(BH, Ns, 64, generator=g) * scale
    v = torch.randn(BH, Ns, 64, generator=g) * 3
    v = v - v.mean(dim=1, keepdim=True)
    x = torch.randn(BH, Nc, 64, generator=g)
    dout = torch.randn(BH, Nc, 64, generator=g)
    ts = [t.double().requires_grad_() for t in (q, k, v, x)]
    ref = _ref(*ts)
    ref.backward(dout.double())
    gs = [t.cuda().contiguous().requires_grad_() for t in (q, k, v, x)]
    out = autograd_path.MHAdaAttnFn.apply(*gs)
    out.backward(dout.cuda())
    # yardstick: the reference's own fp32 autograd (materialised A) on the same device
    fs = [t.cuda().contiguous().requires_grad_() for t in (q, k, v, x)]
    out32 = _ref(*fs)
    out32.backward(dout.cuda())
    torch.cuda.synchronize()
    assert _rel(out.double().cpu(), ref.detach()) < max(2e-4, 2 * _rel(out32.double().cpu(), ref.detach()))
    for name, a, b, c in zip("qkvx", gs, ts, fs):
        err = _rel(a.grad.double().cpu(), b.grad)
        err32 = _rel(c.grad.double().cpu(), b.grad)
        assert err < max(2e-4, 4 * err32), (name, err, err32)


def test_attn_train_bwd_with_clamped_variance():
    """Channels whose attention-weighted variance is below the 1e-6 clamp (constant V' there): the
    clamp's gradient is zero in those channels (mhada_attn_train_bwd_prep), as in fp64 autograd."""
    g = torch.Generator().manual_seed(5)
    BH, Nc, Ns = 2, 128, 96
    q = torch.randn(BH, Nc, 64, generator=g) * 0.4
    k = torch.randn(BH, Ns, 64, generator=g) * 0.4
    v = torch.randn(BH, Ns, 64, generator=g) * 3
    v = v - v.mean(dim=1, keepdim=True)
    v[:, :, :5] = 0.0  # var = 0 < 1e-6: the clamp is active in channels 0-4
    x = torch.randn(BH, Nc, 64, generator=g)
    dout = torch.randn(BH, Nc, 64, generator=g)
    ts = [t.double().requires_grad_() for t in (q, k, v, x)]
    _ref(*ts).backward(dout.double())
    gs = [t.cuda().contiguous().requires_grad_() for t in (q, k, v, x)]
    autograd_path.MHAdaAttnFn.apply(*gs).backward(dout.cuda())
    for name, a, b in zip("qkvx", gs, ts):
        assert _rel(a.grad.double().cpu(), b.grad) < 2e-4, name


@pytest.mark.parametrize("BH,Nc,Ns", [(2, 128, 64), (1, 37, 300), (3, 500, 256), (2, 33, 4)])
def test_attn_train_bwd_ds_spill_matches_recompute(BH, Nc, Ns):
    """dS spilled by the dK/dV' kernel + dQ = dS K as a batched GEMM (ops.attn_train_bwd's default)
    against the recompute path (query-stationary dQ kernel): dK, dV' bit-identical (same kernel,
    same order), dQ to fp32 summation order."""
    g = torch.Generator().manual_seed(BH * 1000 + Nc + Ns)
    q, k, v = (torch.randn(BH, n, 64, generator=g).cuda() * 0.5 for n in (Nc, Ns, Ns))
    v = (v - v.mean(dim=1, keepdim=True)).contiguous()
    x = torch.randn(BH, Nc, 64, generator=g).cuda()
    out, mo, lse = ops.attn_train_fwd(q, k, v, x)
    dmo = torch.randn(BH, Nc, 128, generator=g).cuda()
    dd = (dmo * mo).sum(-1).contiguous()
    a = ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=True)
    b = ops.attn_train_bwd(q, k, v, lse, dmo, dd, spill=False)
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert _rel(a[0].double(), b[0].double()) < 1e-5


@pytest.mark.parametrize("BH,Nc,Ns", [(2, 128, 64), (1, 37, 300), (3, 500, 256), (2, 33, 4), (1, 64, 128), (2, 161, 96)])
def test_attn_train_dkv_dma_kernel_matches_register_staged(BH, Nc, Ns):
    """The LDS-DMA / software-pipelined dK / dV' kernel (tuning train_dkv_dma = 1, the default) against
    the round-3 register-staged kernel: the same products in the same order, so dK, dV' and the
    spilled dS are bit-identical (1..16 query tiles, ragged Nc: padded query rows must give P = 0)."""
    from mhada_hip import _lib
    g = torch.Generator().manual_seed(BH * 31 + Nc + Ns)
    q, k, v = (torch.randn(BH, n, 64, generator=g).cuda() * 0.5 for n in (Nc, Ns, Ns))
    v = (v - v.mean(dim=1, keepdim=True)).contiguous()
    out, mo, lse = ops.attn_train_fwd(q, k, v, torch.randn(BH, Nc, 64, generator=g).cuda())
    dmo = torch.randn(BH, Nc, 128, generator=g).cuda()
    dd = (dmo * mo).sum(-1).contiguous()
    lib = _lib.load()
    res = []
    for dma in (0, 1):
        dk, dv = torch.empty_like(k), torch.empty_like(v)
        ds = torch.full((BH, Nc, Ns), float("nan"), device="cuda")
        with _lib.tuning(train_dkv_dma=dma):
            rc = lib.mhada_attn_train_dkv(q.data_ptr(), k.data_ptr(), v.data_ptr(), lse.data_ptr(), dmo.data_ptr(),
                                          dd.data_ptr(), dk.data_ptr(), dv.data_ptr(), ds.data_ptr(), BH, Nc, Ns,
                                          torch.cuda.current_stream().cuda_stream)
        assert rc == 0, lib.mhada_last_error()
        torch.cuda.synchronize()
        res.append((dk, dv, ds))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert torch.isfinite(res[1][2]).all()  # every dS element written


def test_attn_train_bwd_default_path_is_shape_determined(monkeypatch):
    """the spill / recompute choice depends on shapes and ops.DS_SPILL_BYTES only (not
    on free memory), is recorded in ops.BWD_PATH_COUNTS, and repeated calls give the same bits."""
    g = torch.Generator().manual_seed(9)
    BH, Nc, Ns = 2, 96, 64
    q, k, v = (torch.randn(BH, n, 64, generator=g).cuda() * 0.5 for n in (Nc, Ns, Ns))
    v = (v - v.mean(dim=1, keepdim=True)).contiguous()
    out, mo, lse = ops.attn_train_fwd(q, k, v, torch.randn(BH, Nc, 64, generator=g).cuda())
    dmo = torch.randn(BH, Nc, 128, generator=g).cuda()
    dd = (dmo * mo).sum(-1).contiguous()
    res = {}
    for budget, path in ((ops.DS_SPILL_BYTES, "spill"), (4 * BH * Nc * Ns - 1, "recompute")):
        monkeypatch.setattr(ops, "DS_SPILL_BYTES", budget)
        assert ops.ds_spill_eligible(BH, Nc, Ns) == (path == "spill")
        before = dict(ops.BWD_PATH_COUNTS)
        a = ops.attn_train_bwd(q, k, v, lse, dmo, dd)
        b = ops.attn_train_bwd(q, k, v, lse, dmo, dd)
        assert ops.BWD_PATH_COUNTS[path] == before[path] + 2
        assert all(torch.equal(x, y) for x, y in zip(a, b))
        res[path] = a
    assert torch.equal(res["spill"][1], res["recompute"][1]) and torch.equal(res["spill"][2], res["recompute"][2])


def test_attn_train_lse_and_stats():
    g = torch.Generator().manual_seed(5)
    q, x = torch.randn(2, 96, 64, generator=g), torch.randn(2, 96, 64, generator=g)
    k, v = torch.randn(2, 80, 64, generator=g), torch.randn(2, 80, 64, generator=g)
    out, mo, lse = ops.attn_train_fwd(*(t.cuda() for t in (q, k, v, x)))
    s = (q @ k.transpose(1, 2)).double()
    assert torch.allclose(lse.double().cpu(), torch.logsumexp(s, -1) / torch.log(torch.tensor(2.0, dtype=torch.float64)),
                          atol=1e-4, rtol=1e-5)
    a = torch.softmax(s, -1)
    assert _rel(mo[..., :64].double().cpu(), a @ v.double()) < 1e-5
    assert _rel(mo[..., 64:].double().cpu(), a @ (v.double() ** 2)) < 1e-5


def test_fused_block_grads_match_autograd_block():
    torch.manual_seed(0)
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").cuda()
    blk = ada.adaAttnHead[0]
    fc = (torch.randn(2, 512, 12, 10, device="cuda") * 2).requires_grad_()
    fs = (torch.randn(2, 512, 9, 11, device="cuda") * 2).requires_grad_()
    fcs = (torch.randn(2, 512, 12, 10, device="cuda") * 2).requires_grad_()
    dout = torch.randn(2, 512, 12, 10, device="cuda")
    results = []
    for mode in ("hip", "torch"):
        autograd_path.TRAIN_ATTN = mode
        try:
            for t in (fc, fs, fcs, *blk.parameters()):
                t.grad = None
            y = autograd_path.block_forward(blk, fc, fs, fcs)
            y.backward(dout)
            results.append([y.detach().clone()] + [t.grad.clone() for t in (fc, fs, fcs, *blk.parameters())])
        finally:
            autograd_path.TRAIN_ATTN = "hip"
    # K-bias gradients are zero in exact arithmetic (a per-query constant logit shift): those
    # are held to an absolute floor of 1e-5 of the largest gradient
    gmax = max(b.abs().max().item() for b in results[1])
    for i, (a, b) in enumerate(zip(*results)):
        err = (a.double() - b.double()).abs().max().item()
        assert err <= max(1e-3 * b.abs().max().item(), 1e-5 * gmax), (i, err)


def test_fused_block_under_autocast_runs_fp32_kernels():
    """Training under torch.autocast(bf16): the HIP training ops cast their operands to fp32
    (custom_fwd), so the fused block runs and matches its fp32 result (the bf16
    projection outputs used to crash the fp32-only kernels)."""
    blk = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").cuda().adaAttnHead[0]
    g = torch.Generator().manual_seed(5)
    fc, fs, fcs = (torch.randn(2, 512, 8, 8, generator=g).cuda().requires_grad_() for _ in range(3))
    ys = []
    for amp in (False, True):
        for t in (fc, fs, fcs, *blk.parameters()):
            t.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = autograd_path.block_forward(blk, fc, fs, fcs)
        y.float().sum().backward()
        ys.append((y.detach().float(), fc.grad.clone()))
    assert torch.isfinite(ys[1][0]).all() and torch.isfinite(ys[1][1]).all()
    assert _rel(ys[1][0].double(), ys[0][0].double()) < 5e-2
    assert _rel(ys[1][1].double(), ys[0][1].double()) < 5e-2


@pytest.mark.parametrize("form", ["s3", "vt", "r1"])
@pytest.mark.parametrize("BH,Nc,Ns,scale", [(2, 300, 700, 0.5), (3, 97, 33, 1.0), (1, 512, 4096, 0.35),
                                            (2, 256, 130, 2.5), (2, 600, 1000, 3.0)])
def test_attn_train_fwd_kernels_vs_fp64(monkeypatch, form, BH, Nc, Ns, scale):
    """The three training forwards — mhada_attn_train_fwd_split3 (SPLIT3 products on the bf16 MFMA,
    fixed-shift softmax with the exact recompute, the default), mhada_attn_train_fwd_vt (the inference
    fp32 structure: 64-key tiles, lazy rescale, V'^T | V'^2^T image) and the round-1
    mhada_attn_train_fwd — against fp64: out', [M' | E2'] and lse2 (exact whether the running max is
    rescaled lazily or fixed to the first tile's), ragged key tiles, peaky logits (scale 2.5 / 3: the
    max moves late and by a lot — for the fixed shift past 2^64, so rows are recomputed exactly)."""
    monkeypatch.setattr(ops, "TRAIN_FWD_S3", form == "s3")
    monkeypatch.setattr(ops, "TRAIN_FWD_VT", form == "vt")
    g = torch.Generator().manual_seed(BH * 100 + Ns)
    q = torch.randn(BH, Nc, 64, generator=g) * scale
    k = torch.randn(BH, Ns, 64, generator=g) * scale
    v = torch.randn(BH, Ns, 64, generator=g) * 2
    v = v - v.mean(dim=1, keepdim=True)
    x = torch.randn(BH, Nc, 64, generator=g)
    out, mo, lse = ops.attn_train_fwd(*(t.cuda().contiguous() for t in (q, k, v, x)))
    qd, kd, vd = q.double(), k.double(), v.double()
    s = qd @ kd.transpose(1, 2)
    a = torch.softmax(s, -1)
    assert torch.allclose(lse.double().cpu(), torch.logsumexp(s, -1) / torch.log(torch.tensor(2.0, dtype=torch.float64)),
                          atol=2e-4, rtol=1e-5)
    # M', E2': 2e-5, or 2x the error of the same expressions evaluated in fp32 by torch (at logit std
    # 72, scale 3, an fp32 S is off by ~1e-5 in log2 units and P by as much relative, in any fp32 form)
    a32 = torch.softmax(q @ k.transpose(1, 2), -1)
    for sl, ref64, ref32 in ((slice(0, 64), a @ vd, a32 @ v), (slice(64, 128), a @ vd ** 2, a32 @ (v * v))):
        assert _rel(mo[..., sl].double().cpu(), ref64) < max(2e-5, 2 * _rel(ref32.double(), ref64))
    # out' = sqrt(E2' - M'^2) x + M' cancels where the variance is small: held to the error of the
    # reference expression's own fp32 evaluation on the same inputs (x4), with a 2e-4 floor
    ref = _ref(qd, kd, vd, x.double())
    err32 = _rel(_ref(q, k, v, x).double(), ref)
    assert _rel(out.double().cpu(), ref) < max(2e-4, 4 * err32)


@pytest.mark.parametrize("BH,N", [(3, 300), (2, 64), (1, 4096), (4, 7)])
def test_transpose64_is_the_exact_transpose(BH, N):
    """mhada_transpose64 (K^T for the dS-spill dQ GEMM): [BH][N][64] -> [BH][64][ceil64(N)], the
    transpose bit for bit, the padding columns zero."""
    x = torch.randn(BH, N, 64, generator=torch.Generator().manual_seed(N)).cuda()
    t = ops.transpose64(x)
    ldt = (N + 63) // 64 * 64
    assert t.shape == (BH, 64, ldt)
    assert torch.equal(t[..., :N], x.transpose(1, 2))
    assert bool((t[..., N:] == 0).all())


@pytest.mark.parametrize("BH,Nc,Ns,scale", [(2, 300, 128, 1.0), (8, 256, 1024, 1.0), (3, 1000, 96, 30.0),
                                            (1, 37, 32, 1.0), (16, 520, 4096, 0.01)])
def test_dq_split3_vs_fp64(monkeypatch, BH, Nc, Ns, scale):
    """dQ = dS K of the dS-spill backward on the SPLIT3 GEMM (mhada_gemm_n64_split3: dS split into bf16
    planes in registers, K^T as planes, 6 cross products per K-tile summed from zero and added in fp32)
    against fp64 and against the fp32-MFMA N <= 64 GEMM it replaces: ragged row tiles, 1 .. 128
    K-tiles, problem counts with and without the per-XCD grouping (BH % 8), dS of mixed sign and
    magnitude (as P (dA - D) is)."""
    g = torch.Generator().manual_seed(BH * 7 + Nc + Ns)
    ds = (torch.randn(BH, Nc, Ns, generator=g) * torch.rand(BH, Nc, 1, generator=g) * scale).cuda()
    k = torch.randn(BH, Ns, 64, generator=g).cuda()
    ref = ds.double() @ k.double()
    kt = ops.transpose64(k)
    ldt = kt.shape[-1]
    dq = torch.full((BH, Nc, 64), float("nan"), device="cuda")
    ops.gemm_n64_split3(ds, ops.split3_rows(kt.view(BH * 64, ldt)), dq, BH, Nc, Ns, ldt)
    dq32 = torch.empty_like(dq)
    ops.gemm(a=ds, w=kt, c=dq32, M=Nc, N=64, K=Ns, compute=torch.float32, lda=Ns, sa=(Nc * Ns, 0), nb=(BH, 1),
             ldw=ldt, sw=(64 * ldt, 0), ldc=64, sc=(Nc * 64, 0))
    torch.cuda.synchronize()
    assert torch.isfinite(dq).all()
    e3, e32 = _rel(dq.double(), ref), _rel(dq32.double(), ref)
    assert e3 < 2e-6 and e3 <= 1.5 * e32 + 1e-8, (e3, e32)


@pytest.mark.parametrize("BH,N", [(3, 300), (2, 64), (1, 4096), (4, 7)])
def test_transpose64_split3_is_split_of_transpose(BH, N):
    """mhada_transpose64_split3 (the SPLIT3 dQ GEMM's W operand in one pass) = split3_rows of
    mhada_transpose64 bit for bit, padding columns zero in every plane."""
    x = torch.randn(BH, N, 64, generator=torch.Generator().manual_seed(N + 1)).cuda()
    kt = ops.transpose64(x)
    ldt = kt.shape[-1]
    assert torch.equal(ops.transpose64_split3(x), ops.split3_rows(kt.view(BH * 64, ldt)))
