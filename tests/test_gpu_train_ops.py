"""Training-path HIP kernels (csrc/train_ops.hip + the CONV3X3_ZERO gather of gemm.hip) through
their autograd Functions (mhada_hip/train_fns.py), each against PyTorch fp64 autograd of the same
reference expression: the decoder's ReflectionPad2d(1) + conv3x3 + ReLU (conv.py:23-45), VGG19's
zero-padded conv + ReLU and MaxPool2d(2) (vgg19.py, cfg E), the bilinear x2 upsample (conv.py:71)
and imageNet1k_normalize (vgg19.py:6-12).  fp32 kernels vs fp64: relative L2 < 1e-5."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from mhada_hip import ops, train_fns
from mhada_hip._lib import A_ROWS

DEV = "cuda"


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


@pytest.mark.parametrize("M,N,K", [(64, 576, 5000), (512, 2048, 333), (3, 128, 700), (130, 260, 64)])
def test_gemm_tn_rows(M, N, K):
    a = rnd(K, M, seed=1)
    b = rnd(K, N, seed=2)
    c = ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=N, b_mode=A_ROWS)
    ref = a.double().T @ b.double()
    assert rel(c, ref) < 1e-5
    # deterministic: same bits on a second call
    assert torch.equal(c, ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=N, b_mode=A_ROWS))


@pytest.mark.parametrize("M,N,K", [(64, 576, 5000), (512, 2048, 333), (4, 128, 700), (132, 260, 64), (128, 64, 70000)])
def test_gemm_tn_fused_colsum(M, N, K):
    """The bias gradient from the TN GEMM's own A staging (mhada_gemm_tn_args.colsum): the column
    sums of A against fp64, the GEMM unchanged by it, bits stable across calls (split-K slabs and
    the per-tile partials are summed in a fixed order).  M = 4 takes the unfused fallback."""
    a = rnd(K, M, seed=3)
    b = rnd(K, N, seed=4)
    c, cs = ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=N, b_mode=A_ROWS, colsum=True)
    assert rel(c, a.double().T @ b.double()) < 1e-5
    assert rel(cs, a.double().sum(0)) < 1e-6
    assert torch.equal(c, ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=N, b_mode=A_ROWS))
    c2, cs2 = ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=N, b_mode=A_ROWS, colsum=True)
    assert torch.equal(c, c2) and torch.equal(cs, cs2)


@pytest.mark.parametrize("nb,M,N,K", [(8, 64, 64, 9000), (3, 128, 256, 700)])
def test_gemm_tn_batched(nb, M, N, K):
    """The batched TN form (HeadProjFn's per-head weight gradients in one launch): head i uses
    A = a[i] and B = the column block b[:, N i:], exactly the per-problem results (bits), and the
    column sums."""
    a = rnd(nb, K, M, seed=5)
    b = rnd(K, nb * N, seed=6)
    c, cs = ops.gemm_tn(a, b, M=M, N=N, K=K, lda=M, ldb=nb * N, b_mode=A_ROWS, colsum=True, nb=nb,
                        sza=K * M, szb=N)
    for i in range(nb):
        ci, csi = ops.gemm_tn(a[i], b[:, N * i:], M=M, N=N, K=K, lda=M, ldb=nb * N, b_mode=A_ROWS, colsum=True)
        assert rel(c[i], a[i].double().T @ b[:, N * i:N * (i + 1)].double()) < 1e-5
        assert rel(cs[i], a[i].double().sum(0)) < 1e-6
        assert rel(c[i], ci) < 1e-6 and rel(cs[i], csi) < 1e-6


@pytest.mark.parametrize("rows,C", [(100000, 64), (37, 2048), (4096, 3 * 4)])
def test_colsum(rows, C):
    x = rnd(rows, C, seed=3)
    assert rel(ops.colsum(x), x.double().sum(0)) < 1e-6


def _conv_ref(x_nhwc, w, b, pad_mode, relu):
    x = x_nhwc.permute(0, 3, 1, 2)
    if pad_mode == "reflect":
        y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w, b)
    else:
        y = F.conv2d(x, w, b, padding=1)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("pad_mode", ["reflect", "zero"])
@pytest.mark.parametrize("B,H,W,Ci,Co,cx", [(2, 9, 13, 64, 64, 64), (1, 16, 16, 128, 256, 128), (2, 8, 6, 3, 64, 32),
                                          (1, 20, 17, 64, 3, 64), (2, 3, 5, 32, 32, 32), (1, 32, 32, 512, 256, 512)])
def test_conv3x3_fwd_bwd(pad_mode, B, H, W, Ci, Co, cx):
    x = rnd(B, H, W, cx, seed=H * W)
    if cx > Ci:
        x[..., Ci:] = 0  # VGG's padded input channels are zero
    w = rnd(Co, Ci, 3, 3, seed=2, scale=(9 * Ci) ** -0.5)
    b = rnd(Co, seed=3, scale=0.1)
    gy = rnd(B, H, W, Co, seed=4)
    conv = torch.nn.Conv2d(Ci, Co, 3).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(w)
        conv.bias.copy_(b)
    xg = x.clone().requires_grad_(True)
    y = train_fns.conv3x3(xg, conv, pad_mode, relu=True)
    y.backward(gy)
    x64 = x[..., :Ci].double().requires_grad_(True)  # the reference conv sees the Ci real channels
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    ref = _conv_ref(x64, w64, b64, pad_mode, True)
    ref.backward(gy.double())
    assert rel(y, ref) < 1e-5
    assert rel(xg.grad[..., :Ci], x64.grad) < 1e-5
    assert rel(conv.weight.grad, w64.grad) < 1e-5
    assert rel(conv.bias.grad, b64.grad) < 1e-5


@pytest.mark.parametrize("pad_mode", ["reflect", "zero"])
@pytest.mark.parametrize("B,H,W,C", [(2, 12, 10, 64), (1, 7, 9, 128)])
def test_conv_chain_relu_adjoint_folded_into_dgrad(pad_mode, B, H, W, C):
    """conv a -> ReLU -> conv b with a's ReLU adjoint folded into b's input gradient (Conv3x3Fn
    grad_masked on a, relu_input on b: the Winograd dgrad's output stage / the reflect fold zero
    it where a's output is <= 0) gives the bits of the unfolded chain (relu_bwd pass in a)."""
    x = rnd(B, H, W, C, seed=41)
    convs = []
    for i in range(2):
        conv = torch.nn.Conv2d(C, C, 3).to(DEV)
        with torch.no_grad():
            conv.weight.copy_(rnd(C, C, 3, 3, seed=42 + i, scale=(9 * C) ** -0.5))
            conv.bias.copy_(rnd(C, seed=44 + i, scale=0.1))
        convs.append(conv)
    gy = rnd(B, H, W, C, seed=46)
    grads = []
    for fold in (False, True):
        xg = x.clone().requires_grad_(True)
        h = train_fns.conv3x3(xg, convs[0], pad_mode, relu=True, grad_masked=fold)
        y = train_fns.conv3x3(h, convs[1], pad_mode, relu=True, relu_input=fold)
        for c in convs:
            c.weight.grad = c.bias.grad = None
        y.backward(gy)
        grads.append([xg.grad] + [t.grad.clone() for c in convs for t in (c.weight, c.bias)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_maxpool2_fwd_bwd_with_ties():
    # post-ReLU activations: many zeros, so the first-maximum rule decides most windows
    x = F.relu(rnd(2, 16, 18, 64, seed=5))
    x[0, 0:2, 0:2, :] = 1.5  # a window of four equal maxima
    gy = rnd(2, 8, 9, 64, seed=6)
    xg = x.clone().requires_grad_(True)
    y = train_fns.MaxPool2Fn.apply(xg)
    y.backward(gy)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    yr.backward(gy.permute(0, 3, 1, 2))
    assert torch.equal(y, yr.permute(0, 2, 3, 1))
    assert torch.equal(xg.grad, xr.grad.permute(0, 2, 3, 1))


def test_maxpool2_bwd_with_relu_mask_equals_relu_adjoint_after_pool_adjoint():
    """MaxPool2Fn(relu_input=True): the pool adjoint with the producing ReLU's adjoint applied
    (bits of relu_bwd(maxpool2_bwd(g), x)), odd sizes included."""
    for H, W in ((16, 18), (7, 9)):
        x = F.relu(rnd(2, H, W, 64, seed=31))
        gy = rnd(2, H // 2, W // 2, 64, seed=32)
        ref = ops.relu_bwd(ops.maxpool2_bwd(x, gy), x)
        assert torch.equal(ops.maxpool2_bwd(x, gy, relu_mask=True), ref)
        xg = x.clone().requires_grad_(True)
        train_fns.MaxPool2Fn.apply(xg, True).backward(gy)
        assert torch.equal(xg.grad, ref)


@pytest.mark.parametrize("H,W", [(8, 8), (5, 7), (1, 3), (64, 32)])
def test_upsample2x_adjoint(H, W):
    x = rnd(2, H, W, 64, seed=7)
    gy = rnd(2, 2 * H, 2 * W, 64, seed=8)
    xg = x.clone().requires_grad_(True)
    y = train_fns.Upsample2xFn.apply(xg)
    y.backward(gy)
    x64 = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    r = F.interpolate(x64, scale_factor=2, mode="bilinear", align_corners=False)
    r.backward(gy.double().permute(0, 3, 1, 2))
    assert rel(y, r.permute(0, 2, 3, 1)) < 1e-6
    assert rel(xg.grad, x64.grad.permute(0, 2, 3, 1)) < 1e-6
    xr = F.relu(x)  # relu_input: the producing ReLU's adjoint folded in, bits of relu_bwd after it
    xrg = xr.clone().requires_grad_(True)
    train_fns.Upsample2xFn.apply(xrg, True).backward(gy)
    assert torch.equal(xrg.grad, ops.relu_bwd(ops.upsample2x_bwd(gy), xr))


def test_vgg_input_and_adjoint():
    img = (torch.rand(2, 3, 12, 10, generator=torch.Generator().manual_seed(9)) * 255).to(DEV).requires_grad_(True)
    out = train_fns.VggInputFn.apply(img)
    assert out.shape == (2, 12, 10, 32) and torch.all(out[..., 3:] == 0)
    mean = img.new_tensor([0.485, 0.456, 0.406]).view(-1, 1, 1)
    std = img.new_tensor([0.229, 0.224, 0.225]).view(-1, 1, 1)
    ref = (img.detach().double() / 255.0 - mean.double()) / std.double()  # vgg19.py:11
    assert rel(out[..., :3], ref.permute(0, 2, 3, 1)) < 1e-6
    g = rnd(2, 12, 10, 32, seed=10)
    out.backward(g)
    img64 = img.detach().double().requires_grad_(True)
    ((img64 / 255.0 - mean.double()) / std.double()).backward(g[..., :3].permute(0, 3, 1, 2).double())
    assert rel(img.grad, img64.grad) < 1e-6


def test_vgg19_and_decoder_modules_against_aten_autograd():
    """The HIP training forwards of network.VGG19 and the Decoder (with gradients to the input
    image / features and the decoder parameters) against the same modules evaluated by aten."""
    import network
    from mhada_hip import autograd_path
    from mhada_hip.recipe import load_recipe, recipe_state_dict
    vgg = load_recipe(network.VGG19(), "vgg").to(DEV)
    img = (torch.rand(2, 3, 48, 40, generator=torch.Generator().manual_seed(11)) * 255).to(DEV)
    x1 = img.clone().requires_grad_(True)
    f1 = vgg(x1)
    x2 = img.double().cpu().requires_grad_(True)  # aten fp64 reference on the CPU
    vgg64 = load_recipe(network.VGG19(), "vgg").double()
    f2 = {}
    h = autograd_path.imagenet_normalize(x2).double()
    for i in range(1, 6):
        h = getattr(vgg64, f"slice{i}")(h)
        f2[f"relu{i}_1"] = h
    loss1 = sum((f1[k] * (j + 1)).square().mean() for j, k in enumerate(sorted(f1)))
    loss2 = sum((f2[k] * (j + 1)).square().mean() for j, k in enumerate(sorted(f2)))
    for k in f1:
        assert rel(f1[k].cpu(), f2[k]) < 1e-5, k
    loss1.backward()
    loss2.backward()
    assert rel(x1.grad.cpu(), x2.grad) < 1e-4

    dec = network.Decoder()
    sd = recipe_state_dict("dec", {"decoder." + k: tuple(v.shape) for k, v in dec.state_dict().items()})
    dec.load_state_dict({k[len("decoder."):]: v for k, v in sd.items()}, strict=True)
    # biases shifted by +5: pre-activations then sit far from zero, so fp32 and fp64 never take
    # different ReLU branches (a flip near the input changes a whole neighbourhood of gradients
    # and every weight gradient of the early layers); the masking itself is pinned per layer above
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, torch.nn.Conv2d):
                m.bias.add_(5.0)
    dec64 = network.Decoder().double()  # aten fp64 reference on the CPU
    dec64.load_state_dict(dec.state_dict())
    dec = dec.to(DEV)
    feat = rnd(2, 512, 6, 5, seed=12).requires_grad_(True)
    y1 = autograd_path.decoder_forward(dec, feat)
    feat64 = feat.detach().double().cpu().requires_grad_(True)
    y2 = autograd_path.decoder_forward(dec64, feat64)
    assert rel(y1.cpu(), y2) < 1e-5
    g = rnd(*y1.shape, seed=13)
    y1.backward(g)
    y2.backward(g.double().cpu())
    def close(a, b):
        return rel(a.cpu(), b) < 1e-5
    assert close(feat.grad, feat64.grad)
    for (n, p), (_, p64) in zip(dec.named_parameters(), dec64.named_parameters()):
        assert close(p.grad, p64.grad), n


# ---- AdaAttnForLoss (adaDecoder.py:52-81) on the wide-head HIP kernel (csrc/loss_attn.hip) -------
def _loss_attn_ref(c_x, s_x, c_1x, s_1x, act):
    """adaDecoder.py:52-81 in fp64 (the reference expression, unchunked)."""
    inorm = lambda t: F.instance_norm(t.double(), eps=1e-5)  # noqa: E731
    b, _, h, w = c_1x.shape
    q = inorm(c_1x).reshape(b, -1, h * w).permute(0, 2, 1)
    k = inorm(s_1x).reshape(b, s_1x.shape[1], -1)
    v = s_x.double().reshape(b, s_x.shape[1], -1).permute(0, 2, 1)
    if act == "softmax":
        a = torch.softmax(torch.bmm(q, k), dim=-1)
    else:
        s = torch.bmm(q, k) / torch.bmm(q.norm(dim=-1, keepdim=True), k.norm(dim=1, keepdim=True)) + 1
        a = s / s.sum(dim=-1, keepdim=True)
    m = torch.bmm(a, v)
    sd = torch.sqrt((torch.bmm(a, v * v) - m * m).clamp(min=1e-6))
    bc, _, hc, wc = c_x.shape
    m = m.reshape(bc, hc, wc, -1).permute(0, 3, 1, 2)
    sd = sd.reshape(bc, hc, wc, -1).permute(0, 3, 1, 2)
    return sd * inorm(c_x) + m


@pytest.mark.parametrize("act", ["softmax", "cosine"])
@pytest.mark.parametrize("B,dqk,dv,hc,wc,hs,ws", [(2, 448, 256, 16, 16, 16, 16), (1, 960, 512, 8, 8, 8, 8),
                                                   (2, 1472, 512, 4, 4, 4, 4), (1, 448, 256, 9, 7, 5, 11),
                                                   (1, 96, 64, 20, 3, 6, 6), (2, 448, 256, 40, 33, 21, 37),
                                                   (1, 96, 256, 11, 13, 9, 10)])
def test_loss_attn_against_fp64(act, B, dqk, dv, hc, wc, hs, ws):
    """The three local-feature-loss shapes (relu3/4/5 channel counts) plus ragged token counts;
    VGG-like non-negative features (post-ReLU), fp32 kernel vs fp64 reference: 1e-4 relative."""
    from mhada_hip import autograd_path
    c_x = F.relu(rnd(B, dv, hc, wc, seed=1))
    s_x = F.relu(rnd(B, dv, hs, ws, seed=2))
    c_1x = F.relu(rnd(B, dqk, hc, wc, seed=3))
    s_1x = F.relu(rnd(B, dqk, hs, ws, seed=4))
    with torch.no_grad():
        y = autograd_path.ada_attn_for_loss(c_x, s_x, c_1x, s_1x, act)
    ref = _loss_attn_ref(c_x, s_x, c_1x, s_1x, act)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-4


def test_loss_attn_matches_reference_golden():
    """lf_target4 of the train golden (reference AdaAttnForLoss on reference-VGG features of the
    golden's content/style): the HIP VGG19 features feed the HIP loss attention."""
    import network
    from conftest import load_golden
    from mhada_hip import losses as L
    from mhada_hip.recipe import load_recipe, seeded_image
    g = load_golden("train_64_b2")
    vgg = load_recipe(network.VGG19(), "vgg").to(DEV)
    c = seeded_image(2, 64, 64, int(g["content_seed"])).to(DEV)
    s = seeded_image(2, 64, 64, int(g["style_seed"])).to(DEV)
    with torch.no_grad():
        fc, fs = vgg(c), vgg(s)
        t4 = network.AdaAttnForLoss(512, 960)(fc["relu4_1"], fs["relu4_1"], L.feature_down_sample(fc, 4),
                                               L.feature_down_sample(fs, 4))
    assert torch.allclose(t4.cpu(), torch.from_numpy(g["lf_target4"]), rtol=1e-4, atol=1e-4)


# ---- ViT training kernels: Linear (+ReLU) and the patch embedding ---------------------------------
@pytest.mark.parametrize("M,K,N,relu", [(1000, 512, 1536, False), (777, 512, 2048, True), (300, 2048, 512, False)])
def test_linear_fn_fwd_bwd(M, K, N, relu):
    x = rnd(M, K, seed=21).requires_grad_(True)
    w = rnd(N, K, seed=22, scale=K ** -0.5).requires_grad_(True)
    b = rnd(N, seed=23, scale=0.1).requires_grad_(True)
    gy = rnd(M, N, seed=24)
    y = train_fns.linear(x, w, b, relu=relu)
    y.backward(gy)
    x64, w64, b64 = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    r = F.linear(x64, w64, b64)
    if relu:
        r = F.relu(r)
    r.backward(gy.double())
    assert rel(y, r) < 1e-5
    for a, b_ in ((x.grad, x64.grad), (w.grad, w64.grad), (b.grad, b64.grad)):
        assert rel(a, b_) < 1e-5


@pytest.mark.parametrize("M,K,N", [(1000, 512, 512), (300, 2048, 512)])
def test_linear_fn_fused_residual(M, K, N):
    """LinearFn(residual=r): y = x W^T + b + r in the GEMM epilogue (the ViT's out-projection and
    MLP2 residual adds), the residual's gradient passed through: against fp64 autograd."""
    x = rnd(M, K, seed=25).requires_grad_(True)
    w = rnd(N, K, seed=26, scale=K ** -0.5).requires_grad_(True)
    b = rnd(N, seed=27, scale=0.1).requires_grad_(True)
    r = rnd(M, N, seed=28).requires_grad_(True)
    gy = rnd(M, N, seed=29)
    y = train_fns.linear(x, w, b, residual=r)
    (y * gy).sum().backward()
    x64, w64, b64, r64 = (t.detach().double().requires_grad_(True) for t in (x, w, b, r))
    ref = F.linear(x64, w64, b64) + r64
    (ref * gy.double()).sum().backward()
    assert rel(y, ref) < 1e-5
    for a, b_ in ((x.grad, x64.grad), (w.grad, w64.grad), (b.grad, b64.grad), (r.grad, r64.grad)):
        assert rel(a, b_) < 1e-5


@pytest.mark.parametrize("M,K,N,mode", [(32768, 512, 1536, "plain"), (32768, 512, 2048, "relu"), (32768, 2048, 512, "residual"),
                                         (65536, 512, 512, "residual"), (40000, 512, 2048, "mlp_fold")])
def test_linear_fn_split3_vs_fp64(monkeypatch, M, K, N, mode):
    """LinearFn at the 512^2 training shapes, where its forward and input-gradient GEMMs run as SPLIT3
    products (train_fns.TRAIN_SPLIT3, round 6): output and all gradients against fp64 autograd at an
    fp32-class error (< 2e-6 where no ReLU mask flips dominate) and within 1.75x
    of the fp32-MFMA GEMMs' error (TRAIN_SPLIT3 = False) on the same operands; ReLU, a fused residual,
    and the MLP pair with its ReLU adjoint folded into the
    second layer's input-gradient epilogue (relu = 2 on the SPLIT3 kernel), bit-identical to the
    unfolded pair and to the pair with the plane hand-off (LinearFn planes_out)."""
    from mhada_hip.engine import _split3_fills
    assert _split3_fills(M, min(N, K), torch.device(DEV))  # the shapes take the SPLIT3 path
    errs = {}
    for s3 in (True, False):
        monkeypatch.setattr(train_fns, "TRAIN_SPLIT3", s3)
        x = rnd(M, K, seed=21).requires_grad_(True)
        w = rnd(N, K, seed=22, scale=K ** -0.5).requires_grad_(True)
        b = rnd(N, seed=23, scale=0.1).requires_grad_(True)
        gy = rnd(M, N if mode != "mlp_fold" else K, seed=24)
        ps = [x, w, b]
        if mode == "mlp_fold":
            w2 = rnd(K, N, seed=25, scale=N ** -0.5).requires_grad_(True)
            b2 = rnd(K, seed=26, scale=0.1).requires_grad_(True)
            ps += [w2, b2]
            grads = []
            for fold, hand in ((True, False), (False, False), (True, True)):
                for t in ps:
                    t.grad = None
                used = train_fns.PLANES_HANDOFF["used"]
                h = train_fns.linear(x, w, b, relu=True, grad_masked=fold, planes_out=hand)
                y = train_fns.linear(h, w2, b2, relu_input=fold)
                y.backward(gy)
                grads.append([t.grad.clone() for t in ps])
                # the plane hand-offs on the SPLIT3 path: forward with planes_out (MLP1's epilogue writes h's
                # planes for MLP2), backward with the folded ReLU adjoint (MLP2's input-gradient epilogue
                # writes the planes of h's gradient for MLP1's input-gradient GEMM)
                assert train_fns.PLANES_HANDOFF["used"] - used == s3 * (int(hand) + int(fold))
            for a, c in zip(grads[0], grads[1]):
                assert torch.equal(a, c)
            for a, c in zip(grads[0], grads[2]):  # the hand-off planes are split3_rows' planes bit for bit
                assert torch.equal(a, c)
        elif mode == "residual":
            r = rnd(M, N, seed=27).requires_grad_(True)
            ps.append(r)
            y = train_fns.linear(x, w, b, residual=r)
            y.backward(gy)
        else:
            y = train_fns.linear(x, w, b, relu=(mode == "relu"))
            y.backward(gy)
        p64 = [t.detach().double().requires_grad_(True) for t in ps]
        if mode == "mlp_fold":
            ref = F.linear(F.relu(F.linear(p64[0], p64[1], p64[2])), p64[3], p64[4])
        elif mode == "residual":
            ref = F.linear(p64[0], p64[1], p64[2]) + p64[3]
        else:
            ref = F.linear(p64[0], p64[1], p64[2])
            if mode == "relu":
                ref = F.relu(ref)
        ref.backward(gy.double())
        errs[s3] = [rel(y, ref)] + [rel(t.grad, t64.grad) for t, t64 in zip(ps, p64)]
    for e3, e32 in zip(errs[True], errs[False]):
        # behind a ReLU the gradients carry the mask flips of outputs within rounding of 0 (any fp32
        # evaluation against fp64: ~3e-4 here), so the absolute bound is relative to the fp32 path's
        assert e3 < max(2e-6, 1.75 * e32) and e3 <= 1.75 * e32 + 1e-8, (errs[True], errs[False])


@pytest.mark.parametrize("N,K0", [(1536, 512), (512, 2048), (700, 64)])
def test_split3_weight_dev_matches_host_split(N, K0):
    """mhada_split3_weight (the training step's per-step weight split) is bit-identical to
    ops.split3_weight, for W and for W^T."""
    w = rnd(N, K0, seed=5)
    assert torch.equal(ops.split3_weight_dev(w), ops.split3_weight(w))
    wt = rnd(K0, N, seed=6)
    if N % 64 == 0:
        assert torch.equal(ops.split3_weight_dev(wt, transposed=True), ops.split3_weight(wt.t().contiguous()))


def test_split3_rows_planes_are_exact():
    """mhada_split3_rows: plane 0 is the bf16 rounding, each plane the rounding of what the planes before
    leave, and the three sum to the fp32 input exactly."""
    x = rnd(1000, 384, seed=31) * 7
    pl = ops.split3_rows(x)
    assert pl.shape == (3, 1000, 384) and pl.dtype == torch.bfloat16
    assert torch.equal(pl[0], x.bfloat16())
    r1 = x.double() - pl[0].double()
    assert torch.equal(pl[1], r1.float().bfloat16())
    assert torch.equal(pl[0].double() + pl[1].double() + pl[2].double(), x.double())


@pytest.mark.parametrize("B,H,W,C", [(2, 5, 7, 64), (3, 33, 20, 128), (1, 1, 2, 4), (2, 64, 64, 512), (8, 128, 128, 64),
                                     (2, 1, 1, 8)])
def test_feat_stats_vs_fp64(B, H, W, C):
    """mhada_feat_stats (the losses' per-channel mean / unbiased std and mse in one pass) against
    fp64 torch on channels-last feature maps; a 1x1 map gives the unbiased std's NaN, as torch.std."""
    g = torch.Generator().manual_seed(B * H * W + C)
    x = (torch.rand(B, C, H, W, generator=g) * 3).to(DEV).contiguous(memory_format=torch.channels_last)
    t = (torch.rand(B, C, H, W, generator=g) * 3).to(DEV).contiguous(memory_format=torch.channels_last)
    mu, sd, mse = ops.feat_stats(x.permute(0, 2, 3, 1), t.permute(0, 2, 3, 1))
    xd, td = x.double(), t.double()
    torch.testing.assert_close(mu.double(), xd.mean(dim=(2, 3)), rtol=1e-6, atol=1e-6)
    if H * W > 1:
        torch.testing.assert_close(sd.double(), xd.std(dim=(2, 3)), rtol=1e-5, atol=1e-6)
    else:
        assert bool(torch.isnan(sd).all()) and bool(torch.isnan(xd.std(dim=(2, 3))).all())
    torch.testing.assert_close(mse.double(), ((xd - td) ** 2).mean(), rtol=1e-6, atol=0)
    mu2, sd2, none = ops.feat_stats(x.permute(0, 2, 3, 1))
    assert none is None and torch.equal(mu2, mu)
    assert torch.equal(sd2, sd) if H * W > 1 else bool(torch.isnan(sd2).all())
    _, _, mse2 = ops.feat_stats(x.permute(0, 2, 3, 1), t.permute(0, 2, 3, 1), stats=False)
    assert torch.equal(mse2, mse)


def test_mlp_relu_adjoint_folded_into_dgrad_gemm():
    """ViT MLP: Linear(ReLU) -> Linear with the first layer's ReLU adjoint applied in the second
    layer's input-gradient GEMM epilogue (mhada_gemm relu = 2, the mask in r) gives the bits of the
    unfolded pair (relu_bwd pass), a ragged M / N tile included."""
    for M, K, N in ((1000, 512, 2048), (77, 64, 68)):
        x = rnd(M, K, seed=51)
        w1, b1 = rnd(N, K, seed=52, scale=K ** -0.5), rnd(N, seed=53)
        w2, b2 = rnd(K, N, seed=54, scale=N ** -0.5), rnd(K, seed=55)
        gy = rnd(M, K, seed=56)
        res = []
        for fold in (False, True):
            ps = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
            h = train_fns.linear(ps[0], ps[1], ps[2], relu=True, grad_masked=fold)
            train_fns.linear(h, ps[3], ps[4], relu_input=fold).backward(gy)
            res.append([t.grad for t in ps])
        for a, b in zip(*res):
            assert torch.equal(a, b)


@pytest.mark.parametrize("B,H,W", [(2, 64, 64), (3, 72, 128)])
def test_patch_embed_fn_weight_grad(B, H, W):
    img = (torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(25)) * 255).to(DEV)
    conv = torch.nn.Conv2d(3, 512, 8, stride=8).to(DEV)
    y = train_fns.PatchEmbedFn.apply(img, conv.weight, conv.bias)
    gy = rnd(*y.shape, seed=26)
    y.backward(gy)
    w64 = conv.weight.detach().double().requires_grad_(True)
    b64 = conv.bias.detach().double().requires_grad_(True)
    r = F.conv2d(img.double(), w64, b64, stride=8).flatten(2).transpose(1, 2)
    r.backward(gy.double())
    assert rel(y, r) < 1e-5
    assert rel(conv.weight.grad, w64.grad) < 1e-5 and rel(conv.bias.grad, b64.grad) < 1e-5


def test_vit_training_forward_matches_aten_autograd():
    """network.VisionTransformer under autograd on the HIP training kernels vs the same module
    evaluated by aten in fp64 on the CPU (batch-axis attention, B = 3): outputs and parameter
    gradients."""
    import network
    from mhada_hip import autograd_path
    from mhada_hip.recipe import load_recipe
    vit = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(DEV).train()
    vit64 = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").double().train()
    img = torch.rand(3, 3, 64, 48, generator=torch.Generator().manual_seed(27)) * 255
    outs = vit(img.to(DEV))
    outs64 = autograd_path.vit_forward(vit64, img.double())
    loss = sum((o * (i + 1)).square().mean() for i, o in enumerate(outs))
    loss64 = sum((o * (i + 1)).square().mean() for i, o in enumerate(outs64))
    for a, b in zip(outs, outs64):
        assert rel(a.cpu(), b) < 1e-5
    loss.backward()
    loss64.backward()
    gmax = max(float(p.grad.abs().max()) for p in vit64.parameters())
    for (n, p), (_, p64) in zip(vit.named_parameters(), vit64.named_parameters()):
        err = (p.grad.cpu().double() - p64.grad).norm().item()
        assert err <= 1e-4 * p64.grad.norm().item() + 1e-7 * gmax, n


@pytest.mark.parametrize("M,N,K,mode", [(64, 576, 30000, "reflect"), (4, 576, 20000, "reflect"), (3, 576, 5000, "zero"),
                                        (4, 576, 7500, "zero"), (4, 1152, 5000, "reflect"), (256, 2304, 8000, "zero")])
def test_gemm_tn_conv_tiles(M, N, K, mode):
    """Weight-gradient tiles: the 64-row variant, the skinny (M <= 4) kernels — LDS-tiled for
    Cin % 64 == 0 with 4-float dY rows, the gather form otherwise (M = 3) — and 128 rows; 50 x 50
    images leave ragged 4 x 32 tiles."""
    from mhada_hip._lib import A_CONV3X3, A_CONV3X3_ZERO
    ci = N // 9
    H = W = 50
    B = max(1, K // (H * W))
    K = B * H * W
    x = rnd(B, H, W, ci, seed=31)
    g = rnd(K, M, seed=32)
    c = ops.gemm_tn(g, x, M=M, N=N, K=K, lda=M, b_mode=A_CONV3X3 if mode == "reflect" else A_CONV3X3_ZERO,
                    img=(ci, H, W), pad=1)
    xp = F.pad(x.permute(0, 3, 1, 2).double(), (1, 1, 1, 1), mode="reflect" if mode == "reflect" else "constant")
    cols = F.unfold(xp, 3)  # (B, ci*9, H*W) with k = ci*9 + tap
    cols = cols.view(B, ci, 9, H * W).permute(0, 3, 2, 1).reshape(K, 9 * ci)  # -> [pixel][tap*ci + c]
    ref = g.double().T @ cols
    assert rel(c, ref) < 1e-5
    if M == 4:  # the gather form on the same operands
        from mhada_hip import _lib
        with _lib.tuning(tn_skinny_lds=0):
            c0 = ops.gemm_tn(g, x, M=M, N=N, K=K, lda=M, b_mode=A_CONV3X3 if mode == "reflect" else A_CONV3X3_ZERO,
                             img=(ci, H, W), pad=1)
        assert rel(c0, ref) < 1e-5


@pytest.mark.parametrize("L", [1, 2, 3, 8])
def test_batch_axis_attention_fwd_bwd(L):
    """nn.MultiheadAttention's core over the batch axis (vit.py:48,59) on the HIP kernels vs fp64."""
    N, C, heads = 77, 512, 8
    qkv = rnd(L, N, 3 * C, seed=40 + L).requires_grad_(True)
    out = train_fns.BatchAxisAttnFn.apply(qkv, heads)
    g = rnd(L, N, C, seed=50 + L)
    out.backward(g)
    q64 = qkv.detach().double().requires_grad_(True)
    q, k, v = (z.reshape(L, N, heads, 64).permute(1, 2, 0, 3) for z in q64.split(C, dim=-1))
    a = torch.softmax(q @ k.transpose(-1, -2) / 8.0, dim=-1)
    ref = (a @ v).permute(2, 0, 1, 3).reshape(L, N, C)
    ref.backward(g.double())
    assert rel(out, ref) < 1e-6
    assert rel(qkv.grad, q64.grad) < 1e-6


@pytest.mark.parametrize("T,H", [(300, 8), (4096, 8), (77, 2)])
def test_head_proj_grouped_gemm_vs_fp64(T, H):
    """train_fns.HeadProjFn (the per-head 1x1 convs of adaDecoder.py:188-190 as one grouped GEMM,
    head-major output) against fp64 autograd of the per-head products: output and the gradients of
    x, the stacked weights and biases."""
    from mhada_hip import train_fns
    x = rnd(T, 64 * H, seed=11)
    w = rnd(H, 64, 64, scale=0.125, seed=12)
    b = rnd(H, 64, seed=13)
    gy = rnd(H, T, 64, seed=14)
    xs, ws, bs = (t.clone().requires_grad_() for t in (x, w, b))
    y = train_fns.head_proj(xs, ws, bs)
    y.backward(gy)
    xd, wd, bd = (t.double().clone().requires_grad_() for t in (x, w, b))
    yd = torch.stack([xd[:, 64 * h:64 * h + 64] @ wd[h].T + bd[h] for h in range(H)])
    yd.backward(gy.double())
    assert rel(y, yd) < 2e-6
    for a, r in ((xs.grad, xd.grad), (ws.grad, wd.grad), (bs.grad, bd.grad)):
        assert rel(a, r) < 2e-6


@pytest.mark.parametrize("B,N,C", [(2, 300, 512), (8, 4096, 64), (1, 37, 68)])
def test_instance_norm_tokens_vs_fp64(B, N, C):
    """train_fns.InstanceNormTokensFn (token-major InstanceNorm, adaDecoder.py:147-149) against
    fp64 F.instance_norm autograd on the same values in NCHW: output and input gradient."""
    from mhada_hip import train_fns
    x = rnd(B, N, C, seed=21) * 3 + 1
    dy = rnd(B, N, C, seed=22)
    xs = x.clone().requires_grad_()
    y = train_fns.instance_norm_tokens(xs)
    y.backward(dy)
    xd = x.double().clone().requires_grad_()
    yd = F.instance_norm(xd.transpose(1, 2), eps=1e-5).transpose(1, 2)
    yd.backward(dy.double())
    assert rel(y, yd) < 2e-6
    assert rel(xs.grad, xd.grad) < 2e-5


@pytest.mark.parametrize("M,C", [(32768, 512), (1000, 512), (37, 256), (300, 1024)])
def test_layernorm_fn_vs_fp64(M, C):
    """LayerNormFn (vit.py:54-55,58,62 under autograd) against fp64 F.layer_norm autograd: y, dx,
    dgamma, dbeta; bit-identical on a second run (fixed-order column sums)."""
    ln = torch.nn.LayerNorm(C, eps=1e-6).to(DEV)
    with torch.no_grad():
        ln.weight.copy_(rnd(C, seed=5) * 0.5 + 1)
        ln.bias.copy_(rnd(C, seed=6) * 0.1)
    x = (rnd(M, C, seed=7) * 3 + 1).requires_grad_()
    dy = rnd(M, C, seed=8)
    outs = []
    for _ in range(2):
        ln.zero_grad()
        x.grad = None
        y = train_fns.layernorm(x, ln)
        y.backward(dy)
        outs.append((y.detach(), x.grad.clone(), ln.weight.grad.clone(), ln.bias.grad.clone()))
    xd = x.detach().double().requires_grad_()
    gd, bd = ln.weight.detach().double().requires_grad_(), ln.bias.detach().double().requires_grad_()
    yd = F.layer_norm(xd, (C,), gd, bd, 1e-6)
    yd.backward(dy.double())
    for got, ref in zip(outs[0], (yd, xd.grad, gd.grad, bd.grad)):
        assert rel(got, ref) < 1e-5
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("h,w", [(8, 8), (9, 16), (64, 64), (135, 240), (32, 32), (16, 40), (24, 5)])
def test_pos_embed_fn_vs_fp64(h, w):
    """PosEmbedFn (vit.py:91-92 under autograd): forward and the gather adjoint against fp64
    F.interpolate(bilinear, align_corners=False) autograd; deterministic (bit-identical rerun)."""
    pos = (rnd(1, 512, 32, 32, seed=9) * 0.02).requires_grad_()
    g = rnd(h * w, 512, seed=10)
    grads = []
    for _ in range(2):
        pos.grad = None
        out = train_fns.pos_embed(pos, h, w)
        out.backward(g)
        grads.append(pos.grad.clone())
    pd = pos.detach().double().requires_grad_()
    ref = F.interpolate(pd, size=(h, w), mode="bilinear", align_corners=False)
    ref = ref.reshape(512, h * w).t()
    ref.backward(g.double())
    # fp32 source coordinates (the kernel, as aten's fp32 kernel) vs the fp64 reference's: 1e-5
    assert rel(out, ref) < 1e-5
    assert rel(grads[0], pd.grad) < 1e-5
    assert torch.equal(grads[0], grads[1])


def test_bf16_block_without_autocast_takes_aten_path():
    """a bf16 MHAda block input outside autocast must not reach the fp32-only token
    statistics kernels: it runs the aten formula and matches the fp32 block within bf16 rounding."""
    import network
    from mhada_hip.recipe import load_recipe
    blk = load_recipe(network.AdaAttnMultiHead(512, 8), "blk").to(DEV).train()
    fc, fs = rnd(2, 512, 4, 4, seed=11), rnd(2, 512, 3, 5, seed=12)
    ref = blk(fc, fs, fc).detach()
    blk16 = blk.to(torch.bfloat16)
    out = blk16(fc.bfloat16(), fs.bfloat16(), fc.bfloat16())
    assert out.dtype == torch.bfloat16 and torch.isfinite(out.float()).all()
    assert rel(out.float(), ref) < 5e-2


@pytest.mark.parametrize("stats,target", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("B,C,H,W", [(2, 64, 33, 20), (3, 512, 8, 8)])
def test_feature_loss_fn_matches_aten_autograd(stats, target, B, C, H, W):
    """FeatureLossFn (mhada_feat_loss_bwd) against fp64 autograd of the reference expressions it
    replaces: mse(mean_hw), mse(std_hw) (lossfn.py:7-23) and mse(x, t) (lossfn.py:26-47), each
    term scaled by its own upstream gradient; x an NCHW view of NHWC storage as the VGG emits it."""
    x = rnd(B, H, W, C, seed=11).permute(0, 3, 1, 2).requires_grad_(True)
    ref_f = rnd(B, C, H, W, seed=12) * 0.7 + 0.3
    t = rnd(B, H, W, C, seed=13).permute(0, 3, 1, 2) if target else None
    rm, rsd = (ref_f.mean(dim=(2, 3)), ref_f.std(dim=(2, 3))) if stats else (None, None)
    w = (70.0, 3.5, 15.0)
    lm, ls, lmse = train_fns.feature_loss_terms(x, rm, rsd, t)
    (w[0] * lm + w[1] * ls + w[2] * lmse).backward()
    xd = x.detach().double().requires_grad_(True)
    tot = 0
    refs = []
    if stats:
        a = F.mse_loss(xd.mean(dim=(2, 3)), rm.double())
        b = F.mse_loss(xd.std(dim=(2, 3)), rsd.double())
        tot = tot + w[0] * a + w[1] * b
        refs += [(lm, a), (ls, b)]
    if target:
        c = F.mse_loss(xd, t.double())
        tot = tot + w[2] * c
        refs.append((lmse, c))
    tot.backward()
    for got, want in refs:
        assert abs(got.item() - want.item()) <= 1e-5 * abs(want.item())
    assert rel(x.grad, xd.grad) < 1e-5
    # relu_input: x a ReLU output, the gradient leaves masked by (x > 0) — the bits of relu_bwd after it
    xr = F.relu(x.detach()).requires_grad_(True)
    lm, ls, lmse = train_fns.feature_loss_terms(xr, rm, rsd, t)
    (w[0] * lm + w[1] * ls + w[2] * lmse).backward()
    xm = xr.detach().clone().requires_grad_(True)
    lm, ls, lmse = train_fns.feature_loss_terms(xm, rm, rsd, t, relu_input=True)
    (w[0] * lm + w[1] * ls + w[2] * lmse).backward()
    ref = ops.relu_bwd(xr.grad.permute(0, 2, 3, 1).contiguous(), xr.detach().permute(0, 2, 3, 1).contiguous())
    assert torch.equal(xm.grad.permute(0, 2, 3, 1), ref)


@pytest.mark.parametrize("pad_mode", ["reflect", "zero"])
@pytest.mark.parametrize("B,H,W,Ci,Co,ldg", [(2, 8, 16, 64, 64, 64), (1, 18, 32, 128, 256, 256), (3, 6, 48, 64, 128, 132),
                                              (2, 24, 64, 64, 128, 128)])
def test_conv3x3_wgrad_wino(pad_mode, B, H, W, Ci, Co, ldg):
    """mhada_conv3x3_wgrad_wino (the decoder's weight / bias gradients) against fp64: dW[co][tap][ci]
    = sum_pixels g * x_pad (the same im2col contraction the TN GEMM computes) and db = sum g; a
    padded output-gradient row stride (ldg > Cout) and several tile-chunk splits; bits stable."""
    x = rnd(B, H, W, Ci, seed=41)
    gfull = rnd(B, H, W, ldg, seed=42)
    dw, db = ops.conv3x3_wgrad_wino(x, gfull, Co, pad_mode, bias=True)
    g = gfull[..., :Co].double()
    xp = F.pad(x.permute(0, 3, 1, 2).double(), (1, 1, 1, 1), mode="reflect" if pad_mode == "reflect" else "constant")
    cols = F.unfold(xp, 3).view(B, Ci, 9, H * W).permute(0, 3, 2, 1).reshape(B * H * W, 9 * Ci)
    ref = g.reshape(-1, Co).T @ cols
    assert rel(dw, ref) < 2e-6
    assert rel(db, g.reshape(-1, Co).sum(0)) < 1e-6
    dw2, db2 = ops.conv3x3_wgrad_wino(x, gfull, Co, pad_mode, bias=True)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


def test_cosine_block_training_linear_form_matches_reference_autograd():
    """The cosine activation under autograd on the device (adaDecoder.py:20-34) runs the linear form
    (A V = (q^ (K^ V) + sum v) / l, no N_c x N_s matrix): block output and parameter gradients
    against fp64 autograd of the reference expression on the CPU."""
    import network
    torch.manual_seed(3)
    blk = network.AdaAttnMultiHead(qkv_dim=128, num_heads=2, activation="cosine")
    fc, fs, fcs = (torch.randn(2, 128, 12, 10), torch.randn(2, 128, 8, 14), torch.randn(2, 128, 12, 10))
    ref = network.AdaAttnMultiHead(qkv_dim=128, num_heads=2, activation="cosine").double()
    ref.load_state_dict(blk.state_dict())
    out_ref = ref(fc.double(), fs.double(), fcs.double())
    out_ref.square().sum().backward()
    g = blk.to(DEV)
    out = g(fc.to(DEV), fs.to(DEV), fcs.to(DEV))
    out.square().sum().backward()
    assert rel(out.cpu(), out_ref) < 1e-5
    for (n, p), (_, pr) in zip(g.named_parameters(), ref.named_parameters()):
        assert rel(p.grad.cpu(), pr.grad) < 1e-4, n


# ---- the 3-channel ends of the conv stacks (csrc/rgb_ops.hip) -------------------------------------
@pytest.mark.parametrize("B,H,W", [(2, 2, 2), (1, 3, 5), (2, 37, 70), (1, 64, 130), (3, 9, 64)])
def test_out3_fn_vs_fp64(B, H, W):
    """train_fns.Out3Fn (the decoder's ConvReLU(64, 3), conv.py:94) against aten fp64 autograd:
    the NCHW output, the input gradient (ReLU, transposed conv and ReflectionPad2d adjoints,
    including the mirrored border taps at H, W = 2 and 3) and the weight / bias gradients, whose
    fixed-order reduction gives the same bits on a second call."""
    x = rnd(B, H, W, 64, seed=21)
    w = rnd(3, 64, 3, 3, seed=22, scale=24 ** -1)
    b = rnd(3, seed=23, scale=0.2)
    gy = rnd(B, 3, H, W, seed=24)
    xg = x.clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    bg = b.clone().requires_grad_(True)
    y = train_fns.Out3Fn.apply(xg, wg, bg)
    y.backward(gy)
    x64 = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    ref = F.relu(F.conv2d(F.pad(x64, (1, 1, 1, 1), mode="reflect"), w64, b64))
    ref.backward(gy.double())
    assert rel(y, ref) < 1e-6
    assert rel(xg.grad, x64.grad.permute(0, 2, 3, 1)) < 1e-5
    assert rel(wg.grad, w64.grad) < 1e-5
    assert rel(bg.grad, b64.grad) < 1e-5
    dw2, db2 = ops.out3_wgrad(x, gy, y.detach())
    assert torch.equal(dw2, wg.grad) and torch.equal(db2, bg.grad)
    # relu_input: the producing layer's ReLU adjoint folded into the input gradient
    wd = w.permute(2, 3, 0, 1).reshape(9, 3, 64).contiguous()
    xr = F.relu(x)
    assert torch.equal(ops.out3_dgrad(gy, y.detach(), wd, xr), ops.relu_bwd(ops.out3_dgrad(gy, y.detach(), wd), xr))


@pytest.mark.parametrize("B,H,W", [(2, 2, 2), (1, 5, 7), (2, 37, 70), (1, 64, 130), (2, 40, 48)])
def test_vgg_stem_fn_vs_fp64(B, H, W):
    """train_fns.VggStemFn (imageNet1k_normalize -> Conv2d(3, 64, 3, padding=1) -> ReLU with frozen
    weights, vgg19.py:10-11,25-26) against aten fp64 autograd: the NHWC output and the image
    gradient of mhada_vgg_stem_dgrad (ReLU, zero-padded transposed conv and normalisation
    adjoints in one pass)."""
    img = (torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(25)) * 255).to(DEV)
    w = rnd(64, 3, 3, 3, seed=26, scale=0.2)
    b = rnd(64, seed=27, scale=0.1)
    gy = rnd(B, H, W, 64, seed=28)
    ig = img.clone().requires_grad_(True)
    y = train_fns.VggStemFn.apply(ig, w, b)
    y.backward(gy)
    i64 = img.double().requires_grad_(True)
    mean = i64.new_tensor([0.485, 0.456, 0.406]).view(-1, 1, 1)
    std = i64.new_tensor([0.229, 0.224, 0.225]).view(-1, 1, 1)
    ref = F.relu(F.conv2d((i64 / 255.0 - mean) / std, w.double(), b.double(), padding=1))
    ref.backward(gy.double().permute(0, 3, 1, 2))
    assert rel(y, ref.permute(0, 2, 3, 1)) < 1e-5
    assert rel(ig.grad, i64.grad) < 1e-5


@pytest.mark.parametrize("M,C", [(1000, 512), (32768, 512), (77, 256)])
def test_layernorm_fwd_plane_output_is_split_of_y(M, C):
    """mhada_layernorm_fwd_split3 (round 6): y bit-identical to mhada_layernorm_fwd and the planes exactly
    split3_rows(y) — the QKV / MLP1 SPLIT3 operand handed over by LayerNormFn."""
    x, g, b = rnd(M, C, seed=71), rnd(C, seed=72), rnd(C, seed=73)
    y0, st0 = ops.layernorm_fwd(x, g, b, 1e-6)
    y, st, pl = ops.layernorm_fwd(x, g, b, 1e-6, planes=True)
    assert torch.equal(y, y0) and torch.equal(st, st0)
    assert torch.equal(pl, ops.split3_rows(y))


@pytest.mark.parametrize("L,N,groups", [(8, 300, 1), (16, 129, 2), (3, 64, 1)])
def test_vit_batch_attn_bwd_plane_output_is_split_of_dqkv(L, N, groups):
    """mhada_vit_batch_attn_bwd_split3 (round 6): dqkv bit-identical to mhada_vit_batch_attn_bwd and the
    planes exactly split3_rows(dqkv), also when a grouped call writes its slice of the planes."""
    heads, C = 8, 512
    qkv, dout = rnd(L, N, 3 * C, seed=81), rnd(L, N, C, seed=82)
    d0 = ops.vit_batch_attn_bwd(qkv, dout, L, N, heads, groups)
    d, pl = ops.vit_batch_attn_bwd(qkv, dout, L, N, heads, groups, planes=True)
    assert torch.equal(d, d0)
    assert torch.equal(pl, ops.split3_rows(d.view(L * N, 3 * C)))


def test_vit_training_plane_handoffs_are_bit_identical():
    """The ViT training path at the 512^2 B8 batched-call size (32768 tokens: every linear SPLIT3) with the
    SPLIT3 plane hand-offs (LayerNorm -> QKV / MLP1, MLP1 -> MLP2, and backward the batch-axis attention ->
    QKV, MLP2 -> MLP1) against every linear splitting its own operand: outputs and every gradient bit for
    bit, and the hand-offs actually taken."""
    import network
    from mhada_hip import autograd_path
    from mhada_hip.recipe import load_recipe
    vit = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(DEV).train()
    x = (rnd(8, 3, 512, 512, seed=91) * 40 + 128)
    res = []
    for on in (True, False):
        train_fns.PLANES_HANDOFF_ON = on
        try:
            vit.zero_grad(set_to_none=True)
            used = train_fns.PLANES_HANDOFF["used"]
            outs = autograd_path.vit_forward(vit, x)
            loss = sum((o * rnd(*o.shape, seed=92 + i)).sum() for i, o in enumerate(outs))
            loss.backward()
            res.append(([o.detach().clone() for o in outs], [p.grad.clone() for p in vit.parameters()],
                        train_fns.PLANES_HANDOFF["used"] - used))
        finally:
            train_fns.PLANES_HANDOFF_ON = True
    (o1, g1, u1), (o0, g0, u0) = res
    assert u0 == 0 and u1 == 3 * 5  # per layer: LN1 -> QKV, LN2 -> MLP1, MLP1 -> MLP2, attn -> QKV, MLP2 -> MLP1
    for a, b in zip(o1 + g1, o0 + g0):
        assert torch.equal(a, b)
