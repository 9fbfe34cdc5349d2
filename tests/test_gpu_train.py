"""Training path on the GPU: one train_image.py step against the reference's goldens, and a
full-size (512^2, batch 8) step running forward/backward/Adam with finite losses."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from mhada_hip.recipe import seeded_image
from mhada_hip.train import Trainer, VideoTrainer
from test_train_cpu import VIDEO_GOLDENS, build, check_against_golden, check_video_against_golden


def test_train_step_matches_reference_golden_gpu():
    check_against_golden(Trainer(*build("cuda")), "cuda")


@pytest.mark.parametrize("name", VIDEO_GOLDENS)
def test_video_train_step_matches_reference_golden_gpu(name):
    """One train_video.py step (5 AdaFormer calls, temporal losses with the warp and its adjoint on
    HIP) against the reference's own composition of it (tests/golden/make_video_train_goldens.py),
    square frames and frames of twice the style's width (the grouped calls split by shape)."""
    check_video_against_golden(VideoTrainer(*build("cuda")), "cuda", name)



def test_train_step_256_b2_losses_match_oracle_and_grads_match_cpu():
    """One train_image.py step at 256^2, batch 2 (16x the golden's pixels; every VGG / loss-attention
    level is non-trivial): the five loss terms against the numpy oracle's restatement of
    train_image.py:103-136 (oracle.train_losses, rtol 2e-4), and every parameter's gradient norm
    against the drop-in's CPU autograd path (the reference's aten expression, golden-pinned by
    test_train_cpu) at rtol 2e-3."""
    from oracle import mhada_oracle as O
    from test_train_cpu import grad_summary
    c = seeded_image(2, 256, 256, 41)
    s = seeded_image(2, 256, 256, 42)
    cpu = Trainer(*build("cpu"))
    ref_out = cpu.backward(c, s)
    p = [O.to_numpy_params(m.state_dict()) for m in (cpu.vit_c, cpu.vit_s, cpu.ada, cpu.vgg)]
    ref = np.array(O.train_losses(c.numpy(), s.numpy(), *p))
    tr = Trainer(*build("cuda"))
    out = tr.backward(c.cuda(), s.cuda())
    keys = ("loss_gs", "loss_lf", "loss_id1", "loss_id2", "loss")
    got = np.array([float(out[k].detach()) for k in keys])
    np.testing.assert_allclose(got, ref, rtol=2e-4)
    np.testing.assert_allclose(np.array([float(ref_out[k].detach()) for k in keys]), ref, rtol=2e-4)
    for m_gpu, m_cpu in ((tr.vit_c, cpu.vit_c), (tr.vit_s, cpu.vit_s), (tr.ada, cpu.ada)):
        g_ref = grad_summary(m_cpu)
        np.testing.assert_allclose(grad_summary(m_gpu), g_ref, rtol=2e-3, atol=1e-5 * g_ref.max())


def test_batched_adaformer_step_matches_per_call_step():
    """Trainer.batch_adaformer (the three AdaFormer calls of train_image.py:105-110 as one call
    over the concatenated batch) against the reference's three separate calls: the same losses
    and gradients up to fp32 summation order (the weight gradients reduce over 3B images in one
    GEMM instead of three partial GEMMs added by autograd)."""
    from test_train_cpu import grad_summary
    c = seeded_image(2, 128, 128, 51).cuda()
    s = seeded_image(2, 128, 128, 52).cuda()
    outs, grads = [], []
    for batched in (True, False):
        tr = Trainer(*build("cuda"))
        tr.batch_adaformer = batched
        out = tr.backward(c, s)
        outs.append(np.array([float(out[k].detach()) for k in ("loss_gs", "loss_lf", "loss_id1", "loss_id2")]))
        grads.append(np.concatenate([grad_summary(m) for m in (tr.vit_c, tr.vit_s, tr.ada)]))
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-5)
    np.testing.assert_allclose(grads[0], grads[1], rtol=1e-4, atol=1e-6 * grads[1].max())


def test_batched_vit_step_matches_per_call_step():
    """Trainer.batch_vit (each ViT's two calls of train_image.py:103-104 as one call over the
    concatenated batch, the batch-axis attention per call) against the four separate calls: the
    same ViT features bit for bit, the same losses and gradients up to fp32 summation order."""
    from test_train_cpu import grad_summary
    from mhada_hip.autograd_path import vit_forward
    c = seeded_image(2, 128, 128, 61).cuda()
    s = seeded_image(2, 128, 128, 62).cuda()
    tr = Trainer(*build("cuda"))
    sep = [vit_forward(tr.vit_c, c), vit_forward(tr.vit_c, s)]
    grp = vit_forward(tr.vit_c, torch.cat([c, s]), groups=2)
    for o, a, b in zip(grp, *sep):
        torch.testing.assert_close(o, torch.cat([a, b]), rtol=0, atol=0)
    outs, grads = [], []
    for batched in (True, False):
        tr = Trainer(*build("cuda"))
        tr.batch_vit = batched
        out = tr.backward(c, s)
        outs.append(np.array([float(out[k].detach()) for k in ("loss_gs", "loss_lf", "loss_id1", "loss_id2")]))
        grads.append(np.concatenate([grad_summary(m) for m in (tr.vit_c, tr.vit_s, tr.ada)]))
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-5)
    np.testing.assert_allclose(grads[0], grads[1], rtol=1e-4, atol=1e-6 * grads[1].max())


def test_relu_adjoint_folds_are_bit_identical():
    """The ReLU adjoints folded into consumers (VGG feature maps into the loss backward and the next
    conv's dgrad: Trainer.masked_vgg_features) give the bits of the relu_bwd passes they replace."""
    from test_train_cpu import grad_summary
    c = seeded_image(2, 96, 64, 71).cuda()
    s = seeded_image(2, 96, 64, 72).cuda()
    res = []
    for masked in (False, True):
        tr = Trainer(*build("cuda"))
        tr.masked_vgg_features = masked
        out = tr.backward(c, s)
        res.append(([float(out[k].detach()) for k in ("loss_gs", "loss_lf", "loss_id1", "loss_id2")],
                    [p.grad.clone() for m in (tr.vit_c, tr.vit_s, tr.ada) for p in m.parameters()]))
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


def test_train_step_full_size_runs():
    tr = Trainer(*build("cuda"))
    c = seeded_image(8, 512, 512, 100).cuda()
    s = seeded_image(8, 512, 512, 101).cuda()
    l1 = tr.step(c, s)
    l2 = tr.step(c, s)
    assert all(np.isfinite(v) for v in l1.values()) and all(np.isfinite(v) for v in l2.values())
    assert l2["loss"] < l1["loss"] * 1.5  # one Adam step at lr 1e-4 does not blow up


def test_rccl_data_parallel_grads_match_single_gpu():
    """The RCCL path on the device: a 1-rank "nccl" process group (device_id
    set before any collective) runs Trainer(distributed=True) — post-accumulate-grad hooks
    launching async all-reduces against the HIP compute stream, then finish() — and its
    gradients equal Trainer(distributed=False) on the same 64^2 batch of 2."""
    import socket

    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        assert dist.get_backend() == "nccl"
        c = seeded_image(2, 64, 64, 7).cuda()
        s_img = seeded_image(2, 64, 64, 8).cuda()
        grads = []
        for distributed in (True, False):
            tr = Trainer(*build("cuda"), distributed=distributed)
            assert (tr.reducer is not None) == distributed
            tr.backward(c, s_img)
            torch.cuda.synchronize()
            grads.append({f"{mn}.{n}": p.grad.clone() for mn, m in (("vit_c", tr.vit_c), ("vit_s", tr.vit_s),
                                                                     ("ada", tr.ada))
                          for n, p in m.named_parameters() if p.grad is not None})
            tr.close()
        assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 300
        # same kernels, same inputs, fixed-order reductions everywhere (HIP kernels, deterministic
        # pos-embed adjoint), a 1-rank all-reduce (sum of one) and /1: bit for bit
        for n in grads[1]:
            assert torch.equal(grads[0][n], grads[1][n]), n
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_train_step_512_b1_losses_match_oracle():
    """BASELINE configs[3]'s resolution (512^2), batch 1: the five loss terms of one
    train_image.py:103-136 step on the HIP path against the numpy oracle (oracle.train_losses,
    rtol 2e-4), run here inside the test (about a minute of CPU on the box's 16 threads)."""
    from oracle import mhada_oracle as O
    c = seeded_image(1, 512, 512, 61)
    s = seeded_image(1, 512, 512, 62)
    ms = build("cpu")
    p = [O.to_numpy_params(m.state_dict()) for m in ms]
    ref = np.array(O.train_losses(c.numpy(), s.numpy(), *p))
    tr = Trainer(*build("cuda"))
    out = tr.backward(c.cuda(), s.cuda())
    got = np.array([float(out[k].detach()) for k in ("loss_gs", "loss_lf", "loss_id1", "loss_id2", "loss")])
    np.testing.assert_allclose(got, ref, rtol=2e-4)
