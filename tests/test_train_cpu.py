"""Training path (e) on CPU: one train_image.py step against the reference's
golden losses/gradients, and the data-parallel gradient all-reduce with 2 gloo ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import network
from conftest import load_golden
from mhada_hip.recipe import load_recipe, seeded_image
from mhada_hip.train import Trainer, VideoTrainer


def build(device="cpu"):
    torch.manual_seed(0)
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(device).train()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(device).train()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(device).train()
    vgg = load_recipe(network.VGG19(), "vgg").to(device)
    return vc, vs, ada, vgg


def grad_summary(m):
    return np.array([float(p.grad.double().norm()) if p.grad is not None else 0.0
                     for _, p in sorted(m.named_parameters())])


def check_against_golden(tr, device):
    g = load_golden("train_64_b2")
    c = seeded_image(2, 64, 64, int(g["content_seed"])).to(device)
    s = seeded_image(2, 64, 64, int(g["style_seed"])).to(device)
    out = tr.backward(c, s)
    got = np.array([float(out[k].detach()) for k in ("loss_gs", "loss_lf", "loss_id1", "loss_id2", "loss")])
    np.testing.assert_allclose(got, g["losses"], rtol=2e-4)
    for name, m in (("vit_c", tr.vit_c), ("vit_s", tr.vit_s), ("ada", tr.ada)):
        ref = g[f"grad_{name}"]  # tiny norms (<1e-4 of the largest) are rounding noise
        np.testing.assert_allclose(grad_summary(m), ref, rtol=2e-3, atol=1e-5 * ref.max())
    np.testing.assert_allclose(tr.ada.decoder.conv3[1].conv.conv.weight.grad.cpu().numpy(),
                               g["grad_ada_last_conv_w"], rtol=2e-3, atol=1e-3)


def test_train_step_matches_reference_golden():
    torch.set_num_threads(8)
    check_against_golden(Trainer(*build()), "cpu")


VIDEO_GOLDENS = ["train_video_64_b2", "train_video_64x128_s64_b2"]


def check_video_against_golden(tr, device, name="train_video_64_b2"):
    """One train_video.py:110-166 step against the reference's own composition of it
    (tests/golden/make_video_train_goldens.py): the seven losses and every gradient norm."""
    g = load_golden(name)
    fh, fw = (int(x) for x in g["frame_shape"]) if "frame_shape" in g else (64, 64)
    sh, sw = (int(x) for x in g["style_shape"]) if "style_shape" in g else (64, 64)
    style = seeded_image(2, sh, sw, int(g["seeds"][0])).to(device)
    c1, c2 = (seeded_image(2, fh, fw, int(x)).to(device) for x in g["seeds"][1:])
    flow = torch.from_numpy(g["flow"]).to(device)
    mask = torch.from_numpy(g["mask"]).to(device)
    out = tr.backward(style, c1, c2, flow, mask)
    keys = ("loss_gs", "loss_lf", "loss_ot", "loss_ft", "loss_id1", "loss_id2", "loss")
    got = np.array([float(out[k].detach()) for k in keys])
    np.testing.assert_allclose(got, g["losses"], rtol=2e-4)
    for name, m in (("vit_c", tr.vit_c), ("vit_s", tr.vit_s), ("ada", tr.ada)):
        ref = g[f"grad_{name}"]
        np.testing.assert_allclose(grad_summary(m), ref, rtol=2e-3, atol=1e-5 * ref.max())
    np.testing.assert_allclose(tr.ada.decoder.conv3[1].conv.conv.weight.grad.cpu().numpy(),
                               g["grad_ada_last_conv_w"], rtol=2e-3, atol=1e-3)


@pytest.mark.parametrize("name", VIDEO_GOLDENS)
def test_video_train_step_matches_reference_golden(name):
    """Both video goldens; the 64x128-frame / 64x64-style one splits VideoTrainer's grouped ViT and
    AdaFormer calls by shape as train_video.py's 256x512 / 256x256 shapes do."""
    torch.set_num_threads(8)
    check_video_against_golden(VideoTrainer(*build()), "cpu", name)


@pytest.mark.parametrize("name", VIDEO_GOLDENS)
def test_video_golden_fp32_noise_yardstick(name):
    """The fp32 golden against the float64 run of the same composition (ViTs and AdaFormer in float64,
    VGG19 fp32 as the reference forces): the rtol of check_video_against_golden (2e-3) is 4x the fp32
    noise of these gradient norms (<= 4.9e-4), so a form that fails it is less accurate than fp32."""
    g = load_golden(name)
    for k in ("vit_c", "vit_s", "ada"):
        a, b = g[f"grad_{k}"], g[f"grad_{k}_f64"]
        big = b > 1e-5 * b.max()
        assert np.max(np.abs(a[big] / b[big] - 1)) < 5e-4

def test_checkpoint_dict_roundtrip(tmp_path):
    tr = Trainer(*build())
    ck = tr.checkpoint(epoch=1, batch_size=8)
    assert set(ck) == {"epoch", "batch_size", "model_state", "optim_state"}
    torch.save(ck, tmp_path / "checkpoint_epoch_1_batchSize_8.pth")
    ck2 = torch.load(tmp_path / "checkpoint_epoch_1_batchSize_8.pth", weights_only=True)
    tr2 = Trainer(*build())
    tr2.load_checkpoint(ck2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = Trainer(*build(), distributed=True, bucket_mb=4)  # several buckets
    # a micro-batch of TWO images per rank: the batch-axis ViT attention couples
    # them inside the rank's forward call, never across ranks
    c = seeded_image(2, 64, 64, 200 + rank)
    s = seeded_image(2, 64, 64, 300 + rank)
    tr.backward(c, s)
    if rank == 0:
        grads = {n: p.grad.clone() for n, p in tr.ada.named_parameters()}
        grads.update({"vit_c." + n: p.grad.clone() for n, p in tr.vit_c.named_parameters()})
        torch.save(grads, os.path.join(out_dir, "dp_grads.pt"))
    # after the Adam steps every rank holds the same parameters (bench.py's DP check)
    for o in (tr.opt_vit_c, tr.opt_vit_s, tr.opt_ada):
        o.step()
    import bench
    agree = bench.rank_agreement([tr.vit_c, tr.vit_s, tr.ada])
    torch.save(agree, os.path.join(out_dir, f"agree_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_allreduce_equals_accumulation(tmp_path):
    """2 gloo ranks with 2 images each == one process averaging the gradients of the two B = 2
    micro-batch calls (train_image.py:103-110,139-144).  Control: splitting each
    micro-batch into single-image calls (batch-axis attention uncoupled) gives different
    gradients, so the comparison does see the coupling."""
    world = 2
    mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    dp = torch.load(tmp_path / "dp_grads.pt", weights_only=True)
    torch.set_num_threads(2)  # same intra-op split as the workers: same summation order
    tr = Trainer(*build(), distributed=False)
    def accumulate(calls):
        acc = {}
        for c, s in calls:
            tr.backward(c, s)
            named = dict(("vit_c." + n, p) for n, p in tr.vit_c.named_parameters())
            named.update(dict(tr.ada.named_parameters()))
            for n, p in named.items():
                acc[n] = acc.get(n, 0) + p.grad / len(calls)
        return acc

    micro = [(seeded_image(2, 64, 64, 200 + r), seeded_image(2, 64, 64, 300 + r)) for r in range(world)]
    acc = accumulate(micro)
    single = accumulate([(c[i:i + 1], s[i:i + 1]) for c, s in micro for i in range(2)])
    torch.set_num_threads(8)
    for n, g in acc.items():
        torch.testing.assert_close(dp[n], g, rtol=1e-4, atol=1e-5 * float(g.abs().max()))
    # the ViT's attention weights see the coupling: per-image calls move their gradient by far more
    # than the DP tolerance
    qkv = "vit_c.encoder.0.attention.in_proj_weight"
    assert float((single[qkv] - acc[qkv]).norm()) > 1e-2 * float(acc[qkv].norm())
    for r in range(world):
        agree = torch.load(tmp_path / f"agree_{r}.pt", weights_only=True)
        assert agree["identical"] and agree["backend"] == "gloo" and agree["world"] == world, agree


def _reducer_worker(rank, world, port, out_dir):
    from mhada_hip.parallel import GradAllReducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    used, unused = torch.nn.Linear(4, 3), torch.nn.Linear(4, 3)
    params = list(used.parameters()) + list(unused.parameters())
    red = GradAllReducer(params, bucket_bytes=16)  # one small bucket per parameter or two
    x = torch.full((2, 4), float(rank + 1))
    used(x).sum().backward()
    red.finish()
    res = {"w": used.weight.grad.clone(), "unused_none": unused.weight.grad is None}
    red.remove()
    # a second reducer on the same parameters: the first one's hooks must not fire any more
    red2 = GradAllReducer(params, bucket_bytes=1 << 20)
    for p in params:
        p.grad = None
    used(x).sum().backward()
    red2.finish()
    res["w2"] = used.weight.grad.clone()
    res["n_hooks_first"] = len(red._hooks)
    red2.remove()
    torch.save(res, os.path.join(out_dir, f"red_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_reducer_keeps_unused_grads_none_and_removes_hooks(tmp_path):
    """a parameter no loss reaches keeps grad None (Adam skips it, as in the single-GPU
    reference), and remove() detaches the hooks so a second reducer runs exactly one all-reduce
    per bucket (a stale hook would desynchronise the collectives across ranks)."""
    world = 2
    mp.spawn(_reducer_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(tmp_path / f"red_{r}.pt", weights_only=True)
        # d sum(W x) / dW = 2 rows of x (value rank+1) -> mean over ranks of 2*(r+1) = 3
        torch.testing.assert_close(res["w"], torch.full((3, 4), 3.0))
        torch.testing.assert_close(res["w2"], torch.full((3, 4), 3.0))
        assert res["unused_none"] and res["n_hooks_first"] == 0
