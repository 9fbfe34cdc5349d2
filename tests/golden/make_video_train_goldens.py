"""Golden vectors for one train_video.py step (SURVEY §8f rank 3 + the temporal losses), produced by
the reference's own network/*.py and lossfn.py (imported with the stand-ins of
make_train_goldens.py) composed exactly as train_video.py:110-166 composes them: 5 ViT and 5
AdaFormer calls, VGG19 features, global-style / local-feature / output- and feature-level temporal /
identity losses weighted 100 / 15 / 2 / 2 / 0.05 / 0.1, backward.  Stores the inputs' seeds, the
flow and mask, the seven losses and per-parameter gradient norms.

Two cases: 64x64 frames with a 64x64 style (train_video_64_b2.npz) and 64x128 frames with a 64x64
style (train_video_64x128_s64_b2.npz) — the latter has train_video.py's shape structure (frames of
twice the style's width, 256x512 / 256x256 there), so VideoTrainer's shape grouping splits its ViT and
AdaFormer calls as it does at the real shapes.

Usage:  python tests/golden/make_video_train_goldens.py
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from make_train_goldens import grad_summary, load_reference, np32  # noqa: E402
from make_video_goldens import smooth_flow  # noqa: E402
from mhada_hip.recipe import load_recipe, seeded_image  # noqa: E402


def main(H=64, W=64, Hs=64, Ws=64, name="train_video_64_b2", f64=False):
    """f64: the same composition with the trained modules (ViTs, AdaFormer) and inputs in float64 —
    VGG19 stays fp32, its reference forward casts to float; its gradient norms are added to the fp32
    golden as grad_*_f64 — the yardstick for how far an fp32 evaluation of this step may land from
    the fp32 reference (near-degenerate attention rows make E2' - M'^2 cancel, and sqrt's gradient
    1/(2 S) amplifies that)."""
    torch.set_num_threads(8)
    R = load_reference()
    U, L = R["utilities"], R["lossfn"]
    vit_c = load_recipe(R["vit"].VisionTransformer(pos_embedding=True), "vit_c").train()
    vit_s = load_recipe(R["vit"].VisionTransformer(pos_embedding=False), "vit_s").train()
    ada = load_recipe(R["adaDecoder"].AdaAttnTransformerMultiHead(), "ada").train()
    vgg = R["vgg19"].VGG19()
    load_recipe(vgg, "vgg")
    vgg.eval()
    noLearn = nn.ModuleList([R["adaDecoder"].AdaAttnForLoss(256, 64 + 128 + 256),
                             R["adaDecoder"].AdaAttnForLoss(512, 64 + 128 + 256 + 512),
                             R["adaDecoder"].AdaAttnForLoss(512, 64 + 128 + 256 + 512 + 512)]).eval()
    mse = nn.MSELoss(reduction="mean")
    mseMatrix = nn.MSELoss(reduction="none")
    # batch 2: at batch 1 this CPU PyTorch build's instance_norm backward misreads a gradient with
    # channels-last strides (which the reference's permuted head outputs produce), see DESIGN.md §4
    B = 2
    style = seeded_image(B, Hs, Ws, 201)
    c1 = seeded_image(B, H, W, 202)
    c2 = seeded_image(B, H, W, 203)
    g = torch.Generator().manual_seed(204)
    flow = smooth_flow(g, B, H, W, 3.0)
    # [B][H][W] as the data loader yields it: forward/backward consistency of a noisy inverse flow
    mask = torch.stack([U.flow_warp_mask(flow[b], -flow[b] + 1.0 * torch.randn(2, H, W, generator=g))
                        for b in range(B)])
    if f64:
        # the trained modules in float64; VGG19 stays fp32 (network/vgg19.py:6-12 casts its input to
        # float, so the reference cannot run it in float64) and so do the loss attentions on its features
        for m in (vit_c, vit_s, ada):
            m.double()
        style, c1, c2, flow, mask = (t.double() for t in (style, c1, c2, flow, mask))

    # train_video.py:110-166
    vitc_fc1 = vit_c(c1)
    vitc_fc2 = vit_c(c2)
    vits_fs = vit_s(style)
    ada_fcs1, cs1 = ada(vitc_fc1, vits_fs)
    ada_fcs2, cs2 = ada(vitc_fc2, vits_fs)
    vits_fc1 = vit_s(c1)
    vits_fc2 = vit_s(c2)
    vitc_fs = vit_c(style)
    _, cc1 = ada(vitc_fc1, vits_fc1)
    _, cc2 = ada(vitc_fc2, vits_fc2)
    _, ss = ada(vitc_fs, vits_fs)
    with torch.no_grad():
        vgg_fc1 = vgg(c1)
        vgg_fc2 = vgg(c2)
        vgg_fs = vgg(style)
    vgg_fcs1 = vgg(cs1)
    vgg_fcs2 = vgg(cs2)
    vgg_fcc1 = vgg(cc1)
    vgg_fcc2 = vgg(cc2)
    vgg_fss = vgg(ss)
    loss_gs = (L.global_style_loss(vgg_fcs1, vgg_fs, mse) + L.global_style_loss(vgg_fcs2, vgg_fs, mse)) * 100
    loss_lf = (L.local_feature_loss(vgg_fc1, vgg_fs, vgg_fcs1, noLearn, mse)
               + L.local_feature_loss(vgg_fc2, vgg_fs, vgg_fcs2, noLearn, mse)) * 15
    loss_ot = L.output_level_temporal_loss(c1, c2, cs1, cs2, flow, mask, mseMatrix) * 2
    loss_ft = L.feature_level_temporal_loss(ada_fcs1, ada_fcs2, flow, mask, mseMatrix) * 2
    loss_id1 = (mse(cc1, c1) + mse(cc2, c2) + mse(ss, style)) * 5e-2
    loss_id2 = 0
    for i in [1, 2, 3, 4, 5]:
        loss_id2 += mse(vgg_fcc1[f"relu{i}_1"], vgg_fc1[f"relu{i}_1"])
        loss_id2 += mse(vgg_fcc2[f"relu{i}_1"], vgg_fc2[f"relu{i}_1"])
        loss_id2 += mse(vgg_fss[f"relu{i}_1"], vgg_fs[f"relu{i}_1"])
    loss_id2 *= 1e-1
    loss = loss_gs + loss_lf + loss_ot + loss_ft + loss_id1 + loss_id2
    loss.backward()

    path = os.path.join(HERE, name + ".npz")
    if f64:
        old = dict(np.load(path))
        for n, m in (("vit_c", vit_c), ("vit_s", vit_s), ("ada", ada)):
            old[f"grad_{n}_f64"] = grad_summary(m)
        old["losses_f64"] = np.array([float(v) for v in (loss_gs, loss_lf, loss_ot, loss_ft, loss_id1, loss_id2, loss)])
        np.savez_compressed(path, **old)
        print(f"added the float64 gradient norms to {path}")
        return
    out = {
        "seeds": np.array([201, 202, 203]), "flow": np32(flow), "mask": np32(mask),
        "frame_shape": np.array([H, W]), "style_shape": np.array([Hs, Ws]),
        "losses": np.array([float(v) for v in (loss_gs, loss_lf, loss_ot, loss_ft, loss_id1, loss_id2, loss)]),
        "grad_vit_c": grad_summary(vit_c), "grad_vit_s": grad_summary(vit_s), "grad_ada": grad_summary(ada),
        "grad_ada_last_conv_w": np32(ada.decoder.conv3[1].conv.conv.weight.grad),
    }
    np.savez_compressed(path, **out)
    print(f"wrote {path}: losses {out['losses']}, mask mean {float(mask.mean()):.3f}")


if __name__ == "__main__":
    for args in ((64, 64, 64, 64, "train_video_64_b2"), (64, 128, 64, 64, "train_video_64x128_s64_b2")):
        main(*args)
        main(*args, f64=True)
