"""Which arithmetic form moves the train_video golden's gradient norms: the video-training golden
check (tests/test_train_cpu.check_video_against_golden) under each combination of the SPLIT3 training
attention forward (ops.TRAIN_FWD_S3) and the SPLIT3 inference attention (ops.F32_SPLIT_ATTN), with the
max relative deviation of every gradient-norm group.

    python tools/video_golden_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd"), os.path.join(REPO, "tests")]

import numpy as np
import torch

from conftest import load_golden
from mhada_hip import ops
from mhada_hip.recipe import seeded_image
from mhada_hip.train import VideoTrainer
from test_train_cpu import build, grad_summary


def run(name):
    g = load_golden(name)
    fh, fw = (int(x) for x in g["frame_shape"])
    sh, sw = (int(x) for x in g["style_shape"])
    tr = VideoTrainer(*build("cuda"))
    style = seeded_image(2, sh, sw, int(g["seeds"][0])).cuda()
    c1, c2 = (seeded_image(2, fh, fw, int(x)).cuda() for x in g["seeds"][1:])
    out = tr.backward(style, c1, c2, torch.from_numpy(g["flow"]).cuda(), torch.from_numpy(g["mask"]).cuda())
    keys = ("loss_gs", "loss_lf", "loss_ot", "loss_ft", "loss_id1", "loss_id2", "loss")
    got = np.array([float(out[k].detach()) for k in keys])
    res = {"losses": float(np.max(np.abs(got / g["losses"] - 1)))}
    for n, m in (("vit_c", tr.vit_c), ("vit_s", tr.vit_s), ("ada", tr.ada)):
        ref = g[f"grad_{n}"]
        gs = grad_summary(m)
        big = ref > 1e-5 * ref.max()
        res[n] = float(np.max(np.abs(gs[big] / ref[big] - 1)))
    return res


for name in ("train_video_64_b2", "train_video_64x128_s64_b2"):
    for s3t in (True, False):
        for s3i in (True, False):
            ops.TRAIN_FWD_S3, ops.F32_SPLIT_ATTN = s3t, s3i
            r = run(name)
            print(f"{name:28s} train_fwd_s3={s3t!s:5s} infer_s3={s3i!s:5s} " +
                  " ".join(f"{k} {v:.2e}" for k, v in r.items()), flush=True)
