"""Training path on the GPU: one train_image.py step against the reference's goldens, and a
full-size (512^2, batch 8) step running forward/backward/Adam with finite losses."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from mhada_hip.recipe import seeded_image
from mhada_hip.train import Trainer
from test_train_cpu import build, check_against_golden


def test_train_step_matches_reference_golden_gpu():
    check_against_golden(Trainer(*build("cuda")), "cuda")


def test_train_step_full_size_runs():
    tr = Trainer(*build("cuda"))
    c = seeded_image(8, 512, 512, 100).cuda()
    s = seeded_image(8, 512, 512, 101).cuda()
    l1 = tr.step(c, s)
    l2 = tr.step(c, s)
    assert all(np.isfinite(v) for v in l1.values()) and all(np.isfinite(v) for v in l2.values())
    assert l2["loss"] < l1["loss"] * 1.5  # one Adam step at lr 1e-4 does not blow up
