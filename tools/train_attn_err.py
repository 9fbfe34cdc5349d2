"""Errors of the training attention (forward + backward through MHAdaAttnFn) against fp64 autograd
for each training forward (ops.TRAIN_FWD_S3 / TRAIN_FWD_VT), with the reference's fp32 autograd as
the yardstick — over several seeds of tests/test_gpu_train_attn.py's shapes, so a form's
systematic error can be told from one draw's noise.

    python tools/train_attn_err.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import autograd_path, ops


def ref(q, k, v, x):
    a = torch.softmax(q @ k.transpose(1, 2), dim=-1)
    m = a @ v
    e2 = a @ (v * v)
    return torch.sqrt((e2 - m * m).clamp(min=1e-6)) * x + m


def rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-30)).item()


def main():
    cases = [(2, 128, 64, 0.4), (1, 37, 300, 0.6), (2, 256, 129, 1.5), (2, 600, 1000, 3.0), (2, 512, 4096, 1.0)]
    for BH, Nc, Ns, scale in cases:
        for seed in range(4):
            g = torch.Generator().manual_seed(Nc * 7 + Ns + 1000 * seed)
            q = torch.randn(BH, Nc, 64, generator=g) * scale
            k = torch.randn(BH, Ns, 64, generator=g) * scale
            v = torch.randn(BH, Ns, 64, generator=g) * 3
            v = v - v.mean(dim=1, keepdim=True)
            x = torch.randn(BH, Nc, 64, generator=g)
            dout = torch.randn(BH, Nc, 64, generator=g)
            ts = [t.double().requires_grad_() for t in (q, k, v, x)]
            r = ref(*ts)
            r.backward(dout.double())
            fs = [t.cuda().requires_grad_() for t in (q, k, v, x)]
            ref(*fs).backward(dout.cuda())
            line = f"BH {BH} Nc {Nc:4d} Ns {Ns:4d} scale {scale} seed {seed} | f32 " + " ".join(
                f"{n} {rel(c.grad.double().cpu(), b.grad):.1e}" for n, c, b in zip("qkvx", fs, ts))
            for form in ("s3", "vt"):
                ops.TRAIN_FWD_S3, ops.TRAIN_FWD_VT = form == "s3", form == "vt"
                gs = [t.cuda().requires_grad_() for t in (q, k, v, x)]
                out = autograd_path.MHAdaAttnFn.apply(*gs)
                out.backward(dout.cuda())
                line += f" | {form} out {rel(out.detach().double().cpu(), r.detach()):.1e} " + " ".join(
                    f"{n} {rel(a.grad.double().cpu(), b.grad):.1e}" for n, a, b in zip("qkvx", gs, ts))
            print(line, flush=True)


if __name__ == "__main__":
    main()
