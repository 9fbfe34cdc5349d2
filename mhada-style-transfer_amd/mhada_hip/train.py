"""One training iteration of ``train_image.py:93-144`` on the drop-in modules, optionally data
parallel (one process per GPU, gradient all-reduce over RCCL — mhada_hip.parallel).

    trainer = Trainer(vit_c, vit_s, ada, vgg)            # 3 Adam optimisers, lr 1e-4
    losses = trainer.step(content, style)               # dict of the 4 weighted losses + total

The step: 4 ViT forwards, 3 AdaFormer forwards, 5 VGG19 forwards, global-style / local-feature
/ identity losses weighted 70 / 15 / 0.05 / 0.1, backward, (all-reduce), 3 Adam steps.
Checkpoints use the reference's dict layout (train_image.py:172-186).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import losses as L

LAMBDA_GS, LAMBDA_LF, LAMBDA_ID1, LAMBDA_ID2 = 70.0, 15.0, 5e-2, 1e-1  # train_image.py:19-22
# train_video.py:20-25
VIDEO_LAMBDA_GS, VIDEO_LAMBDA_LF, VIDEO_LAMBDA_OT, VIDEO_LAMBDA_FT = 100.0, 15.0, 2.0, 2.0
VIDEO_LAMBDA_ID1, VIDEO_LAMBDA_ID2 = 5e-2, 1e-1


class Trainer:
    def __init__(self, vit_c: nn.Module, vit_s: nn.Module, ada: nn.Module, vgg: nn.Module, lr: float = 1e-4,
                 activation: str = "softmax", distributed: Optional[bool] = None, bucket_mb: int = 25):
        import network
        self.vit_c, self.vit_s, self.ada, self.vgg = vit_c, vit_s, ada, vgg
        dev = next(vit_c.parameters()).device
        self.no_learn = nn.ModuleList([  # train_image.py:52-58
            network.AdaAttnForLoss(256, 64 + 128 + 256, activation),
            network.AdaAttnForLoss(512, 64 + 128 + 256 + 512, activation),
            network.AdaAttnForLoss(512, 64 + 128 + 256 + 512 + 512, activation),
        ]).to(dev).eval()
        self.vgg.eval()
        for p in self.vgg.parameters():
            p.requires_grad_(False)
        self.mse = nn.MSELoss(reduction="mean")
        self.batch_adaformer = True  # see losses()
        self.batch_vit = True  # see losses()
        # one backward pass per VGG feature map for the gs / lf / id2 terms (HIP; see _feature_losses)
        self.fused_feature_losses = dev.type == "cuda"
        # with the fused losses: the ReLU adjoints of the VGG feature maps relu2_1 .. relu5_1 applied by
        # their consumers (FeatureLossFn / the next conv's dgrad) instead of a relu_bwd pass (bit-identical)
        self.masked_vgg_features = True
        self.opt_vit_c = torch.optim.Adam(vit_c.parameters(), lr=lr)
        self.opt_vit_s = torch.optim.Adam(vit_s.parameters(), lr=lr)
        self.opt_ada = torch.optim.Adam(ada.parameters(), lr=lr)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.reducer = None
        if distributed:
            from .parallel import GradAllReducer
            params = list(vit_c.parameters()) + list(vit_s.parameters()) + list(ada.parameters())
            self.reducer = GradAllReducer(params, bucket_bytes=bucket_mb << 20)

    def close(self) -> None:
        """Remove the all-reduce hooks from the parameters (a new Trainer on the same modules
        installs its own)."""
        if self.reducer is not None:
            self.reducer.remove()
            self.reducer = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def losses(self, content: torch.Tensor, style: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Forward + weighted losses (train_image.py:103-136).

        The reference's three AdaFormer calls (cs, cc, ss: train_image.py:105,109-110) run as ONE
        call over their concatenated batch when ``batch_adaformer`` is set (the default): every op
        of the MHAda blocks and the decoder is per sample (InstanceNorm statistics, attention and
        convolutions never mix images), so the outputs are the same, while each AdaFormer
        parameter gets one weight-gradient reduction over 3B images instead of three gradients
        summed by autograd (~640 small add launches per step) and every launch is 3x larger.
        Likewise ``batch_vit`` (the default, on the GPU) runs each ViT's two calls (vit_c on content
        and style, vit_s on style and content) as one call over the concatenated batch; their
        batch-axis attention (vit.py:48) couples the images of ONE call, so it runs per call
        (vit_forward(groups=2)) while every other op (per token) sees the 2B images at once."""
        if self.batch_vit and content.is_cuda and content.shape == style.shape:
            # each ViT's two calls as one over the concatenated batch, the batch-axis attention
            # per call (autograd_path.vit_forward groups): the same outputs, one weight-gradient
            # GEMM per parameter instead of two partial ones summed by autograd (~150 add launches)
            from .autograd_path import vit_forward
            B = content.shape[0]
            fc_vc, fs_vc = zip(*(o.split(B) for o in vit_forward(self.vit_c, torch.cat([content, style]), groups=2)))
            fs_vs, fc_vs = zip(*(o.split(B) for o in vit_forward(self.vit_s, torch.cat([style, content]), groups=2)))
            fc_vc, fs_vc, fs_vs, fc_vs = (list(t) for t in (fc_vc, fs_vc, fs_vs, fc_vs))
        else:
            fc_vc = self.vit_c(content)
            fs_vs = self.vit_s(style)
            fc_vs = self.vit_s(content)
            fs_vc = self.vit_c(style)
        if self.batch_adaformer:
            B = content.shape[0]
            _, out = self.ada([torch.cat(t) for t in zip(fc_vc, fc_vc, fs_vc)],
                              [torch.cat(t) for t in zip(fs_vs, fc_vs, fs_vs)])
            cs, cc, ss = out.split(B)
        else:
            _, cs = self.ada(fc_vc, fs_vs)
            _, cc = self.ada(fc_vc, fc_vs)
            _, ss = self.ada(fs_vc, fs_vs)
        vgg_fs = self.vgg(style)
        vgg_fc = self.vgg(content)
        if self.fused_feature_losses and self.masked_vgg_features:
            # the three feature dicts that take gradients feed only _feature_losses' FeatureLossFn
            # (relu_input=True): the ReLU adjoints of relu2_1 .. relu5_1 are applied by their consumers
            from .autograd_path import vgg19_forward
            vgg_fcs, vgg_fcc, vgg_fss = (vgg19_forward(self.vgg, x, masked_features=True) for x in (cs, cc, ss))
        else:
            vgg_fcs = self.vgg(cs)
            vgg_fcc = self.vgg(cc)
            vgg_fss = self.vgg(ss)
        if self.fused_feature_losses:
            gs, lf, id2 = self._feature_losses(vgg_fc, vgg_fs, vgg_fcs, vgg_fcc, vgg_fss)
            gs, lf, id2 = gs * LAMBDA_GS, lf * LAMBDA_LF, id2 * LAMBDA_ID2
        else:
            gs = L.global_style_loss(vgg_fcs, vgg_fs, self.mse) * LAMBDA_GS
            lf = L.local_feature_loss(vgg_fc, vgg_fs, vgg_fcs, self.no_learn, self.mse) * LAMBDA_LF
            id2 = L.identity_loss_2(vgg_fcc, vgg_fc, vgg_fss, vgg_fs, self.mse) * LAMBDA_ID2
        id1 = L.identity_loss_1(cc, content, ss, style, self.mse) * LAMBDA_ID1
        return {"loss_gs": gs, "loss_lf": lf, "loss_id1": id1, "loss_id2": id2, "loss": gs + lf + id1 + id2}

    def _feature_losses(self, fc, fs, fcs, fcc, fss):
        """global_style_loss, local_feature_loss and identity_loss_2 (lossfn.py:7-47) with each
        VGG feature map's terms on train_fns.FeatureLossFn: the same loss values, summed in the
        reference's order, and one backward pass per feature map."""
        from .train_fns import feature_loss_terms, feature_mean_std
        gs = lf = id2 = 0
        for i in (1, 2, 3, 4, 5):
            k = f"relu{i}_1"
            t = None
            if i >= 3:  # lossfn.py:26-34: the AdaAttN target of the content / style features
                t = self.no_learn[i - 3](fc[k], fs[k], L.feature_down_sample(fc, i), L.feature_down_sample(fs, i))
            m = i >= 2 and self.masked_vgg_features  # relu2_1 .. relu5_1 from vgg19_forward(masked_features=True)
            lm, ls, lmse = feature_loss_terms(fcs[k], *feature_mean_std(fs[k]), t, relu_input=m)
            gs = gs + (lm + ls)  # lossfn.py:21: loss += mean_dist + std_dist
            if t is not None:
                lf = lf + lmse
            a = feature_loss_terms(fcc[k], t=fc[k], relu_input=m)[2]
            b = feature_loss_terms(fss[k], t=fs[k], relu_input=m)[2]
            id2 = id2 + a + b
        return gs, lf, id2

    def zero_grad(self) -> None:
        for o in (self.opt_vit_c, self.opt_vit_s, self.opt_ada):
            o.zero_grad()

    def backward(self, content: torch.Tensor, style: torch.Tensor) -> Dict[str, torch.Tensor]:
        """zero_grad + forward + backward + (all-reduce); no optimizer step."""
        self.zero_grad()
        out = self.losses(content, style)
        out["loss"].backward()
        if self.reducer is not None:
            self.reducer.finish()
        return out

    def step(self, content: torch.Tensor, style: torch.Tensor) -> Dict[str, float]:
        out = self.backward(content, style)
        self.opt_vit_c.step()
        self.opt_vit_s.step()
        self.opt_ada.step()
        return {k: float(v.detach()) for k, v in out.items()}

    def checkpoint(self, epoch: int, batch_size: int) -> dict:
        """The reference's checkpoint dict (train_image.py:172-186)."""
        return {
            "epoch": epoch,
            "batch_size": batch_size,
            "model_state": {"adaFormer": self.ada.state_dict(), "vit_c": self.vit_c.state_dict(),
                            "vit_s": self.vit_s.state_dict()},
            "optim_state": {"adaFormer": self.opt_ada.state_dict(), "vit_c": self.opt_vit_c.state_dict(),
                            "vit_s": self.opt_vit_s.state_dict()},
        }

    def load_checkpoint(self, ckpt: dict) -> None:
        """Resume (train_image.py:75-84)."""
        self.ada.load_state_dict(ckpt["model_state"]["adaFormer"])
        self.vit_c.load_state_dict(ckpt["model_state"]["vit_c"])
        self.vit_s.load_state_dict(ckpt["model_state"]["vit_s"])
        self.opt_ada.load_state_dict(ckpt["optim_state"]["adaFormer"])
        self.opt_vit_c.load_state_dict(ckpt["optim_state"]["vit_c"])
        self.opt_vit_s.load_state_dict(ckpt["optim_state"]["vit_s"])


class VideoTrainer(Trainer):
    """One iteration of ``train_video.py:110-171`` (fine-tuning on frame pairs with optical flow):
    5 AdaFormer calls (cs1, cs2, cc1, cc2, ss), VGG19 of the 3 inputs (no grad) and the 5 outputs,
    global-style / local-feature losses of both frames, the output- and feature-level temporal
    losses (lossfn.py:50-86: the warps and their adjoints on HIP, video.WarpFn), identity losses,
    weighted 100 / 15 / 2 / 2 / 0.05 / 0.1.

        trainer = VideoTrainer(vit_c, vit_s, ada, vgg)
        losses = trainer.step(style, c1, c2, flow, mask)   # the data loader's tuple order

    Data parallel as Trainer (gradient all-reduce = mean over ranks); the temporal losses normalise
    by each rank's own nonzero-mask count, so N ranks equal one process only when the counts match
    (the reference trains video on one GPU)."""

    def video_losses(self, style, c1, c2, flow, mask) -> Dict[str, torch.Tensor]:
        """train_video.py:110-166.  As in Trainer.losses, calls of one module on inputs of one shape
        run as one call over the concatenated batch (train_video.py's frames are 256x512 and its
        style 256x256: each ViT's two frame calls, the AdaFormer's (frame, style) pair cs1 / cs2 and
        its (frame, frame) pair cc1 / cc2)."""
        fc1_c, fc2_c, fs_c = self._vit_calls(self.vit_c, (c1, c2, style))
        fs_s, fc1_s, fc2_s = self._vit_calls(self.vit_s, (style, c1, c2))
        (ada_fcs1, cs1), (ada_fcs2, cs2), (_, cc1), (_, cc2), (_, ss) = self._ada_calls(
            ((fc1_c, fs_s), (fc2_c, fs_s), (fc1_c, fc1_s), (fc2_c, fc2_s), (fs_c, fs_s)))
        with torch.no_grad():
            vgg_fc1, vgg_fc2, vgg_fs = self.vgg(c1), self.vgg(c2), self.vgg(style)
        if self.fused_feature_losses and self.masked_vgg_features:
            from .autograd_path import vgg19_forward
            vgg_fcs1, vgg_fcs2, vgg_fcc1, vgg_fcc2, vgg_fss = (vgg19_forward(self.vgg, x, masked_features=True)
                                                               for x in (cs1, cs2, cc1, cc2, ss))
        else:
            vgg_fcs1, vgg_fcs2, vgg_fcc1, vgg_fcc2, vgg_fss = (self.vgg(x) for x in (cs1, cs2, cc1, cc2, ss))
        if self.fused_feature_losses:
            gs, lf, id2 = self._video_feature_losses(vgg_fc1, vgg_fc2, vgg_fs, vgg_fcs1, vgg_fcs2, vgg_fcc1,
                                                     vgg_fcc2, vgg_fss)
        else:
            gs = L.global_style_loss(vgg_fcs1, vgg_fs, self.mse) + L.global_style_loss(vgg_fcs2, vgg_fs, self.mse)
            lf = (L.local_feature_loss(vgg_fc1, vgg_fs, vgg_fcs1, self.no_learn, self.mse)
                  + L.local_feature_loss(vgg_fc2, vgg_fs, vgg_fcs2, self.no_learn, self.mse))
            id2 = 0
            for i in (1, 2, 3, 4, 5):
                k = f"relu{i}_1"
                id2 = id2 + self.mse(vgg_fcc1[k], vgg_fc1[k]) + self.mse(vgg_fcc2[k], vgg_fc2[k]) \
                    + self.mse(vgg_fss[k], vgg_fs[k])
        mse_matrix = nn.MSELoss(reduction="none")
        ot = L.output_level_temporal_loss(c1, c2, cs1, cs2, flow, mask, mse_matrix) * VIDEO_LAMBDA_OT
        ft = L.feature_level_temporal_loss(ada_fcs1, ada_fcs2, flow, mask, mse_matrix) * VIDEO_LAMBDA_FT
        id1 = (self.mse(cc1, c1) + self.mse(cc2, c2) + self.mse(ss, style)) * VIDEO_LAMBDA_ID1
        gs, lf, id2 = gs * VIDEO_LAMBDA_GS, lf * VIDEO_LAMBDA_LF, id2 * VIDEO_LAMBDA_ID2
        return {"loss_gs": gs, "loss_lf": lf, "loss_ot": ot, "loss_ft": ft, "loss_id1": id1, "loss_id2": id2,
                "loss": gs + lf + ot + ft + id1 + id2}

    def _vit_calls(self, vit, xs):
        """vit(x) for each x; inputs of one shape as one grouped call (batch-axis attention per call,
        autograd_path.vit_forward groups) when batch_vit is set on the device."""
        out = [None] * len(xs)
        for idx in _shape_groups([x.shape for x in xs]):
            if len(idx) > 1 and self.batch_vit and xs[idx[0]].is_cuda:
                from .autograd_path import vit_forward
                B = xs[idx[0]].shape[0]
                parts = zip(*(o.split(B) for o in vit_forward(vit, torch.cat([xs[i] for i in idx]), groups=len(idx))))
                for i, p in zip(idx, parts):
                    out[i] = list(p)
            else:
                for i in idx:
                    out[i] = vit(xs[i])
        return out

    def _ada_calls(self, calls):
        """self.ada(fc, fs) for each call; calls whose features have one shape as one call over the
        concatenated batch when batch_adaformer is set (every AdaFormer op is per image)."""
        out = [None] * len(calls)
        for idx in _shape_groups([(fc[0].shape, fs[0].shape) for fc, fs in calls]):
            if len(idx) > 1 and self.batch_adaformer:
                B = calls[idx[0]][0][0].shape[0]
                fcs, cs = self.ada([torch.cat(t) for t in zip(*(calls[i][0] for i in idx))],
                                   [torch.cat(t) for t in zip(*(calls[i][1] for i in idx))])
                for i, a, b in zip(idx, fcs.split(B), cs.split(B)):
                    out[i] = (a, b)
            else:
                for i in idx:
                    out[i] = self.ada(*calls[i])
        return out

    def _video_feature_losses(self, fc1, fc2, fs, fcs1, fcs2, fcc1, fcc2, fss):
        """The gs / lf / id2 sums of train_video.py:133-165 on train_fns.FeatureLossFn (one backward
        pass per feature map and output), in the reference's summation order."""
        from .train_fns import feature_loss_terms, feature_mean_std
        gs1 = gs2 = lf1 = lf2 = id2 = 0
        for i in (1, 2, 3, 4, 5):
            k = f"relu{i}_1"
            m = i >= 2 and self.masked_vgg_features
            ref = feature_mean_std(fs[k])
            t1 = t2 = None
            if i >= 3:
                fds = L.feature_down_sample(fs, i)
                t1 = self.no_learn[i - 3](fc1[k], fs[k], L.feature_down_sample(fc1, i), fds)
                t2 = self.no_learn[i - 3](fc2[k], fs[k], L.feature_down_sample(fc2, i), fds)
            lm1, ls1, lmse1 = feature_loss_terms(fcs1[k], *ref, t1, relu_input=m)
            lm2, ls2, lmse2 = feature_loss_terms(fcs2[k], *ref, t2, relu_input=m)
            gs1, gs2 = gs1 + (lm1 + ls1), gs2 + (lm2 + ls2)
            if i >= 3:
                lf1, lf2 = lf1 + lmse1, lf2 + lmse2
            id2 = id2 + feature_loss_terms(fcc1[k], t=fc1[k], relu_input=m)[2] \
                + feature_loss_terms(fcc2[k], t=fc2[k], relu_input=m)[2] + feature_loss_terms(fss[k], t=fs[k], relu_input=m)[2]
        return gs1 + gs2, lf1 + lf2, id2

    def backward(self, style, c1, c2, flow, mask) -> Dict[str, torch.Tensor]:
        """zero_grad + forward + backward + (all-reduce); no optimizer step."""
        self.zero_grad()
        out = self.video_losses(style, c1, c2, flow, mask)
        out["loss"].backward()
        if self.reducer is not None:
            self.reducer.finish()
        return out

    def step(self, style, c1, c2, flow, mask) -> Dict[str, float]:
        out = self.backward(style, c1, c2, flow, mask)
        self.opt_vit_c.step()
        self.opt_vit_s.step()
        self.opt_ada.step()
        return {k: float(v.detach()) for k, v in out.items()}


def _shape_groups(keys):
    """Indices grouped by equal key, groups in order of first appearance."""
    groups = {}
    for i, k in enumerate(keys):
        groups.setdefault(k, []).append(i)
    return list(groups.values())
