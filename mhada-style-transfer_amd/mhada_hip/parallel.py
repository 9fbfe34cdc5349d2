"""Data parallelism for the training path: one process per GPU, ONE exchange
step per iteration — the gradient all-reduce (sum, then / world) over RCCL (torch.distributed
backend "nccl" on ROCm; "gloo" for CPU tests).

The reference trains single-GPU (train_image.py:31-186); this is the build's only collective.
Gradients are packed into ~25 MB flat buckets in reverse parameter order (the order backward
produces them) and each bucket's all-reduce is launched asynchronously from the parameter
post-accumulate-grad hook of its last gradient, so communication overlaps the rest of the
backward pass.  `finish()` waits, averages and scatters the results back into `.grad`.

Exactness: every image loss is a mean over equal-size shards, so the average of per-rank
gradients equals the gradient of the global-batch mean — the single-process oracle is
micro-batch gradient accumulation (the ViT's batch-axis attention couples only the images of
one forward call, so a rank's micro-batch is one reference forward call).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


class GradAllReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_bytes: int = 25 << 20,
                 group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self._bucket_of[id(p)] = bi
        self._flat = [None] * len(self.buckets)
        self._pending = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.reset()

    def reset(self) -> None:
        self._pending = [len(b) for b in self.buckets]
        self._handles = [None] * len(self.buckets)

    def _launch(self, bi: int) -> None:
        ps = self.buckets[bi]
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
        flat = self._flat[bi]
        if flat is None or flat.device != grads[0].device or flat.dtype != grads[0].dtype:
            flat = torch.empty(sum(g.numel() for g in grads), device=grads[0].device, dtype=grads[0].dtype)
            self._flat[bi] = flat
        torch.cat([g.reshape(-1) for g in grads], out=flat)
        self._handles[bi] = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        bi = self._bucket_of[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def finish(self) -> None:
        """Wait for every bucket (launching those whose parameters got no gradient this step),
        average, and write the reduced values back into .grad.  A parameter that got no gradient
        (grad None: unused by this step's graph, the same on every rank) contributes zeros to its
        bucket and KEEPS grad None, so Adam skips it exactly as in the single-GPU reference."""
        for bi in range(len(self.buckets)):
            if self._handles[bi] is None:
                self._launch(bi)
        for bi, ps in enumerate(self.buckets):
            self._handles[bi].wait()
            flat = self._flat[bi]
            flat.div_(self.world)
            off = 0
            for p in ps:
                n = p.numel()
                if p.grad is not None:
                    p.grad.copy_(flat[off:off + n].view_as(p))
                off += n
        self.reset()

    def remove(self) -> None:
        """Detach the gradient hooks (Trainer.close): a later reducer on the same parameters must
        not share them, or extra all-reduces would mismatch the collectives across ranks."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
