"""Flat-buffer Adam for the generator / discriminator (train_multi_gpu.py:295-296).

All parameters of a model live in ONE contiguous fp32 buffer (views), and their grads in one
more, so the optimiser step is a single encx_adam_step launch over the whole model and the
data-parallel gradient exchange is one RCCL all-reduce of one buffer (no bucketing needed at
59 MB on xGMI). Autograd accumulates into the pre-zeroed grad views in place.
"""
import torch

from . import distrib
from ._lib import call, ptr, stream


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (amsgrad off, no weight decay), one param group."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        params = [p for p in params if p.requires_grad]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.flat = torch.empty(n, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=torch.float32)
        self.n_step = 0
        o = 0
        self._views = []
        for p in params:
            k = p.numel()
            v = self.flat[o:o + k].view_as(p)
            v.copy_(p.data)
            p.data = v
            g = self.flat_grad[o:o + k].view_as(p)
            p.grad = g
            p._encx_flat = True  # encx ops accumulate this param's grad in place
            self._views.append((p, g))
            o += k

    def zero_grad(self, set_to_none: bool = False):
        self.flat_grad.zero_()
        for p, g in self._views:
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def gather_grads(self):
        """If autograd replaced a grad view with a fresh tensor, fold it back into the flat
        buffer (a safety net; normally a no-op)."""
        for p, g in self._views:
            if p.grad is not None and p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g

    def all_reduce_grads(self):
        if distrib.is_distributed():
            torch.distributed.all_reduce(self.flat_grad)
            self.flat_grad.div_(distrib.world_size())

    @torch.no_grad()
    def step(self, closure=None):
        self.gather_grads()
        self.n_step += 1
        grp = self.param_groups[0]
        b1, b2 = grp['betas']
        call('encx_adam_step', ptr(self.flat), ptr(self.flat_grad), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), self.flat.numel(), float(grp['lr']), float(b1), float(b2),
             float(grp['eps']), self.n_step, stream())
