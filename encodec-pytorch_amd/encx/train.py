"""One training step with the semantics of train_multi_gpu.py:train_one_step (:56-129).

The step is: forward -> (discriminator on real / fake) -> total_loss -> Balancer -> ONE backward
over [output, loss_w] with grads [balanced, 1] -> RCCL all-reduce of the flat generator grads
(world > 1) -> Adam; then, for the GAN configs, the discriminator update. It never reads a
device value on the host, so consecutive steps queue back to back.

Documented deviations: #7 a single combined backward (identical at
world_size 1; at world_size > 1 the commit-loss grads are all-reduced too, true DP);
#9 the discriminator is trained with an explicit probability instead of eval(bool).
"""
import random

import torch

from .balancer import Balancer
from . import distrib
from .losses import total_loss, disc_loss
from .model import EncodecModel
from .optim import FlatAdam
from .scheduler import WarmupCosineLrScheduler

DEFAULT_WEIGHTS = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}  # config/config.yaml:55-60


class Trainer:
    def __init__(self, model: EncodecModel, disc=None, lr=3e-4, disc_lr=3e-4, betas=(0.5, 0.9),
                 weights=None, max_iter=100000, warmup_iter=0, disc_prob=1.0, sample_rate=24000,
                 scheduler=True):
        self.model = model
        self.disc = disc
        self.sample_rate = sample_rate
        if distrib.is_distributed():
            distrib.broadcast_tensors(model.parameters())
            if disc is not None:
                distrib.broadcast_tensors(disc.parameters())
        self.opt = FlatAdam(model.parameters(), lr=lr, betas=betas)
        self.opt_d = FlatAdam(disc.parameters(), lr=disc_lr, betas=betas) if disc is not None else None
        w = dict(weights or DEFAULT_WEIGHTS)
        if disc is None:
            w = {k: w[k] for k in ('l_t', 'l_f')}
        self.balancer = Balancer(w)
        self.sched = self.sched_d = None
        if scheduler:
            self.sched = WarmupCosineLrScheduler(self.opt, max_iter=max_iter, eta_ratio=0.1,
                                                 warmup_iter=warmup_iter, warmup_ratio=1e-4)
            if disc is not None:
                self.sched_d = WarmupCosineLrScheduler(self.opt_d, max_iter=max_iter, eta_ratio=0.1,
                                                       warmup_iter=warmup_iter, warmup_ratio=1e-4)
        self.disc_prob = disc_prob

    def step(self, x):
        model, disc = self.model, self.disc
        model.train()
        self.opt.zero_grad()
        y, loss_w, _ = model(x)
        if disc is not None:
            disc.train()
            logits_real, fmap_real = disc(x, param_grads=False)
            logits_fake, fmap_fake = disc(y, param_grads=False)
            losses = total_loss(fmap_real, logits_fake, fmap_fake, x, y, self.sample_rate)
        else:
            losses = total_loss(None, None, None, x, y, self.sample_rate)
        out_grad = self.balancer.compute(losses, y)
        torch.autograd.backward([y, loss_w], [out_grad, torch.ones_like(loss_w)])
        self.opt.all_reduce_grads()
        self.opt.step()
        out = dict(losses)
        out['loss_w'] = loss_w
        if disc is not None:
            train_d = random.random() < self.disc_prob
            if distrib.is_distributed() and self.disc_prob < 1.0:
                t = torch.tensor([train_d], device=x.device)
                torch.distributed.broadcast(t, 0)
                train_d = bool(t.item())
            if train_d:
                self.opt_d.zero_grad()
                lr_, _ = disc(x)
                lf_, _ = disc(y.detach())
                ld = disc_loss(lr_, lf_)
                ld.backward()
                self.opt_d.all_reduce_grads()
                self.opt_d.step()
                out['l_d'] = ld
        if self.sched is not None:
            self.sched.step()
        if self.sched_d is not None:
            self.sched_d.step()
        return out
