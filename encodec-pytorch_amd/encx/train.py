"""One training step with the semantics of train_multi_gpu.py:train_one_step (:56-129).

The step is: forward -> (discriminator on real / fake) -> total_loss -> Balancer -> ONE backward
over [output, loss_w] with grads [balanced, 1] -> RCCL all-reduce of the flat generator grads
(world > 1) -> Adam; then, for the GAN configs, the discriminator update. It never reads a
device value on the host, so consecutive steps queue back to back.

The discriminator runs forward ONCE per step on the real and on the fake audio. The reference
runs it twice on each (train_multi_gpu.py:62-63 in the generator phase, :114-116 in the
discriminator phase); the discriminator's weights and the generator output are unchanged in
between (only the generator's Adam step runs there), so the second pair of forwards is
value-identical recomputation. Here the generator phase differentiates the shared graph w.r.t.
the audio only and the discriminator phase w.r.t. the weights only (ops.DiscGradMode); the
fake branch is fed a detached leaf of the output, so the discriminator phase never reaches the
generator graph, as the reference's output.detach() (:116).

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
from .ops import DiscGradMode
from .optim import FlatAdam
from .scheduler import WarmupCosineLrScheduler

DEFAULT_WEIGHTS = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}  # config/config.yaml:55-60


class Trainer:
    def __init__(self, model: EncodecModel, disc=None, lr=3e-4, disc_lr=3e-4, betas=(0.5, 0.9),
                 weights=None, max_iter=100000, warmup_iter=0, disc_prob=1.0, sample_rate=24000,
                 scheduler=True, balancer_kwargs=None):
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
        self.balancer = Balancer(w, **(balancer_kwargs or {}))
        self.sched = self.sched_d = None
        if scheduler:
            self.sched = WarmupCosineLrScheduler(self.opt, max_iter=max_iter, eta_ratio=0.1,
                                                 warmup_iter=warmup_iter, warmup_ratio=1e-4)
            if disc is not None:
                self.sched_d = WarmupCosineLrScheduler(self.opt_d, max_iter=max_iter, eta_ratio=0.1,
                                                       warmup_iter=warmup_iter, warmup_ratio=1e-4)
        self.disc_prob = disc_prob
        self.disc_mode = DiscGradMode()

    def step(self, x):
        model, disc = self.model, self.disc
        model.train()
        self.opt.zero_grad()
        y, loss_w, _ = model(x)
        if disc is not None:
            disc.train()
            # generator phase: the balancer's autograd.grad calls differentiate the shared
            # discriminator graph w.r.t. the fake audio only
            self.disc_mode.set(params=False, input=True)
            yd = y.detach().requires_grad_()
            logits_real, fmap_real = disc(x, mode=self.disc_mode)
            logits_fake, fmap_fake = disc(yd, mode=self.disc_mode)
            losses = total_loss(fmap_real, logits_fake, fmap_fake, x, yd, self.sample_rate)
            out_grad = self.balancer.compute(losses, yd)
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
                # discriminator phase on the same graph: weight grads only (train_multi_gpu.py:112-124)
                self.disc_mode.set(params=True, input=False)
                self.opt_d.zero_grad()
                ld = disc_loss(logits_real, logits_fake)
                ld.backward()
                self.opt_d.all_reduce_grads()
                self.opt_d.step()
                out['l_d'] = ld
            del logits_real, fmap_real, logits_fake, fmap_fake
        if self.sched is not None:
            self.sched.step()
        if self.sched_d is not None:
            self.sched_d.step()
        return out

    # ------------------------------------------------------------------ checkpoints
    def state_dicts(self):
        """The four state dicts the reference checkpoints (utils.py:132-148)."""
        return {'optimizer': self.opt.state_dict(),
                'scheduler': self.sched.state_dict() if self.sched is not None else None,
                'disc_optimizer': self.opt_d.state_dict() if self.opt_d is not None else None,
                'disc_scheduler': self.sched_d.state_dict() if self.sched_d is not None else None}

    def load_state_dicts(self, optimizer=None, scheduler=None, disc_optimizer=None, disc_scheduler=None):
        """train_multi_gpu.py:303-307."""
        if optimizer is not None:
            self.opt.load_state_dict(optimizer)
        if scheduler is not None and self.sched is not None:
            self.sched.load_state_dict(scheduler)
        if disc_optimizer is not None and self.opt_d is not None:
            self.opt_d.load_state_dict(disc_optimizer)
        if disc_scheduler is not None and self.sched_d is not None:
            self.sched_d.load_state_dict(disc_scheduler)
