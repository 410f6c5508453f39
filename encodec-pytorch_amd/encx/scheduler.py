"""Learning-rate schedules (scheduler.py of the reference): host-side, no device work."""
import math

from torch.optim.lr_scheduler import _LRScheduler


class WarmupLrScheduler(_LRScheduler):
    """scheduler.py:27-63: ratio = warmup_ratio ** (1 - it/warmup_iter) ('exp') or linear."""

    def __init__(self, optimizer, warmup_iter=500, warmup_ratio=5e-4, warmup='exp', last_epoch=-1):
        self.warmup_iter = warmup_iter
        self.warmup_ratio = warmup_ratio
        self.warmup = warmup
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        ratio = self.get_lr_ratio()
        return [ratio * lr for lr in self.base_lrs]

    def get_lr_ratio(self):
        if self.last_epoch < self.warmup_iter:
            return self.get_warmup_ratio()
        return self.get_main_ratio()

    def get_main_ratio(self):
        raise NotImplementedError

    def get_warmup_ratio(self):
        assert self.warmup in ('linear', 'exp')
        alpha = self.last_epoch / self.warmup_iter
        if self.warmup == 'linear':
            return self.warmup_ratio + (1 - self.warmup_ratio) * alpha
        return self.warmup_ratio ** (1. - alpha)


class WarmupCosineLrScheduler(WarmupLrScheduler):
    """scheduler.py:112-132. The cosine phase uses last_epoch (not last_epoch - warmup_iter),
    reproduced as in the reference."""

    def __init__(self, optimizer, max_iter, eta_ratio=0, warmup_iter=500, warmup_ratio=5e-4,
                 warmup='exp', last_epoch=-1):
        self.eta_ratio = eta_ratio
        self.max_iter = max_iter
        super().__init__(optimizer, warmup_iter, warmup_ratio, warmup, last_epoch)

    def get_main_ratio(self):
        real_max_iter = self.max_iter - self.warmup_iter
        return self.eta_ratio + (1 - self.eta_ratio) * (
            1 + math.cos(math.pi * self.last_epoch / real_max_iter)) / 2
