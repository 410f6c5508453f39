"""Loss balancer (balancer.py of the reference) with its statistics kept on the device.

Per-item gradient norms, the EMA `averager` (fp64, like the reference's Python floats), the
cross-rank `average_metrics` all-reduce and the rescaled gradient sum all run as encx kernels
(and one RCCL all-reduce of nl+1 floats), so the balancer adds no host synchronisation.
"""
import torch
from torch import autograd

from . import distrib
from ._lib import call, ptr, stream, lib, ENCX_BALANCER_MAX_LOSSES


class Balancer:
    """balancer.py:31-118."""

    def __init__(self, weights, rescale_grads: bool = True, total_norm: float = 1.,
                 ema_decay: float = 0.999, per_batch_item: bool = True, epsilon: float = 1e-12,
                 monitor: bool = False):
        if len(weights) > ENCX_BALANCER_MAX_LOSSES:
            raise ValueError(f'encx Balancer combines up to {ENCX_BALANCER_MAX_LOSSES} losses')
        self.weights = weights
        self.per_batch_item = per_batch_item
        self.total_norm = total_norm
        self.beta = ema_decay
        self.epsilon = epsilon
        self.monitor = monitor
        self.rescale_grads = rescale_grads
        self._metrics = {}
        self._state = None

    @property
    def metrics(self):
        return self._metrics

    def _buffers(self, names, device):
        if self._state is None or self._state['names'] != names:
            nl = len(names)
            tw = sum(self.weights[k] for k in names)
            self._state = {
                'names': names,
                'total': torch.zeros(nl, device=device, dtype=torch.float64),
                'fix': torch.zeros(nl, device=device, dtype=torch.float64),
                'avg': torch.zeros(nl, device=device, dtype=torch.float64),
                'red': torch.zeros(nl + 1, device=device, dtype=torch.float32),
                'ratio': torch.tensor([self.weights[k] / tw for k in names], device=device,
                                      dtype=torch.float64),
                'plain': torch.tensor([float(self.weights[k]) for k in names], device=device,
                                      dtype=torch.float32),
                'norms': torch.zeros(nl, device=device, dtype=torch.float32),
                'scales': torch.zeros(nl, device=device, dtype=torch.float32),
                # five or more losses: the combine runs in calls of four grads, each later call
                # taking the previous out as g0 with scale 1 (the same left-to-right sum)
                'chain': torch.ones(max(0, -(-(nl - 4) // 3)), 4, device=device, dtype=torch.float32),
            }
        return self._state

    def combine(self, grads):
        """grads: ordered dict name -> d loss / d input. Returns the out_grad of :110-118."""
        self.combine_start(grads)
        self.reduce_stats()
        return self.combine_finish()

    # combine() in three parts, so a HIP-graph-captured step can run the cross-rank statistics
    # all-reduce eagerly between two captured segments (Trainer, graphs=True).
    def combine_start(self, grads):
        """Per-item norms and the EMA update (balancer.py:88-101) up to the all-reduce."""
        names = tuple(grads)
        g0 = next(iter(grads.values()))
        st = self._buffers(names, g0.device)
        s = stream()
        self._gl = [g.contiguous() for g in grads.values()]
        if self.rescale_grads:
            B = g0.shape[0] if self.per_batch_item else 1
            L = g0.numel() // B
            ws = torch.empty(lib.encx_item_norm_workspace(B) // 4, device=g0.device, dtype=torch.float32)
            for i, g in enumerate(self._gl):
                call('encx_item_norm_mean', ptr(g), ptr(st['norms'][i:i + 1]), ptr(ws), B, L, s)
            call('encx_balancer_update', ptr(st['norms']), ptr(st['total']), ptr(st['fix']),
                 ptr(st['avg']), ptr(st['red']), len(names), float(self.beta), float(B), s)

    def reduce_stats(self):
        """average_metrics (distrib.py:112-124): one all-reduce of nl+1 floats."""
        if self.rescale_grads and distrib.is_distributed():
            torch.distributed.all_reduce(self._state['red'])

    def combine_finish(self):
        """Scales and the rescaled gradient sum (balancer.py:102-118)."""
        st, gl, s = self._state, self._gl, stream()
        names = st['names']
        if self.rescale_grads:
            call('encx_balancer_scales', ptr(st['avg']), ptr(st['red']), ptr(st['ratio']),
                 ptr(st['scales']), len(names), float(self.total_norm), float(self.epsilon),
                 int(distrib.is_distributed()), s)
            scales = st['scales']
        else:
            scales = st['plain']
        out = torch.empty_like(gl[0])
        gp = [ptr(g) for g in gl[:4]] + [None] * (4 - len(gl[:4]))
        call('encx_balancer_combine', gp[0], gp[1], gp[2], gp[3], ptr(scales), ptr(out), out.numel(), s)
        for j, k0 in enumerate(range(4, len(gl), 3)):  # out += s_k g_k for the losses after the 4th
            k1 = min(k0 + 3, len(gl))
            sc = st['chain'][j]
            sc[1:1 + k1 - k0].copy_(scales[k0:k1])
            gp = [ptr(g) for g in gl[k0:k1]] + [None] * (3 - (k1 - k0))
            call('encx_balancer_combine', ptr(out), gp[0], gp[1], gp[2], ptr(sc), ptr(out), out.numel(), s)
        self._gl = None
        if self.monitor:
            avg = st['avg'].tolist()
            tot = sum(avg)
            self._metrics = {f'ratio_{k}': v / tot for k, v in zip(names, avg)}
        return out

    def grads(self, losses, input):
        return {name: autograd.grad(loss, [input], retain_graph=True)[0] for name, loss in losses.items()}

    def compute(self, losses, input):
        return self.combine(self.grads(losses, input))

    def backward(self, losses, input, retain_graph=False):
        input.backward(self.compute(losses, input), retain_graph=retain_graph)
