"""Flat-buffer Adam for the generator / discriminator (train_multi_gpu.py:295-296).

All parameters of a model live in ONE contiguous fp32 buffer (views), and their grads in one
more, so the optimiser step is a single encx_adam_step launch over the whole model and the
data-parallel gradient exchange is a handful of RCCL all-reduces over slices of one buffer.
Autograd accumulates into the pre-zeroed grad views in place.

state_dict / load_state_dict use torch.optim.Adam's layout (per-parameter 'step', 'exp_avg',
'exp_avg_sq'; one param group with Adam's keys), so checkpoints interchange with the
reference's `optimizer_state_dict` (train_multi_gpu.py:303-308, utils.py:132-148).
"""
import torch

from . import distrib
from ._lib import call, ptr, stream

_ADAM_GROUP_DEFAULTS = dict(weight_decay=0, amsgrad=False, maximize=False, foreach=None,
                            capturable=False, differentiable=False, fused=None)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (amsgrad off, no weight decay), one param group."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        params = [p for p in params if p.requires_grad]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, **_ADAM_GROUP_DEFAULTS))
        dev = params[0].device
        n = sum(p.numel() for p in params)
        self.flat = torch.empty(n, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=torch.float32)
        self.hp = torch.zeros(8, device=dev, dtype=torch.float32)  # per-step scalars (encx_adam_hyper)
        self.n_step = 0
        o = 0
        self._views = []
        self.offsets = []
        for p in params:
            k = p.numel()
            v = self.flat[o:o + k].view_as(p)
            v.copy_(p.data)
            p.data = v
            g = self.flat_grad[o:o + k].view_as(p)
            p.grad = g
            p._encx_flat = True  # encx ops accumulate this param's grad in place
            self._views.append((p, g))
            self.offsets.append((o, k))
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

    def span(self, params):
        """(start, end) of the flat-grad slice holding `params` (must be contiguous)."""
        ids = {id(p) for p in params}
        offs = [(o, k) for (p, _), (o, k) in zip(self._views, self.offsets) if id(p) in ids]
        a, b = min(o for o, _ in offs), max(o + k for o, k in offs)
        if sum(k for _, k in offs) != b - a:
            raise ValueError('encx FlatAdam.span: params are not contiguous in the flat buffer')
        return a, b

    def reduce_async(self, a=0, b=None):
        """Start the RCCL sum of flat_grad[a:b] over the ranks and return its work handle. The
        collective runs on the communicator's stream, ordered after the work already queued on
        the current stream, so it overlaps whatever the current stream does next (the rest of
        the backward, the discriminator phase); work.wait() orders the current stream after it."""
        return torch.distributed.all_reduce(self.flat_grad[a:b], async_op=True)

    def all_reduce_grads(self, scale=True):
        """Sum flat_grad over ranks in one collective, then divide by the world size unless
        scale=False."""
        if not distrib.is_distributed():
            return
        self.reduce_async().wait()
        if scale:
            self.flat_grad.div_(distrib.world_size())

    def prepare(self):
        """Host half of a step: advance the step count and write this step's scalars into
        self.hp with one small launch (its arguments are fixed at launch time, so the host may
        run steps ahead of the device)."""
        self.n_step += 1
        self._opt_called = True  # what torch's LR-scheduler step-order check looks for
        grp = self.param_groups[0]
        b1, b2 = grp['betas']
        call('encx_adam_hyper', ptr(self.hp), float(grp['lr']), float(b1), float(b2),
             float(grp['eps']), self.n_step, stream())

    def launch(self):
        """Device half: the update itself, reading self.hp (HIP-graph capturable)."""
        self.gather_grads()
        call('encx_adam_step_dev', ptr(self.flat), ptr(self.flat_grad), ptr(self.exp_avg),
             ptr(self.exp_avg_sq), self.flat.numel(), ptr(self.hp), stream())

    @torch.no_grad()
    def step(self, closure=None):
        self.prepare()
        self.launch()

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self):
        """torch.optim.Adam.state_dict() layout: {'state': {i: {'step', 'exp_avg',
        'exp_avg_sq'}}, 'param_groups': [{..., 'params': [0..n-1]}]} (no state before the first
        step, as torch's Adam)."""
        state = {}
        if self.n_step > 0:
            for i, ((p, _), (o, k)) in enumerate(zip(self._views, self.offsets)):
                state[i] = {'step': torch.tensor(float(self.n_step)),
                            'exp_avg': self.exp_avg[o:o + k].view_as(p).clone(),
                            'exp_avg_sq': self.exp_avg_sq[o:o + k].view_as(p).clone()}
        grp = {k: v for k, v in self.param_groups[0].items() if k != 'params'}
        grp['params'] = list(range(len(self._views)))
        return {'state': state, 'param_groups': [grp]}

    @torch.no_grad()
    def load_state_dict(self, state_dict):
        """Accepts FlatAdam's or torch.optim.Adam's state dict (same layout)."""
        groups = state_dict['param_groups']
        if len(groups) != 1 or len(groups[0]['params']) != len(self._views):
            raise ValueError('encx FlatAdam: state dict must hold one param group with '
                             f'{len(self._views)} params')
        g = groups[0]
        if g.get('weight_decay', 0) != 0 or g.get('amsgrad', False) or g.get('maximize', False):
            raise ValueError('encx FlatAdam: weight_decay / amsgrad / maximize are not supported')
        for k, v in g.items():
            if k != 'params':
                self.param_groups[0][k] = v
        ids = g['params']
        state = state_dict['state']
        if not state:
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            self.n_step = 0
            return
        steps = set()
        for (p, _), (o, k), pid in zip(self._views, self.offsets, ids):
            s = state[pid]
            steps.add(int(float(s['step'])))
            self.exp_avg[o:o + k].copy_(s['exp_avg'].reshape(-1))
            self.exp_avg_sq[o:o + k].copy_(s['exp_avg_sq'].reshape(-1))
        if len(steps) != 1:
            raise ValueError(f'encx FlatAdam: one shared step count expected, got {sorted(steps)}')
        self.n_step = steps.pop()
