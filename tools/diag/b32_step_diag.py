"""Diagnostic for tests/test_gpu_fullsize.py::test_config3_b32_step_vs_oracle_fp64: the second
step's output, per-loss grads w.r.t. the output and the balanced out_grad, ours against the fp64
oracle's (oracle.STEP_TRACE) from the same state. Run on a GPU box from the repo root."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), ROOT,
                os.path.join(ROOT, 'encodec-pytorch_amd')]
import steputil as S  # noqa: E402
from oracle import encodec_oracle as O  # noqa: E402
from synth import synth_wave  # noqa: E402

DEV = 'cuda:0'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def main():
    from encx.train import Trainer, DEFAULT_WEIGHTS
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from fixtures import disc_state
    from test_gpu_model import build
    m, p, cbs, cfg = build((6.0,), True, 3, np.stack([np.zeros((2, 128)), np.full((2, 128), 0.05)], 1)
                           .astype(np.float32)[[0] * 8], 4, 8)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.to(DEV)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False)
    x = torch.as_tensor(synth_wave((32, 1, 24000), 607)).to(DEV)
    tr.step(x)
    torch.cuda.synchronize()
    orig = S.oracle_step
    traces = []

    def traced(*a, **k):
        O.STEP_TRACE = tr_ = {}
        try:
            return orig(*a, **k)
        finally:
            O.STEP_TRACE = None
            traces.append(tr_)
    S.oracle_step = traced
    try:
        S.check_step(tr, x, cfg, 6.0, DEFAULT_WEIGHTS, device=DEV)
        print('check_step passed')
    except AssertionError as e:
        print('check_step failed:', str(e)[:600])
    t64, t32 = traces[0], traces[1]
    print('y: ours vs fp64', rel(tr.last_y, t64['y']), ' fp32 oracle vs fp64', rel(t32['y'], t64['y']))
    for k in t64['grads']:
        print(f'grad {k}: ours {rel(tr.last_loss_grads[k], t64["grads"][k]):.3e}  fp32 oracle '
              f'{rel(t32["grads"][k], t64["grads"][k]):.3e}')
    print(f'out_grad: ours {rel(tr.last_out_grad, t64["out_grad"]):.3e}  fp32 oracle '
          f'{rel(t32["out_grad"], t64["out_grad"]):.3e}')
    # a uniform scale error?
    for k in list(t64['grads']) + ['out_grad']:
        a = (tr.last_out_grad if k == 'out_grad' else tr.last_loss_grads[k]).double().cpu()
        b = (t64['out_grad'] if k == 'out_grad' else t64['grads'][k]).double().cpu()
        print(f'{k}: sum ratio - 1 = {float(a.sum() / b.sum() - 1):.3e}, norm ratio - 1 = {float(a.norm() / b.norm() - 1):.3e}, '
              f'per-item sums rel {float(((a.sum(-1) - b.sum(-1)).abs().max() / b.sum(-1).abs().max())):.3e}')


if __name__ == '__main__':
    main()
