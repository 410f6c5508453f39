"""Diagnostic: tests/test_gpu_48k.py::test_forward_48k_vs_oracle_fp64's grads, every parameter's
error vs fp64 and its ratio to the fp32 oracle's, in model order. Run on a GPU box from the repo
root (env ENCX_CONV2 etc. select the kernels)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), ROOT,
                os.path.join(ROOT, 'encodec-pytorch_amd')]
from oracle import encodec_oracle as O  # noqa: E402
from fixtures import load, T  # noqa: E402
from synth import rng  # noqa: E402
from test_gpu_48k import build48k, rel  # noqa: E402

DEV = 'cuda:0'


def main():
    d = load('g9_step48k.npz')
    m, p, cbs, cfg = build48k(d, 'gen/')
    m.train()
    x = T(d['gen/x']).to(DEV)
    y, loss_w, frames = m(x)
    gy = T(rng(95).standard_normal(size=tuple(y.shape)).astype(np.float32)).to(DEV)
    torch.autograd.backward([y, loss_w], [gy, torch.ones_like(loss_w)])
    out = {}
    for dt in (torch.float64, torch.float32):
        pp = {k: v.to(dt).requires_grad_(True) for k, v in p.items()}
        cc = [{k: v.to(dt) for k, v in cb.items()} for cb in cbs]
        yo, lw, _, _, _ = O.encodec_forward_train(T(d['gen/x']).to(dt), pp, cc, cfg, 3.0)
        torch.autograd.backward([yo, lw], [gy.cpu().to(dt), torch.ones_like(lw)])
        out[dt] = (yo, pp)
    print('y rel', rel(y, out[torch.float64][0]), flush=True)
    params = dict(m.named_parameters())
    for k in p:
        e = rel(params[k].grad, out[torch.float64][1][k].grad)
        e32 = rel(out[torch.float32][1][k].grad, out[torch.float64][1][k].grad)
        print(f'{k:60s} {e:.2e} {e32:.2e} {e / max(e32, 1e-12):8.1f}', flush=True)


if __name__ == '__main__':
    main()
