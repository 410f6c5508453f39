"""Capture pieces of the train step into a HIP graph and compare with eager execution (debug aid
for encx.train.Trainer(graphs=True))."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'encodec-pytorch_amd'), os.path.join(ROOT, 'tests', 'golden')]
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from test_gpu_train_state import make_trainer, batches  # noqa: E402

DEV = 'cuda:0'


def snap(m):
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def restore(m, s):
    with torch.no_grad():
        for k, v in m.state_dict().items():
            v.copy_(s[k])


def cmp(name, a, b):
    a, b = a.detach().double(), b.detach().double()
    d = float((a - b).abs().max())
    print(f'{name:30s} max|diff| {d:.3e}  ref max {float(b.abs().max()):.3e}', flush=True)


def main():
    tr = make_trainer()
    xs = batches(2)
    tr.step(xs[0])
    m = tr.model
    m.train()
    s0 = snap(m)
    # 1) generator forward
    y_e, lw_e, _ = m(xs[1], bandwidth=6.0)
    codes_e = m.last_codes[0].clone()
    torch.cuda.synchronize()
    restore(m, s0)
    xs_static = xs[1].clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_g, lw_g, _ = m(xs_static, bandwidth=6.0)
        codes_g = m.last_codes[0]
    restore(m, s0)
    g.replay()
    torch.cuda.synchronize()
    cmp('fwd y', y_g, y_e)
    cmp('fwd loss_w', lw_g, lw_e)
    print('codes equal', bool(torch.equal(codes_g, codes_e)), flush=True)
    for k in s0:
        if '_codebook' in k:
            pass
    # 2) encoder only
    restore(m, s0)
    e_e = m.encoder(xs[1])
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        e_g = m.encoder(xs_static)
    g2.replay()
    torch.cuda.synchronize()
    cmp('encoder', e_g, e_e)
    # 3) decoder only
    q = e_e.detach().clone()
    d_e = m.decoder(q)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3):
        d_g = m.decoder(q)
    g3.replay()
    torch.cuda.synchronize()
    cmp('decoder', d_g, d_e)


def capture_mutation():
    """Does capturing the whole step (without replaying it) change any parameter / buffer?"""
    tr = make_trainer(graphs=True)
    xs = batches(2)
    tr.step(xs[0])
    torch.cuda.synchronize()
    before = snap(tr.model)
    before_d = snap(tr.disc)
    fb = tr.opt.flat.clone()
    orig = torch.cuda.CUDAGraph.replay
    torch.cuda.CUDAGraph.replay = lambda self: None
    tr.opt.prepare()
    tr.opt_d.prepare()
    tr._capture((6.0, True, tuple(xs[1].shape)), xs[1])
    torch.cuda.CUDAGraph.replay = orig
    torch.cuda.synchronize()
    after = snap(tr.model)
    for k in before:
        if not torch.equal(before[k], after[k]):
            cmp('MUTATED ' + k, after[k], before[k])
    after_d = snap(tr.disc)
    for k in before_d:
        if not torch.equal(before_d[k], after_d[k]):
            cmp('MUTATED disc ' + k, after_d[k], before_d[k])
    cmp('flat', tr.opt.flat, fb)
    print('capture_mutation done', flush=True)


def bisect():
    """Run the first n segments of the step eagerly and from one captured graph, from the same
    state; compare what they produce."""
    tr = make_trainer(graphs=True)
    xs = batches(2)
    tr.step(xs[0])
    torch.cuda.synchronize()
    s_m, s_d = snap(tr.model), snap(tr.disc)
    st = {k: getattr(tr.opt, k).clone() for k in ('flat', 'flat_grad', 'exp_avg', 'exp_avg_sq')}
    st_d = {k: getattr(tr.opt_d, k).clone() for k in ('flat', 'flat_grad', 'exp_avg', 'exp_avg_sq')}
    bst = {k: v.clone() for k, v in tr.balancer._state.items() if torch.is_tensor(v)}
    tr.opt.prepare()
    tr.opt_d.prepare()

    def reset():
        restore(tr.model, s_m)
        restore(tr.disc, s_d)
        for k, v in st.items():
            getattr(tr.opt, k).copy_(v)
        for k, v in st_d.items():
            getattr(tr.opt_d, k).copy_(v)
        for k, v in bst.items():
            tr.balancer._state[k].copy_(v)
        torch.cuda.synchronize()

    def grab(c):
        out = {}
        for k in ('y', 'loss_w'):
            if k in c:
                out[k] = c[k].detach().clone()
        for k, v in c.get('losses', {}).items():
            out['loss ' + k] = v.detach().clone()
        for k, v in c.get('out', {}).items():
            out['out ' + k] = v.detach().clone()
        out['flat'] = tr.opt.flat.clone()
        out['flat_grad'] = tr.opt.flat_grad.clone()
        out['disc flat'] = tr.opt_d.flat.clone()
        out['disc grad'] = tr.opt_d.flat_grad.clone()
        out['bal red'] = tr.balancer._state['red'].clone()
        return out

    for n in (1, 2, 3, 4):
        reset()
        segs, c = tr._segments(xs[1], 6.0, True, False)
        for sg, _ in segs[:n]:
            sg()
        torch.cuda.synchronize()
        e = grab(c)
        reset()
        xs_static = xs[1].clone()
        segs, c = tr._segments(xs_static, 6.0, True, False)
        parts = [sg for sg, _ in segs[:n]]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for sg in parts:
                sg()
        reset()
        g.replay()
        torch.cuda.synchronize()
        gr = grab(c)
        print(f'--- first {n} segment(s)', flush=True)
        for k in e:
            if k in gr:
                cmp(k, gr[k], e[k])
        del g


if __name__ == '__main__':
    bisect()
