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


def decoder_walk(m, x, seg, x64=None):
    """The decoder layer by layer on the real latent: each conv / block against its fp64
    restatement from the same fp32 input (test_gpu_fullsize._fp64_layer), and the chained error
    (our chain vs the fp64 chain from the same latent)."""
    from test_gpu_fullsize import _fp64_layer
    from encx.modules.conv import SConv1d, SConvTranspose1d
    from encx.modules.seanet import SEANetResnetBlock
    from encx.modules.lstm import SLSTM
    act = None
    x64 = x.double() if x64 is None else x64
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
        for i, mod in enumerate(m.decoder.model):
            if isinstance(mod, torch.nn.ELU):
                act = 'elu'
                continue
            if isinstance(mod, SLSTM):
                y = mod(x)
                pp = {'m.' + k: v.double() for k, v in mod.named_parameters()}
                y1 = O.slstm(x.double(), pp, 'm', mod.lstm.num_layers)
                yc = O.slstm(x64, pp, 'm', mod.lstm.num_layers)
            else:
                y = mod(x) if isinstance(mod, SEANetResnetBlock) else mod(x, act=act)
                y1, _ = _fp64_layer(mod, x.double(), act)
                yc, _ = _fp64_layer(mod, x64, act)
            print(f'  seg {seg} decoder.model.{i} {type(mod).__name__} {tuple(x.shape)}: layer rel {rel(y, y1):.2e} '
                  f'chain rel {rel(y, yc):.2e}', flush=True)
            x, x64, act = y, yc.detach(), None


def main():
    d = load('g9_step48k.npz')
    m, p, cbs, cfg = build48k(d, 'gen/')
    m.train()
    x = T(d['gen/x']).to(DEV)
    from encx.modules.conv import SConv1d, SConvTranspose1d
    from encx.modules.seanet import SEANetResnetBlock
    from encx.modules.lstm import SLSTM
    from test_gpu_fullsize import _fp64_layer
    seen, hooks = [], []
    for name, mod in m.named_modules():
        if isinstance(mod, (SConv1d, SConvTranspose1d, SEANetResnetBlock, SLSTM)) and '.block.' not in name \
                and '.shortcut' not in name:
            def hook(mod_, args, kwargs, out, name=name):
                seen.append((name, mod_, args[0].detach().clone(), kwargs.get('act'), out.detach().clone()))
            hooks.append(mod.register_forward_hook(hook, with_kwargs=True))
    decs = []
    hooks.append(m.decoder.register_forward_hook(
        lambda mod_, args, out: decs.append((args[0].detach().clone(), out.detach().clone()))))
    y, loss_w, frames = m(x)
    for h in hooks:
        h.remove()
    for name, mod, xin, act, yo in seen:
        with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
            if isinstance(mod, SLSTM):
                y64 = O.slstm(xin.double(), {'m.' + k: v.double() for k, v in mod.named_parameters()}, 'm',
                              mod.lstm.num_layers)
            else:
                y64, _ = _fp64_layer(mod, xin.double(), act)
        print(f'  in-model {name} {tuple(xin.shape)} act {act}: rel {rel(yo, y64):.2e}', flush=True)
    gy = T(rng(95).standard_normal(size=tuple(y.shape)).astype(np.float32)).to(DEV)
    torch.cuda.synchronize()
    y_fwd = y.detach().clone()
    torch.autograd.backward([y, loss_w], [gy, torch.ones_like(loss_w)])
    torch.cuda.synchronize()
    print('y changed by the backward: max', float((y.detach() - y_fwd).abs().max()), flush=True)
    out = {}
    for dt in (torch.float64, torch.float32):
        pp = {k: v.to(dt).requires_grad_(True) for k, v in p.items()}
        cc = [{k: v.to(dt) for k, v in cb.items()} for cb in cbs]
        yo, lw, _, _, _ = O.encodec_forward_train(T(d['gen/x']).to(dt), pp, cc, cfg, 3.0)
        torch.autograd.backward([yo, lw], [gy.cpu().to(dt), torch.ones_like(lw)])
        out[dt] = (yo, pp)
    print('y rel', rel(y, out[torch.float64][0]), 'before the backward', rel(y_fwd, out[torch.float64][0]), flush=True)
    # segment by segment: our encoder output vs the fp64 oracle's, and the RVQ codes each picks
    cbs64 = [{k: v.double() for k, v in cb.items()} for cb in cbs]
    p64 = {k: v.double() for k, v in p.items()}
    xd = T(d['gen/x']).double()
    for i, (off, seg) in enumerate(O.segments(cfg, xd.shape[-1])):
        xn, _ = O.normalize(xd[:, :, off:off + seg])
        e64 = O.run_plan(xn, p64, cfg.enc_plan, cfg.causal, cfg.norm)
        emb = frames[i][0].detach().double().cpu()
        n_q = O.rvq_num_quantizers(3.0, cfg.frame_rate, n_q_max=cfg.n_q)
        _, c64, _, _ = O.rvq_train(e64, cbs64, n_q)
        _, cm, _, _ = O.rvq_train(emb, cbs64, n_q)
        print(f'segment {i}: emb rel {rel(emb, e64):.2e}, codes differing {int((c64 != cm).sum())} of {c64.numel()}',
              flush=True)
        q64, _, _, cbs64 = O.rvq_train(e64, cbs64, n_q)
        qin, dout = decs[i]
        print(f'  model decoder input vs oracle q: {rel(qin, q64):.2e}', flush=True)
        d64 = O.run_plan(q64, p64, cfg.dec_plan, cfg.causal, cfg.norm)
        print(f'  model decoder output vs oracle decoder(q64): {rel(dout, d64):.2e}', flush=True)
        decoder_walk(m, q64.float().to(DEV), i)
    params = dict(m.named_parameters())
    for k in p:
        e = rel(params[k].grad, out[torch.float64][1][k].grad)
        e32 = rel(out[torch.float32][1][k].grad, out[torch.float64][1][k].grad)
        print(f'{k:60s} {e:.2e} {e32:.2e} {e / max(e32, 1e-12):8.1f}', flush=True)


if __name__ == '__main__':
    main()
