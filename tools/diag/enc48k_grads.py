"""Where along the backward does the 48 kHz GAN step's encoder-grad excess start?

One Trainer step of the g9 GAN fixture (48 kHz stereo, two segments) with the intermediate
gradients retained: the balancer's combined output grad, the grad of each segment's decoder
input (the quantized latent) and of each segment's encoder output (emb, after the STE and the
commit loss), and the encoder layer grads. The same step is restated from the oracle's pieces
(O.run_plan / O.rvq_train / O.msstft_forward with our LeakyReLU slopes / O.Balancer) in fp64 and
fp32 with the same tensors retained. Each row: our error vs fp64, the plain fp32 oracle's, ratio.
python tools/diag/enc48k_grads.py (GPU box) -> gpurun_out/enc48k_grads.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, 'encodec-pytorch_amd'), os.path.join(ROOT, 'tests', 'golden'),
          os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402

import steputil  # noqa: E402
from oracle import encodec_oracle as O  # noqa: E402
from test_gpu_48k import build48k, load, T, DEV, disc_state  # noqa: E402

W = {'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4}
FEAT = os.environ.get('ENC48K_FEAT_SIGNS', '1') != '0'  # impose our feature-L1 signs (oracle._l1_feat)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def oracle_gen(snap, x, cfg, bw, masks, dtype):
    """The generator phase of O.train_step with intermediate grads retained."""
    p = {k: v.to(dtype).requires_grad_(True) for k, v in snap['gen']['p'].items()}
    cbs = [{k: v.to(dtype) for k, v in cb.items()} for cb in snap['cbs']]
    dp = {k: v.to(dtype) for k, v in snap['disc']['p'].items()}
    x = x.detach().cpu().to(dtype)
    n_q = O.rvq_num_quantizers(bw, cfg.frame_rate, n_q_max=cfg.n_q)
    loss_w = torch.zeros(1, dtype=dtype)
    frames, embs, qs = [], [], []
    for off, seg in O.segments(cfg, x.shape[-1]):
        xn, scale = O.normalize(x[:, :, off:off + seg])
        emb = O.run_plan(xn, p, cfg.enc_plan, cfg.causal, cfg.norm)
        emb.retain_grad()
        q, codes, pen, cbs = O.rvq_train(emb, cbs, n_q)
        q.retain_grad()
        loss_w = loss_w + pen
        frames.append((q, scale))
        embs.append(emb)
        qs.append(q)
    outs = []
    for q, scale in frames:
        outs.append(O.run_plan(q, p, cfg.dec_plan, cfg.causal, cfg.norm) * scale.view(-1, 1, 1))
    stride = max(1, int((1 - cfg.overlap) * int(cfg.segment * cfg.sample_rate)))
    y = O.linear_overlap_add(outs, stride)[:, :, :x.shape[-1]]
    lr_, fr = O.msstft_forward(x, dp, masks=masks['real'])
    lf_, ff = O.msstft_forward(y, dp, masks=masks['fake'])
    losses = O.total_loss(fr, lf_, ff, x, y, cfg.sample_rate, feat_signs=masks.get('feat') if FEAT else None)
    grads = {k: torch.autograd.grad(l.sum(), [y], retain_graph=True)[0] for k, l in losses.items()}
    bal = O.Balancer(W)
    if snap['bal'] is not None:
        for name, t, f in zip(*snap['bal']):
            bal.total[name], bal.fix[name] = t, f
    out_grad = bal.combine(grads)
    extra = {f'g_{k}': v for k, v in grads.items()}
    extra.update({f'loss_{k}': v.detach().reshape(1) for k, v in losses.items()})
    extra.update({f'bal_avg_{k}': torch.tensor([bal.total[k] / bal.fix[k]], dtype=torch.float64) for k in grads})
    torch.autograd.backward([y, loss_w], [out_grad, torch.ones_like(loss_w)])
    return {**extra, 'out_grad': out_grad, **{f'seg{i}.q_grad': q.grad for i, q in enumerate(qs)},
            **{f'seg{i}.emb_grad': e.grad for i, e in enumerate(embs)},
            **{f'param:{k}': v.grad for k, v in p.items() if k.startswith('encoder.')},
            **{f'seg{i}.emb': e.detach() for i, e in enumerate(embs)}}


def main():
    from encx.train import Trainer
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from encx import balancer as B
    d = load('g9_step48k.npz')
    m, p, cbs, cfg = build48k(d, 'gan/')
    disc = MultiScaleSTFTDiscriminator(filters=32, in_channels=2, out_channels=2)
    disc.load_state_dict(disc_state(94, 2, 2), strict=False)
    disc = disc.to(DEV)
    tr = Trainer(m, disc, lr=1e-4, disc_lr=1e-4, scheduler=False, weights=W, sample_rate=48000)
    x = T(d['gan/x']).to(DEV)
    lines = []
    for it in range(2):
        snap = steputil.snapshot(tr)
        mine = {}
        embs, qs = [], []
        enc_fwd = m.encoder.forward
        q_fwd = m.quantizer.forward

        def enc_hook(xx, _f=enc_fwd):
            e = _f(xx)
            e.retain_grad()
            embs.append(e)
            return e

        def q_hook(*a, _f=q_fwd, **k):
            r = _f(*a, **k)
            r.quantized.retain_grad()
            qs.append(r.quantized)
            return r
        m.encoder.forward = enc_hook
        m.quantizer.forward = q_hook
        fin = B.Balancer.combine_finish
        cst = B.Balancer.combine_start

        def cf(self, _f=fin):
            g = _f(self)
            mine['out_grad'] = g.detach().clone()
            st = self._state
            for i, k in enumerate(st['names']):
                mine[f'bal_avg_{k}'] = st['avg'][i:i + 1].detach().clone()
            return g

        def cs(self, grads, _f=cst):
            for k, v in grads.items():
                mine[f'g_{k}'] = v.detach().clone()
            return _f(self, grads)
        B.Balancer.combine_finish = cf
        B.Balancer.combine_start = cs
        store = []
        hooks = steputil.disc_mask_hooks(tr.disc, store)
        try:
            out_losses = tr.step(x)
            torch.cuda.synchronize()
        finally:
            for h in hooks:
                h.remove()
            m.encoder.forward = enc_fwd
            m.quantizer.forward = q_fwd
            B.Balancer.combine_finish = fin
            B.Balancer.combine_start = cst
        masks = steputil.split_masks(store, len(tr.disc.discriminators))
        for k, v in out_losses.items():
            mine[f'loss_{k}'] = v.detach().reshape(1)
        for i, (e, q) in enumerate(zip(embs, qs)):
            mine[f'seg{i}.emb_grad'] = e.grad
            mine[f'seg{i}.q_grad'] = q.grad
            mine[f'seg{i}.emb'] = e.detach()
        names = [k for k, q in m.named_parameters() if q.requires_grad]
        for k, (q, g, _, _) in steputil._flat_views(tr.opt, names).items():
            if k.startswith('encoder.'):
                mine['param:' + k] = g
        nt = torch.get_num_threads()
        torch.set_num_threads(steputil.ORACLE_THREADS)
        o64 = oracle_gen(snap, x, cfg, 3.0, masks, torch.float64)
        o32 = oracle_gen(snap, x, cfg, 3.0, masks, torch.float32)
        torch.set_num_threads(nt)
        lines.append(f'# step {it}   {"tensor":56s} {"ours":>10s} {"fp32":>10s} {"ratio":>7s}')
        for k in o64:
            if k not in mine or mine[k] is None:
                lines.append(f'  {k}: missing on our side')
                continue
            e, e32 = rel(mine[k], o64[k]), rel(o32[k], o64[k])
            lines.append(f'  {k:64s} {e:10.3e} {e32:10.3e} {e / max(e32, 1e-30):7.2f}')
    os.makedirs('gpurun_out', exist_ok=True)
    txt = '\n'.join(lines)
    open('gpurun_out/enc48k_grads.txt', 'w').write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main()
