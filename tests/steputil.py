"""One Trainer step against the CPU oracle's step from the SAME state, element by element.

Test infrastructure (GPU tests only). Before a HIP step the trainer's state -- parameters, Adam
moments and step count, codebook buffers, balancer statistics, learning rate -- is copied to
the host; the oracle (oracle/encodec_oracle.py train_step, pinned to the reference's g7 / g9
fixtures by tests/test_oracle.py) then runs the same step from that state in fp64, and once more
in fp32. The HIP step is compared with the fp64 step:

  * grads, per tensor: max |g - g64| / max |g64| within 4x what the plain fp32 oracle achieves
    on the same tensor, or 4x the fp32 oracle's MEDIAN error over the model's tensors where that
    is larger (floor 1e-6), and (with >= 5 tensors) the median over tensors of (our error / the
    fp32 oracle's) at most 4 (MEDIAN_RATIO): the HIP path must be about as accurate as a
    straightforward fp32 implementation of the reference's arithmetic. The median term exists because a tensor's fp32-oracle error is one
    sample of the rounding accumulated over every layer above it: on the 48 kHz GAN step a few
    tensors' samples fall 2-4x under their neighbours' (encoder.model.3 norm.weight 2.5e-5 beside
    5-6e-5), and the lucky sample is not a bound on fp32 arithmetic. The table of achieved errors
    is returned (and printed).
  * post-Adam parameters, element-wise: an element whose fp64 grad lies within 4x of its OWN fp32
    rounding (|g32 - g64| at that element, the plain fp32 oracle's error there) of zero can take
    either sign in fp32 (Adam then steps it either way by ~lr): it is "undecided" and skipped.
    Every decided element must match within 4 * lr * max(|g - g64|, |g32 - g64|) / |g64| + 2e-6,
    Adam's sensitivity to the grad deviation at that element, plus fp32 rounding of the
    parameter. At least 97 % of the elements must be decided.
  * codebook EMA buffers (cluster_size, embed_avg, embed): element-wise within 1e-5 of the
    buffer's largest magnitude.
No global slack: every bound is per element or per tensor.
"""
import contextlib

import numpy as np
import torch

from oracle import encodec_oracle as O


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _flat_views(opt, names):
    out = {}
    for k, (p, _), (o, n) in zip(names, opt._views, opt.offsets):
        out[k] = (p, opt.flat_grad[o:o + n].view_as(p), opt.exp_avg[o:o + n].view_as(p),
                  opt.exp_avg_sq[o:o + n].view_as(p))
    return out


def snapshot(tr):
    """The trainer's state before a step, on the host."""
    s = {}
    for tag, mod, opt in (('gen', tr.model, tr.opt), ('disc', tr.disc, tr.opt_d)):
        if mod is None:
            continue
        names = [k for k, p in mod.named_parameters() if p.requires_grad]
        v = _flat_views(opt, names)
        s[tag] = {'p': {k: t[0].detach().cpu().clone() for k, t in v.items()},
                  'm': {k: t[2].detach().cpu().clone() for k, t in v.items()},
                  'v': {k: t[3].detach().cpu().clone() for k, t in v.items()},
                  'step': opt.n_step, 'lr': float(opt.param_groups[0]['lr'])}
    s['cbs'] = [{k: getattr(layer._codebook, k).detach().cpu().clone()
                 for k in ('inited', 'cluster_size', 'embed', 'embed_avg')}
                for layer in tr.model.quantizer.vq.layers]
    st = tr.balancer._state
    s['bal'] = None if st is None else (list(st['names']), st['total'].cpu().tolist(), st['fix'].cpu().tolist())
    return s


def disc_mask_hooks(disc, store):
    """Forward hooks collecting every LeakyReLU'd discriminator map of a step (on the host), in
    call order: the Trainer runs the discriminator on the real audio, then on the fake."""
    hs = []
    for d in disc.discriminators:
        for layer in d.convs:
            hs.append(layer.register_forward_hook(lambda mod, inp, out: store.append(out.detach().cpu())))
    return hs


def split_masks(store, n_disc):
    """[real maps..., fake maps...] -> {'real': [disc][layer] slope masks (map > 0), 'fake': the
    same, 'feat': [disc][layer] signs of fake - real (the feature-matching L1's derivative)}"""
    per = len(store) // (2 * n_disc)
    grid = [store[i * per:(i + 1) * per] for i in range(2 * n_disc)]
    real, fake = grid[:n_disc], grid[n_disc:]
    return {'real': [[m > 0 for m in ms] for ms in real], 'fake': [[m > 0 for m in ms] for ms in fake],
            'feat': [[torch.sign(f - r) for r, f in zip(rs, fs)] for rs, fs in zip(real, fake)]}


@contextlib.contextmanager
def lrelu_audit(feat=None):
    """Collect (pre-activation, imposed mask) of every masked LeakyReLU the oracle evaluates;
    with a `feat` list also (fake - real, imposed sign) of every feature-matching L1."""
    O.LRELU_AUDIT = log = []
    O.FEAT_AUDIT = feat
    try:
        yield log
    finally:
        O.LRELU_AUDIT = None
        O.FEAT_AUDIT = None


def _local_max(e):
    """max of e over each element's 3-wide neighbourhood along the last axis and, for maps of
    4 or more dims ([B, C, T, F]), the second-to-last axis too."""
    F = torch.nn.functional
    shape = e.shape
    x = F.max_pool1d(e.reshape(-1, 1, shape[-1]), 3, 1, 1).reshape(shape)
    if e.dim() >= 4:
        xt = x.transpose(-1, -2).contiguous()
        x = F.max_pool1d(xt.reshape(-1, 1, shape[-2]), 3, 1, 1).reshape(xt.shape).transpose(-1, -2)
    return x


def check_masks(a64, a32, what):
    """Our LeakyReLU slope masks (imposed on the oracle) against the fp64 oracle's OWN signs of
    the same pre-activations. Per element: a sign may differ only where |z64| is within 8x that
    element's fp32 rounding estimate, i.e. where fp32 arithmetic may legitimately land on the other
    side of 0. The estimate is the plain fp32 oracle's error |z32 - z64| at the element and its
    neighbours (max over 3 along f and t), floored at the map's median error. One run's error at a
    single element is one draw and can be near 0 by luck: with the element's own draw only, a
    weight-grad summation-order change put one feature-L1 element of the 48 kHz step at 4.4x, and
    a later one another at 8.8x (round 5). A sign error in a HIP epilogue lands far from 0 and
    fails here. Reports the flips per map. a64 / a32: the lrelu_audit logs of the fp64 and fp32
    oracle runs."""
    assert a64 and len(a64) == len(a32), (what, len(a64), len(a32))
    flips = total = 0
    worst = 0.0
    per_map = []
    for i, ((z64, m), (z32, _)) in enumerate(zip(a64, a32)):
        z64 = z64.double()
        bad = m != (z64 > 0) if m.dtype == torch.bool else m.double() != torch.sign(z64)
        n = int(bad.sum())
        if n:
            err = (z32.double() - z64).abs()
            nz = err[z64 != 0]
            med = float(nz.median()) if nz.numel() else 0.0
            bound = 8 * _local_max(err)[bad].clamp_min(med)
            mag = z64.abs()[bad]
            ratio = mag / bound.clamp_min(1e-300)
            assert bool((mag <= bound).all()), (what, f'map {i}: slope mask off the fp64 sign beyond that '
                                                'element\'s rounding', float(ratio.max()), n)
            worst = max(worst, float(ratio.max()))
            per_map.append(f'{i}:{n}/{m.numel()}')
        flips += n
        total += m.numel()
    print(f'{what}: {flips} of {total} imposed signs differ from the fp64 signs, each within 8x its '
          f'own rounding estimate (worst at {worst:.2f} of its bound); per map: {" ".join(per_map) or "none"}')
    return flips


def oracle_step(snap, x, cfg, bandwidth, weights, dtype, disc_masks=None):
    """O.train_step from the snapshot in `dtype` -> (out, params, codebooks, disc params)."""
    p = {k: v.to(dtype) for k, v in snap['gen']['p'].items()}
    adam = {k: {'step': snap['gen']['step'], 'm': snap['gen']['m'][k].to(dtype),
                'v': snap['gen']['v'][k].to(dtype)} for k in p}
    cbs = [{k: v.to(dtype) for k, v in cb.items()} for cb in snap['cbs']]
    bal = O.Balancer(weights)
    if snap['bal'] is not None:
        for name, t, f in zip(*snap['bal']):
            bal.total[name], bal.fix[name] = t, f
    dp = dadam = dlr = None
    if 'disc' in snap:
        d = snap['disc']
        dp = {k: v.to(dtype) for k, v in d['p'].items()}
        dadam = {k: {'step': d['step'], 'm': d['m'][k].to(dtype), 'v': d['v'][k].to(dtype)} for k in dp}
        dlr = d['lr']
    nt = torch.get_num_threads()
    torch.set_num_threads(ORACLE_THREADS)
    try:
        out = O.train_step(x.detach().cpu().to(dtype), p, cbs, cfg, bandwidth, bal, adam, snap['gen']['lr'],
                           disc_p=dp, disc_adam_state=dadam, disc_lr=dlr, disc_masks=disc_masks)
    finally:
        torch.set_num_threads(nt)
    return out, p, cbs, dp


# The fp32 oracle's own error is one sample of fp32 summation order: the same oracle step on 8
# vs 16 host threads (oneDNN's blocking follows the thread count) moved the 48 kHz GAN step's
# median ratio from 1.9 to 3.2. The oracle therefore runs on a fixed thread count (ORACLE_THREADS,
# reproducible bounds), and the median ratio is held to the per-tensor factor, 4.
MEDIAN_RATIO = 4.0
ORACLE_THREADS = 8


def _grad_bounds(errs, floor=1e-6):
    """errs: name -> (our err, fp32 oracle err) -> rows [(name, err, err32, bound)], and the
    median-ratio assertion (see the module docstring)."""
    med32 = float(np.median([e32 for _, e32 in errs.values()])) if errs else 0.0
    rows = [(k, e, e32, max(4 * max(e32, med32), floor)) for k, (e, e32) in errs.items()]
    ratios = [e / e32 for e, e32 in errs.values() if e32 > floor]
    if len(ratios) >= 5:
        assert float(np.median(ratios)) <= MEDIAN_RATIO, ('median error ratio vs the fp32 oracle',
                                                           float(np.median(ratios)))
    return rows


def _check_opt(tag, mod, opt, g64, g32, p64, lr, table, floor=1e-6):
    names = [k for k, p in mod.named_parameters() if p.requires_grad]
    views = {k: v for k, v in _flat_views(opt, names).items() if k in g64}
    errs = {k: (_rel(v[1], g64[k]), _rel(g32[k], g64[k])) for k, v in views.items()}
    table.extend((f'{tag}:{k}', e, e32, b) for k, e, e32, b in _grad_bounds(errs, floor))
    decided_n = total_n = 0
    for k, (p, g, _, _) in views.items():
        gd = g64[k].double()
        e_own = (g32[k].double() - gd).abs()
        e_mine = (g.detach().double().cpu() - gd).abs()
        decided = (gd.abs() > 4 * e_own) & (gd.abs() > 1e-12 * float(gd.abs().max()))
        decided_n += int(decided.sum())
        total_n += gd.numel()
        tol = 4 * lr * torch.maximum(e_mine, e_own) / gd.abs().clamp_min(1e-30) + 2e-6
        diff = (p.detach().double().cpu() - p64[k].double()).abs()
        bad = decided & (diff > tol)
        assert not bool(bad.any()), (tag, k, float(diff[decided].max()), int(bad.sum()))
    assert decided_n >= 0.97 * total_n, (tag, decided_n, total_n)


def _assert_table(table, what):
    """Every row within its bound; on failure the whole table's violators, worst first."""
    bad = sorted((r for r in table if not r[1] <= r[3]), key=lambda r: -r[1] / r[3])
    if bad:
        lines = '\n'.join(f'  {n}: err {e:.3e} fp32-oracle {e32:.3e} bound {b:.3e}' for n, e, e32, b in bad[:20])
        raise AssertionError(f'{what}: {len(bad)} of {len(table)} tensors over their bound\n{lines}')


def check_grads(mine, g64, g32, what, floor=1e-6):
    """Per tensor: rel err of `mine` vs fp64 within 4x the fp32 oracle's (floor `floor`).
    mine / g64 / g32: name -> tensor. Returns the table [(name, err, err_fp32, bound)]."""
    table = _grad_bounds({k: (_rel(mine[k], g64[k]), _rel(g32[k], g64[k])) for k in g64}, floor)
    _assert_table(table, what)
    worst = max(table, key=lambda r: r[1] / r[3])
    print(f'{what}: {len(table)} tensors, worst err {max(r[1] for r in table):.2e}; '
          f'tightest {worst[0]} {worst[1]:.2e} vs fp32 oracle {worst[2]:.2e}')
    return table


def check_step(tr, x, cfg, bandwidth, weights, verbose=True, floor=1e-6):
    """tr.step(x) against the oracle's step from the same state; returns (out, table). floor:
    the smallest per-tensor grad bound (relative to the tensor's fp64 magnitude)."""
    snap = snapshot(tr)
    store, hooks = [], []
    if tr.disc is not None:
        hooks = disc_mask_hooks(tr.disc, store)
    try:
        out = tr.step(x)
        torch.cuda.synchronize()
    finally:
        for h in hooks:
            h.remove()
    # the oracle's discriminator LeakyReLU slopes follow OUR maps' signs (oracle._lrelu): a
    # pre-activation within rounding of 0 may take either slope in fp32, a discrete outcome that
    # no rounding bound covers
    masks = split_masks(store, len(tr.disc.discriminators)) if tr.disc is not None else None
    f64, f32 = [], []
    with lrelu_audit(f64) as a64:
        o64, p64, cbs64, dp64 = oracle_step(snap, x, cfg, bandwidth, weights, torch.float64, masks)
    with lrelu_audit(f32) as a32:
        o32, _, _, _ = oracle_step(snap, x, cfg, bandwidth, weights, torch.float32, masks)
    if masks is not None:
        check_masks(a64, a32, 'step slope masks')
        if 'l_feat' in weights:
            check_masks(f64, f32, 'step feature-L1 signs')
    table = []
    _check_opt('gen', tr.model, tr.opt, o64['grads'], o32['grads'], p64, snap['gen']['lr'], table, floor)
    if tr.disc is not None and 'disc_grads' in o64:
        _check_opt('disc', tr.disc, tr.opt_d, o64['disc_grads'], o32['disc_grads'], dp64, snap['disc']['lr'], table,
                   floor)
    for i, layer in enumerate(tr.model.quantizer.vq.layers):
        cb = layer._codebook
        for k in ('cluster_size', 'embed_avg', 'embed'):
            e = _rel(getattr(cb, k), cbs64[i][k])
            table.append((f'codebook{i}:{k}', e, float('nan'), 1e-5))
    _assert_table(table, 'step vs oracle')
    for k in weights:
        np.testing.assert_allclose(float(out[k]), o64[k], rtol=2e-5, err_msg=k)
    if verbose:
        worst = max(table, key=lambda r: r[1] / r[3])
        print(f'step vs oracle: {len(table)} tensors, worst grad err {max(r[1] for r in table):.2e}, '
              f'tightest {worst[0]} {worst[1]:.2e} / bound {worst[3]:.2e}')
    return out, table
