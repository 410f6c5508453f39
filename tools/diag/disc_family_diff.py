"""Diagnose a kernel-family-dependent discriminator result: run the MS-STFT discriminator
(config-3 size, B 32) forward + the l_g input-grad backward with each conv2d family forced
(encx_conv2d_select 0 auto / 1 register-window / 2 tiled) and print, per feature map and per
feature-map grad, the relative difference against the tiled run. GPU box only."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, 'encodec-pytorch_amd'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)


def run(family, disc, x):
    from encx._lib import lib
    prev = lib.encx_conv2d_select(family)
    try:
        xd = x.clone().requires_grad_(True)
        logits, fmaps = disc(xd)
        for fm in fmaps:
            for t in fm:
                t.retain_grad()
        l_g = sum(torch.relu(1 - l).mean() for l in logits) / len(logits) / len(logits)
        l_g.backward()
        torch.cuda.synchronize()
        return ([l.detach().clone() for l in logits], [[t.detach().clone() for t in fm] for fm in fmaps],
                [[t.grad.clone() if t.grad is not None else None for t in fm] for fm in fmaps], xd.grad.clone())
    finally:
        lib.encx_conv2d_select(prev)


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def main():
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from fixtures import disc_state
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    torch.manual_seed(0)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.cuda()
    x = 0.1 * torch.randn(B, 1, 24000, device='cuda')
    ref = run(2, disc, x)
    for fam in (1, 0, 2):
        r = run(fam, disc, x)
        print(f'== family {fam} vs tiled: dx {rel(r[3], ref[3]):.2e}')
        for k in range(len(r[0])):
            print(f'  disc {k}: logits {rel(r[0][k], ref[0][k]):.2e}; maps ' +
                  ' '.join(f'{rel(a, b):.1e}' for a, b in zip(r[1][k], ref[1][k])) + '; map grads ' +
                  ' '.join('-' if a is None else f'{rel(a, b):.1e}' for a, b in zip(r[2][k], ref[2][k])))


if __name__ == '__main__':
    main()


def replay_layer1(B=32):
    """Disc 0, layer 1: the composed run's own inputs (map 0, map 1's grad) through one
    standalone Conv2d backward per family."""
    from encx import ops
    from encx._lib import lib
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from fixtures import disc_state
    torch.manual_seed(0)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.cuda()
    x = 0.1 * torch.randn(B, 1, 24000, device='cuda')
    outs = {}
    for fam in (2, 1):
        lib.encx_conv2d_select(fam)
        xd = x.clone().requires_grad_(True)
        logits, fmaps = disc(xd)
        for t in fmaps[0]:
            t.retain_grad()
        l_g = sum(torch.relu(1 - l).mean() for l in logits) / len(logits) / len(logits)
        l_g.backward()
        m0, m1 = fmaps[0][0].detach(), fmaps[0][1].detach()
        g0, g1 = fmaps[0][0].grad.clone(), fmaps[0][1].grad.clone()
        c = disc.discriminators[0].convs[1]
        conv = c.conv
        for fam2 in (2, 1):
            lib.encx_conv2d_select(fam2)
            xi = m0.clone().requires_grad_(True)
            w = conv.weight_v if hasattr(conv, 'weight_v') else conv.weight
            gg = getattr(conv, 'weight_g', None)
            y = ops.conv2d(xi, w, gg, conv.bias, (3, 9), (1, 2), (1, 1), (1, 4), True)
            y.backward(g1)
            print(f'composed family {fam}, standalone family {fam2}: y vs map1 {rel(y, m1):.2e}; '
                  f'dx vs composed map0 grad {rel(xi.grad, g0):.2e}')
            outs[(fam, fam2)] = xi.grad.clone()
    print(f'standalone rw vs standalone tiled on the tiled run inputs: {rel(outs[(2, 1)], outs[(2, 2)]):.2e}')
    # fp64 truth for the tiled run's inputs, with each family's own LeakyReLU mask
    import torch.nn.functional as F
    wv, wg = conv.weight_v.detach().double(), conv.weight_g.detach().double()
    w64 = wg * wv / wv.reshape(wv.shape[0], -1).norm(dim=1).reshape(-1, 1, 1, 1)
    x64 = m0.double().requires_grad_(True)
    p64 = F.conv2d(x64, w64, conv.bias.detach().double(), stride=(1, 2), padding=(1, 4))
    mask = torch.where(m1 > 0, 1.0, 0.2).double()
    gx, = torch.autograd.grad(p64, (x64,), g1.double() * mask)
    # per-element backward error: |dx - dx64| / (|W| conv^T |dy'|), the sum of the magnitudes of
    # the terms each dx element adds up (a bug shows as ratios ~1 at its elements, rounding as
    # ratios ~1e-7..1e-5)
    xa = torch.zeros_like(x64).requires_grad_(True)
    pa = F.conv2d(xa, w64.abs(), None, stride=(1, 2), padding=(1, 4))
    scale, = torch.autograd.grad(pa, (xa,), (g1.double() * mask).abs())
    for fam2 in (2, 1):
        e = (outs[(2, fam2)].double() - gx).abs() / scale.clamp_min(1e-300)
        i = torch.nonzero(e == e.max())[0].tolist()
        print(f'family {fam2} dx vs fp64: {rel(outs[(2, fam2)], gx):.2e}; per-element backward error max '
              f'{float(e.max()):.2e} at {i}, 99.99% {float(torch.quantile(e.flatten()[::97].float(), 0.9999)):.2e}; '
              f'|dx64| max {float(gx.abs().max()):.2e}, term scale max {float(scale.max()):.2e}')
    # the same weights and map with a random output grad; the real output grad with random weights
    dyr = torch.randn_like(g1)
    for what, dy_, wv_, wg_ in (('random dy, real weights', dyr, conv.weight_v, conv.weight_g),
                                ('real dy, random weights', g1, 0.2 * torch.randn_like(conv.weight_v), None)):
        res = {}
        for fam2 in (2, 1):
            lib.encx_conv2d_select(fam2)
            xi = m0.clone().requires_grad_(True)
            y = ops.conv2d(xi, wv_.detach(), None if wg_ is None else wg_.detach(), conv.bias.detach(),
                           (3, 9), (1, 2), (1, 1), (1, 4), True)
            y.backward(dy_)
            res[fam2] = xi.grad.clone()
        print(f'{what}: rw vs tiled {rel(res[1], res[2]):.2e}')
    # scale: how large / how concentrated is the real output grad
    a = g1.abs()
    print(f'g1: max {float(a.max()):.3e} mean {float(a.mean()):.3e} zero frac {float((a == 0).float().mean()):.3f}; '
          f'per-t max {a.amax(dim=(0, 1, 3))[:4].tolist()} .. {a.amax(dim=(0, 1, 3))[-4:].tolist()}; '
          f'per-f max first {a.amax(dim=(0, 1, 2))[:3].tolist()} last {a.amax(dim=(0, 1, 2))[-3:].tolist()}')
    d = (outs[(2, 1)] - outs[(2, 2)]).abs()
    idx = torch.nonzero(d == d.max())[0].tolist()
    print(f'largest rw-tiled difference at [b, ci, t, f] = {idx} of {list(d.shape)}; per-f max of diff: '
          f'first {d.amax(dim=(0, 1, 2))[:6].tolist()} last {d.amax(dim=(0, 1, 2))[-6:].tolist()}; '
          f'per-t max first {d.amax(dim=(0, 1, 3))[:3].tolist()} last {d.amax(dim=(0, 1, 3))[-3:].tolist()}')
    lib.encx_conv2d_select(0)


if __name__ == '__main__' and os.environ.get('REPLAY'):
    replay_layer1()
