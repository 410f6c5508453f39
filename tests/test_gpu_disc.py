"""GPU parity of the MS-STFT discriminator path (csrc/disc.hip through the C ABI): the G5
fixture generated from the reference, the fp64 oracle at 1 s clips (forward, input grad,
weight grads), the adversarial / feature / discriminator losses, and the GAN train step."""
import numpy as np
import pytest
import torch

from oracle import encodec_oracle as O
from fixtures import load, T, disc_state, model_state, codebooks_from_stats

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def make_disc(seed):
    from encx.msstftd import MultiScaleSTFTDiscriminator
    d = MultiScaleSTFTDiscriminator(filters=32)
    p = disc_state(seed)
    missing, unexpected = d.load_state_dict(p, strict=False)
    assert not unexpected and all(k.endswith('spec_transform.window') for k in missing)
    return d.to(DEV), p


def test_disc_fixture():
    """G5: logits, feature maps and d/dx of sum(logits*w) + sum(mean(fmap)) (msstftd.py:131-149)."""
    d = load('g5_disc.npz')
    disc, _ = make_disc(51)
    x = T(d['x']).to(DEV).requires_grad_(True)
    logits, fmaps = disc(x)
    r = np.random.Generator(np.random.PCG64(53))
    f = 0
    for k, lg in enumerate(logits):
        assert rel(lg, T(d[f'logits{k}'])) < 1e-4, k
        wl = T(r.standard_normal(size=tuple(lg.shape)).astype(np.float32)).to(DEV)
        f = f + (lg * wl).sum()
        for j, fm in enumerate(fmaps[k]):
            assert tuple(fm.shape) == tuple(d[f'fmap{k}_{j}_shape'])
            np.testing.assert_allclose(fm.double().sum().item(), d[f'fmap{k}_{j}_sum'], rtol=1e-4)
            np.testing.assert_allclose(fm.double().pow(2).sum().item(), d[f'fmap{k}_{j}_sq'], rtol=1e-4)
            assert rel(fm.reshape(-1)[:256], T(d[f'fmap{k}_{j}_head'])) < 1e-4
            f = f + fm.mean()
    f.backward()
    assert rel(x.grad, T(d['dx'])) < 1e-3


@pytest.mark.parametrize('B,Tn', [(2, 24000), (3, 7001)])
def test_disc_vs_oracle_fp64(B, Tn):
    """Full 1 s clips (all three scales at their real sizes) and a ragged length: every
    parameter grad and the input grad against the oracle in fp64."""
    disc, p = make_disc(7)
    g = torch.Generator().manual_seed(B * 31 + Tn)
    x64 = (0.1 * torch.randn(B, 1, Tn, generator=g, dtype=torch.float64)).requires_grad_(True)
    p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
    lg64, fm64 = O.msstft_forward(x64, p64)
    ws = [torch.randn(l.shape, generator=g, dtype=torch.float64) for l in lg64]
    wf = [[torch.randn(f.shape, generator=g, dtype=torch.float64) for f in fm] for fm in fm64]
    f64 = sum((l * w).sum() for l, w in zip(lg64, ws)) + \
        sum((f * w).sum() for fm, wm in zip(fm64, wf) for f, w in zip(fm, wm))
    f64.backward()

    x = x64.detach().float().to(DEV).requires_grad_(True)
    lg, fm = disc(x)
    for a, b in zip(lg, lg64):
        assert rel(a, b) < 1e-4
    for fa, fb in zip(fm, fm64):
        for a, b in zip(fa, fb):
            assert rel(a, b) < 1e-4
    f = sum((l * w.float().to(DEV)).sum() for l, w in zip(lg, ws)) + \
        sum((f_ * w.float().to(DEV)).sum() for fa, wm in zip(fm, wf) for f_, w in zip(fa, wm))
    f.backward()
    torch.cuda.synchronize()
    # the same in plain fp32 (the oracle): each grad's bound is 4x the fp32 oracle's error
    from steputil import check_grads
    x32 = x64.detach().float().requires_grad_(True)
    p32 = {k: v.detach().float().requires_grad_(True) for k, v in p64.items()}
    lg32, fm32 = O.msstft_forward(x32, p32)
    f32 = sum((l * w.float()).sum() for l, w in zip(lg32, ws)) + \
        sum((f_ * w.float()).sum() for fa, wm in zip(fm32, wf) for f_, w in zip(fa, wm))
    f32.backward()
    params = dict(disc.named_parameters())
    check_grads({'x': x.grad, **{k: params[k].grad for k in p64}}, {'x': x64.grad, **{k: v.grad for k, v in p64.items()}},
                {'x': x32.grad, **{k: v.grad for k, v in p32.items()}}, 'disc grads vs fp64')


def masked_msstft(x, p, fmaps_mine):
    """The oracle's MS-STFT forward in fp64 with every LeakyReLU slope taken from the sign of
    OUR feature maps: a pre-activation within fp32 rounding of 0 can land on either side, and
    the generator-side seed (uniform over the logits) is what makes such flips visible in
    d l / dy; with the masks shared, the backward is linear and must agree to fp32 accuracy."""
    import torch.nn.functional as F
    logits = []
    for k, (n, h) in enumerate(zip(O.DISC_CFG['n_ffts'], O.DISC_CFG['hops'])):
        pre = f'discriminators.{k}'
        z = O.spectrogram(x, n, h, n)
        z = torch.cat([z.real, z.imag], dim=1).permute(0, 1, 3, 2)
        masks = [torch.where(f.detach().cpu() > 0, 1.0, 0.2).double() for f in fmaps_mine[k]]
        z = F.conv2d(z, p[pre + '.convs.0.conv.weight'], p[pre + '.convs.0.conv.bias'], padding=(1, 4)) * masks[0]
        for i, d in enumerate((1, 2, 4)):
            q = f'{pre}.convs.{i + 1}.conv'
            w = O.weight_norm(p[q + '.weight_v'], p[q + '.weight_g'])
            z = F.conv2d(z, w, p[q + '.bias'], stride=(1, 2), dilation=(d, 1), padding=(d, 4)) * masks[i + 1]
        q = f'{pre}.convs.4.conv'
        z = F.conv2d(z, O.weight_norm(p[q + '.weight_v'], p[q + '.weight_g']), p[q + '.bias'], padding=(1, 1)) * masks[4]
        q = f'{pre}.conv_post.conv'
        logits.append(F.conv2d(z, O.weight_norm(p[q + '.weight_v'], p[q + '.weight_g']), p[q + '.bias'], padding=(1, 1)))
    return logits


def test_gan_losses_vs_oracle():
    """l_g / l_feat (losses.py:44-56, incl. the double division by K) and disc_loss (:65-80)
    values against the oracle; the generator-side grads d l_g / dy and d l_feat / dy through
    the discriminator against the fp64 oracle evaluated with our LeakyReLU masks."""
    from encx.losses import total_loss, disc_loss
    disc, p = make_disc(9)
    g = torch.Generator().manual_seed(5)
    x64 = 0.1 * torch.randn(2, 1, 24000, generator=g, dtype=torch.float64)
    y64 = (x64 + 0.05 * torch.randn(2, 1, 24000, generator=g, dtype=torch.float64)).requires_grad_(True)
    p64 = {k: v.double() for k, v in p.items()}
    lr64, fr64 = O.msstft_forward(x64, p64)
    lf64, ff64 = O.msstft_forward(y64, p64)
    ref = O.total_loss(fr64, lf64, ff64, x64, y64)
    ld64 = O.disc_loss(lr64, [l.detach() for l in lf64])

    x = x64.float().to(DEV)
    y = y64.detach().float().to(DEV).requires_grad_(True)
    lr, fr = disc(x, param_grads=False)
    lf, ff = disc(y, param_grads=False)
    out = total_loss(fr, lf, ff, x, y)
    for k in ('l_g', 'l_feat'):
        np.testing.assert_allclose(out[k].item(), ref[k].item(), rtol=1e-4)
    gg, = torch.autograd.grad(out['l_g'], [y], retain_graph=True)
    gf, = torch.autograd.grad(out['l_feat'], [y], retain_graph=True)
    ld = disc_loss(lr, [l.detach() for l in lf])
    np.testing.assert_allclose(ld.item(), ld64.item(), rtol=1e-5)

    # sign disagreements with fp64 only where the fp64 activation is ~0
    flips = 0
    for fa, fb in zip(ff, ff64):
        for a, b in zip(fa, fb):
            bad = (a.detach().cpu() > 0) != (b.detach() > 0)
            flips += int(bad.sum())
            if bad.any():
                assert float(b.detach()[bad].abs().max()) < 1e-5 * float(b.detach().abs().max())
    lfm = masked_msstft(y64, p64, ff)
    K = len(lfm)
    lg_m = sum(torch.relu(1 - l).mean() for l in lfm) / (K * K)
    gg64, = torch.autograd.grad(lg_m, [y64], retain_graph=True)
    gf64, = torch.autograd.grad(ref['l_feat'].sum(), [y64], retain_graph=True)
    print(f'mask flips {flips}; d l_g/dy rel {rel(gg, gg64):.2e}; d l_feat/dy rel {rel(gf, gf64):.2e}')
    assert rel(gg, gg64) < 1e-4
    assert rel(gf, gf64) < 2e-3  # sign(ff - fr) kinks: elements with ff ~ fr


def test_train_step_gan_fixture():
    """G7 GAN: two full train steps (generator with the 4-loss balancer, then the
    discriminator update): each step's losses against the reference's (g7), and each step
    element by element against the oracle's step from the same state (tests/steputil.py:
    generator and discriminator grads per tensor, post-Adam parameters, codebook buffers)."""
    from encx.train import Trainer
    from encx.model import EncodecModel
    from steputil import check_step
    d = load('g7_step.npz')
    cfg = O.Config(target_bandwidths=(1.5,), audio_normalize=True)
    m = EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    p = model_state(cfg, 71)
    cbs = codebooks_from_stats(d['gan/stats'], 73, 2, cfg.n_q)
    sd = dict(p)
    for i, cb in enumerate(cbs):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m = m.to(DEV)
    disc, _ = make_disc(74)
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=weights)
    x = T(d['gan/x']).to(DEV)
    for it in range(2):
        out, _ = check_step(tr, x, cfg, 1.5, weights)
        for k in ('l_t', 'l_f', 'l_g', 'l_feat'):
            np.testing.assert_allclose(float(out[k]), float(d[f'gan/it{it}_{k}'].reshape(-1)[0]), rtol=2e-4)
        np.testing.assert_allclose(float(out['l_d']), float(d[f'gan/it{it}_l_d'].reshape(-1)[0]), rtol=1e-4)


# (Ci, Co, kernel, stride, dilation, padding) of the DiscriminatorSTFT layers (msstftd.py:67-84)
LAYERS = [(2, 32, (3, 9), (1, 1), (1, 1), (1, 4)),
          (32, 32, (3, 9), (1, 2), (1, 1), (1, 4)),
          (32, 32, (3, 9), (1, 2), (2, 1), (2, 4)),
          (32, 32, (3, 9), (1, 2), (4, 1), (4, 4)),
          (32, 32, (3, 3), (1, 1), (1, 1), (1, 1)),
          (32, 1, (3, 3), (1, 1), (1, 1), (1, 1)),
          (4, 32, (3, 9), (1, 1), (1, 1), (1, 4)),  # first layer of the 48 kHz stereo disc
          (32, 1, (3, 3), (1, 2), (2, 1), (2, 1))]  # one output channel, strided + dilated (+ act)


@pytest.fixture(params=[0, 1, 2], ids=['auto', 'regwin', 'tiled'])
def conv2d_family(request):
    """encx_conv2d_select: the per-layer cost model, then each kernel family forced, so both
    families are checked at every size (the cost model alone picks the tiled kernels for small
    maps)."""
    from encx._lib import lib
    prev = lib.encx_conv2d_select(request.param)
    yield request.param
    lib.encx_conv2d_select(prev)


@pytest.mark.parametrize('li', range(len(LAYERS)))
@pytest.mark.parametrize('T2,Fi', [(7, 33), (23, 65), (5, 129), (3, 513), (40, 257), (12, 1025), (15, 513)])
def test_conv2d_vs_torch_fp64(li, T2, Fi, conv2d_family):
    """One NormConv2d (+ LeakyReLU except conv_post): output, input grad and weight/bias
    grads against torch.nn.functional.conv2d in fp64, with a random output grad, for each
    kernel family."""
    import torch.nn.functional as F
    from encx import ops
    Ci, Co, k, s, d, pad = LAYERS[li]
    act = li != 5
    g = torch.Generator().manual_seed(li * 100 + T2)
    x64 = torch.randn(2, Ci, T2, Fi, generator=g, dtype=torch.float64).requires_grad_(True)
    v64 = (0.2 * torch.randn((Co, Ci) + k, generator=g, dtype=torch.float64)).requires_grad_(True)
    b64 = (0.1 * torch.randn(Co, generator=g, dtype=torch.float64)).requires_grad_(True)
    p64 = F.conv2d(x64, v64, b64, stride=s, dilation=d, padding=pad)  # pre-activation
    dy64 = torch.randn(p64.shape, generator=g, dtype=torch.float64)
    x = x64.detach().float().to(DEV).requires_grad_(True)
    v = v64.detach().float().to(DEV).requires_grad_(True)
    b = b64.detach().float().to(DEV).requires_grad_(True)
    y = ops.conv2d(x, v, None, b, k, s, d, pad, act)
    y.backward(dy64.float().to(DEV))
    assert rel(y, F.leaky_relu(p64, 0.2) if act else p64) < 1e-5
    # LeakyReLU': the fp32 pre-activation may take the other sign than fp64's where |p| is within
    # fp32 rounding of 0 (then the mask is 1 against 0.2 at that element, a legitimate fp32
    # outcome). Such flips are allowed only there; the reference grads use OUR mask.
    mask = 1.0
    if act:
        mine = y.detach().double().cpu() > 0
        flips = mine != (p64.detach() > 0)
        assert bool((p64.detach().abs()[flips] <= 1e-5 * float(p64.detach().abs().max())).all())
        mask = torch.where(mine, 1.0, 0.2).double()
    dyl = dy64 * mask
    gx, gv, gb = torch.autograd.grad(p64, (x64, v64, b64), dyl)
    assert rel(x.grad, gx) < 1e-5, rel(x.grad, gx)
    assert rel(v.grad, gv) < 1e-5, rel(v.grad, gv)
    # the bias grad is a plain sum of dy' (thousands of O(1) terms that largely cancel): bound
    # its error by the fp32 summation scale as well as relatively
    bscale = float(dyl.abs().sum(dim=(0, 2, 3)).max())
    berr = float((b.grad.double().cpu() - gb).abs().max())
    assert rel(b.grad, gb) < 1e-5 or berr <= 1e-7 * bscale, (rel(b.grad, gb), berr, bscale)


@pytest.mark.parametrize('params,inp', [(False, True), (True, False), (True, True)])
def test_premask_bit_identical(params, inp):
    """DiscGradMode.premask (the Trainer's setting: each Conv2d's bwd-data hands its input's
    producer the grad of that producer's pre-activation) changes where the LeakyReLU' mask is
    applied, not its value: grads of l_g + l_feat and of the hinge disc loss w.r.t. the fake
    audio and every discriminator parameter are bit-identical to the unmasked protocol."""
    from encx.ops import DiscGradMode
    from encx.msstftd import adversarial_losses, hinge_disc_loss
    disc, _ = make_disc(11)
    g = torch.Generator().manual_seed(5)
    x = (0.1 * torch.randn(2, 1, 24000, generator=g)).to(DEV)
    y0 = (0.1 * torch.randn(2, 1, 24000, generator=g)).to(DEV)
    outs = []
    for premask in (False, True):
        y = y0.clone().requires_grad_(True)
        mode = DiscGradMode(params=params, input=inp, premask=premask)
        lr, fr = disc(x, mode=mode)
        lf, ff = disc(y, mode=mode)
        l_g, l_feat = adversarial_losses(fr, lf, ff)
        l_d = hinge_disc_loss(lr, lf)
        wrt = ([y] if inp else []) + ([q for q in disc.parameters()] if params else [])
        res = []
        for loss in (l_g, l_feat, l_g + l_feat, l_d):
            gs = torch.autograd.grad(loss, wrt, retain_graph=True, allow_unused=True)
            res.append([t.clone() if t is not None else None for t in gs])
        outs.append(res)
    for a, b in zip(*outs):
        for ta, tb in zip(a, b):
            assert (ta is None) == (tb is None)
            if ta is not None:
                assert torch.equal(ta, tb)


def _disc_layer_shapes(B=32, T=24000, C=1):
    """(n_fft, li, x shape, layer) of every Conv2d of the config-3 MS-STFT discriminator at full
    size (msstftd.py:131-149: n_fft 1024 / 2048 / 512, hop n/4, 32 filters)."""
    out = []
    for n in (1024, 2048, 512):
        T2, F = (T - n) // (n // 4) + 1, n // 2 + 1
        for li in range(6):
            Ci, Co, k, s, d, pad = LAYERS[li]
            if li == 0:
                Ci = 2 * C
            out.append((n, li, (B, Ci, T2, F), (Ci, Co, k, s, d, pad)))
            F = (F + 2 * pad[1] - k[1]) // s[1] + 1
    for n in (1024, 2048, 512):  # the first layer of the 48 kHz stereo discriminator (config 5)
        T2 = (2 * T - n) // (n // 4) + 1
        out.append((n, 6, (B, 4, T2, n // 2 + 1), LAYERS[6]))
    return out


@pytest.mark.parametrize('family', [1, 2], ids=['regwin', 'tiled'])
def test_conv2d_full_size_vs_torch_fp64(family):
    """Every Conv2d of the config-3 discriminator at its real size (B 32, 1 s clips: up to 4.8 M
    output positions per layer, many work items per wave of the persistent register-window
    kernels) for one forced kernel family: output, input grad, weight and bias grads against
    torch's fp64 conv2d on the GPU (test-only checker), relative to the tensor's largest
    magnitude."""
    import torch.nn.functional as F
    from encx import ops
    from encx._lib import lib
    def rel(a, b):  # on the device: up to 48 M elements per tensor
        a, b = a.detach().double(), b.detach().double()
        return float((a - b).abs().max() / (b.abs().max() + 1e-30))

    prev = lib.encx_conv2d_select(family)
    try:
        bad = []
        for n, li, xs, (Ci, Co, k, s, d, pad) in _disc_layer_shapes():
            act = li != 5
            torch.cuda.empty_cache()
            g = torch.Generator(device=DEV).manual_seed(li * 100 + n)
            x64 = torch.randn(xs, generator=g, device=DEV, dtype=torch.float64)
            v64 = 0.2 * torch.randn((Co, Ci) + k, generator=g, device=DEV, dtype=torch.float64)
            b64 = 0.1 * torch.randn(Co, generator=g, device=DEV, dtype=torch.float64)
            x = x64.float().requires_grad_(True)
            v = v64.float().requires_grad_(True)
            b = b64.float().requires_grad_(True)
            y = ops.conv2d(x, v, None, b, k, s, d, pad, act)
            dy = torch.randn(y.shape, generator=g, device=DEV, dtype=torch.float64)
            y.backward(dy.float())
            # the reference in fp64 from the same fp32 operands, with OUR LeakyReLU mask
            xr, vr, br = (t.detach().double().requires_grad_(True) for t in (x, v, b))
            p = F.conv2d(xr, vr, br, stride=s, dilation=d, padding=pad)
            mask = torch.where(y.detach() > 0, 1.0, 0.2).double() if act else 1.0
            want_y = torch.where(y.detach() > 0, p, 0.2 * p) if act else p
            gx, gv, gb = torch.autograd.grad(p, (xr, vr, br), dy * mask)
            errs = {'y': rel(y, want_y), 'dx': rel(x.grad, gx), 'dw': rel(v.grad, gv), 'db': rel(b.grad, gb)}
            print(f'n {n} layer {li} {tuple(xs)}: ' + ' '.join(f'{k_} {e:.1e}' for k_, e in errs.items()))
            bad += [(n, li, k_, e) for k_, e in errs.items() if not e < 2e-5]
            del x64, x, y, dy, p, gx, gv, gb, xr
        assert not bad, bad
    finally:
        lib.encx_conv2d_select(prev)


@pytest.mark.parametrize('family', [1, 2], ids=['regwin', 'tiled'])
@pytest.mark.parametrize('li,T2,Fi', [(1, 43, 1025), (2, 90, 257), (3, 184, 129), (4, 90, 65)])
def test_feat_code_epilogue_bit_identical(li, T2, Fi, family):
    """encx_conv2d_bwd_data_feat with the pair's 1-byte code (encx_feat_loss_code: sign(ff - fr),
    ff > 0) against the same call reading both float maps: dx bit for bit, with the LeakyReLU'
    mask from the fake map (premask) and without, accumulating and not, at config-3 layer sizes
    (B 32) for each kernel family; and the loss and denominator of encx_feat_loss_code equal
    encx_feat_loss's."""
    from encx import ops
    from encx._lib import lib, call, ptr, stream
    Ci, Co, k, s, d, pad = LAYERS[li]
    KT, KF, sf, dt, pt, pf, Fo = ops.conv2d_geometry(Fi, k, s, d, pad)
    B = 32
    g = torch.Generator(device=DEV).manual_seed(li * 7 + T2)
    dy = torch.randn(B, Co, T2, Fo, generator=g, device=DEV)
    y = torch.randn(B, Co, T2, Fo, generator=g, device=DEV)
    ff = torch.randn(B, Ci, T2, Fi, generator=g, device=DEV)
    fr = ff + 0.3 * torch.randn(B, Ci, T2, Fi, generator=g, device=DEV)
    fr.view(-1)[::97] = ff.view(-1)[::97]  # ties: sign 0
    wf = 0.1 * torch.randn(Co * Ci * KT * KF, generator=g, device=DEV)
    wp = ops._wpoly(wf, Co, Ci, KT, KF, sf, dy)
    den = torch.rand(1, generator=g, device=DEV) + 0.5
    fg = torch.rand(1, generator=g, device=DEV) + 0.5
    n = ff.numel()
    code = torch.empty(n, device=DEV, dtype=torch.uint8)
    outs, dens = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    ws = torch.empty(lib.encx_disc_loss_workspace() // 4, device=DEV)
    call('encx_feat_loss', ptr(fr), ptr(ff), n, 3.0, ptr(outs[0:1]), ptr(dens[0:1]), 0, ptr(ws), stream())
    call('encx_feat_loss_code', ptr(fr), ptr(ff), n, 3.0, ptr(outs[1:2]), ptr(dens[1:2]), 0, ptr(ws), ptr(code),
         stream())
    assert torch.equal(outs[0], outs[1]) and torch.equal(dens[0], dens[1])
    dims = (B, Ci, T2, Fi, Co, Fo, KT, KF, sf, dt, pt, pf)
    prev = lib.encx_conv2d_select(family)
    try:
        for xact in (None, ff):
            for acc in (0, 1):
                res = []
                for c in (None, code):
                    dx = torch.full_like(ff, 0.5)
                    call('encx_conv2d_bwd_data_feat', ptr(dy), ptr(y), ptr(wp), ptr(xact), ptr(dx), acc, ptr(fr),
                         ptr(ff), ptr(den), ptr(fg), 3.0, ptr(c), *dims, stream())
                    res.append(dx)
                assert torch.equal(res[0], res[1]), (xact is not None, acc, float((res[0] - res[1]).abs().max()))
        # a LeakyReLU map other than the fake map is refused (the epilogues read one map for both)
        other = ff.clone()
        rc = lib.encx_conv2d_bwd_data_feat(ptr(dy), ptr(y), ptr(wp), ptr(other), ptr(dx), 0, ptr(fr), ptr(ff),
                                           ptr(den), ptr(fg), 3.0, None, *dims, stream())
        assert rc != 0
    finally:
        lib.encx_conv2d_select(prev)
