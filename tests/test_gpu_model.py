"""GPU parity of the whole model / train step (encx EncodecModel + Trainer) against the golden
fixtures generated from the reference and against the CPU oracle at full size."""
import numpy as np
import pytest
import torch

from oracle import encodec_oracle as O
from fixtures import load, T, model_state, codebooks_from_stats, certified, rvq_certified
from synth import synth_wave

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def G(a):
    return T(a).to(DEV)


def rel(a, b):
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.as_tensor(a, dtype=torch.float64)
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def build(target_bandwidths, audio_normalize, seed, stats, cb_seed, n_used):
    from encx.model import EncodecModel
    m = EncodecModel._get_model(list(target_bandwidths), 24000, 1, causal=True, model_norm='weight_norm',
                                audio_normalize=audio_normalize)
    cfg = O.Config(target_bandwidths=target_bandwidths, audio_normalize=audio_normalize)
    p = model_state(cfg, seed)
    cbs = codebooks_from_stats(stats, cb_seed, n_used, cfg.n_q)
    sd = dict(p)
    for i, cb in enumerate(cbs):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    return m.to(DEV), p, cbs, cfg


def test_eval_model_fixture():
    d = load('g1_eval24k.npz')
    m, p, cbs, cfg = build((1.5, 3., 6., 12., 24.), False, 1, d['stats'], 77, 2)
    m.eval()
    m.set_target_bandwidth(1.5)
    x = G(d['x'])
    with torch.no_grad():
        emb = m.encoder(x)
        codes = m.encode(x)[0][0]
        y = m(x)
    assert rel(emb, d['emb']) < 1e-4, rel(emb, d['emb'])
    ref = d['codes'].astype(np.int64)
    e2 = max(float((cb['embed'] ** 2).sum(1).max()) for cb in cbs[:2])
    cert = certified(d['gaps'], float((emb.cpu() ** 2).sum(1).max()), e2)
    mine = codes.cpu().numpy()
    # layer 0 against the reference's own codes, on the frames the fixture's fp64 gap certifies
    assert (mine[0][cert] == ref[0][cert]).all()
    # every layer against the fp64 RVQ of our latent, on every certified frame
    for factor in (256, 32):
        want, cert_all = rvq_certified(emb, [cb['embed'] for cb in cbs[:2]], factor)
        assert cert_all.any()
        assert torch.equal(torch.from_numpy(mine).transpose(0, 1)[cert_all], want[cert_all]), factor
    # decode unconditionally from the reference's codes (model.py:170-193)
    with torch.no_grad():
        y_ref_codes = m.decode([(G(ref).view(1, 2, -1), None)])
    assert rel(y_ref_codes, d['y']) < 1e-3, rel(y_ref_codes, d['y'])


def test_train_step_gen_fixture():
    """Two generator steps (config 2's step, B 2): each step's losses against the reference's
    (g7), and each step element by element against the oracle's step from the same state
    (tests/steputil.py: grads per tensor, post-Adam parameters, codebook EMA buffers)."""
    from encx.train import Trainer
    from steputil import check_step
    d = load('g7_step.npz')
    m, p, cbs, cfg = build((1.5,), True, 71, d['gen/stats'], 73, 2)
    weights = {'l_t': 0.1, 'l_f': 1}
    tr = Trainer(m, None, lr=3e-4, scheduler=False, weights=weights)
    x = G(d['gen/x'])
    for it in range(2):
        out, _ = check_step(tr, x, cfg, 1.5, weights)
        for k in ('l_t', 'l_f'):
            np.testing.assert_allclose(float(out[k]), float(d[f'gen/it{it}_{k}'].reshape(-1)[0]), rtol=1e-4)
        # the commit loss is a mean of (q - x)^2 over residuals ~10x smaller than x, so the
        # latent's ~1e-6 fp32 rounding is amplified; step 0 against the fp32 reference to 1e-4
        # (the oracle step above pins it to 2e-5 of fp64); the reference's own step 1 starts from
        # weights moved by its own Adam sign flips
        np.testing.assert_allclose(float(out['loss_w']), float(d[f'gen/it{it}_loss_w'].reshape(-1)[0]),
                                   rtol=1e-4 if it == 0 else 2e-3)


def test_full_size_forward_vs_oracle():
    """Config-2 shapes (B=32, 1 s @ 24 kHz, n_q=8): encoder/decoder parity at full size,
    codes bit-exact on every fp64-certified frame."""
    torch.manual_seed(0)
    from encx.model import EncodecModel
    cfg = O.Config(target_bandwidths=(6.0,), audio_normalize=True)
    p = model_state(cfg, 5)
    m = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    x0 = synth_wave((32, 1, 24000), 1234)
    xn, _ = O.normalize(T(x0))
    with torch.no_grad():
        emb_ref = O.run_plan(xn, p, cfg.enc_plan)
    e = emb_ref.permute(0, 2, 1).reshape(-1, 128).double()
    stats = np.zeros((8, 2, 128), np.float32)
    for i in range(8):
        stats[i, 0] = e.mean(0).float().numpy() * (1 if i == 0 else 0)
        stats[i, 1] = e.std(0).float().numpy() * (0.6 ** i)
    cbs = codebooks_from_stats(stats, 9, 8, cfg.n_q)
    sd = dict(p)
    for i, cb in enumerate(cbs):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    from encx import ops
    x = G(x0)
    with torch.no_grad():
        emb = m.encoder(ops.normalize(x)[0])
    assert rel(emb, emb_ref) < 2e-4, rel(emb, emb_ref)
    # RVQ layer 0 codes: bit-exact on certified frames
    idx = ops.rvq_argmin(emb.contiguous(), m.quantizer.vq.layers[0]._codebook.embed).cpu().numpy()
    xr = emb_ref.permute(0, 2, 1).reshape(-1, 128).double()
    E = cbs[0]['embed'].double()
    dist = (xr ** 2).sum(1, keepdim=True) - 2 * xr @ E.t() + (E ** 2).sum(1)[None]
    s = torch.sort(dist, 1).values
    cert = certified((s[:, 1] - s[:, 0]).numpy(), float((xr ** 2).sum(1).max()), float((E ** 2).sum(1).max()))
    ref_idx = O.codebook_quantize(emb_ref.permute(0, 2, 1).reshape(-1, 128), cbs[0]['embed']).numpy()
    assert cert.mean() > 0.9, cert.mean()
    assert (idx[cert] == ref_idx[cert]).all()
    # decoder on the same latent
    with torch.no_grad():
        y = m.decoder(emb)
        y_ref = O.run_plan(emb_ref, p, cfg.dec_plan)
    assert rel(y, y_ref) < 1e-3, rel(y, y_ref)


def test_full_size_train_steps_run():
    """Fresh model (kmeans init on the first batch), 3 config-2 steps at full size."""
    torch.manual_seed(0)
    from encx.model import EncodecModel
    from encx.train import Trainer
    m = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                audio_normalize=True).to(DEV)
    tr = Trainer(m, None, lr=3e-4, warmup_iter=10)
    x = G(synth_wave((32, 1, 24000), 77))
    hist = []
    for _ in range(3):
        out = tr.step(x)
        hist.append({k: float(v) for k, v in out.items()})
    for h in hist:
        assert all(np.isfinite(v) for v in h.values()), h
    cb = m.quantizer.vq.layers[0]._codebook
    assert float(cb.inited) == 1.0 and torch.isfinite(cb.embed).all()
    assert torch.isfinite(tr.opt.flat).all()
    assert hist[-1]['l_f'] < hist[0]['l_f'] * 1.05


def test_train_grads_vs_oracle_fp64():
    """Element-level check of the whole generator backward (balanced l_t + l_f + commit, ONE
    backward as in Trainer.step) against the oracle run in fp64, on the G7 fixture's model,
    codebooks and clip. Adam is left out so near-zero grads cannot hide behind sign flips."""
    from encx.losses import total_loss
    from encx.train import Trainer
    d = load('g7_step.npz')
    m, p, cbs, cfg = build((1.5,), True, 71, d['gen/stats'], 73, 2)
    tr = Trainer(m, None, lr=3e-4, scheduler=False, weights={'l_t': 0.1, 'l_f': 1})
    x = G(d['gen/x'])
    m.train()
    tr.opt.zero_grad()
    y, loss_w, _ = m(x)
    codes = m.last_codes[0]
    losses = total_loss(None, None, None, x, y, 24000)
    out_grad = tr.balancer.compute(losses, y)
    torch.autograd.backward([y, loss_w], [out_grad, torch.ones_like(loss_w)])
    torch.cuda.synchronize()

    x64 = T(d['gen/x']).double()
    p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
    cbs64 = [{k: v.double() for k, v in cb.items()} for cb in cbs]
    y64, lw64, codes64, _, _ = O.encodec_forward_train(x64, p64, cbs64, cfg, 1.5)
    l64 = {'l_t': O.loss_t(x64, y64), 'l_f': O.loss_f(x64, y64, 24000)}
    g64 = {k: torch.autograd.grad(l, [y64], retain_graph=True)[0] for k, l in l64.items()}
    og = O.Balancer({'l_t': 0.1, 'l_f': 1}).combine(g64)
    torch.autograd.backward([y64, lw64], [og, torch.ones_like(lw64)])

    assert torch.equal(codes.cpu().long(), torch.as_tensor(codes64).long().reshape(codes.shape))
    assert rel(y, y64) < 1e-4
    lw_err = rel(loss_w, lw64)
    print(f'loss_w rel err vs fp64 {lw_err:.3e}')
    assert lw_err < 2e-5, lw_err
    # the same backward in plain fp32 (the oracle): each tensor's bound is 4x its error
    p32 = {k: v.float().requires_grad_(True) for k, v in p.items()}
    cbs32 = [{k: v.float() for k, v in cb.items()} for cb in cbs]
    x32 = T(d['gen/x']).float()
    y32, lw32, _, _, _ = O.encodec_forward_train(x32, p32, cbs32, cfg, 1.5)
    l32 = {'l_t': O.loss_t(x32, y32), 'l_f': O.loss_f(x32, y32, 24000)}
    g32 = {k: torch.autograd.grad(l, [y32], retain_graph=True)[0] for k, l in l32.items()}
    torch.autograd.backward([y32, lw32], [O.Balancer({'l_t': 0.1, 'l_f': 1}).combine(g32), torch.ones_like(lw32)])
    from steputil import check_grads
    params = dict(m.named_parameters())
    check_grads({k: params[k].grad for k in p64}, {k: v.grad for k, v in p64.items()},
                {k: v.grad for k, v in p32.items()}, 'generator grads vs fp64')


def test_config3_b32_step_and_input_grads_vs_fp64():
    """Config 3 at its real size (B 32, 1 s, n_q 8, the MS-STFT discriminator, all four losses
    balanced): two Trainer steps stay finite; and the generator phase's per-loss grads w.r.t.
    the fake audio (l_t, l_f, l_g through the discriminator; what the balancer combines) for one
    clip of the B 32 batch against the fp64 oracle run on that clip alone (each loss is a batch
    mean, so clip 0's grad in the batch is 1/32 of its single-clip grad), each within 4x of the
    fp32 oracle's error (the oracle's LeakyReLU slopes taken from our maps)."""
    from encx.train import Trainer
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from encx.losses import total_loss
    from fixtures import disc_state
    from steputil import check_grads
    m, p, cbs, cfg = build((6.0,), True, 3, np.stack([np.zeros((2, 128)), np.full((2, 128), 0.05)], 1)
                           .astype(np.float32)[[0] * 8], 4, 8)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.to(DEV)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, max_iter=100, warmup_iter=0)
    x = G(synth_wave((32, 1, 24000), 606))
    for _ in range(2):
        out = tr.step(x)
        assert all(np.isfinite(float(v)) for v in out.values()), out
    assert torch.isfinite(tr.opt.flat).all() and torch.isfinite(tr.opt_d.flat).all()
    # the generator phase on the stepped weights
    m.train()
    y, _, _ = m(x)
    yd = y.detach().requires_grad_()
    from steputil import disc_maps
    lr_, fr = disc(x)
    with disc_maps(disc, DEV) as (ins, outs):
        lf_, ff = disc(yd)
    losses = total_loss(fr, lf_, ff, x, yd, 24000)
    mine = {k: torch.autograd.grad(losses[k], [yd], retain_graph=True)[0][0] for k in ('l_t', 'l_f', 'l_g')}
    dp = {k: v.detach().cpu() for k, v in disc.state_dict().items() if not k.endswith('spec_transform.window')}
    # LeakyReLU slopes from OUR fp32 maps of clip 0 (a pre-activation within rounding of 0 may
    # take either slope in fp32: a discrete, legitimate outcome that a rounding bound cannot
    # cover; oracle._lrelu), so the comparison measures rounding only
    masks = [[fm[:1].detach().cpu() > 0 for fm in fms] for fms in ff]
    from steputil import lrelu_audit, check_flips
    ref, audit = {}, {}
    for dt in (torch.float64, torch.float32):
        x0 = x[:1].detach().cpu().to(dt)
        y0 = yd[:1].detach().cpu().to(dt).requires_grad_(True)
        pd = {k: v.to(dt) for k, v in dp.items()}
        with lrelu_audit() as audit[dt]:
            lg, _ = O.msstft_forward(y0, pd, masks=masks)
        ls = {'l_t': O.loss_t(x0, y0), 'l_f': O.loss_f(x0, y0, 24000),
              'l_g': sum(torch.relu(1 - l).mean() for l in lg) / len(lg) / len(lg)}
        ref[dt] = {k: torch.autograd.grad(l, [y0], retain_graph=True)[0][0] / 32 for k, l in ls.items()}
    check_flips(disc, dict(disc.named_parameters()), [t[:1] for t in ins], [t[:1] for t in outs],
                audit[torch.float64], None, 'config-3 B32 clip-0 slope masks')
    check_grads(mine, ref[torch.float64], ref[torch.float32], 'config-3 B32 input grads of clip 0')
