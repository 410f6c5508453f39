"""Pin the CPU oracle to the golden fixtures generated from the real reference (CPU only).

These tests are what make the oracle trustworthy as the parity checker for the HIP path.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import encodec_oracle as O
from fixtures import load, T, model_state, disc_state, codebooks_from_stats, g3_codebooks, certified
from synth import synth_state

torch.set_num_threads(min(8, torch.get_num_threads()))


def close(a, b, rtol=1e-5, atol=1e-6):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


# --------------------------------------------------------------------------- mel filters
def test_mel_filterbank_matches_fixture_and_transformers():
    d = load('g4_mel.npz')
    for i in range(5, 12):
        n = 2 ** i
        mine = O.mel_filterbank(24000, n, 64)
        close(mine, d[f'melbasis{n}'], rtol=0, atol=0)
    try:
        from transformers.audio_utils import mel_filter_bank
    except Exception:  # pragma: no cover
        pytest.skip('transformers not importable')
    for i in range(5, 12):
        n = 2 ** i
        ref = mel_filter_bank(num_frequency_bins=n // 2 + 1, num_mel_filters=64, min_frequency=0.0,
                              max_frequency=12000.0, sampling_rate=24000, norm='slaney',
                              mel_scale='slaney').T
        np.testing.assert_allclose(O.mel_filterbank(24000, n, 64), ref, rtol=1e-5, atol=1e-9)
    # a band-limited bank (Audio2Mel's mel_fmin / mel_fmax, audio_to_mel.py:24), 80 mels
    for n, sr, lo, hi in [(1024, 22050, 0.0, 8000.0), (2048, 24000, 50.0, 9000.0), (512, 16000, 125.0, None)]:
        ref = mel_filter_bank(num_frequency_bins=n // 2 + 1, num_mel_filters=80, min_frequency=lo,
                              max_frequency=sr / 2 if hi is None else hi, sampling_rate=sr, norm='slaney',
                              mel_scale='slaney').T
        np.testing.assert_allclose(O.mel_filterbank(sr, n, 80, lo, hi), ref, rtol=1e-5, atol=1e-9)


# --------------------------------------------------------------------------- convs
CASES = [
    ('c_k7_1to8', 'conv', 1, 8, 7, 1, True, False, 480),
    ('c_k3_16to8_elu', 'conv', 16, 8, 3, 1, True, True, 480),
    ('c_k1_8to16_elu', 'conv', 8, 16, 1, 1, True, True, 480),
    ('c_k1_16to16', 'conv', 16, 16, 1, 1, True, False, 480),
    ('c_k4s2_16to32_elu', 'conv', 16, 32, 4, 2, True, True, 480),
    ('c_k10s5_16to32_elu', 'conv', 16, 32, 10, 5, True, True, 480),
    ('c_k16s8_32to64_elu', 'conv', 32, 64, 16, 8, True, True, 480),
    ('c_k7_64to16_elu', 'conv', 64, 16, 7, 1, True, True, 30),
    ('c_k7_short_reflect', 'conv', 8, 8, 7, 1, True, False, 5),
    ('c_k7s1_nc', 'conv', 8, 8, 7, 1, False, False, 100),
    ('c_k10s5_nc_odd', 'conv', 8, 16, 10, 5, False, True, 97),
    ('t_k4s2_32to16_elu', 'convtr', 32, 16, 4, 2, True, True, 240),
    ('t_k10s5_32to16_elu', 'convtr', 32, 16, 10, 5, True, True, 96),
    ('t_k16s8_64to32_elu', 'convtr', 64, 32, 16, 8, True, True, 60),
    ('t_k8s4_nc', 'convtr', 16, 8, 8, 4, False, False, 50),
]


def conv_case_state(ci, kind, cin, cout, K):
    pre = 'convtr.convtr' if kind == 'convtr' else 'conv.conv'
    wshape = (cin, cout, K) if kind == 'convtr' else (cout, cin, K)
    shapes = {pre + '.bias': (cout,), pre + '.weight_g': (wshape[0], 1, 1), pre + '.weight_v': wshape}
    st = synth_state(shapes, 100 + ci)
    return {('m.' + k): T(v) for k, v in st.items()}, pre


@pytest.mark.parametrize('ci', range(len(CASES)))
def test_oracle_conv_fixture(ci):
    d = load('g2_convs.npz')
    name, kind, cin, cout, K, s, causal, pre_elu, Tn = CASES[ci]
    p, pre = conv_case_state(ci, kind, cin, cout, K)
    p = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    x = T(d[name + '/x']).clone().requires_grad_(True)
    xin = F.elu(x) if pre_elu else x
    if kind == 'conv':
        y = O.sconv1d(xin, p, 'm', K, s, causal=causal)
    else:
        y = O.sconvtr1d(xin, p, 'm', K, s, causal=causal)
    close(y, d[name + '/y'])
    y.backward(T(d[name + '/gy']))
    close(x.grad, d[name + '/dx'], rtol=1e-4, atol=1e-5)
    close(p['m.' + pre + '.weight_v'].grad, d[name + '/dv'], rtol=1e-4, atol=1e-5)
    close(p['m.' + pre + '.weight_g'].grad, d[name + '/dg'], rtol=1e-4, atol=1e-5)
    close(p['m.' + pre + '.bias'].grad, d[name + '/db'], rtol=1e-4, atol=1e-4)


# --------------------------------------------------------------------------- G1 eval model
def test_oracle_eval_24k_fixture():
    d = load('g1_eval24k.npz')
    cfg = O.Config(audio_normalize=False)
    p = model_state(cfg, 1)
    cbs = codebooks_from_stats(d['stats'], 77, 2, cfg.n_q)
    with torch.no_grad():
        y, codes, emb = O.encodec_forward_eval(T(d['x']), p, cbs, cfg, 1.5)
    close(emb, d['emb'], rtol=1e-4, atol=1e-6)
    ref_codes = d['codes'].astype(np.int64)
    mine = codes.numpy()
    assert mine.shape == ref_codes.shape
    e2 = max(float((cb['embed'] ** 2).sum(1).max()) for cb in cbs[:2])
    x2 = float((emb ** 2).sum(1).max())
    cert = certified(d['gaps'], x2, e2)
    assert cert.sum() > 0
    assert (mine[0][cert] == ref_codes[0][cert]).all()
    # where every code agrees, the decoded waveform must agree too
    if (mine == ref_codes).all():
        close(y, d['y'], rtol=1e-3, atol=1e-6)


# --------------------------------------------------------------------------- G3 RVQ
def test_oracle_rvq_train_fixture():
    d = load('g3_rvq.npz')
    cbs = g3_codebooks(d)
    emb = T(d['emb']).clone().requires_grad_(True)
    q, codes, penalty, new = O.rvq_train(emb, cbs, 2)
    assert (codes.numpy() == d['codes']).all()
    close(q, d['quantized'])
    close(penalty, d['penalty'])
    torch.autograd.backward([q, penalty], [T(d['gq']), torch.tensor(1.0)])
    close(emb.grad, d['demb'], rtol=1e-5, atol=1e-6)
    for i in range(2):
        close(new[i]['cluster_size'], d[f'cluster_size{i}'], rtol=1e-6, atol=1e-7)
        close(new[i]['embed_avg'], d[f'embed_avg{i}'], rtol=1e-5, atol=1e-6)
        close(new[i]['embed'], d[f'embed{i}'], rtol=1e-5, atol=1e-6)


def test_oracle_kmeans_fixture():
    d = load('g3_rvq.npz')
    means, bins = O.kmeans(T(d['km_samples']), 64, 10, T(d['km_init']))
    close(means, d['km_means'], rtol=1e-5, atol=1e-6)
    assert (bins.numpy() == d['km_bins']).all()


# --------------------------------------------------------------------------- G4 mel
def test_oracle_mel_and_spec_fixture():
    d = load('g4_mel.npz')
    x = T(d['x'])
    for i in range(5, 12):
        n = 2 ** i
        close(O.audio2mel(x, n, n // 4, n, 24000), d[f'mel{n}'], rtol=1e-4, atol=1e-4)
    for n, h in zip((1024, 2048, 512), (256, 512, 128)):
        close(torch.view_as_real(O.spectrogram(x, n, h, n)), d[f'spec{n}'], rtol=1e-4, atol=1e-5)


def test_oracle_losses_fixture():
    d = load('g4_mel.npz')
    x = T(d['x'])
    y = T(d['y']).clone().requires_grad_(True)
    lt = O.loss_t(x, y)
    lf = O.loss_f(x, y)
    close(lt, d['l_t'])
    close(lf, d['l_f'], rtol=1e-5)
    gf, = torch.autograd.grad(lf, [y])
    gt, = torch.autograd.grad(lt, [y])
    close(gf, d['dlf_dy'], rtol=1e-4, atol=1e-7)
    close(gt, d['dlt_dy'])


# --------------------------------------------------------------------------- G5 disc
def test_oracle_disc_fixture():
    d = load('g5_disc.npz')
    p = disc_state(51)
    x = T(d['x']).clone().requires_grad_(True)
    logits, fmaps = O.msstft_forward(x, p)
    r = np.random.Generator(np.random.PCG64(53))
    f = 0
    for k, lg in enumerate(logits):
        close(lg, d[f'logits{k}'], rtol=1e-4, atol=1e-5)
        wl = T(r.standard_normal(size=tuple(lg.shape)).astype(np.float32))
        f = f + (lg * wl).sum()
        for j, fm in enumerate(fmaps[k]):
            assert tuple(fm.shape) == tuple(d[f'fmap{k}_{j}_shape'])
            np.testing.assert_allclose(fm.detach().double().sum().item(), d[f'fmap{k}_{j}_sum'], rtol=1e-4)
            np.testing.assert_allclose(fm.detach().double().pow(2).sum().item(), d[f'fmap{k}_{j}_sq'], rtol=1e-4)
            close(fm.reshape(-1)[:256], d[f'fmap{k}_{j}_head'], rtol=1e-4, atol=1e-5)
            f = f + fm.mean()
    f.backward()
    close(x.grad, d['dx'], rtol=1e-3, atol=1e-5)


def test_sign_audit_flags_only_real_sign_errors():
    """steputil.check_flips, the a-priori sign audit: with the maps of a fp32 evaluation standing
    in for the HIP maps (their signs imposed on the fp64 oracle), every flipped element's fp32
    pre-activation lies within gamma_n sum|w x| of its fp64 recompute from the same inputs and the
    audit passes; a sign error planted at one element (the map's largest |z| negated: what a wrong
    epilogue does) fails it, and so does an imposed mask that is not the map's own sign."""
    import pytest
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from steputil import lrelu_audit, check_flips
    d = load('g5_disc.npz')
    p = disc_state(51)
    x = T(d['x'])[:1, :, :6000]
    disc = MultiScaleSTFTDiscriminator(filters=32)  # the layer geometry (CPU module, no kernels)
    ins, outs = [], []
    for k, (n, h, w) in enumerate(zip(O.DISC_CFG['n_ffts'], O.DISC_CFG['hops'], O.DISC_CFG['wins'])):
        z = O.spectrogram(x, n, h, w)
        z = torch.cat([z.real, z.imag], dim=1).permute(0, 1, 3, 2)
        _, fm = O.disc_stft_forward(x, p, f'discriminators.{k}', n, h, w)
        ins += [z] + fm[:-1]
        outs += fm

    def audit(maps):
        masks = [[maps[5 * k + j] > 0 for j in range(5)] for k in range(3)]
        with lrelu_audit() as a64:
            O.msstft_forward(x.double(), {k: v.double() for k, v in p.items()}, masks=masks)
        return a64
    assert check_flips(disc, p, ins, outs, audit(outs), None, 'fp32 maps') >= 0
    y = outs[3]
    zh = torch.where(y > 0, y, y / 0.2)
    # a flip within rounding of 0 (the element of smallest nonzero |z|, negated) is legitimate
    j = int(torch.where(zh != 0, zh.abs(), torch.full_like(zh, float('inf'))).reshape(-1).argmin())
    znear = zh.clone().reshape(-1)
    znear[j] = -znear[j]
    znear = znear.view_as(zh)
    near = list(outs)
    near[3] = torch.where(znear > 0, znear, 0.2 * znear)
    assert check_flips(disc, p, ins, near, audit(near), None, 'one flip within rounding of 0') >= 1
    i = int(zh.abs().reshape(-1).argmax())
    zbad = zh.clone().reshape(-1)
    zbad[i] = -zbad[i]
    zbad = zbad.view_as(zh)
    bad = list(outs)
    bad[3] = torch.where(zbad > 0, zbad, 0.2 * zbad)
    with pytest.raises(AssertionError, match='a-priori'):
        check_flips(disc, p, ins, bad, audit(bad), None, 'one planted sign error')
    a64 = audit(outs)
    z64, m = a64[3]
    mb = m.clone().reshape(-1)
    mb[i] = ~mb[i]
    a64[3] = (z64, mb.view_as(m))
    with pytest.raises(AssertionError, match='sign'):
        check_flips(disc, p, ins, outs, a64, None, 'a mask that is not the map\'s sign')


# --------------------------------------------------------------------------- G6 balancer
def test_oracle_balancer_fixture():
    d = load('g6_balancer.npz')
    # known answer, balancer.py:121-139 (rescale off: plain weighted sum)
    assert float(d['kat_0'][0]) == 99.0 and float(d['kat_1'][0]) == 0.0
    b = O.Balancer({'1': 1, '2': 1})
    out = b.combine({'1': torch.tensor([-1.0]), '2': torch.tensor([100.0])})
    assert abs(float(out)) < 1e-6
    b = O.Balancer({'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3})
    for it in range(3):
        grads = {k: T(d[f'it{it}_{k}']) for k in ('l_t', 'l_f', 'l_g', 'l_feat')}
        close(b.combine(grads), d[f'it{it}_out'], rtol=1e-5, atol=1e-8)


# --------------------------------------------------------------------------- G7 train step
@pytest.mark.parametrize('gan', [False, True])
def test_oracle_train_step_fixture(gan):
    d = load('g7_step.npz')
    pre = 'gan/' if gan else 'gen/'
    cfg = O.Config(target_bandwidths=(1.5,), audio_normalize=True)
    p = model_state(cfg, 71)
    cbs = codebooks_from_stats(d[pre + 'stats'], 73, 2, cfg.n_q)
    dp = disc_state(74) if gan else None
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3} if gan else {'l_t': 0.1, 'l_f': 1}
    bal = O.Balancer(weights)
    st, dst = {}, {}
    x = T(d[pre + 'x'])
    for it in range(2):
        out = O.train_step(x, p, cbs, cfg, 1.5, bal, st, 3e-4, disc_p=dp, disc_adam_state=dst, disc_lr=3e-4)
        for k in weights:
            np.testing.assert_allclose(out[k], float(d[f'{pre}it{it}_{k}'].reshape(-1)[0]), rtol=2e-4)
        np.testing.assert_allclose(out['loss_w'], float(d[f'{pre}it{it}_loss_w'].reshape(-1)[0]), rtol=2e-3, atol=1e-7)
        if gan:
            np.testing.assert_allclose(out['l_d'], float(d[f'{pre}it{it}_l_d'].reshape(-1)[0]), rtol=1e-5)
    keys = [k[len(pre) + 2:] for k in d.files if k.startswith(pre + 'p/')]
    names = set(p) | {f'quantizer.vq.layers.{i}._codebook.{b}' for i in range(cfg.n_q)
                      for b in ('inited', 'cluster_size', 'embed', 'embed_avg')}
    assert set(keys) == names
    for k in p:
        ref = d[pre + 'p/' + k]
        v = p[k].double()
        np.testing.assert_allclose([v.sum().item(), v.abs().sum().item()], ref, rtol=2e-4, atol=2e-5)
    for i in range(2):
        for b in ('cluster_size', 'embed', 'embed_avg'):
            ref = d[f'{pre}p/quantizer.vq.layers.{i}._codebook.{b}']
            v = cbs[i][b].double()
            np.testing.assert_allclose([v.sum().item(), v.abs().sum().item()], ref, rtol=1e-4, atol=1e-4)
    if gan:
        for k in dp:
            np.testing.assert_allclose([dp[k].double().sum().item(), dp[k].double().abs().sum().item()],
                                       d['gan/d/' + k], rtol=2e-4, atol=2e-5)


# --------------------------------------------------------------------------- G9 48 kHz stereo
@pytest.mark.parametrize('gan', [False, True])
def test_oracle_train_step_48k_fixture(gan):
    """Config-5 model shape: 48 kHz stereo, non-causal, GroupNorm, two segments overlap-added
    (model.py:122-181, utils.py:22-61); mel losses at 48 kHz; stereo discriminator."""
    from fixtures import cfg48k
    d = load('g9_step48k.npz')
    pre = 'gan/' if gan else 'gen/'
    cfg = cfg48k()
    assert cfg.n_q == 2 and cfg.frame_rate == 150
    assert len(O.segments(cfg, 4800)) == int(d[pre + 'it0_nframes']) == 2
    p = model_state(cfg, 91)
    cbs = codebooks_from_stats(d[pre + 'stats'], 93, 2, cfg.n_q)
    dp = disc_state(94, 2, 2) if gan else None
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4} if gan else {'l_t': 0.1, 'l_f': 1}
    bal = O.Balancer(weights)
    st, dst = {}, {}
    x = T(d[pre + 'x'])
    for it in range(2):
        out = O.train_step(x, p, cbs, cfg, 3.0, bal, st, 1e-4, disc_p=dp, disc_adam_state=dst, disc_lr=1e-4)
        for k in weights:
            np.testing.assert_allclose(out[k], float(d[f'{pre}it{it}_{k}'].reshape(-1)[0]), rtol=2e-4)
        np.testing.assert_allclose(out['loss_w'], float(d[f'{pre}it{it}_loss_w'].reshape(-1)[0]), rtol=2e-3, atol=1e-7)
        if gan:
            np.testing.assert_allclose(out['l_d'], float(d[f'{pre}it{it}_l_d'].reshape(-1)[0]), rtol=1e-5)
    # Adam's first steps move each weight by ~lr * sign(g): a weight whose grad is ~0 can flip
    # sign under fp reordering (2 lr per flip), so the signed sums get a few flips of slack
    flips = 4 * 2 * 1e-4 * 2
    for k in p:
        ref = d[pre + 'p/' + k]
        v = p[k].double()
        assert abs(v.sum().item() - ref[0]) <= 2e-4 * abs(ref[0]) + flips, (k, v.sum().item(), ref)
        np.testing.assert_allclose(v.abs().sum().item(), ref[1], rtol=2e-4, atol=2e-5, err_msg=k)
    for i in range(2):
        for b in ('cluster_size', 'embed', 'embed_avg'):
            ref = d[f'{pre}p/quantizer.vq.layers.{i}._codebook.{b}']
            v = cbs[i][b].double()
            np.testing.assert_allclose([v.sum().item(), v.abs().sum().item()], ref, rtol=1e-4, atol=1e-4)
    if gan:
        for k in dp:
            v = dp[k].double()
            assert abs(v.sum().item() - d['gan/d/' + k][0]) <= 2e-4 * abs(d['gan/d/' + k][0]) + flips, k
            np.testing.assert_allclose(v.abs().sum().item(), d['gan/d/' + k][1], rtol=2e-4, atol=2e-5, err_msg=k)


def test_oracle_overlap_add_matches_reference_rule():
    """utils.py:22-61 on hand-checkable frames: a lone frame passes through; where two frames
    overlap the weights are the first frame's triangle, normalised."""
    f0 = torch.ones(1, 10)
    assert torch.allclose(O.linear_overlap_add([f0], 10), f0)
    f1 = 3 * torch.ones(1, 4)
    out = O.linear_overlap_add([f0, f1], 8)
    assert out.shape[-1] == 12
    t = torch.linspace(0, 1, 12)[1:-1]
    w = 0.5 - (t - 0.5).abs()
    exp = torch.cat([torch.ones(8), (w[8:10] + 3 * w[:2]) / (w[8:10] + w[:2]), 3 * torch.ones(2)])
    assert torch.allclose(out[0], exp)


# --------------------------------------------------------------------------- G8 scheduler
def test_oracle_scheduler_fixture():
    d = load('g8_sched.npz')
    lrs = [O.warmup_cosine_lr(3e-4, i, 400, 50) for i in range(400)]
    np.testing.assert_allclose(lrs, d['lr'], rtol=1e-12)


def test_rvq_bandwidth_rule():
    # vq.py:101-113 at 75 Hz
    assert [O.rvq_num_quantizers(b, 75) for b in (1.5, 3., 6., 12., 24.)] == [2, 4, 8, 16, 32]
    assert [O.rvq_num_quantizers(b, 150) for b in (3., 6., 12., 24.)] == [2, 4, 8, 16]
    assert math.isclose(O.Config().frame_rate, 75)


# --------------------------------------------------------------------------- g12 LM coder
def test_oracle_quantized_cdf_and_coder_fixture():
    from oracle import ac_oracle as A
    from fixtures import g12_ac_rows
    d = load('g12_lm.npz')
    for card, bits, pdf, cdf, sym, data, eof in g12_ac_rows(d):
        for p, c in zip(pdf, cdf):
            assert np.array_equal(A.quantized_cdf(p, bits, check=False), c)
        assert A.encode(sym, cdf, bits) == data
        dec = A.Decoder(data, bits)
        assert [dec.pull(c) for c in cdf] == sym.tolist()
        assert dec.bytes_read == len(data)
        if eof == 1:
            assert dec.pull(np.zeros(1, np.int64)) is None
        else:
            with pytest.raises(RuntimeError):
                dec.pull(np.zeros(1, np.int64))
    # near-certain pdfs whose cdf total exceeds 2^bits: check=True rejects, the coder asserts
    o = 0
    for card, bits in zip(d['ac_over_card'], d['ac_over_bits']):
        p, c = d['ac_over_pdf'][o:o + card], d['ac_over_cdf'][o:o + card]
        o += card
        assert np.array_equal(A.quantized_cdf(p, int(bits), check=False), c)
        assert c[-1] > 2 ** int(bits)
        with pytest.raises(AssertionError):
            A.quantized_cdf(p, int(bits), check=True)
        with pytest.raises(AssertionError):
            A.encode([card - 1], [c], int(bits))


@pytest.mark.parametrize('name', ['a', 'b'])
def test_oracle_lm_fixture(name):
    from oracle import lm_oracle as L
    from fixtures import g12_lm_config
    d = load('g12_lm.npz')
    cfg, st = g12_lm_config(name)
    codes = T(d[f'lm_{name}/codes'])
    ref = d[f'lm_{name}/probs']                       # [B][T][K][card]
    B, K, Tn = codes.shape
    states, offset = None, 0
    inp = torch.zeros(B, K, 1, dtype=torch.long)
    got = []
    for t in range(Tn):
        p, states, offset = L.lm_step(st, inp, states, offset, cfg)
        inp = 1 + codes[:, :, t:t + 1]
        got.append(p[:, :, :, 0].permute(0, 2, 1))
    close(torch.stack(got, 1), ref, rtol=1e-4, atol=1e-7)
    # the one-pass form (teacher-forced, phantom zero key) gives the same probabilities
    allp = L.lm_all(st, codes, cfg).permute(0, 3, 2, 1)   # [B][T][K][card]
    close(allp, ref, rtol=1e-4, atol=1e-7)


def test_oracle_lm_compress_fixture():
    """compress(use_lm=True) bytes of the reference (g1 model, 1.5 kbps, 0.2 s): the oracle's
    cdfs from the reference's pdfs and its coder reproduce the payload bit for bit, and the
    oracle LM reproduces the pdfs."""
    from oracle import ac_oracle as A, ecdc_oracle as E, lm_oracle as L
    from fixtures import g12_lm_config
    d = load('g12_lm.npz')
    data = d['e2e_bytes'].tobytes()
    meta, off = E.parse_header(data)
    codes = d['e2e_codes']                            # [1][K][T]
    K, Tn = codes.shape[1:]
    assert meta == {'m': 'encodec_24khz', 'al': 4800, 'nc': int(K), 'lm': True, 'fr': int(Tn)}
    cdfs = [A.quantized_cdf(p, 24, check=False) for p in d['e2e_pdf']]
    assert all(np.array_equal(a, b) for a, b in zip(cdfs, d['e2e_cdf']))
    syms = codes[0].T.reshape(-1)                     # push order: t-major, then codebook
    assert A.encode(syms, cdfs) == data[off:]
    cfg, st = g12_lm_config('a')
    p = L.lm_all(st, T(codes), cfg)                   # [1][card][K][T]
    close(p[0].permute(2, 1, 0).reshape(-1, cfg.card), d['e2e_pdf'], rtol=1e-4, atol=1e-7)


def test_code_impose_and_tie_audit():
    """steputil.code_impose / check_code_ties (the GPU step checks' nearest-code audit): the
    oracle's rvq_train takes the imposed codes in order, logs its own picks, and the audit passes
    a flip between two codes at the same distance (within our latent's distance from the fp64
    one) and refuses a flip to a far code."""
    from steputil import code_impose, check_code_ties
    g = torch.Generator().manual_seed(3)
    B, D, Tn, K, n_q = 2, 8, 5, 16, 2
    emb = torch.randn(B, D, Tn, generator=g, dtype=torch.float64)
    cbs = [{'inited': torch.ones(1), 'cluster_size': torch.ones(K, dtype=torch.float64),
            'embed': torch.randn(K, D, generator=g, dtype=torch.float64),
            'embed_avg': torch.randn(K, D, generator=g, dtype=torch.float64)} for _ in range(n_q)]
    # row 0's first-layer target made equidistant from codes 3 and 5
    x0 = 0.5 * (cbs[0]['embed'][3] + cbs[0]['embed'][5])
    emb[0, :, 0] = x0
    _, own, _, _ = O.rvq_train(emb, cbs, n_q)
    assert int(own[0, 0, 0]) in (3, 5)
    seg = [(own.reshape(n_q, -1).clone(), emb.float())]
    with code_impose(seg) as log:
        _, got, _, _ = O.rvq_train(emb, cbs, n_q)
    assert torch.equal(got, own) and len(log) == n_q
    assert check_code_ties(log, seg, n_q, 'same') == 0
    flip = own.reshape(n_q, -1).clone()
    flip[0, 0] = 8 - int(own[0, 0, 0])  # the other of the tied pair
    with code_impose([(flip, emb.float())]) as log:  # layer 1's picks after the flip
        O.rvq_train(emb, cbs, n_q)
    flip[1] = log[1][2]
    seg = [(flip, emb.float())]
    with code_impose(seg) as log:
        _, got, _, _ = O.rvq_train(emb, cbs, n_q)
    assert int(got[0, 0, 0]) == int(flip[0, 0])
    assert check_code_ties(log, seg, n_q, 'tie') >= 1
    far = own.reshape(n_q, -1).clone()
    d = ((emb[0, :, 1][None] - cbs[0]['embed']) ** 2).sum(1)
    far[0, 1] = int(d.argmax())
    seg = [(far, emb.float())]
    with code_impose(seg) as log:
        O.rvq_train(emb, cbs, n_q)
    with pytest.raises(AssertionError):
        check_code_ties(log, seg, n_q, 'far')
    assert O.CODES is None and O.CODE_AUDIT is None


def test_l1_sign_impose_and_audit():
    """steputil.l1_impose / check_l1_flips: with our own signs imposed the oracle's reconstruction
    L1 has F.l1_loss's value and gradient; a flipped sign at a near tie passes the audit and moves
    that element's gradient; a flip at a large difference is refused."""
    from steputil import l1_impose, check_l1_flips
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 1, 4000, generator=g, dtype=torch.float64)
    y = (x + 0.1 * torch.randn(2, 1, 4000, generator=g, dtype=torch.float64)).requires_grad_(True)
    with torch.no_grad():
        y[0, 0, 7] = x[0, 0, 7] + 1e-9  # a near tie
    ref = F.l1_loss(x, y)
    gref, = torch.autograd.grad(ref, y)
    sig = {'t': torch.sign(x - y.detach()), 'f': None}
    with l1_impose(sig) as log:
        v = O.loss_t(x, y)
    gv, = torch.autograd.grad(v, y)
    assert torch.allclose(v, ref) and torch.equal(gv, gref) and check_l1_flips(log, 'same') == 0
    sig['t'] = sig['t'].clone()
    sig['t'][0, 0, 7] *= -1
    with l1_impose(sig) as log:
        v = O.loss_t(x, y)
    gv, = torch.autograd.grad(v, y)
    assert check_l1_flips(log, 'tie') == 1 and float(gv[0, 0, 7]) == -float(gref[0, 0, 7])
    sig['t'][0, 0, 100] *= -1
    with l1_impose(sig) as log:
        O.loss_t(x, y)
    with pytest.raises(AssertionError):
        check_l1_flips(log, 'far')
    assert O.L1_SIGNS is None and O.L1_AUDIT is None
