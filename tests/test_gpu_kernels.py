"""GPU parity of the HIP kernels (through the libencx C ABI) against the golden fixtures and the
CPU oracle. Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import encodec_oracle as O
from fixtures import load, T, model_state, codebooks_from_stats, g3_codebooks, certified
from synth import synth_state, synth_wave

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def G(a):
    return T(a).to(DEV)


def close(a, b, rtol=1e-5, atol=1e-6, what=''):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b)
    bad = err > tol
    assert not bad.any(), f'{what}: {bad.sum()}/{bad.size} off, max abs err {err.max():.3e}, ' \
                          f'max rel {(err / (np.abs(b) + 1e-30)).max():.3e}'


# --------------------------------------------------------------------------- conv fixtures
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


def _case_params(ci, kind, cin, cout, K):
    pre = 'convtr.convtr' if kind == 'convtr' else 'conv.conv'
    wshape = (cin, cout, K) if kind == 'convtr' else (cout, cin, K)
    shapes = {pre + '.bias': (cout,), pre + '.weight_g': (wshape[0], 1, 1), pre + '.weight_v': wshape}
    st = synth_state(shapes, 100 + ci)
    return (G(st[pre + '.weight_v']).requires_grad_(True), G(st[pre + '.weight_g']).requires_grad_(True),
            G(st[pre + '.bias']).requires_grad_(True))


@pytest.mark.parametrize('ci', range(len(CASES)))
def test_conv_fixture(ci):
    from encx import ops
    d = load('g2_convs.npz')
    name, kind, cin, cout, K, s, causal, pre_elu, Tn = CASES[ci]
    v, g, b = _case_params(ci, kind, cin, cout, K)
    x = G(d[name + '/x']).requires_grad_(True)
    act = 'elu' if pre_elu else None
    if kind == 'conv':
        y = ops.conv1d(x, v, g, b, K, s, 1, causal, 'reflect', act)
    else:
        y = ops.convtr1d(x, v, g, b, K, s, causal, 1.0, act)
    close(y, d[name + '/y'], 1e-5, 1e-5, name + ' y')
    y.backward(G(d[name + '/gy']))
    close(x.grad, d[name + '/dx'], 1e-4, 1e-5, name + ' dx')
    close(v.grad, d[name + '/dv'], 1e-4, 1e-5, name + ' dv')
    close(g.grad, d[name + '/dg'], 1e-4, 1e-5, name + ' dg')
    close(b.grad, d[name + '/db'], 1e-4, 1e-4, name + ' db')


# the real SEANet layer shapes (B=2, shorter T) against the oracle, fwd + all grads
MODEL_LAYERS = [
    # kind, cin, cout, K, s, pre_elu, T_in
    ('conv', 1, 32, 7, 1, False, 4800), ('conv', 32, 16, 3, 1, True, 4800),
    ('conv', 16, 32, 1, 1, True, 4800), ('conv', 32, 32, 1, 1, False, 4800),
    ('conv', 32, 64, 4, 2, True, 4800), ('conv', 64, 128, 8, 4, True, 2400),
    ('conv', 128, 256, 10, 5, True, 600), ('conv', 256, 512, 16, 8, True, 120),
    ('conv', 512, 128, 7, 1, True, 15), ('conv', 128, 512, 7, 1, False, 15),
    ('conv', 256, 128, 3, 1, True, 120), ('conv', 128, 256, 1, 1, True, 120),
    ('conv', 32, 1, 7, 1, True, 4800),
    ('convtr', 512, 256, 16, 8, True, 15), ('convtr', 256, 128, 10, 5, True, 120),
    ('convtr', 128, 64, 8, 4, True, 600), ('convtr', 64, 32, 4, 2, True, 2400),
    # the 1x1 layers on the pointwise GEMM kernels (fwd / bwd-data for T <= 1024, weight grad
    # for T <= 3000 at >= 64 channels) at their real widths and lengths
    ('conv', 256, 256, 1, 1, True, 600), ('conv', 128, 256, 1, 1, False, 600),
    ('conv', 64, 128, 1, 1, True, 3000), ('conv', 128, 128, 1, 1, True, 1000),
    ('conv', 128, 128, 1, 1, True, 3000),  # the 1x1 GEMM past PW_TMAX (>= 128-channel reduction)
]


@pytest.mark.parametrize('li', range(len(MODEL_LAYERS)))
def test_conv_model_shapes_vs_oracle(li):
    from encx import ops
    kind, cin, cout, K, s, pre_elu, Tin = MODEL_LAYERS[li]
    v0, g0, b0 = _case_params(500 + li, kind, cin, cout, K)
    x0 = synth_wave((2, cin, Tin), 900 + li, amp=1.0)
    act = 'elu' if pre_elu else None
    x = G(x0).requires_grad_(True)
    if kind == 'conv':
        y = ops.conv1d(x, v0, g0, b0, K, s, 1, True, 'reflect', act)
    else:
        y = ops.convtr1d(x, v0, g0, b0, K, s, True, 1.0, act)
    gy = synth_wave(tuple(y.shape), 950 + li, amp=1.0)
    y.backward(G(gy))
    # oracle on CPU in fp64; tolerances are relative per element plus a floor relative to the
    # tensor's max (fp32 accumulation order differs: elements that cancel to ~0 keep an
    # absolute error of the order of eps32 * the summands)
    pre = 'convtr.convtr' if kind == 'convtr' else 'conv.conv'
    p = {'m.' + pre + '.weight_v': v0.detach().cpu().double().requires_grad_(True),
         'm.' + pre + '.weight_g': g0.detach().cpu().double().requires_grad_(True),
         'm.' + pre + '.bias': b0.detach().cpu().double().requires_grad_(True)}
    xc = T(x0).double().requires_grad_(True)
    xin = F.elu(xc) if pre_elu else xc
    yc = O.sconv1d(xin, p, 'm', K, s) if kind == 'conv' else O.sconvtr1d(xin, p, 'm', K, s)
    yc.backward(T(gy).double())
    tag = f'{kind} {cin}->{cout} K{K} s{s}'

    def near(a, b, rtol, nrel, what):
        b = b.detach()
        close(a, b, rtol, nrel * float(b.abs().max()), what)
    near(y, yc, 1e-4, 1e-6, tag + ' y')
    near(x.grad, xc.grad, 1e-4, 1e-5, tag + ' dx')
    near(v0.grad, p['m.' + pre + '.weight_v'].grad, 1e-4, 1e-5, tag + ' dv')
    near(g0.grad, p['m.' + pre + '.weight_g'].grad, 1e-4, 1e-5, tag + ' dg')
    near(b0.grad, p['m.' + pre + '.bias'].grad, 1e-4, 1e-5, tag + ' db')


DILATED_LAYERS = [
    # cin, cout, K, s, d, causal, pad_mode, pre_elu, T_in: SEANetResnetBlock's k3 conv at
    # dilation_base ** j (modules/seanet.py:114-117, n_residual_layers > 1), both paddings, a
    # short input (the reflect pad's zero extension), a strided dilated conv, residual widths
    (16, 8, 3, 1, 2, True, 'reflect', True, 300), (32, 16, 3, 1, 4, False, 'reflect', True, 257),
    (8, 8, 3, 1, 8, True, 'zero', False, 100), (8, 4, 3, 1, 3, True, 'reflect', True, 5),
    (8, 16, 4, 2, 2, True, 'reflect', True, 97), (64, 32, 3, 1, 2, True, 'reflect', True, 1200),
]


@pytest.mark.parametrize('li', range(len(DILATED_LAYERS)))
def test_dilated_conv1d_vs_oracle(li):
    """nn.Conv1d(dilation=d) inside SConv1d (modules/conv.py:195-210): forward (the implicit GEMM
    takes d), backward-data (encx_conv1d_bwd_data_dilated) and the weight / bias grads against
    the fp64 oracle."""
    from encx import ops
    cin, cout, K, s, d, causal, pad, pre_elu, Tin = DILATED_LAYERS[li]
    v0, g0, b0 = _case_params(700 + li, 'conv', cin, cout, K)
    x0 = synth_wave((3, cin, Tin), 720 + li, amp=1.0)
    act = 'elu' if pre_elu else None
    x = G(x0).requires_grad_(True)
    y = ops.conv1d(x, v0, g0, b0, K, s, d, causal, pad, act)
    gy = synth_wave(tuple(y.shape), 740 + li, amp=1.0)
    y.backward(G(gy))
    p = {'m.conv.conv.weight_v': v0.detach().cpu().double().requires_grad_(True),
         'm.conv.conv.weight_g': g0.detach().cpu().double().requires_grad_(True),
         'm.conv.conv.bias': b0.detach().cpu().double().requires_grad_(True)}
    xc = T(x0).double().requires_grad_(True)
    yc = O.sconv1d(F.elu(xc) if pre_elu else xc, p, 'm', K, s, d, causal, pad)
    yc.backward(T(gy).double())
    tag = f'{cin}->{cout} K{K} s{s} d{d} {pad}'
    for a, b, what in [(y, yc, 'y'), (x.grad, xc.grad, 'dx'), (v0.grad, p['m.conv.conv.weight_v'].grad, 'dv'),
                       (g0.grad, p['m.conv.conv.weight_g'].grad, 'dg'), (b0.grad, p['m.conv.conv.bias'].grad, 'db')]:
        b = b.detach()
        close(a, b, 1e-4, 1e-5 * float(b.abs().max()), f'{tag} {what}')


# --------------------------------------------------------------------------- RVQ
class _CB:
    def __init__(self, d):
        for k, v in d.items():
            setattr(self, k, v)
        self.training = True
        self.decay, self.epsilon = 0.99, 1e-5

    def init_embed_(self, x):
        pass


def test_rvq_commitment_weight_scales_penalty_and_its_grad():
    """VectorQuantization(commitment_weight=w) (core_vq.py:267: loss += commit_loss * w): the
    penalty and its gradient into the input scale by w; codes, quantized and the codebook updates
    do not change."""
    from encx import ops
    d = load('g3_rvq.npz')
    outs = {}
    for w in (1.0, 0.25):
        cbs = [_CB({k: v.to(DEV).contiguous() for k, v in cb.items()}) for cb in g3_codebooks(d)]
        emb = G(d['emb']).requires_grad_(True)
        q, codes, pen = ops.RVQTrainFn.apply(emb, cbs, 0.99, 1e-5, False, w)
        torch.autograd.backward([pen], [torch.ones((), device=DEV)])  # dq = 0: the commit grad alone
        outs[w] = (q.detach(), codes, pen.detach(), emb.grad, cbs[0].embed)
    (q1, c1, p1, g1, e1), (qw, cw_, pw, gw, ew) = outs[1.0], outs[0.25]
    assert torch.equal(c1, cw_) and torch.equal(q1, qw) and torch.equal(e1, ew)
    close(pw, 0.25 * p1, 1e-6, 0, 'penalty * w')
    close(gw, 0.25 * g1, 1e-6, 1e-12, 'd penalty / d emb * w')


def test_rvq_train_fixture():
    from encx import ops
    d = load('g3_rvq.npz')
    cbs = [_CB({k: v.to(DEV).contiguous() for k, v in cb.items()}) for cb in g3_codebooks(d)]
    emb = G(d['emb']).requires_grad_(True)
    q, codes, pen = ops.RVQTrainFn.apply(emb, cbs, 0.99, 1e-5)
    assert (codes.cpu().numpy() == d['codes']).all()
    close(q, d['quantized'], 1e-6, 1e-6, 'quantized')
    close(pen, d['penalty'], 1e-5, 1e-7, 'penalty')
    torch.autograd.backward([q, pen], [G(d['gq']), torch.ones((), device=DEV)])
    close(emb.grad, d['demb'], 1e-5, 1e-6, 'demb')
    for i in range(2):
        close(cbs[i].cluster_size, d[f'cluster_size{i}'], 1e-6, 1e-7, f'cluster_size{i}')
        close(cbs[i].embed_avg, d[f'embed_avg{i}'], 1e-5, 1e-6, f'embed_avg{i}')
        close(cbs[i].embed, d[f'embed{i}'], 1e-5, 1e-6, f'embed{i}')


def test_rvq_argmin_full_size_certified():
    from encx import ops
    r = np.random.Generator(np.random.PCG64(7))
    emb = r.standard_normal((32, 128, 75)).astype(np.float32)
    E = r.standard_normal((1024, 128)).astype(np.float32)
    idx = ops.rvq_argmin(G(emb), G(E)).cpu().numpy()
    x = emb.transpose(0, 2, 1).reshape(-1, 128).astype(np.float64)
    dist = (x ** 2).sum(1)[:, None] - 2 * x @ E.T.astype(np.float64) + (E.astype(np.float64) ** 2).sum(1)[None]
    srt = np.sort(dist, 1)
    gap = srt[:, 1] - srt[:, 0]
    cert = certified(gap, float((x ** 2).sum(1).max()), float((E.astype(np.float64) ** 2).sum(1).max()))
    ref = O.codebook_quantize(T(emb.transpose(0, 2, 1).reshape(-1, 128)), T(E)).numpy()
    assert cert.mean() > 0.99
    assert (idx[cert] == ref[cert]).all()
    assert (idx[cert] == dist.argmin(1)[cert]).all()


def test_rvq_argmin_ties_first_index():
    from encx import ops
    E = np.zeros((1024, 128), np.float32)
    E[5] = 1.0
    E[700] = 1.0  # exact duplicate of code 5 -> tie, first index wins
    x = np.ones((1, 128, 3), np.float32)
    idx = ops.rvq_argmin(G(x), G(E)).cpu().numpy()
    assert (idx == 5).all()


def test_kmeans_fixture():
    from encx._lib import call, ptr, stream
    d = load('g3_rvq.npz')
    samples = G(d['km_samples'])
    means = samples[T(d['km_init']).to(DEV)].contiguous()
    bins = torch.zeros(64, dtype=torch.int64, device=DEV)
    idx = torch.empty(600, dtype=torch.int64, device=DEV)
    keys = torch.empty(600, dtype=torch.int64, device=DEV)
    from encx._lib import lib
    ws = torch.empty(lib.encx_rvq_bucket_workspace(600, 128, 64) // 4 + 1, device=DEV)
    for _ in range(10):
        call('encx_kmeans_step', ptr(samples), ptr(means), ptr(bins), ptr(idx), ptr(keys), ptr(ws),
             600, 128, 64, stream())
    close(means, d['km_means'], 1e-5, 1e-6, 'kmeans means')
    assert (bins.cpu().numpy() == d['km_bins']).all()


def test_sample_rows_is_a_permutation_prefix():
    from encx import ops
    from encx._lib import call, ptr, stream
    s = torch.arange(600 * 4, dtype=torch.float32, device=DEV).view(600, 4)
    out = torch.empty(256, 4, device=DEV)
    call('encx_sample_rows', ptr(s), ptr(out), 600, 4, 256, 12345, stream())
    rows = (out[:, 0] / 4).long().cpu().numpy()
    assert len(set(rows.tolist())) == 256 and rows.min() >= 0 and rows.max() < 600
    means, bins = ops.kmeans(G(synth_wave((300, 8), 3, amp=1.0)), 16, 5, 99)
    assert int(bins.sum()) == 300


# --------------------------------------------------------------------------- mel / losses
def test_mel_fixture():
    from encx import ops
    d = load('g4_mel.npz')
    x = G(d['x'])
    for i in range(5, 12):
        n = 2 ** i
        close(ops.logmel(x, n, 64, 24000), d[f'mel{n}'], 1e-4, 2e-4, f'logmel {n}')


@pytest.fixture(params=[True, False], ids=['fused', 'per_scale'])
def mel_path(request):
    """l_f through the fused multi-scale launches (encx_mel_loss_multi) and through the
    per-scale ones (encx_mel_loss)."""
    from encx import ops
    prev = ops.MEL_FUSED
    ops.MEL_FUSED = request.param
    yield request.param
    ops.MEL_FUSED = prev


def test_losses_fixture(mel_path):
    from encx import losses
    d = load('g4_mel.npz')
    x = G(d['x'])
    y = G(d['y']).requires_grad_(True)
    lt, lf = losses.reconstruction_losses(x, y)
    close(lt.view(1), d['l_t'].reshape(1), 1e-5, 1e-7, 'l_t')
    close(lf.view(1), d['l_f'].reshape(1), 1e-5, 1e-6, 'l_f')
    gf, = torch.autograd.grad(lf, [y])
    gt, = torch.autograd.grad(lt, [y])
    close(gt, d['dlt_dy'], 1e-6, 1e-9, 'dl_t/dy')
    close(gf, d['dlf_dy'], 2e-3, 2e-7, 'dl_f/dy')


def test_mel_loss_full_size_vs_oracle(mel_path):
    from encx import losses
    x0 = synth_wave((4, 1, 24000), 11)
    y0 = synth_wave((4, 1, 24000), 12)
    y = G(y0).requires_grad_(True)
    lt, lf = losses.reconstruction_losses(G(x0), y)
    gf, = torch.autograd.grad(lf, [y])
    yc = T(y0).requires_grad_(True)
    lfc = O.loss_f(T(x0), yc)
    gfc, = torch.autograd.grad(lfc, [yc])
    close(lf.view(1), lfc.detach().view(1), 1e-5, 1e-6, 'l_f full')
    close(gf, gfc, 5e-3, 1e-4 * float(gfc.abs().max()), 'dl_f/dy full')


@pytest.mark.parametrize('n,hop,win,sr,lo,hi', [
    (1024, 256, 1024, 22050, 0.0, 8000.0), (512, 128, 512, 24000, 50.0, 9000.0),  # the loss framing
    (1024, 256, 800, 22050, 0.0, None), (512, 160, 400, 16000, 0.0, 8000.0), (2048, 300, 2048, 24000, 30.0, None)])
def test_audio2mel_band_vs_oracle_fp64(n, hop, win, sr, lo, hi):
    """Audio2Mel(n_fft, hop_length, win_length, mel_fmin, mel_fmax) (audio_to_mel.py:7-55; the
    filters librosa.filters.mel builds for that band, :24) against the oracle's restatement in fp64
    (its filter bank pinned to transformers' slaney bank, test_oracle.py): the loss framing on the
    fused mel kernels, any other through encx_mel_logmel_framed."""
    from encx.audio_to_mel import Audio2Mel
    m = Audio2Mel(n_fft=n, hop_length=hop, win_length=win, sampling_rate=sr, n_mel_channels=80,
                  mel_fmin=lo, mel_fmax=hi).to(DEV)
    x0 = synth_wave((3, 1, 6000), n + int(lo) + win, amp=0.3)
    ref = O.audio2mel(T(x0).double(), n, hop, win, sr, 80, lo, hi)
    out = m(G(x0))
    assert out.shape == ref.shape
    close(out, ref, 1e-4, 2e-4, f'logmel n {n} hop {hop} win {win} band [{lo}, {hi}]')


def test_balancer_fixture():
    from encx.balancer import Balancer
    d = load('g6_balancer.npz')
    b = Balancer({'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3})
    for it in range(3):
        grads = {k: G(d[f'it{it}_{k}']) for k in ('l_t', 'l_f', 'l_g', 'l_feat')}
        close(b.combine(grads), d[f'it{it}_out'], 1e-4, 1e-8, f'balancer it{it}')
    b = Balancer({'1': 1, '2': 1}, rescale_grads=False)
    out = b.combine({'1': torch.full((1, 1), -1.0, device=DEV), '2': torch.full((1, 1), 100.0, device=DEV)})
    assert float(out) == 99.0
    b = Balancer({'1': 1, '2': 1})
    out = b.combine({'1': torch.full((1, 1), -1.0, device=DEV), '2': torch.full((1, 1), 100.0, device=DEV)})
    assert abs(float(out)) < 1e-6


@pytest.mark.parametrize('nl', [5, 7, 8])
def test_balancer_many_losses_vs_oracle(nl):
    """balancer.py:83-118 takes any number of losses; encx chains its 4-grad combine calls."""
    from encx.balancer import Balancer
    r = np.random.Generator(np.random.PCG64(nl))
    w = {f'l{k}': float(k % 3 + 1) * 0.5 for k in range(nl)}
    b, bo = Balancer(w), O.Balancer(w)
    for it in range(3):
        gs = {k: r.standard_normal((4, 1, 300)).astype(np.float32) * (k_i + 1)
              for k_i, k in enumerate(w)}
        out = b.combine({k: G(v) for k, v in gs.items()})
        ref = bo.combine({k: T(v) for k, v in gs.items()})
        close(out, ref, 1e-5, 1e-7, f'balancer nl={nl} it{it}')
    # rescale_grads=False: out = sum_k w_k g_k, left to right as `out_grad += grad`
    b = Balancer(w, rescale_grads=False)
    gs = {k: r.standard_normal((2, 1, 50)).astype(np.float32) for k in w}
    ref = 0
    for k, v in gs.items():
        ref = ref + T(v) * w[k]
    out = b.combine({k: G(v) for k, v in gs.items()})
    assert torch.equal(out.cpu(), ref), 'plain weighted sum not bit-exact'


def test_adam_vs_oracle():
    from encx.optim import FlatAdam
    r = np.random.Generator(np.random.PCG64(5))
    p0 = {'a': r.standard_normal((33, 7)).astype(np.float32), 'b': r.standard_normal((100,)).astype(np.float32)}
    ps = [torch.nn.Parameter(G(p0['a'])), torch.nn.Parameter(G(p0['b']))]
    opt = FlatAdam(ps, lr=3e-4, betas=(0.5, 0.9))
    pc = {k: T(v).clone() for k, v in p0.items()}
    st = {}
    for it in range(3):
        gs = {k: r.standard_normal(v.shape).astype(np.float32) for k, v in p0.items()}
        opt.zero_grad()
        ps[0].grad.copy_(G(gs['a']))
        ps[1].grad.copy_(G(gs['b']))
        opt.step()
        O.adam_step(pc, {k: T(v) for k, v in gs.items()}, st, 3e-4)
    close(ps[0], pc['a'], 1e-6, 1e-7, 'adam a')
    close(ps[1], pc['b'], 1e-6, 1e-7, 'adam b')


def test_normalize_and_scale():
    from encx import ops
    x0 = synth_wave((3, 1, 1000), 21, amp=0.3)
    xn, sc = ops.normalize(G(x0))
    xr, scr = O.normalize(T(x0))
    close(xn, xr, 1e-6, 1e-7, 'xn')
    close(sc, scr, 1e-6, 1e-9, 'scale')


# --------------------------------------------------------------------------- LSTM
@pytest.mark.parametrize('B,H,Tn,L,fuse,persist,wgs', [
    (3, 32, 7, 1, 0, 1, 32), (17, 64, 20, 2, 0, 1, 32), (5, 48, 9, 3, 0, 1, 32), (32, 512, 75, 2, 0, 1, 32),
    (32, 512, 75, 2, 0, 0, 32), (17, 64, 20, 2, 1, 0, 32), (32, 512, 75, 2, 1, 0, 32), (17, 128, 20, 2, 0, 1, 32),
    (5, 256, 9, 3, 0, 1, 32), (40, 384, 11, 1, 0, 1, 32), (17, 256, 20, 2, 0, 1, 1),
    # batches above one launch's 64 rows: run as chunks (ops.lstm)
    (80, 64, 12, 2, 0, 1, 32), (130, 128, 9, 1, 0, 1, 32), (96, 512, 6, 2, 0, 0, 32)])
def test_lstm_vs_oracle(B, H, Tn, L, fuse, persist, wgs):
    """encx LSTM (csrc/lstm.hip) forward + backward against the oracle's step-by-step
    restatement of SLSTM (modules/lstm.py:22-28) run in fp64 on the CPU, for 1, 2 and 3 layers:
    every output and grad within 4x the error of the same restatement run in plain fp32.
    persist: the one-launch recurrences (option LSTM_PERSIST; used where H % 128 == 0, H <= 512
    and the workgroups fit the CUs, else the launch-per-step wavefront); fuse: the opt-in fused
    backward step of the wavefront (option LSTM_FUSE); wgs: the weight grad's k-split cap
    (LSTM_WG_SPLITS; 1 = one GEMM storing straight into the grads)."""
    import ctypes
    from encx import ops
    from encx._lib import option, call
    gen = torch.Generator().manual_seed(B * 1000 + H)
    k = 1.0 / np.sqrt(H)
    names = ['weight_ih', 'weight_hh', 'bias_ih', 'bias_hh']
    shapes = [(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]
    p64, wts = {}, []
    for l in range(L):
        for n, s in zip(names, shapes):
            w = (torch.rand(s, generator=gen, dtype=torch.float64) * 2 - 1) * k
            p64[f'm.lstm.{n}_l{l}'] = w.requires_grad_(True)
            wts.append(w.detach().float().to(DEV).requires_grad_(True))
    x64 = torch.randn(B, H, Tn, generator=gen, dtype=torch.float64).requires_grad_(True)
    r64 = torch.randn(B, H, Tn, generator=gen, dtype=torch.float64)
    y64 = O.slstm(x64, p64, 'm', L)
    (y64 * r64).sum().backward()
    x = x64.detach().float().to(DEV).requires_grad_(True)
    with option(LSTM_FUSE=fuse, LSTM_PERSIST=persist, LSTM_WG_SPLITS=wgs):
        y = ops.lstm(x, wts, skip=True)
        (y * r64.float().to(DEV)).sum().backward()
        torch.cuda.synchronize()
    nerr = ctypes.c_int64()
    call('encx_lstm_sync_errors', ctypes.byref(nerr))
    assert nerr.value == 0, f'{nerr.value} hand-off spins timed out'

    def rel_close(a, b, what, tol=2e-4):
        b = b.detach()
        scale = b.abs().max().item() + 1e-12
        close(a, b, rtol=tol, atol=tol * scale, what=what)

    # the same SLSTM in plain fp32 on the host (the oracle's loop): what fp32 arithmetic achieves
    p32 = {k: v.detach().float().requires_grad_(True) for k, v in p64.items()}
    x32 = x64.detach().float().requires_grad_(True)
    y32 = O.slstm(x32, p32, 'm', L)
    (y32 * r64.float()).sum().backward()

    def err(a, b):
        b = b.detach().double().cpu()
        return float((a.detach().double().cpu() - b).abs().max() / (b.abs().max() + 1e-12))
    rows = [('y', err(y, y64), err(y32, y64)), ('dx', err(x.grad, x64.grad), err(x32.grad, x64.grad))]
    rows += [(n.split('.')[-1], err(wts[i].grad, w.grad), err(p32[n].grad, w.grad)) for i, (n, w) in enumerate(p64.items())]
    print('LSTM rel err vs fp64 (encx / plain fp32): ' + ', '.join(f'{n} {a:.1e}/{b:.1e}' for n, a, b in rows))
    # as accurate as plain fp32: within 4x of its error (floor 1e-6 of the tensor's magnitude;
    # measured 0.5-2.6x at (32, 512, 75, 2))
    bad = [(n, a, b) for n, a, b in rows if not a <= max(4 * b, 1e-6)]
    assert not bad, bad
    rel_close(y, y64, 'y')
    rel_close(x.grad, x64.grad, 'dx')
    for i, (n, w) in enumerate(p64.items()):
        rel_close(wts[i].grad, w.grad, n, tol=5e-4)


@pytest.mark.parametrize('B,H,Tn,L', [(17, 256, 20, 2), (32, 512, 75, 2), (3, 128, 5, 3)])
def test_lstm_persistent_bit_identical(B, H, Tn, L):
    """The one-launch forward and backward (option LSTM_PERSIST) produce the same bits as the launch-per-step wavefront: h, c,
    the gates, the gate grads DA and dx (same k-group order, same LDS sum order, same cell
    arithmetic), with no hand-off spin timing out. The persistent buffers are reused over three
    rounds of fresh inputs, so a stale line of the previous round read anywhere would show."""
    import ctypes
    from encx._lib import call, ptr, option, lib
    gen = torch.Generator().manual_seed(7 * B + H)
    k = H ** -0.5
    f = lambda *s: ((torch.rand(*s, generator=gen) * 2 - 1) * k).to(DEV)
    e = lambda n: torch.empty(n, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    wcat, wcatT, bsum = e(L * 8 * H * H), e(L * 8 * H * H), e(L * 4 * H)
    for l in range(L):
        call('encx_lstm_pack', *(ptr(f(*s)) for s in [(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]),
             ptr(wcat), ptr(wcatT), ptr(bsum), H, l, st)
    x = torch.empty(B, H, Tn, device=DEV)
    dout = torch.empty(B, H, Tn, device=DEV)
    bufs = {}
    for rnd in range(3):
        x.copy_(torch.randn(B, H, Tn, generator=gen))
        dout.copy_(torch.randn(B, H, Tn, generator=gen))
        res = []
        for persist in (0, 1):
            if persist not in bufs:
                bufs[persist] = (e(B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * 4 * H),
                                 torch.empty_like(x), e(L * B * Tn * 4 * H), torch.empty_like(x),
                                 torch.empty(lib.encx_lstm_bwd_workspace(B, Tn, H, L), dtype=torch.uint8, device=DEV))
            xt, Y, Cs, Gs, out, DA, dx, ws = bufs[persist]
            with option(LSTM_PERSIST=persist):
                call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out), 1,
                     B, Tn, H, L, st)
                call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), 0, ptr(ws),
                     B, Tn, H, L, st)
            torch.cuda.synchronize()
            res.append([t.clone() for t in (out, Y, Cs, Gs, DA, dx)])
        nerr = ctypes.c_int64()
        call('encx_lstm_sync_errors', ctypes.byref(nerr))
        assert nerr.value == 0
        for name, a, b in zip(['out', 'h', 'c', 'gates', 'DA', 'dx'], *res):
            assert torch.equal(a, b), (rnd, name, float((a - b).abs().max()))


@pytest.mark.parametrize('form', ['persist', 'fused_step'])
def test_lstm_persistent_graph_replays(form):
    """The recurrences captured in a HIP graph and replayed (the training step's form): every
    replay, on fresh inputs, gives the bits of an eager call, and no hand-off spin times out (the
    counters must be zero at every launch, captured or not). 'persist': the persistent kernels;
    'fused_step': the opt-in step form whose backward fuses E(k+1) into G(k) by last-arriver
    counters (zeroed by a kernel: a captured hipMemsetAsync was not ordered before the next kernel
    in replays)."""
    import ctypes
    from encx._lib import call, ptr, option, lib
    B, H, Tn, L = 4, 512, 75, 2
    gen = torch.Generator().manual_seed(11)
    k = H ** -0.5
    f = lambda *s: ((torch.rand(*s, generator=gen) * 2 - 1) * k).to(DEV)
    e = lambda n: torch.empty(n, device=DEV)
    wcat, wcatT, bsum = e(L * 8 * H * H), e(L * 8 * H * H), e(L * 4 * H)
    st0 = torch.cuda.current_stream().cuda_stream
    for l in range(L):
        call('encx_lstm_pack', *(ptr(f(*s)) for s in [(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]),
             ptr(wcat), ptr(wcatT), ptr(bsum), H, l, st0)
    x, dout = torch.zeros(B, H, Tn, device=DEV), torch.zeros(B, H, Tn, device=DEV)
    bufs = (e(B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * 4 * H), torch.empty_like(x),
            e(L * B * Tn * 4 * H), torch.empty_like(x),
            torch.empty(lib.encx_lstm_bwd_workspace(B, Tn, H, L), dtype=torch.uint8, device=DEV))

    def run():
        xt, Y, Cs, Gs, out, DA, dx, ws = bufs
        st = torch.cuda.current_stream().cuda_stream
        call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out), 1, B, Tn, H, L, st)
        call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), 0, ptr(ws), B, Tn, H, L, st)

    opts = dict(LSTM_PERSIST=1) if form == 'persist' else dict(LSTM_PERSIST=0, LSTM_FUSE=1)
    with option(**opts):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                run()
        torch.cuda.current_stream().wait_stream(s)
        for rnd in range(4):
            x.copy_(torch.randn(B, H, Tn, generator=gen))
            dout.copy_(torch.randn(B, H, Tn, generator=gen))
            g.replay()
            torch.cuda.synchronize()
            got = [t.clone() for t in bufs[:7]]
            run()
            torch.cuda.synchronize()
            nerr = ctypes.c_int64()
            call('encx_lstm_sync_errors', ctypes.byref(nerr))
            assert nerr.value == 0, (rnd, nerr.value)
            for name, a, b in zip(['xt', 'h', 'c', 'gates', 'out', 'DA', 'dx'], got, bufs[:7]):
                assert torch.equal(a, b), (rnd, name)


def test_lstm_handoff_failure_is_loud():
    """A persistent-LSTM hand-off that fails (option LSTM_FAULT: one workgroup of each launch
    never publishes; LSTM_SPIN 6: every poll gives up after 64 tries) is reported: directly
    through encx_lstm_sync_errors, through the capturable encx_lstm_sync_read, and by the
    Trainer -- check_sync() raises, and so does the next step() once the failed step's
    error-word copy has landed. Without the fault the same calls report 0."""
    import ctypes
    from encx._lib import call, ptr, option, lib, lstm_sync_errors
    from encx.model import EncodecModel
    from encx.train import Trainer
    B, H, Tn, L = 4, 512, 75, 2
    gen = torch.Generator().manual_seed(12)
    k = H ** -0.5
    f = lambda *s: ((torch.rand(*s, generator=gen) * 2 - 1) * k).to(DEV)
    e = lambda n: torch.empty(n, device=DEV)
    wcat, wcatT, bsum = e(L * 8 * H * H), e(L * 8 * H * H), e(L * 4 * H)
    st = torch.cuda.current_stream().cuda_stream
    for l in range(L):
        call('encx_lstm_pack', *(ptr(f(*s)) for s in [(4 * H, H), (4 * H, H), (4 * H,), (4 * H,)]),
             ptr(wcat), ptr(wcatT), ptr(bsum), H, l, st)
    x, dout = torch.randn(B, H, Tn, device=DEV), torch.randn(B, H, Tn, device=DEV)
    xt, Y, Cs, Gs, out, DA, dx = (e(B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * H), e(L * B * Tn * 4 * H),
                                  torch.empty_like(x), e(L * B * Tn * 4 * H), torch.empty_like(x))
    ws = torch.empty(lib.encx_lstm_bwd_workspace(B, Tn, H, L), dtype=torch.uint8, device=DEV)
    assert lstm_sync_errors() == 0
    for direction in ('fwd', 'bwd'):
        for fault in (0, 1):
            # (the healthy runs with the default spin bound: 64 polls can time out on a hand-off
            # that is merely slow, e.g. while workgroups of the previous launch still drain)
            spin = 6 if fault else 0
            with option(LSTM_PERSIST=1, LSTM_SPIN=spin, LSTM_FAULT=fault if direction == 'fwd' else 0):
                call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out), 1,
                     B, Tn, H, L, st)
            with option(LSTM_PERSIST=1, LSTM_SPIN=spin, LSTM_FAULT=fault if direction == 'bwd' else 0):
                call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), 0, ptr(ws),
                     B, Tn, H, L, st)
            cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
            call('encx_lstm_sync_read', ptr(cnt), st)
            torch.cuda.synchronize()
            assert (int(cnt) > 0) == bool(fault), (direction, fault, int(cnt))
            assert lstm_sync_errors() == 0  # the read cleared the word
    # the same failure inside a training step: the Trainer raises
    model = EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True).to(DEV)
    tr = Trainer(model, None, lr=3e-4, scheduler=False)
    xb = torch.randn(B, 1, 24000, device=DEV) * 0.1
    tr.step(xb)
    tr.check_sync()  # healthy
    with option(LSTM_SPIN=6, LSTM_FAULT=1):
        tr.step(xb)
    with pytest.raises(RuntimeError, match='hand-off'):
        tr.check_sync()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match='hand-off'):
        tr.step(xb)  # the failed step's copy has landed: the next step refuses to go on
    assert lstm_sync_errors() == 0


# --------------------------------------------------------------------------- fused residual block
@pytest.mark.parametrize('C,T,B', [(32, 2048, 3), (32, 24000, 2), (64, 12000, 2), (64, 3001, 3), (32, 2113, 1)])
def test_fused_resblock_vs_torch_fp64(C, T, B):
    """ops.ResBlockFn (csrc/resblock.hip: SEANetResnetBlock, modules/seanet.py:46-63, as one
    kernel per direction) against torch's fp64 restatement of the block: ELU -> reflect-padded
    causal k3 conv (C -> C/2) -> ELU -> 1x1 conv (C/2 -> C), plus the 1x1 shortcut, all weight
    normed. Output, input grad and every weight / bias grad under a seeded output grad, relative to
    each tensor's largest magnitude; incl. T not a multiple of the 64-position tile."""
    from encx import ops
    g = torch.Generator().manual_seed(C * 7 + T)
    HD = C // 2

    def par(co, ci, k):
        v = (torch.randn(co, ci, k, generator=g, dtype=torch.float64) / (ci * k) ** 0.5)
        gg = v.reshape(co, -1).norm(dim=1).reshape(co, 1, 1) * (1 + 0.1 * torch.randn(co, 1, 1, generator=g, dtype=torch.float64))
        b = 0.1 * torch.randn(co, generator=g, dtype=torch.float64)
        return [v, gg, b]
    ps64 = [par(HD, C, 3), par(C, HD, 1), par(C, C, 1)]
    x64 = 0.5 * torch.randn(B, C, T, generator=g, dtype=torch.float64)
    dy64 = torch.randn(B, C, T, generator=g, dtype=torch.float64)
    leaves64 = [x64.requires_grad_(True)] + [t.requires_grad_(True) for p in ps64 for t in p]

    def wn(v, gg):
        return v * (gg / v.reshape(v.shape[0], -1).norm(dim=1).reshape(-1, 1, 1))
    (v1, g1, b1), (v2, g2, b2), (vs, gs, bs) = ps64
    e = F.pad(F.elu(x64), (2, 0), mode='reflect')
    h = F.conv1d(e, wn(v1, g1), b1)
    y64 = F.conv1d(F.elu(h), wn(v2, g2), b2) + F.conv1d(x64, wn(vs, gs), bs)
    ref = torch.autograd.grad(y64, leaves64, dy64)
    leaves = [t.detach().float().to(DEV).requires_grad_(True) for t in leaves64]
    x = leaves[0]
    p = [leaves[1:4], leaves[4:7], leaves[7:10]]
    y = ops.resblock(x, *p)
    mine = torch.autograd.grad(y, leaves, dy64.float().to(DEV))

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double()
        return float((a - b).abs().max() / (b.abs().max() + 1e-30))
    names = ['x', 'v1', 'g1', 'b1', 'v2', 'g2', 'b2', 'vs', 'gs', 'bs']
    errs = {'y': rel(y, y64)} | {f'd{n}': rel(m, r) for n, m, r in zip(names, mine, ref)}
    print(f'C {C} T {T} B {B}: ' + ' '.join(f'{k} {v:.1e}' for k, v in errs.items()))
    assert errs['y'] < 1e-5, errs
    assert all(v < 1e-4 for v in errs.values()), errs


@pytest.mark.parametrize('C', [32, 64])
def test_fused_resblock_matches_unfused_block(C):
    """The SEANet block with the fused kernels vs the same block on the three separate conv kernels
    (ENCX_RESBLOCK=0): forward and every grad within fp32 rounding of each other."""
    import os
    from encx.modules.seanet import SEANetResnetBlock
    torch.manual_seed(3)
    blk = SEANetResnetBlock(C, norm='weight_norm', causal=True, true_skip=False).to(DEV)
    x0 = (0.5 * torch.randn(2, C, 4800)).to(DEV)
    dy = torch.randn(2, C, 4800).to(DEV)
    outs = []
    for fused in ('1', '0'):
        os.environ['ENCX_RESBLOCK'] = fused
        try:
            x = x0.clone().requires_grad_(True)
            y = blk(x)
            gs = torch.autograd.grad(y, [x] + list(blk.parameters()), dy)
            outs.append([y.detach()] + [g.detach() for g in gs])
        finally:
            os.environ.pop('ENCX_RESBLOCK', None)
    for a, b in zip(*outs):
        assert float((a - b).abs().max()) <= 2e-5 * float(b.abs().max()) + 1e-7, (float((a - b).abs().max()), float(b.abs().max()))


@pytest.mark.parametrize('fft', [1, 0], ids=['fft', 'dft_gemm'])
@pytest.mark.parametrize('n', [32, 64, 128, 256, 512, 1024, 2048])
def test_spectrogram_fft_vs_torch_fp64(n, fft):
    """The real-FFT spectrogram (csrc/fft.h, the discriminator's Spectrogram: hann window,
    center=False, normalized, msstftd.py:62-64, 97-99) and its transpose, at every power-of-2
    size the mel loss and the discriminator use, against torch.stft / autograd in fp64: relative
    to each tensor's largest magnitude. fft = 0: the framed-DFT GEMM path (option FFT)."""
    from encx import ops
    from encx._lib import option
    B, C, Tn = 2, 2, 6000
    x64 = torch.from_numpy(synth_wave((B, C, Tn), n)).double().requires_grad_(True)
    w = torch.hann_window(n, dtype=torch.float64)
    st = torch.stft(x64.reshape(B * C, Tn), n_fft=n, hop_length=n // 4, window=w, center=False,
                    return_complex=True) / w.pow(2).sum().sqrt()  # [BC][nb][Fr]
    ref = torch.cat([st.real, st.imag], 0).reshape(2, B, C, n // 2 + 1, -1).permute(1, 0, 2, 4, 3)
    ref = ref.reshape(B, 2 * C, -1, n // 2 + 1)  # [b][re c | im c][fr][k]
    xg = x64.detach().float().to(DEV).requires_grad_(True)
    dz = torch.randn(ref.shape, generator=torch.Generator().manual_seed(n), dtype=torch.float64)
    with option(FFT=fft):
        z = ops.DiscSpecFn.apply(xg, n, n // 4, 24000)
        gx, = torch.autograd.grad(z, [xg], dz.float().to(DEV))
    gref, = torch.autograd.grad(ref, [x64], dz)

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double()
        return float((a - b).abs().max() / (b.abs().max() + 1e-30))
    ez, eg = rel(z, ref), rel(gx, gref)
    print(f'n {n}: spectrogram {ez:.1e}, its transpose {eg:.1e}')
    assert ez < 2e-6 and eg < 2e-6, (ez, eg)


@pytest.mark.parametrize('n,wl,normalized,fft', [(1024, 600, True, 1), (512, 512, False, 1), (256, 200, False, 1),
                                                 (1024, 1000, True, 0), (2048, 1500, True, 1)])
def test_disc_spectrogram_window_vs_stft_fp64(n, wl, normalized, fft):
    """torchaudio Spectrogram(n_fft, win_length < n_fft, hann, normalized on / off, center=False,
    power=None) of DiscriminatorSTFT (msstftd.py:62-64): torch.stft centres the hann(win_length)
    window in n_fft zeros; normalized divides by sqrt(sum w^2). Through DiscriminatorSTFT's own
    window tables (ops.spec_window_tables), spectrogram and transpose vs fp64 torch.stft."""
    from encx import ops
    from encx._lib import option
    B, C, Tn = 2, 1, 5000
    x64 = torch.from_numpy(synth_wave((B, C, Tn), n + wl)).double().requires_grad_(True)
    w = torch.hann_window(wl, dtype=torch.float64)
    st = torch.stft(x64.reshape(B * C, Tn), n_fft=n, hop_length=n // 4, win_length=wl, window=w, center=False,
                    return_complex=True)
    if normalized:
        st = st / w.pow(2).sum().sqrt()
    ref = torch.cat([st.real, st.imag], 0).reshape(2, B, C, n // 2 + 1, -1).permute(1, 0, 2, 4, 3)
    ref = ref.reshape(B, 2 * C, -1, n // 2 + 1)
    xg = x64.detach().float().to(DEV).requires_grad_(True)
    dz = torch.randn(ref.shape, generator=torch.Generator().manual_seed(wl), dtype=torch.float64)
    win = ops.spec_window_tables(torch.hann_window(wl).to(DEV), n, normalized)
    with option(FFT=fft):
        z = ops.DiscSpecFn.apply(xg, n, n // 4, 24000, win)
        gx, = torch.autograd.grad(z, [xg], dz.float().to(DEV))
    gref, = torch.autograd.grad(ref, [x64], dz)

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double()
        return float((a - b).abs().max() / (b.abs().max() + 1e-30))
    ez, eg = rel(z, ref), rel(gx, gref)
    print(f'n {n} win {wl} normalized {normalized}: spectrogram {ez:.1e}, its transpose {eg:.1e}')
    assert ez < 2e-6 and eg < 2e-6, (ez, eg)


def test_disc_stft_win_length_module_vs_oracle():
    """DiscriminatorSTFT(n_fft=1024, win_length=800) end to end against the oracle's forward
    (torch.stft with win_length): logits and feature maps."""
    from encx.msstftd import DiscriminatorSTFT
    d = DiscriminatorSTFT(32, n_fft=1024, hop_length=256, win_length=800).to(DEV)
    p = {f'd.{k}': v.detach().cpu().double() for k, v in d.state_dict().items()}
    x0 = synth_wave((2, 1, 8000), 77, amp=0.3)
    with torch.no_grad():
        lg, fm = d(G(x0), param_grads=False)
        lr, fr = O.disc_stft_forward(T(x0).double(), p, 'd', 1024, 256, 800)
    close(lg, lr, 1e-4, 1e-4 * float(lr.abs().max()), 'logits')
    for i, (a, b) in enumerate(zip(fm, fr)):
        close(a, b, 1e-4, 1e-4 * float(b.abs().max()), f'fmap {i}')
