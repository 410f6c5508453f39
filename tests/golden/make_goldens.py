"""Generate the golden fixtures in tests/golden/*.npz by RUNNING THE REFERENCE.

Test infrastructure; runs only in the build container, where /root/reference exists
(`python tests/golden/make_goldens.py`). The reference is imported with the shims of
ref_shims.py; every parameter / input is synthesised by synth.py from PCG64 seeds so the
tests can regenerate them bit-identically without any weight file.

Fixture map:
  g1_eval24k.npz   config 1: 24 kHz causal weight-norm model, eval forward, bw 1.5 (n_q 2)
  g2_convs.npz     SConv1d / SConvTranspose1d outputs + grads (dx, dv, dg, db)
  g3_rvq.npz       RVQ train forward (n_q 2, K 1024) + EMA buffers + emb grad; kmeans
  g4_mel.npz       Audio2Mel 7 scales, Spectrogram 3 scales, l_t / l_f and d l_f / d y
  g5_disc.npz      MS-STFT discriminator logits, fmap checksums, input grad
  g6_balancer.npz  Balancer known-answer test (balancer.py:121-139) + a 4-loss case
  g7_step.npz      one full train step (gen-only and GAN), B 2, T 4800, n_q 2
  g8_sched.npz     WarmupCosineLrScheduler learning-rate trace
  g10_ecdc.npz     .ecdc: reference BitPacker vectors (bits 1..32), header, compress/decompress
                   bytes + waves for the g1 model and the g9 48 kHz model (one / two segments)
  g11_data.npz     customAudioDataset crop (seeded random) + mono expand + collate_fn
  g12_lm.npz       LM entropy coder: build_stable_quantized_cdf + ArithmeticCoder/Decoder vectors
                   (ac.py), LMModel streaming probabilities with synthetic weights (real dims and
                   a small past_context), and compress(use_lm=True) bytes of the g1 model
  g9_step48k.npz   config-5 analogue: 48 kHz stereo, non-causal, time_group_norm, segment 0.1 s
                   (two frames: 4800 + 48 samples, linear overlap-add), gen-only and GAN steps
  g13_ddp.npz      the reference's train_one_step under DDP, 2 ranks over gloo (G13 below)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from ref_shims import import_reference  # noqa: E402
from synth import synth_state, synth_wave, synth_codebooks, rng  # noqa: E402

torch.set_num_threads(8)
R = import_reference()


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def load_synth(module, seed):
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()
              if v.dtype == torch.float32 and '_codebook' not in k and 'spec_transform' not in k}
    st = synth_state(shapes, seed)
    new = dict(sd)
    for k, v in st.items():
        new[k] = t(v)
    module.load_state_dict(new)
    return st


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print('wrote', path, os.path.getsize(path) // 1024, 'KB')


def fill_codebooks(model, stats, seed, n_used):
    cbs = synth_codebooks(stats, seed)
    g = rng(seed + 1)
    for i, layer in enumerate(model.quantizer.vq.layers):
        c = layer._codebook
        if i < n_used:
            c.embed.data.copy_(t(cbs[i]))
            cs = g.uniform(0.5, 4.0, size=(1024,)).astype(np.float32)
            c.cluster_size.data.copy_(t(cs))
            c.embed_avg.data.copy_(t((cbs[i] * cs[:, None]).astype(np.float32)))
        c.inited.data.fill_(1.0)


def emb_stats(model, x, n_q):
    """Per-dim mean/std of the encoder output and of each RVQ residual (used to synthesise
    codebooks near the data)."""
    model.eval()
    with torch.no_grad():
        xn = x / (1e-8 + x.mean(1, keepdim=True).pow(2).mean(2, keepdim=True).sqrt())
        emb = model.encoder(xn)
    return emb


def top2_gaps(emb, embeds, codes):
    """fp64 certificate per frame and layer: distance of the 2nd-best code minus the best,
    along the residual chain the reference's own codes define (eval: residual -= q)."""
    res = emb.double().permute(0, 2, 1).reshape(-1, emb.shape[1])
    gaps = []
    for i, E in enumerate(embeds):
        E = E.double()
        d = (res ** 2).sum(1, keepdim=True) - 2 * res @ E.t() + (E ** 2).sum(1)[None]
        s = torch.sort(d, dim=1).values
        gaps.append((s[:, 1] - s[:, 0]).numpy())
        ind = codes[:, i].reshape(-1).long() if codes.dim() == 3 else codes[i].reshape(-1).long()
        res = res - E[ind]
    return np.stack(gaps)


# ------------------------------------------------------------------------------------ G1
def g1():
    m = R.model.EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True,
                                        model_norm='weight_norm', audio_normalize=False,
                                        segment=None, name='encodec_24khz')
    load_synth(m, 1)
    x = t(synth_wave((1, 1, 24000), 1234))
    m.eval()
    with torch.no_grad():
        emb = m.encoder(x)
    e = emb[0].t().double()
    stats = np.zeros((2, 2, 128), np.float32)
    stats[0, 0] = e.mean(0).float().numpy()
    stats[0, 1] = e.std(0).float().numpy()
    cb0 = synth_codebooks(stats[:1], 77)[0]
    # residual after layer 0 with that codebook
    xf = emb[0].t()
    ind = R.quantization.core_vq.EuclideanCodebook.quantize(
        type('o', (), {'embed': t(cb0)})(), xf)
    r1 = (xf - t(cb0)[ind]).double()
    stats[1, 0] = r1.mean(0).float().numpy()
    stats[1, 1] = r1.std(0).float().numpy()
    fill_codebooks(m, stats, 77, 2)
    m.set_target_bandwidth(1.5)
    with torch.no_grad():
        y = m(x)
        codes = m.encode(x)[0][0]
        gaps = top2_gaps(emb, [m.quantizer.vq.layers[i]._codebook.embed for i in range(2)], codes)
    save('g1_eval24k.npz', x=x.numpy(), emb=emb.numpy(), codes=codes.numpy().astype(np.int16),
         y=y.numpy(), stats=stats, gaps=gaps)


# ------------------------------------------------------------------------------------ G2
CONV_CASES = [
    # name, kind, cin, cout, K, s, causal, pre_elu, T
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


def g2():
    out = {}
    for ci, (name, kind, cin, cout, K, s, causal, pre_elu, T) in enumerate(CONV_CASES):
        if kind == 'conv':
            mod = R.modules.SConv1d(cin, cout, K, stride=s, causal=causal, norm='weight_norm')
        else:
            mod = R.modules.SConvTranspose1d(cin, cout, K, stride=s, causal=causal, norm='weight_norm')
        load_synth(mod, 100 + ci)
        x = t(synth_wave((2, cin, T), 200 + ci, amp=1.0)).requires_grad_(True)
        xin = torch.nn.functional.elu(x) if pre_elu else x
        y = mod(xin)
        gy = t(synth_wave(tuple(y.shape), 300 + ci, amp=1.0))
        y.backward(gy)
        params = dict(mod.named_parameters())
        pre = [k for k in params if k.endswith('weight_v')][0][:-len('weight_v')]
        out[name + '/x'] = x.detach().numpy()
        out[name + '/y'] = y.detach().numpy()
        out[name + '/gy'] = gy.numpy()
        out[name + '/dx'] = x.grad.numpy()
        out[name + '/dv'] = params[pre + 'weight_v'].grad.numpy()
        out[name + '/dg'] = params[pre + 'weight_g'].grad.numpy()
        out[name + '/db'] = params[pre + 'bias'].grad.numpy()
    save('g2_convs.npz', **out)


# ------------------------------------------------------------------------------------ G3
def g3():
    q = R.quantization.ResidualVectorQuantizer(dimension=128, n_q=2, bins=1024)
    emb = t(synth_wave((2, 128, 75), 31, amp=1.0))
    stats = np.zeros((2, 2, 128), np.float32)
    stats[0, 1] = 1.0
    stats[1, 1] = 0.6
    cbs = synth_codebooks(stats, 32)
    g = rng(33)
    init = {}
    for i, layer in enumerate(q.vq.layers):
        c = layer._codebook
        c.embed.data.copy_(t(cbs[i]))
        cs = g.uniform(0.0, 4.0, size=(1024,)).astype(np.float32)
        c.cluster_size.data.copy_(t(cs))
        ea = g.standard_normal(size=(1024, 128)).astype(np.float32)
        c.embed_avg.data.copy_(t(ea))
        c.inited.data.fill_(1.0)
        init[f'cs{i}'] = cs
        init[f'ea{i}'] = ea
    q.train()
    x = emb.clone().requires_grad_(True)
    res = q(x, 75, 1.5)
    gq = t(synth_wave(tuple(res.quantized.shape), 34, amp=1.0))
    torch.autograd.backward([res.quantized, res.penalty], [gq, torch.tensor(1.0)])
    outs = dict(emb=emb.numpy(), stats=stats, quantized=res.quantized.detach().numpy(),
                codes=res.codes.numpy().astype(np.int16), penalty=res.penalty.detach().numpy(),
                gaps=top2_gaps(emb, [t(cbs[0]), t(cbs[1])], res.codes),
                gq=gq.numpy(), demb=x.grad.numpy())
    for i, layer in enumerate(q.vq.layers):
        c = layer._codebook
        outs[f'cs_init{i}'] = init[f'cs{i}']
        outs[f'ea_init{i}'] = init[f'ea{i}']
        outs[f'cluster_size{i}'] = c.cluster_size.numpy()
        outs[f'embed_avg{i}'] = c.embed_avg.numpy()
        outs[f'embed{i}'] = c.embed.numpy()
    # kmeans with the sample_vectors draw injected (core_vq.py:69-77, 80-102)
    samples = t(synth_wave((600, 128), 35, amp=1.0))
    init_idx = torch.from_numpy(rng(36).permutation(600)[:64].astype(np.int64))
    orig = R.quantization.core_vq.sample_vectors
    R.quantization.core_vq.sample_vectors = lambda s, n: s[init_idx]
    means, bins = R.quantization.core_vq.kmeans(samples, 64, 10)
    R.quantization.core_vq.sample_vectors = orig
    outs.update(km_samples=samples.numpy(), km_init=init_idx.numpy(), km_means=means.numpy(),
                km_bins=bins.numpy())
    save('g3_rvq.npz', **outs)


# ------------------------------------------------------------------------------------ G4
def g4():
    x = t(synth_wave((2, 1, 4800), 41))
    y = t(synth_wave((2, 1, 4800), 42)).requires_grad_(True)
    out = {'x': x.numpy(), 'y': y.detach().numpy()}
    for i in range(5, 12):
        n = 2 ** i
        a2m = R.audio_to_mel.Audio2Mel(n_fft=n, win_length=n, hop_length=n // 4,
                                       n_mel_channels=64, sampling_rate=24000)
        out[f'mel{n}'] = a2m(x).numpy()
        out[f'melbasis{n}'] = a2m.mel_basis.numpy()
    for n, h in zip((1024, 2048, 512), (256, 512, 128)):
        sp = sys.modules['torchaudio'].transforms.Spectrogram(
            n_fft=n, hop_length=h, win_length=n, window_fn=torch.hann_window,
            normalized=True, center=False, pad_mode=None, power=None)
        z = sp(x)
        out[f'spec{n}'] = torch.view_as_real(z).numpy()
    losses = R.losses.total_loss([[torch.ones(1)]], [torch.zeros(1)], [[torch.ones(1)]], x, y)
    out['l_t'] = losses['l_t'].detach().numpy()
    out['l_f'] = losses['l_f'].detach().numpy()
    gf, = torch.autograd.grad(losses['l_f'], [y])
    gt, = torch.autograd.grad(losses['l_t'], [y])
    out['dlf_dy'] = gf.numpy()
    out['dlt_dy'] = gt.numpy()
    save('g4_mel.npz', **out)


# ------------------------------------------------------------------------------------ G5
def g5():
    d = R.msstftd.MultiScaleSTFTDiscriminator(filters=32)
    load_synth(d, 51)
    x = t(synth_wave((1, 1, 4800), 52)).requires_grad_(True)
    logits, fmaps = d(x)
    r = rng(53)
    f = 0
    out = {'x': x.detach().numpy()}
    for k, lg in enumerate(logits):
        out[f'logits{k}'] = lg.detach().numpy()
        wl = t(r.standard_normal(size=tuple(lg.shape)).astype(np.float32))
        f = f + (lg * wl).sum()
        for j, fm in enumerate(fmaps[k]):
            out[f'fmap{k}_{j}_sum'] = fm.detach().double().sum().numpy()
            out[f'fmap{k}_{j}_sq'] = fm.detach().double().pow(2).sum().numpy()
            out[f'fmap{k}_{j}_shape'] = np.array(fm.shape)
            out[f'fmap{k}_{j}_head'] = fm.detach().reshape(-1)[:256].numpy()
            f = f + fm.mean()
    f.backward()
    out['dx'] = x.grad.numpy()
    save('g5_disc.npz', **out)


# ------------------------------------------------------------------------------------ G6
def g6():
    out = {}
    # balancer.py:121-139 known answer
    from torch.nn import functional as F
    for rescale in (False, True):
        x = torch.zeros(1, requires_grad=True)
        one = torch.ones_like(x)
        losses = {'1': F.l1_loss(x, one), '2': 100 * F.l1_loss(x, -one)}
        R.balancer.Balancer(weights={'1': 1, '2': 1}, rescale_grads=rescale).backward(losses, x)
        out[f'kat_{int(rescale)}'] = x.grad.numpy()
    # 4 losses, 3 consecutive calls (EMA state), per-item norms on [B,1,T]
    r = rng(61)
    b = R.balancer.Balancer(weights={'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3})
    for it in range(3):
        y = torch.zeros(4, 1, 300, requires_grad=True)
        gs = {k: t(r.standard_normal(size=(4, 1, 300)).astype(np.float32) * s)
              for k, s in (('l_t', 0.01), ('l_f', 1.0), ('l_g', 0.1), ('l_feat', 3.0))}
        losses = {k: (y * g).sum() for k, g in gs.items()}
        b.backward(losses, y)
        for k, g in gs.items():
            out[f'it{it}_{k}'] = g.numpy()
        out[f'it{it}_out'] = y.grad.numpy()
    save('g6_balancer.npz', **out)


# ------------------------------------------------------------------------------------ G7
def one_step(gan):
    m = R.model.EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm',
                                        audio_normalize=True, segment=None, name='x')
    load_synth(m, 71)
    x = t(synth_wave((2, 1, 4800), 72))
    with torch.no_grad():
        emb = m.encoder(x / (1e-8 + x.pow(2).mean(2, keepdim=True).sqrt()))
    e = emb.permute(0, 2, 1).reshape(-1, 128).double()
    stats = np.zeros((2, 2, 128), np.float32)
    stats[0, 0] = e.mean(0).float().numpy()
    stats[0, 1] = e.std(0).float().numpy()
    stats[1, 1] = 0.5 * stats[0, 1]
    fill_codebooks(m, stats, 73, 2)
    d = R.msstftd.MultiScaleSTFTDiscriminator(filters=32)
    load_synth(d, 74)
    opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=3e-4, betas=(0.5, 0.9))
    optd = torch.optim.Adam([p for p in d.parameters() if p.requires_grad], lr=3e-4, betas=(0.5, 0.9))
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3} if gan else {'l_t': 0.1, 'l_f': 1}
    bal = R.balancer.Balancer(weights)
    m.train()
    d.train()
    out = {'x': x.numpy(), 'stats': stats}
    for it in range(2):
        opt.zero_grad()
        y, loss_w, _ = m(x)
        if gan:
            lr_, fr = d(x)
            lf_, ff = d(y)
            losses = R.losses.total_loss(fr, lf_, ff, x, y, sample_rate=24000)
        else:
            l_t = torch.nn.functional.l1_loss(x, y)
            l_f = R.losses.total_loss([[torch.ones(1)]], [torch.zeros(1)], [[torch.ones(1)]], x, y)['l_f']
            losses = {'l_t': l_t, 'l_f': l_f}
        bal.backward(losses, y, retain_graph=True)
        loss_w.backward()
        opt.step()
        for k, v in losses.items():
            out[f'it{it}_{k}'] = v.detach().numpy()
        out[f'it{it}_loss_w'] = loss_w.detach().numpy()
        out[f'it{it}_y'] = y.detach().numpy()
        if gan:
            optd.zero_grad()
            lr2, _ = d(x)
            lf2, _ = d(y.detach())
            ld = R.losses.disc_loss(lr2, lf2)
            ld.backward()
            optd.step()
            out[f'it{it}_l_d'] = ld.detach().numpy()
    for k, v in m.state_dict().items():
        if v.dtype == torch.float32:
            out['p/' + k] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    if gan:
        for k, v in d.state_dict().items():
            out['d/' + k] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    # a few full tensors for sharper checks
    sd = m.state_dict()
    for k in ('encoder.model.0.conv.conv.weight_v', 'decoder.model.15.conv.conv.weight_v',
              'quantizer.vq.layers.0._codebook.cluster_size'):
        out['full/' + k] = sd[k].numpy()
    return out


def g7():
    out = {}
    for gan in (False, True):
        o = one_step(gan)
        out.update({('gan/' if gan else 'gen/') + k: v for k, v in o.items()})
    save('g7_step.npz', **out)


G9_SEG = 0.1  # seconds: frames of 4800 samples at stride 4752 -> 4800 + 48 (the 48000 + 480 of 1 s)


def one_step_48k(gan):
    m = R.model.EncodecModel._get_model([3.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                        audio_normalize=True, segment=G9_SEG, name='encodec_48khz')
    load_synth(m, 91)
    x = t(synth_wave((2, 2, 4800), 92))
    with torch.no_grad():
        emb = m.encoder(x / (1e-8 + x.mean(1, keepdim=True).pow(2).mean(2, keepdim=True).sqrt()))
    e = emb.permute(0, 2, 1).reshape(-1, 128).double()
    stats = np.zeros((2, 2, 128), np.float32)
    stats[0, 0] = e.mean(0).float().numpy()
    stats[0, 1] = e.std(0).float().numpy()
    stats[1, 1] = 0.5 * stats[0, 1]
    fill_codebooks(m, stats, 93, 2)
    d = R.msstftd.MultiScaleSTFTDiscriminator(filters=32, in_channels=2, out_channels=2)
    load_synth(d, 94)
    opt = torch.optim.Adam([p for p in m.parameters() if p.requires_grad], lr=1e-4, betas=(0.5, 0.9))
    optd = torch.optim.Adam([p for p in d.parameters() if p.requires_grad], lr=1e-4, betas=(0.5, 0.9))
    # scripts/train.sbatch:32-33: l_g = l_feat = 4
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4} if gan else {'l_t': 0.1, 'l_f': 1}
    bal = R.balancer.Balancer(weights)
    m.train()
    d.train()
    out = {'x': x.numpy(), 'stats': stats}
    for it in range(2):
        opt.zero_grad()
        y, loss_w, frames = m(x)
        out[f'it{it}_nframes'] = np.array(len(frames))
        if gan:
            lr_, fr = d(x)
            lf_, ff = d(y)
            losses = R.losses.total_loss(fr, lf_, ff, x, y, sample_rate=48000)
        else:
            l_t = torch.nn.functional.l1_loss(x, y)
            l_f = R.losses.total_loss([[torch.ones(1)]], [torch.zeros(1)], [[torch.ones(1)]], x, y,
                                      sample_rate=48000)['l_f']
            losses = {'l_t': l_t, 'l_f': l_f}
        bal.backward(losses, y, retain_graph=True)
        loss_w.backward()
        opt.step()
        for k, v in losses.items():
            out[f'it{it}_{k}'] = v.detach().numpy()
        out[f'it{it}_loss_w'] = loss_w.detach().numpy()
        out[f'it{it}_y'] = y.detach().numpy()
        if gan:
            optd.zero_grad()
            lr2, _ = d(x)
            lf2, _ = d(y.detach())
            ld = R.losses.disc_loss(lr2, lf2)
            ld.backward()
            optd.step()
            out[f'it{it}_l_d'] = ld.detach().numpy()
    for k, v in m.state_dict().items():
        if v.dtype == torch.float32:
            out['p/' + k] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    if gan:
        for k, v in d.state_dict().items():
            out['d/' + k] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    return out


def g9():
    out = {}
    for gan in (False, True):
        o = one_step_48k(gan)
        out.update({('gan/' if gan else 'gen/') + k: v for k, v in o.items()})
    save('g9_step48k.npz', **out)


def g8():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=3e-4)
    s = R.scheduler.WarmupCosineLrScheduler(opt, max_iter=400, eta_ratio=0.1, warmup_iter=50, warmup_ratio=1e-4)
    lrs = []
    for _ in range(400):
        lrs.append(opt.param_groups[0]['lr'])
        opt.step()
        s.step()
    save('g8_sched.npz', lr=np.array(lrs))


# ------------------------------------------------------------------------------------ G10
# (bits, count) cases for the reference BitPacker: the model's 10 bits, the reference test's
# 1..15 range (binary.py:130-147), the ABI's 16..32, empty / single-value / ragged counts
G10_CASES = [(10, 600), (10, 1), (10, 0), (1, 13), (2, 5), (3, 1000), (7, 17), (8, 64), (9, 71),
             (11, 333), (13, 999), (15, 257), (16, 100), (20, 77), (31, 9), (32, 33)]


def g10():
    import io
    import binary as ref_binary
    import compress as ref_compress
    out = {}
    g = rng(1010)
    tokens, packed, ghosts = [], [], []
    for bits, n in G10_CASES:
        tok = g.integers(0, 1 << bits, size=n, dtype=np.int64)
        buf = io.BytesIO()
        pk = ref_binary.BitPacker(bits, buf)
        for v in tok.tolist():
            pk.push(v)
        pk.flush()
        b = buf.getvalue()
        buf.seek(0)
        up = ref_binary.BitUnpacker(bits, buf)
        pulled = []
        while True:
            v = up.pull()
            if v is None:
                break
            pulled.append(v)
        assert pulled[:n] == tok.tolist()
        tokens.append(tok)
        packed.append(np.frombuffer(b, np.uint8))
        ghosts.append(len(pulled) - n)
    out['bp_cases'] = np.array(G10_CASES, np.int64)
    out['bp_tokens'] = np.concatenate(tokens)
    out['bp_bytes'] = np.concatenate(packed)
    out['bp_nbytes'] = np.array([len(p) for p in packed], np.int64)
    out['bp_ghosts'] = np.array(ghosts, np.int64)
    hb = io.BytesIO()
    ref_binary.write_ecdc_header(hb, {'m': 'encodec_24khz', 'al': 24000, 'nc': 2, 'lm': False, 'fr': 75})
    out['header'] = np.frombuffer(hb.getvalue(), np.uint8)

    # 24 kHz: the g1 model and clip, bandwidth 1.5 (n_q 2), one frame, no scale
    d1 = np.load(os.path.join(HERE, 'g1_eval24k.npz'))
    m = R.model.EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True,
                                        model_norm='weight_norm', audio_normalize=False,
                                        segment=None, name='encodec_24khz')
    load_synth(m, 1)
    fill_codebooks(m, d1['stats'], 77, 2)
    m.eval()
    m.set_target_bandwidth(1.5)
    x = t(d1['x'])[0]
    b24 = ref_compress.compress(m, x, use_lm=False)
    with torch.no_grad():
        y24, sr = ref_compress.decompress_from_file(m, io.BytesIO(b24), device='cpu')
    out['c24_bytes'] = np.frombuffer(b24, np.uint8)
    out['c24_y'] = y24.numpy()

    # 48 kHz stereo, normalised, 0.1 s segments (the g9 model): a 4752-sample clip is one
    # segment (scale + codes); a 4800-sample clip is two (4800 + 48), and decompress reads the
    # short one with the first frame's length -> EOFError (compress.py:126, 137-138)
    d9 = np.load(os.path.join(HERE, 'g9_step48k.npz'))
    m = R.model.EncodecModel._get_model([3.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                        audio_normalize=True, segment=G9_SEG, name='encodec_48khz')
    load_synth(m, 91)
    fill_codebooks(m, d9['gen/stats'], 93, 2)
    m.eval()
    m.set_target_bandwidth(3.0)
    w = t(synth_wave((2, 4800), 1011))
    b48 = ref_compress.compress(m, w[:, :4752], use_lm=False)
    with torch.no_grad():
        y48, _ = ref_compress.decompress_from_file(m, io.BytesIO(b48), device='cpu')
        codes48 = m.encode(w[None, :, :4752])[0][0]
    out['c48_x'] = w.numpy()
    out['c48_bytes'] = np.frombuffer(b48, np.uint8)
    out['c48_y'] = y48.numpy()
    out['c48_codes'] = codes48.numpy().astype(np.int16)
    b48s = ref_compress.compress(m, w, use_lm=False)
    out['c48s_bytes'] = np.frombuffer(b48s, np.uint8)
    try:
        ref_compress.decompress_from_file(m, io.BytesIO(b48s), device='cpu')
        out['c48s_eof'] = np.array(0)
    except EOFError:
        out['c48s_eof'] = np.array(1)
    save('g10_ecdc.npz', **out)


# ------------------------------------------------------------------------------------ G11
def g11():
    """customAudioDataset.__getitem__ (random tensor_cut crop, mono expand) + collate_fn, run
    on preset decoded clips (the file decode, librosa.load, is replaced by `get`)."""
    import random
    import types as _types
    sys.modules.setdefault('audioread', _types.ModuleType('audioread'))
    import customAudioDataset as ref_ds
    g = rng(1111)
    out = {}
    for name, channels, cut, lens in [('mono', 1, 2400, [5000, 2400, 2401, 7777, 1200, 3000]),
                                      ('stereo', 2, 4800, [9000, 4800, 12000, 700])]:
        clips = []
        for i, L in enumerate(lens):
            mono = channels == 1 or i % 2 == 1     # stereo set: odd clips are mono, expanded
            clips.append(g.standard_normal(L if mono else (channels, L)).astype(np.float32))
        ds = object.__new__(ref_ds.CustomAudioDataset)
        ds.transform, ds.tensor_cut, ds.channels, ds.sample_rate = None, cut, channels, 24000
        ds.fixed_length = 0

        def get(idx=None, _clips=clips, _ds=ds):
            w = torch.as_tensor(_clips[idx])
            if len(w.shape) == 1:                       # customAudioDataset.py:51-54
                w = w.unsqueeze(0).expand(_ds.channels, -1)
            return w, 24000
        ds.get = get
        order = [int(v) for v in g.permutation(len(lens))]
        random.seed(1212)
        items = [ds[i] for i in order]
        batch = ref_ds.collate_fn(items)
        out[f'{name}/clips'] = np.concatenate([c.reshape(-1) for c in clips])
        out[f'{name}/lens'] = np.array(lens, np.int64)
        out[f'{name}/mono'] = np.array([c.ndim == 1 for c in clips])
        out[f'{name}/order'] = np.array(order, np.int64)
        out[f'{name}/cut'] = np.array(cut)
        out[f'{name}/channels'] = np.array(channels)
        out[f'{name}/batch'] = batch.numpy()
    save('g11_data.npz', **out)


# ------------------------------------------------------------------------------------ G12
# (cardinality, steps, total_range_bits, logit scale, symbols): pdf = softmax(scale * randn(card));
# symbols drawn from the pdf (0, as ac.py:277) or uniformly (1: mostly improbable symbols, long
# codes, the range straddling a power of two for many steps)
G12_AC_CASES = [(1024, 32, 24, 3.0, 0), (37, 64, 24, 1.0, 0), (2, 40, 24, 4.0, 0), (3, 6, 24, 1.0, 0),
                (3000, 8, 24, 6.0, 0), (64, 50, 16, 2.0, 0), (256, 48, 24, 6.0, 1), (1024, 24, 30, 8.0, 1)]
# LM configs: real dims (model.py:221-226 at 24 kHz) and a small one whose past_context
# window truncates within the sequence
G12_LM = {'a': dict(n_q=32, card=1024, dim=200, num_heads=8, num_layers=5, past_context=262,
                    seed=121, B=1, K=8, T=10),
          'b': dict(n_q=4, card=64, dim=64, num_heads=4, num_layers=2, past_context=5,
                    seed=122, B=2, K=3, T=14)}


def g12_lm_module(c):
    from oracle.lm_oracle import LMConfig, lm_param_shapes
    from synth import synth_lm_state
    lm = R.model.LMModel(c['n_q'], c['card'], dim=c['dim'], num_heads=c['num_heads'],
                         num_layers=c['num_layers'], past_context=c['past_context'])
    cfg = LMConfig(n_q=c['n_q'], card=c['card'], dim=c['dim'], num_heads=c['num_heads'],
                   num_layers=c['num_layers'], past_context=c['past_context'])
    shapes = lm_param_shapes(cfg)
    sd = lm.state_dict()
    assert set(sd) == set(shapes), set(sd) ^ set(shapes)
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in shapes.items())
    lm.load_state_dict({k: t(v) for k, v in synth_lm_state(shapes, c['seed']).items()})
    lm.eval()
    return lm


def g12():
    import io
    import random
    import compress as ref_compress
    import quantization.ac as ref_ac
    out = {}
    # ---- arithmetic coder vectors (the structure of ac.py:263-288, smaller)
    pdfs, cdfs, syms, datas, eofs = [], [], [], [], []
    over_p, over_c, over_b = [], [], []
    for i, (card, steps, bits, scale, uni) in enumerate(G12_AC_CASES):
        torch.manual_seed(1234 + i)
        fo = io.BytesIO()
        enc = ref_ac.ArithmeticCoder(fo, total_range_bits=bits)
        cp, cc, cs = [], [], []
        while len(cs) < steps:
            pdf = torch.softmax(scale * torch.randn(card), dim=0)
            # check=False as compress.py:84-85 calls it. A near-certain pdf can round to a
            # total above 2^bits; check=True rejects it and the coder would then assert
            # (ac.py:116): such rows are kept apart (ac_over_*) and redrawn
            q = ref_ac.build_stable_quantized_cdf(pdf, enc.total_range_bits, check=False)
            if int(q[-1]) > 2 ** bits:
                over_p.append(pdf.numpy())
                over_c.append(q.numpy())
                over_b.append(bits)
                continue
            s = torch.multinomial(pdf, 1).item() if not uni else int(torch.randint(card, (1,)))
            enc.push(s, q)
            cp.append(pdf.numpy())
            cc.append(q.numpy())
            cs.append(s)
        enc.flush()
        fo.seek(0)
        dec = ref_ac.ArithmeticDecoder(fo, total_range_bits=bits)
        for q, s in zip(cc, cs):
            assert dec.pull(torch.from_numpy(q)) == s
        # one pull past the end (ac.py:288): None if the decoder needs bits the stream no
        # longer has (1), else the binary search over a one-entry zero cdf fails (2)
        try:
            eofs.append(1 if dec.pull(torch.zeros(1)) is None else 0)
        except RuntimeError:
            eofs.append(2)
        pdfs.append(np.concatenate(cp))
        cdfs.append(np.concatenate(cc))
        syms.append(np.array(cs, np.int64))
        datas.append(np.frombuffer(fo.getvalue(), np.uint8))
    out['ac_cases'] = np.array([c[:3] + c[4:] for c in G12_AC_CASES], np.int64)
    out['ac_scale'] = np.array([c[3] for c in G12_AC_CASES], np.float32)
    out['ac_pdf'] = np.concatenate(pdfs).astype(np.float32)
    out['ac_cdf'] = np.concatenate(cdfs).astype(np.int32)
    out['ac_sym'] = np.concatenate(syms)
    out['ac_bytes'] = np.concatenate(datas)
    out['ac_nbytes'] = np.array([len(d) for d in datas], np.int64)
    out['ac_eof'] = np.array(eofs, np.int64)
    out['ac_over_pdf'] = np.concatenate(over_p).astype(np.float32)
    out['ac_over_cdf'] = np.concatenate(over_c).astype(np.int64)
    out['ac_over_card'] = np.array([len(a) for a in over_p], np.int64)
    out['ac_over_bits'] = np.array(over_b, np.int64)

    # ---- LM streaming probabilities (compress.py:74-78 call pattern)
    for name, c in G12_LM.items():
        lm = g12_lm_module(c)
        g = rng(c['seed'] + 1000)
        codes = t(g.integers(0, c['card'], size=(c['B'], c['K'], c['T']), dtype=np.int64))
        states, offset = None, 0
        inp = torch.zeros(c['B'], c['K'], 1, dtype=torch.long)
        probs = []
        with torch.no_grad():
            for ti in range(c['T']):
                p, states, offset = lm(inp, states, offset)
                inp = 1 + codes[:, :, ti:ti + 1]
                probs.append(p[:, :, :, 0].permute(0, 2, 1).numpy())   # [B][K][card]
        out[f'lm_{name}/codes'] = codes.numpy()
        out[f'lm_{name}/probs'] = np.stack(probs, 1).astype(np.float32)  # [B][T][K][card]

    # ---- compress(use_lm=True) of the g1 model at 1.5 kbps on a 0.2 s clip
    d1 = np.load(os.path.join(HERE, 'g1_eval24k.npz'))
    m = R.model.EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True,
                                        model_norm='weight_norm', audio_normalize=False,
                                        segment=None, name='encodec_24khz')
    load_synth(m, 1)
    fill_codebooks(m, d1['stats'], 77, 2)
    m.eval()
    m.set_target_bandwidth(1.5)
    lm = g12_lm_module(G12_LM['a'])
    m.get_lm_model = lambda: lm
    x = t(d1['x'])[0][:, :4800]
    rec_p, rec_c = [], []
    orig = ref_compress.build_stable_quantized_cdf

    def recorder(pdf, bits, **kw):
        q = orig(pdf, bits, **kw)
        rec_p.append(pdf.numpy().copy())
        rec_c.append(q.numpy().copy())
        return q
    ref_compress.build_stable_quantized_cdf = recorder
    try:
        data = ref_compress.compress(m, x, use_lm=True)
        n_enc = len(rec_p)
        with torch.no_grad():
            y, _ = ref_compress.decompress_from_file(m, io.BytesIO(data), device='cpu')
        assert [a.tolist() for a in rec_c[n_enc:]] == [a.tolist() for a in rec_c[:n_enc]]
    finally:
        ref_compress.build_stable_quantized_cdf = orig
    with torch.no_grad():
        codes = m.encode(x[None])[0][0]
    out['e2e_x'] = x.numpy()
    out['e2e_bytes'] = np.frombuffer(data, np.uint8)
    out['e2e_codes'] = codes.numpy()
    out['e2e_pdf'] = np.stack(rec_p[:n_enc]).astype(np.float32)
    out['e2e_cdf'] = np.stack(rec_c[:n_enc]).astype(np.int32)
    out['e2e_y'] = y.numpy()
    save('g12_lm.npz', **out)


# ------------------------------------------------------------------------------------ G13
# The reference's OWN data-parallel step: train_multi_gpu.train_one_step (:32-142) on models
# wrapped as train() wraps them (DDP, broadcast_buffers=False, :310-325), 2 ranks over gloo on
# the CPU, one batch of G13_B clips per rank, bandwidth fixed (n_q 2), the discriminator trained
# (p = 1). Recorded per rank, by wrapping (not editing) the reference's objects:
#   g_bal  : the generator grads right after balancer.backward (DDP-averaged, equal on both ranks)
#   commit : the grads loss_w.backward() (:94) then adds (rank-local under DDP)
#   disc   : the discriminator grads at optimizer_disc.step (DDP-averaged)
#   the losses, the post-Adam parameters and codebook buffers (sync off: each rank's own EMA)
# Generator tensors are stored as per-tensor sums / abs-sums / squared sums plus G13_S evenly
# spaced elements of every parameter (the 14.85 M-element vectors themselves are 59 MB each).
G13_B, G13_T = 2, 4800
from fixtures import g13_samples  # noqa: E402  (64 evenly spaced elements per tensor)


def _g13_rank(rank, world, port, outdir):
    import random
    import types as _types
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(4)
    # off-path imports of train_multi_gpu.py absent from this image: hydra (the CLI decorator),
    # tensorboard (the logging writer; a no-op one is passed in), audioread (datasets)
    for name in ('hydra', 'audioread', 'torch.utils.tensorboard'):
        mod = _types.ModuleType(name)
        mod.main = lambda **kw: (lambda f: f)
        mod.SummaryWriter = object
        sys.modules.setdefault(name, mod)
    import train_multi_gpu as tmg
    torch.manual_seed(0)
    random.seed(0)
    m = R.model.EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm',
                                        audio_normalize=True, segment=None, name='x')
    load_synth(m, 71)
    stats = np.load(os.path.join(HERE, 'g7_step.npz'))['gan/stats']
    fill_codebooks(m, stats, 73, 2)
    d = R.msstftd.MultiScaleSTFTDiscriminator(filters=32)
    load_synth(d, 74)
    x = t(synth_wave((world * G13_B, 1, G13_T), 131))[rank * G13_B:(rank + 1) * G13_B]
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    gparams = [p for p in m.parameters() if p.requires_grad]
    rec = {}

    def snap(ps):
        return [p.grad.detach().clone() for p in ps]

    class RecBalancer(R.balancer.Balancer):
        def backward(self, losses, input, retain_graph=False):
            super().backward(losses, input, retain_graph=retain_graph)
            rec['g_bal'] = snap(gparams)
            rec['losses'] = {k: float(v) for k, v in losses.items()}

    class RecAdam(torch.optim.Adam):
        def __init__(self, *a, tag, **kw):
            super().__init__(*a, **kw)
            self.tag = tag

        def step(self, closure=None):
            rec[self.tag] = snap([p for grp in self.param_groups for p in grp['params']])
            return super().step(closure)

    model = torch.nn.parallel.DistributedDataParallel(m, broadcast_buffers=False, find_unused_parameters=False)
    disc = torch.nn.parallel.DistributedDataParallel(d, broadcast_buffers=False, find_unused_parameters=False)
    opt = RecAdam([{'params': gparams, 'lr': 3e-4}], betas=(0.5, 0.9), tag='g_total')
    optd = RecAdam([{'params': [p for p in d.parameters() if p.requires_grad], 'lr': 3e-4}], betas=(0.5, 0.9),
                   tag='g_disc')
    sched = R.scheduler.WarmupCosineLrScheduler(opt, max_iter=100, eta_ratio=0.1, warmup_iter=0, warmup_ratio=1e-4)
    dsched = R.scheduler.WarmupCosineLrScheduler(optd, max_iter=100, eta_ratio=0.1, warmup_iter=0, warmup_ratio=1e-4)
    ns = _types.SimpleNamespace
    config = ns(common=ns(amp=False, log_interval=1), model=ns(train_discriminator='1.0', sample_rate=24000),
                lr_scheduler=ns(warmup_epoch=0), distributed=ns(data_parallel=True))
    writer = ns(add_scalar=lambda *a, **kw: None)
    bal = RecBalancer({'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3})
    tmg.train_one_step(1, opt, optd, model, disc, [x], config, sched, dsched, writer=writer, balancer=bal)
    out = {}
    for i, (k, p) in enumerate(zip(names, gparams)):
        idx = g13_samples(p.numel())
        for tag, v in (('bal', rec['g_bal'][i]), ('commit', rec['g_total'][i] - rec['g_bal'][i]),
                       ('total', rec['g_total'][i]), ('param', p.detach())):
            v = v.double().reshape(-1)
            out[f'{tag}/{k}'] = v[torch.from_numpy(idx)].numpy()
            out[f'{tag}_sum/{k}'] = np.array([v.sum().item(), v.abs().sum().item(), v.pow(2).sum().item()])
    out['disc_grad'] = torch.cat([g.reshape(-1) for g in rec['g_disc']]).numpy()
    for k, p in d.named_parameters():
        if p.requires_grad:
            out[f'dparam/{k}'] = p.detach().reshape(-1)[torch.from_numpy(g13_samples(p.numel()))].numpy()
    for k, v in rec['losses'].items():
        out[f'loss/{k}'] = np.array(v)
    sd = m.state_dict()
    for i in range(2):
        pre = f'quantizer.vq.layers.{i}._codebook.'
        out[f'cb{i}/cluster_size'] = sd[pre + 'cluster_size'].numpy()
        out[f'cb{i}/embed_avg_rows'] = sd[pre + 'embed_avg'][::16].numpy()
        out[f'cb{i}/embed_rows'] = sd[pre + 'embed'][::16].numpy()
    np.savez(os.path.join(outdir, f'r{rank}.npz'), **out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def g13():
    import socket
    import tempfile
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    outdir = tempfile.mkdtemp(prefix='g13_')
    mp.spawn(_g13_rank, args=(2, port, outdir), nprocs=2, join=True)
    r = [dict(np.load(os.path.join(outdir, f'r{i}.npz'))) for i in range(2)]
    for k in r[0]:
        if k.startswith(('bal', 'disc_grad', 'dparam')):  # DDP-averaged: one value for both ranks
            assert np.array_equal(r[0][k], r[1][k]), k
    out = {'stats': np.load(os.path.join(HERE, 'g7_step.npz'))['gan/stats']}
    for k, v in r[0].items():
        if k.startswith(('bal', 'disc_grad', 'dparam')):
            out[k] = v
        else:
            out['r0/' + k] = v
            out['r1/' + k] = r[1][k]
    save('g13_ddp.npz', **out)


if __name__ == '__main__':
    which = sys.argv[1:] or ['g1', 'g2', 'g3', 'g4', 'g5', 'g6', 'g7', 'g8', 'g9', 'g10', 'g11', 'g12', 'g13']
    for w in which:
        torch.manual_seed(0)
        globals()[w]()
