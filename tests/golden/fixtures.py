"""Loaders that rebuild the exact synthetic states behind each golden fixture.

Test infrastructure. Mirrors the synthesis in make_goldens.py (same seeds, same sorted
generation order) without touching /root/reference, so it works on the GPU box too.
"""
import os

import numpy as np
import torch

from synth import synth_state, synth_wave, synth_codebooks, rng

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def model_state(cfg, seed):
    from oracle.encodec_oracle import model_param_shapes
    return {k: T(v) for k, v in synth_state(model_param_shapes(cfg), seed).items()}


def disc_state(seed, in_channels=1, out_channels=1):
    from oracle.encodec_oracle import disc_param_shapes
    shapes = disc_param_shapes(in_channels=in_channels, out_channels=out_channels)
    return {k: T(v) for k, v in synth_state(shapes, seed).items()}


def cfg48k(**kw):
    """The g9 fixture's model: config 5's 48 kHz stereo SEANet (scripts/train.sbatch:18-30:
    non-causal, time_group_norm) with segment 0.1 s instead of 1 s (same two-frame shape)."""
    from oracle.encodec_oracle import Config
    return Config(sample_rate=48000, channels=2, causal=False, norm='time_group_norm',
                  target_bandwidths=kw.pop('target_bandwidths', (3.0,)), audio_normalize=True,
                  segment=kw.pop('segment', 0.1), **kw)


def codebooks_from_stats(stats, seed, n_used, n_total):
    """Same draws as make_goldens.fill_codebooks."""
    cbs = synth_codebooks(stats, seed)
    g = rng(seed + 1)
    out = []
    for i in range(n_total):
        if i < n_used:
            cs = g.uniform(0.5, 4.0, size=(1024,)).astype(np.float32)
            out.append({'inited': torch.ones(1), 'cluster_size': T(cs), 'embed': T(cbs[i]),
                        'embed_avg': T((cbs[i] * cs[:, None]).astype(np.float32))})
        else:
            out.append({'inited': torch.ones(1), 'cluster_size': torch.zeros(1024),
                        'embed': torch.zeros(1024, 128), 'embed_avg': torch.zeros(1024, 128)})
    return out


def g3_codebooks(d):
    stats = d['stats']
    cbs = synth_codebooks(stats, 32)
    return [{'inited': torch.ones(1), 'cluster_size': T(d[f'cs_init{i}']), 'embed': T(cbs[i]),
             'embed_avg': T(d[f'ea_init{i}'])} for i in range(2)]


def certified(gaps, x_norm2, e_norm2, factor=256):
    """Rows whose fp64 top-2 distance gap exceeds fp32 rounding of the expanded distance
    (factor * eps32 * (|x|^2 + |e|^2)): there the argmin is decided, and codes must match
    bit-exactly. Returns a bool mask."""
    eps = np.finfo(np.float32).eps
    return gaps > factor * eps * (x_norm2 + e_norm2)


def rvq_certified(emb, embeds, factor=256):
    """Eval-mode RVQ (core_vq.py:357-367) of emb [B, D, T] in fp64 -> (codes [n_q, B, T] int64,
    cert [n_q, B, T] bool). A frame's code at layer l is certified when its fp64 top-2 distance
    gap clears fp32 rounding (certified()) AND every earlier layer's code of that frame is
    certified (otherwise its residual may differ). Where cert holds, an fp32 implementation
    fed the same emb must produce exactly these codes. factor 256 = 2 x the worst-case
    rounding bound of a 128-term fp32 dot product (n eps (|x| + |e|)^2 per distance) -- a proof;
    smaller factors (e.g. 32, about 3 sigma of random-walk rounding) certify far more frames
    of the synthetic codebooks and are used as a second, statistical check."""
    x = torch.as_tensor(emb).detach().cpu().double().permute(0, 2, 1)  # [B, T, D]
    B, Tn, D = x.shape
    r = x.reshape(-1, D).clone()
    ok = torch.ones(B * Tn, dtype=torch.bool)
    codes, certs = [], []
    for E in embeds:
        E = torch.as_tensor(E).detach().cpu().double()
        dist = (r ** 2).sum(1, keepdim=True) - 2 * r @ E.t() + (E ** 2).sum(1)[None]
        s, idx = torch.sort(dist, 1)
        gap = (s[:, 1] - s[:, 0]).numpy()
        c = certified(gap, (r ** 2).sum(1).numpy(), float((E ** 2).sum(1).max()), factor)
        ok = ok & torch.from_numpy(c)
        k = idx[:, 0]
        codes.append(k.view(B, Tn))
        certs.append(ok.view(B, Tn).clone())
        r = r - E[k]
    return torch.stack(codes), torch.stack(certs)


def g13_samples(n, count=64):
    """The evenly spaced element indices of an n-element tensor that g13_ddp.npz stores."""
    return np.unique(np.linspace(0, n - 1, min(n, count)).round().astype(np.int64))


__all__ = ['load', 'g13_samples', 'T', 'model_state', 'disc_state', 'cfg48k', 'codebooks_from_stats', 'g3_codebooks',
           'certified', 'rvq_certified', 'synth_wave', 'rng']


# ---------------------------------------------------------------- g12: LM entropy coder
def g12_lm_config(name):
    """The LMConfig + synthetic state of make_goldens.G12_LM[name] (same seeds)."""
    from oracle.lm_oracle import LMConfig, lm_param_shapes
    from synth import synth_lm_state
    c = {'a': dict(n_q=32, card=1024, dim=200, num_heads=8, num_layers=5, past_context=262, seed=121),
         'b': dict(n_q=4, card=64, dim=64, num_heads=4, num_layers=2, past_context=5, seed=122)}[name]
    seed = c.pop('seed')
    cfg = LMConfig(**c)
    st = {k: T(v) for k, v in synth_lm_state(lm_param_shapes(cfg), seed).items()}
    return cfg, st


def g12_ac_rows(d):
    """-> list of (card, bits, pdfs [steps][card], cdfs [steps][card], syms [steps], data bytes,
    eof flag) per coder case of g12_lm.npz."""
    out, po, so, bo = [], 0, 0, 0
    for i, (card, steps, bits, uni) in enumerate(d['ac_cases']):
        n = int(card) * int(steps)
        pdf = d['ac_pdf'][po:po + n].reshape(steps, card)
        cdf = d['ac_cdf'][po:po + n].reshape(steps, card).astype(np.int64)
        sym = d['ac_sym'][so:so + steps]
        nb = int(d['ac_nbytes'][i])
        data = d['ac_bytes'][bo:bo + nb].tobytes()
        out.append((int(card), int(bits), pdf, cdf, sym, data, int(d['ac_eof'][i])))
        po, so, bo = po + n, so + int(steps), bo + nb
    return out
