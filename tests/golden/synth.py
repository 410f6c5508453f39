"""Deterministic synthetic weights / inputs shared by the golden generator and the tests.

Test infrastructure only. The reference's pretrained weights are remote-only
(`/root/reference/model.py:289`), so every fixture is produced from parameters that both
sides regenerate bit-identically from a numpy PCG64 seed: no weight file is committed.

Scales follow torch's default init (U(+-1/sqrt(fan_in))) and torch.nn.utils.weight_norm's
initialisation (g = ||v|| over dims != 0, `torch/nn/utils/weight_norm.py`), so activations
behave like a freshly built reference model.
"""
import numpy as np


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def _fan_in(shape):
    if len(shape) < 2:
        return shape[0]
    f = shape[1]
    for s in shape[2:]:
        f *= s
    return f


def synth_state(named_shapes, seed, lstm_hidden=None):
    """named_shapes: dict name -> shape of float parameters. Returns name -> float32 ndarray.

    Parameters are generated in sorted-name order; every `*.weight_g` is set to the row norm
    of its sibling `*.weight_v` so w == v at init, exactly like weight_norm's own init.
    """
    g = rng(seed)
    out = {}
    names = sorted(named_shapes)
    for name in names:
        if name.endswith('weight_g'):
            continue
        shape = tuple(named_shapes[name])
        if 'lstm' in name:
            h = lstm_hidden or shape[-1]
            bound = 1.0 / np.sqrt(h)
        elif name.endswith('bias'):
            wname = name[:-4] + ('weight_v' if (name[:-4] + 'weight_v') in named_shapes else 'weight')
            wshape = named_shapes.get(wname, shape)
            bound = 1.0 / np.sqrt(_fan_in(wshape))
        else:
            bound = 1.0 / np.sqrt(_fan_in(shape))
        out[name] = g.uniform(-bound, bound, size=shape).astype(np.float32)
    for name in names:
        if not name.endswith('weight_g'):
            continue
        v = out[name[:-1] + 'v'].astype(np.float64)
        n = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(1))
        out[name] = n.reshape(named_shapes[name]).astype(np.float32)
    return out


def synth_wave(shape, seed, amp=0.1):
    """x = amp * N(0,1) fp32 (SURVEY.md §8d synthetic inputs)."""
    return (amp * rng(seed).standard_normal(size=shape)).astype(np.float32)


def synth_codebooks(stats, seed):
    """Rebuild codebooks from stored per-dimension (mean, std) of each layer's residual.

    stats: float32 [n_q, 2, D]. Returns float32 [n_q, K=1024, D].
    """
    g = rng(seed)
    n_q, _, d = stats.shape
    cb = np.empty((n_q, 1024, d), np.float32)
    for i in range(n_q):
        z = g.standard_normal(size=(1024, d))
        cb[i] = (stats[i, 0][None, :].astype(np.float64)
                 + stats[i, 1][None, :].astype(np.float64) * z).astype(np.float32)
    return cb


def synth_lm_state(named_shapes, seed, sharp=6.0):
    """Synthetic LMModel weights (model.py:27-45; the pretrained LM is remote-only,
    model.py:221-240): synth_state, then LayerNorm gains 1 + u (instead of u) and the
    per-codebook output projections scaled by `sharp` so the softmax is peaked like a trained
    model's (the entropy coder then sees both near-certain and rare symbols)."""
    out = synth_state(named_shapes, seed)
    for k in list(out):
        if k.endswith('weight') and ('norm' in k):
            out[k] = (1.0 + out[k].astype(np.float64)).astype(np.float32)
        elif k.startswith('linears.') and k.endswith('weight'):
            out[k] = (out[k] * np.float32(sharp)).astype(np.float32)
    return out
