"""CPU ORACLE for the EnCodec entropy-coding language model -- TEST INFRASTRUCTURE ONLY.

Only `tests/` may import this module, as the checker. The product (`encx.lm`) never imports
it; the LM runs in csrc/lm.hip and fails loudly without the HIP library.

A functional torch-CPU restatement of LMModel (model.py:27-65) over
StreamingTransformerEncoder (modules/transformer.py:62-119), post-norm layers
(`norm_first=False`, transformer.py:31-41) with windowed self-attention (:44-59):

  * `lm_step`: the reference's streaming call `lm(indices, states, offset)` exactly as
    compress.py:76-78 makes it (states = list of per-layer past inputs, a zero vector at first);
  * `lm_all`: the same probabilities for all T steps of a known code sequence in one pass. Row
    t's query attends sequence positions [max(0, s - P), s], s = t + 1, of [phantom zero input,
    x_0, x_1, ...]: the zero state the reference starts every layer with (transformer.py:106) is
    a real key/value (k = in_proj bias, v = its bias), and each layer keeps the last P =
    past_context inputs (:117-118). tests/test_oracle.py checks lm_all == lm_step.

Parity pinning: tests/test_oracle.py checks both against tests/golden/g12_lm.npz, whose
probabilities make_goldens.py (g12) took from the reference's own LMModel with synthetic
weights (the pretrained LM is remote-only, model.py:221-240).
"""
import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass
class LMConfig:
    n_q: int = 32
    card: int = 1024
    dim: int = 200
    num_heads: int = 8
    num_layers: int = 5
    hidden_scale: float = 4.0
    past_context: int = 262        # int(3.5 * frame_rate), model.py:225
    max_period: float = 10000.0

    @property
    def hidden(self):
        return int(self.dim * self.hidden_scale)


def lm_param_shapes(cfg: LMConfig):
    """state-dict keys / shapes of LMModel (model.py:38-45, transformer.py:88-99,
    torch.nn.TransformerEncoderLayer / MultiheadAttention)."""
    D, Fh = cfg.dim, cfg.hidden
    s = {'transformer.norm_in.weight': (D,), 'transformer.norm_in.bias': (D,)}
    for i in range(cfg.num_layers):
        p = f'transformer.layers.{i}.'
        s.update({p + 'self_attn.in_proj_weight': (3 * D, D), p + 'self_attn.in_proj_bias': (3 * D,),
                  p + 'self_attn.out_proj.weight': (D, D), p + 'self_attn.out_proj.bias': (D,),
                  p + 'linear1.weight': (Fh, D), p + 'linear1.bias': (Fh,),
                  p + 'linear2.weight': (D, Fh), p + 'linear2.bias': (D,),
                  p + 'norm1.weight': (D,), p + 'norm1.bias': (D,),
                  p + 'norm2.weight': (D,), p + 'norm2.bias': (D,)})
    for k in range(cfg.n_q):
        s[f'emb.{k}.weight'] = (cfg.card + 1, D)
        s[f'linears.{k}.weight'] = (cfg.card, D)
        s[f'linears.{k}.bias'] = (cfg.card,)
    return s


def sin_embedding(positions, dim, max_period):
    """create_sin_embedding (transformer.py:16-27)."""
    half = dim // 2
    adim = torch.arange(half).view(1, 1, -1)
    phase = positions / (max_period ** (adim / (half - 1)))
    return torch.cat([torch.cos(phase), torch.sin(phase)], dim=-1)


def _attn(st, p, q_in, kv_in, mask, cfg):
    """nn.MultiheadAttention forward (batch_first, need_weights=False) with a boolean mask
    (True = blocked), as _sa_block calls it (transformer.py:44-59)."""
    D, H = cfg.dim, cfg.num_heads
    hd = D // H
    W, b = st[p + 'self_attn.in_proj_weight'], st[p + 'self_attn.in_proj_bias']
    q = F.linear(q_in, W[:D], b[:D])
    k = F.linear(kv_in, W[D:2 * D], b[D:2 * D])
    v = F.linear(kv_in, W[2 * D:], b[2 * D:])
    B, Tq, _ = q.shape
    Tk = k.shape[1]
    q = q.view(B, Tq, H, hd).transpose(1, 2)
    k = k.view(B, Tk, H, hd).transpose(1, 2)
    v = v.view(B, Tk, H, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    s = s.masked_fill(mask, float('-inf'))
    o = torch.softmax(s, dim=-1) @ v
    o = o.transpose(1, 2).reshape(B, Tq, D)
    return F.linear(o, st[p + 'self_attn.out_proj.weight'], st[p + 'self_attn.out_proj.bias'])


def _layer(st, i, x, keys_in, mask, cfg):
    """StreamingTransformerEncoderLayer.forward, norm_first=False (transformer.py:31-41)."""
    p = f'transformer.layers.{i}.'
    D = cfg.dim
    x = F.layer_norm(x + _attn(st, p, x, keys_in, mask, cfg), (D,),
                     st[p + 'norm1.weight'], st[p + 'norm1.bias'])
    ff = F.linear(F.gelu(F.linear(x, st[p + 'linear1.weight'], st[p + 'linear1.bias'])),
                  st[p + 'linear2.weight'], st[p + 'linear2.bias'])
    return F.layer_norm(x + ff, (D,), st[p + 'norm2.weight'], st[p + 'norm2.bias'])


def _input(st, indices, offset, cfg):
    """LMModel.forward input sum (model.py:59-60) + norm_in + position (transformer.py:104-113)."""
    B, K, T = indices.shape
    x = sum([F.embedding(indices[:, k], st[f'emb.{k}.weight']) for k in range(K)])
    x = F.layer_norm(x, (cfg.dim,), st['transformer.norm_in.weight'], st['transformer.norm_in.bias'])
    pos = torch.arange(T).view(1, -1, 1) + offset
    return x + sin_embedding(pos, cfg.dim, cfg.max_period)


def _heads(st, out, K, cfg):
    """model.py:62-64 -> probabilities [B, card, K, T]."""
    logits = torch.stack([F.linear(out, st[f'linears.{k}.weight'], st[f'linears.{k}.bias'])
                          for k in range(K)], dim=1).permute(0, 3, 1, 2)
    return torch.softmax(logits, dim=1)


@torch.no_grad()
def lm_step(st, indices, states, offset, cfg: LMConfig):
    """lm(indices, states, offset) (model.py:47-65): -> (probas [B, card, K, T], states, offset)."""
    B, K, T = indices.shape
    x = _input(st, indices, offset, cfg)
    if states is None:
        states = [torch.zeros_like(x[:, :1]) for _ in range(1 + cfg.num_layers)]
    new_states = []
    for i in range(cfg.num_layers):
        past = states[i]
        Hp = past.shape[1]
        qpos = torch.arange(Hp, T + Hp).view(-1, 1)
        kpos = torch.arange(T + Hp).view(1, -1)
        delta = qpos - kpos
        valid = (delta >= 0) & (delta <= cfg.past_context)
        sa_input = x
        x = _layer(st, i, x, torch.cat([past, x], dim=1), ~valid, cfg)
        new_states.append(torch.cat([past, sa_input], dim=1)[:, -cfg.past_context:, :])
    return _heads(st, x, K, cfg), new_states, offset + T


@torch.no_grad()
def lm_all(st, codes, cfg: LMConfig):
    """Probabilities of every step of compress.py:74-86's loop in one pass: step t's input is
    1 + codes[:, :, t-1] (0 at t = 0). codes: int64 [B, K, T] -> probas [B, card, K, T]."""
    B, K, T = codes.shape
    inp = torch.zeros_like(codes)
    inp[:, :, 1:] = codes[:, :, :-1] + 1
    x = _input(st, inp, 0, cfg)
    P = cfg.past_context
    s = torch.arange(1, T + 1).view(-1, 1)           # query sequence positions
    j = torch.arange(T + 1).view(1, -1)              # key positions, 0 = phantom zero input
    valid = (j <= s) & (j >= s - P)
    for i in range(cfg.num_layers):
        keys_in = torch.cat([torch.zeros_like(x[:, :1]), x], dim=1)
        x = _layer(st, i, x, keys_in, ~valid, cfg)
    return _heads(st, x, K, cfg)


def compress_lm_symbols(st, codes, cfg: LMConfig, total_range_bits=24):
    """The (symbol, quantized cdf) sequence compress.py:74-89 pushes for one frame [1, K, T]
    with the streaming LM, in push order (t-major, then codebook)."""
    from oracle.ac_oracle import quantized_cdf
    _, K, T = codes.shape
    states, offset = None, 0
    inp = torch.zeros(1, K, 1, dtype=torch.long)
    syms, cdfs = [], []
    for t in range(T):
        probas, states, offset = lm_step(st, inp, states, offset, cfg)
        inp = 1 + codes[:, :, t:t + 1]
        for k in range(K):
            cdfs.append(quantized_cdf(probas[0, :, k, 0].numpy(), total_range_bits, check=False))
            syms.append(int(codes[0, k, t]))
    return syms, cdfs
