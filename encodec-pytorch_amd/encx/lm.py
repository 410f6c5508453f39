"""LMModel of the reference (model.py:27-65) over StreamingTransformerEncoder
(modules/transformer.py:62-119), on the encx HIP kernels (csrc/lm.hip, csrc/ac.hip).

The module tree (and so the state dict) is the reference's: `transformer.norm_in`,
`transformer.layers.{i}.self_attn.{in_proj_weight,in_proj_bias,out_proj}`, `linear1`,
`linear2`, `norm1`, `norm2`, `emb.{k}`, `linears.{k}`; torch modules serve only as parameter
holders and no torch arithmetic runs. `forward(indices, states, offset)` keeps the reference's
streaming contract; `states` is an opaque `LMState` (each layer's key/value cache) instead of
the list of past layer inputs, and is passed back the same way.

`encode_streams` / `decode_streams` are the entropy coder of compress.py:67-89 / 128-155 for a
batch of equal-shape frames: the encoder runs all T steps of a frame as one pass (every code
is known), the decoder one step per launch sequence; csrc/lm.hip computes every row in a
fixed order that does not depend on the rows sharing the launch, so both sides produce the
same cdfs bit for bit.
"""
import typing as tp

import torch
from torch import nn

from ._lib import call, lib, stream, ensure_device, ENCX_AC_POS
from .ac import new_decoder_state

TOTAL_RANGE_BITS = 24   # ArithmeticCoder default (ac.py:96), as compress.py uses it
ROUNDOFF = 1e-8         # build_stable_quantized_cdf defaults (ac.py:18-20)
MIN_RANGE = 2


class StreamingTransformerEncoderLayer(nn.Module):
    """Parameter holder with nn.TransformerEncoderLayer's names (transformer.py:30)."""

    def __init__(self, d_model, nhead, dim_feedforward):
        super().__init__()
        self.self_attn = nn.MultiheadAttention(d_model, nhead, batch_first=True)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)


class StreamingTransformerEncoder(nn.Module):
    """transformer.py:62-99 (post-norm layers, GELU, LayerNorm input, no dropout)."""

    def __init__(self, dim, hidden_scale: float = 4., num_heads: int = 8, num_layers: int = 5,
                 max_period: float = 10000, past_context: int = 1000, gelu: bool = True,
                 norm_in: bool = True, dropout: float = 0., **kwargs):
        super().__init__()
        assert dim % num_heads == 0
        if not gelu or not norm_in or dropout or kwargs:
            raise NotImplementedError('encx LM: GELU, norm_in and dropout 0 only (the configuration '
                                      'EncodecModel.get_lm_model builds, model.py:224-225)')
        self.dim, self.num_heads = dim, num_heads
        self.hidden = int(dim * hidden_scale)
        self.max_period = max_period
        self.past_context = past_context
        self.norm_in = nn.LayerNorm(dim)
        self.layers = nn.ModuleList([StreamingTransformerEncoderLayer(dim, num_heads, self.hidden)
                                     for _ in range(num_layers)])


class LMState:
    """Streaming state: per layer a key/value cache [B][capacity][2*dim] of sequence positions
    0 (the zero initial state, transformer.py:106) .. offset, and the step offset."""

    def __init__(self, B, num_layers, dim, capacity, device):
        self.B, self.dim = B, dim
        self.kv = [torch.empty(B, capacity, 2 * dim, device=device) for _ in range(num_layers)]
        self.offset = 0

    @property
    def capacity(self):
        return self.kv[0].shape[1]

    def reserve(self, n):
        if n > self.capacity:
            cap = max(n, 2 * self.capacity)
            for i, kv in enumerate(self.kv):
                nkv = torch.empty(self.B, cap, 2 * self.dim, device=kv.device)
                nkv[:, :self.offset + 1] = kv[:, :self.offset + 1]
                self.kv[i] = nkv


class LMModel(nn.Module):
    """model.py:27-45."""

    def __init__(self, n_q: int = 32, card: int = 1024, dim: int = 200, **kwargs):
        super().__init__()
        self.card = card
        self.n_q = n_q
        self.dim = dim
        self.transformer = StreamingTransformerEncoder(dim=dim, **kwargs)
        self.emb = nn.ModuleList([nn.Embedding(card + 1, dim) for _ in range(n_q)])
        self.linears = nn.ModuleList([nn.Linear(dim, card) for _ in range(n_q)])
        self._packed_key = None

    # ------------------------------------------------------------------ weights
    def _packed(self):
        """The K embedding tables and output heads stacked into contiguous [n_q][.][dim]
        buffers (rebuilt only when a parameter changes)."""
        ps = [e.weight for e in self.emb] + [l.weight for l in self.linears] + [l.bias for l in self.linears]
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if key != self._packed_key:
            with torch.no_grad():
                self._emb = torch.stack([e.weight for e in self.emb]).contiguous()
                self._lin_w = torch.stack([l.weight for l in self.linears]).contiguous()
                self._lin_b = torch.stack([l.bias for l in self.linears]).contiguous()
            self._packed_key = key
        return self._emb, self._lin_w, self._lin_b

    def _check_device(self):
        p = self._emb
        if not p.is_cuda or p.dtype != torch.float32:
            raise RuntimeError('encx LM: parameters must be float32 on the GPU (no CPU fallback)')
        ensure_device(p.device)
        for t in self.parameters():
            if not t.is_contiguous():
                raise RuntimeError('encx LM: parameters must be contiguous')

    def new_state(self, B, capacity=64):
        tr = self.transformer
        return LMState(B, len(tr.layers), self.dim, max(int(capacity), 2), self._emb.device)

    # ------------------------------------------------------------------ core
    def _body(self, idx, strides, B, K, T, shifted, state: LMState, dev_step=None):
        """input + transformer over rows [B][T] continuing `state` -> x [B*T][dim]. With
        dev_step (an int64 device counter) the step offset is read on the device and the host
        offset stays put (a graph-captured decode step; the caller reserved the cache)."""
        tr = self.transformer
        D, Fh = self.dim, tr.hidden
        dev = self._emb.device
        st = stream()
        dptr = dev_step.data_ptr() if dev_step is not None else None
        if dev_step is None:
            state.reserve(state.offset + T + 1)
        x = torch.empty(B * T, D, device=dev)
        call('encx_lm_input', idx.data_ptr(), strides[0], strides[1], strides[2], B, K, T, int(shifted),
             self._emb.data_ptr(), self.card + 1, D, tr.norm_in.weight.data_ptr(), tr.norm_in.bias.data_ptr(),
             state.offset, dptr, float(tr.max_period), x.data_ptr(), st)
        work = torch.empty((int(lib.encx_lm_layer_workspace(B * T, D, Fh)) + 3) // 4, device=dev)
        for i, layer in enumerate(tr.layers):
            y = torch.empty_like(x)
            a = layer.self_attn
            call('encx_lm_layer', x.data_ptr(), y.data_ptr(), B, T, state.kv[i].data_ptr(), state.capacity,
                 state.offset + 1, dptr, tr.past_context, D, tr.num_heads, Fh,
                 a.in_proj_weight.data_ptr(), a.in_proj_bias.data_ptr(),
                 a.out_proj.weight.data_ptr(), a.out_proj.bias.data_ptr(),
                 layer.linear1.weight.data_ptr(), layer.linear1.bias.data_ptr(),
                 layer.linear2.weight.data_ptr(), layer.linear2.bias.data_ptr(),
                 layer.norm1.weight.data_ptr(), layer.norm1.bias.data_ptr(),
                 layer.norm2.weight.data_ptr(), layer.norm2.bias.data_ptr(), work.data_ptr(), st)
            x = y
        if dev_step is None:
            state.offset += T
        return x

    def _heads(self, x, B, T, K, probas=None, cdf=None, sym=None, lohi=None, err=None):
        dev = x.device
        work = torch.empty((int(lib.encx_lm_heads_workspace(B * T, K, self.card)) + 3) // 4, device=dev)
        s = sym.stride() if sym is not None else (0, 0, 0)
        call('encx_lm_heads', x.data_ptr(), B, T, self.dim, self._lin_w.data_ptr(), self._lin_b.data_ptr(),
             K, self.card, work.data_ptr(), probas.data_ptr() if probas is not None else None,
             cdf.data_ptr() if cdf is not None else None, TOTAL_RANGE_BITS, ROUNDOFF, MIN_RANGE,
             sym.data_ptr() if sym is not None else None, s[0], s[1], s[2],
             lohi.data_ptr() if lohi is not None else None, err.data_ptr() if err is not None else None,
             stream())

    @torch.no_grad()
    def forward(self, indices: torch.Tensor, states: tp.Optional[LMState] = None, offset: int = 0):
        """model.py:47-65: indices [B, n_q, T] (1 + code, 0 = missing) -> (probabilities
        [B, card, n_q, T], states, offset + T)."""
        self._packed()
        self._check_device()
        if indices.dtype != torch.int64 or indices.dim() != 3 or not indices.is_cuda:
            raise RuntimeError('encx LM: indices must be int64 [B, K, T] on the GPU')
        B, K, T = indices.shape
        if K > self.n_q:
            raise ValueError(f'{K} codebooks for an LM of n_q={self.n_q}')
        if states is None:
            states = self.new_state(B, T + 1)
            states.offset = int(offset)
            if states.offset:
                raise ValueError('encx LM: a fresh state starts at offset 0')
        elif states.offset != int(offset):
            raise ValueError(f'encx LM: offset {offset} does not continue the state (at {states.offset})')
        x = self._body(indices, indices.stride(), B, K, T, False, states)
        probas = torch.empty(B, T, K, self.card, device=x.device)
        self._heads(x, B, T, K, probas=probas)
        return probas.permute(0, 3, 2, 1), states, states.offset

    # ------------------------------------------------------------------ entropy coder
    @torch.no_grad()
    def encode_streams(self, codes: torch.Tensor) -> tp.List[bytes]:
        """compress.py:67-89 (use_lm=True) for B frames [B, K, T] of codes: the arithmetic
        coded payload of each frame. One LM pass over all T steps, the coding intervals from the
        fused softmax + cdf kernel, then one coder thread per stream."""
        self._packed()
        self._check_device()
        if codes.dtype != torch.int64 or codes.dim() != 3 or not codes.is_cuda:
            raise RuntimeError('encx LM: codes must be int64 [B, K, T] on the GPU')
        B, K, T = codes.shape
        if K > self.n_q:
            raise ValueError(f'{K} codebooks for an LM of n_q={self.n_q}')
        dev = codes.device
        state = self.new_state(B, T + 1)
        x = self._body(codes, codes.stride(), B, K, T, True, state)
        lohi = torch.empty(B, T, K, 2, device=dev, dtype=torch.int32)
        err = torch.zeros(1, device=dev, dtype=torch.int32)
        self._heads(x, B, T, K, sym=codes, lohi=lohi, err=err,
                    cdf=torch.empty(B, T, K, self.card, device=dev, dtype=torch.int32))
        cap = int(lib.encx_ac_encode_capacity(T * K, TOTAL_RANGE_BITS))
        out = torch.empty(B, cap, device=dev, dtype=torch.uint8)
        nbytes = torch.empty(B, device=dev, dtype=torch.int64)
        serr = torch.empty(B, device=dev, dtype=torch.int32)
        call('encx_ac_encode', lohi.data_ptr(), B, T * K, TOTAL_RANGE_BITS, out.data_ptr(), cap,
             nbytes.data_ptr(), serr.data_ptr(), stream())
        host, nb, e, e0 = out.cpu(), nbytes.cpu().tolist(), serr.cpu().tolist(), int(err.item())
        if e0 & 2:
            raise ValueError(f'a code is outside [0, {self.card})')
        if e0 & 1 or any(v == 1 for v in e):
            raise AssertionError('quantized cdf total above 2^total_range_bits (ac.py:50, 116)')
        if any(e):
            raise RuntimeError(f'encx arithmetic coder failed: {e}')
        return [host[b, :nb[b]].numpy().tobytes() for b in range(B)]

    @torch.no_grad()
    def decode_streams(self, datas: tp.Sequence[bytes], K: int, T: int, graph: bool = True,
                       dev_span=None):
        """compress.py:128-155 (use_lm=True) for B streams of K codebooks x T steps: ->
        (codes int64 [B, K, T] on the GPU, bytes consumed per stream). Raises EOFError where
        the reference's decoder runs dry, RuntimeError where its binary search fails.

        One step = LM input, 5 layers, heads + cdf, arithmetic decode of the K codes (whose
        + 1 is the next step's input, compress.py:154-155). With graph=True the step's ~40
        launches are captured once into a HIP graph (offsets from a device-side step counter)
        and replayed T times, with one host sync at the end.
        dev_span = (uint8 device tensor, byte offset, byte count): decode ONE stream of that many
        bytes at that offset of a buffer already on the device (datas is then ignored), so a
        file's segments are decoded from one upload of the file."""
        self._packed()
        self._check_device()
        if K > self.n_q:
            raise ValueError(f'{K} codebooks for an LM of n_q={self.n_q}')
        dev = self._emb.device
        if dev_span is not None:
            src, off, count = dev_span
            if off < 0 or count < 0 or off + count > src.numel():
                raise ValueError('encx decode_streams: dev_span outside its buffer')
            B, stride = 1, max(count, 1)
            data_ptr = src.data_ptr() + off
            nbytes = torch.tensor([count], dtype=torch.int64).to(dev)
        else:
            B = len(datas)
            stride = max([len(d) for d in datas] + [1])
            buf = torch.zeros(B, stride, dtype=torch.uint8)
            for b, d in enumerate(datas):
                if len(d):
                    buf[b, :len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
            data = buf.to(dev)
            data_ptr = data.data_ptr()
            nbytes = torch.tensor([len(d) for d in datas], dtype=torch.int64).to(dev)
        dstate = new_decoder_state(B, dev)
        err = torch.zeros(B, dtype=torch.int32, device=dev)
        codes = torch.zeros(B, K, T, dtype=torch.int64, device=dev)
        idx = torch.zeros(B, K, dtype=torch.int64, device=dev)      # step input, 0 at t = 0
        cdf = torch.empty(B, 1, K, self.card, device=dev, dtype=torch.int32)
        state = self.new_state(B, T + 1)
        step = torch.zeros(1, dtype=torch.int64, device=dev)

        def one_step(t, dstep):
            st = stream()
            x = self._body(idx, (K, 1, 1), B, K, 1, False, state, dev_step=dstep)
            self._heads(x, B, 1, K, cdf=cdf)
            call('encx_ac_decode', data_ptr, stride, nbytes.data_ptr(), B, dstate.data_ptr(),
                 cdf.data_ptr(), K, self.card, TOTAL_RANGE_BITS, codes.data_ptr(), K * T, T, 1, t,
                 dstep.data_ptr() if dstep is not None else None, idx.data_ptr(), err.data_ptr(), st)
            if dstep is not None:
                call('encx_lm_step_advance', dstep.data_ptr(), 1, st)

        if graph and T > 2:
            one_step(0, step)                    # eager first step (loads every kernel)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                one_step(0, step)
            for _ in range(T - 1):
                g.replay()
        else:
            for t in range(T):
                one_step(t, None)
        e = err.cpu().tolist()
        if any(v == 1 for v in e):
            raise EOFError("The stream ended sooner than expected.")
        if any(v == 2 for v in e):
            raise RuntimeError("Binary search failed")
        if any(e):
            raise RuntimeError(f'encx arithmetic decoder failed: {e}')
        return codes, [(p + 7) // 8 for p in dstate[:, ENCX_AC_POS].cpu().tolist()]
