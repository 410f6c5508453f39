"""Autograd ops over the libencx C ABI. Every op runs the HIP kernels; none has a CPU path.

Each Function below replaces the device work of one reference module (file:line in the
docstrings); the nn.Module mirrors in encx.modules / encx.quantization / encx.losses call these.
"""
import contextlib
import ctypes
import os
import math

import numpy as np
import torch

from ._lib import (call, ptr, stream, lib, ensure_device, ENCX_PAD_ZERO, ENCX_PAD_REFLECT,
                   ENCX_ACT_NONE, ENCX_ACT_ELU)

ACT = {None: ENCX_ACT_NONE, 'none': ENCX_ACT_NONE, 'elu': ENCX_ACT_ELU}
PAD = {'reflect': ENCX_PAD_REFLECT, 'zero': ENCX_PAD_ZERO, 'constant': ENCX_PAD_ZERO}


def _f32(n, like):
    return torch.empty(int(n), device=like.device, dtype=torch.float32)


def _ws(nbytes, like):
    """Caller-owned workspace (PyTorch caching allocator); None when the kernel needs none."""
    if nbytes == 0:
        return None
    return torch.empty((nbytes + 3) // 4, device=like.device, dtype=torch.float32)


def _check(x, name='x'):
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError(f'encx: {name} must be a float32 tensor on the GPU '
                           f'(got {x.dtype} on {x.device}); the HIP path has no CPU fallback')
    ensure_device(x.device)


# ---------------------------------------------------------------------------- geometry
def extra_padding_for_conv1d(length, kernel_size, stride, padding_total=0):
    """modules/conv.py:54-61."""
    n_frames = (length - kernel_size + padding_total) / stride + 1
    ideal_length = (math.ceil(n_frames) - 1) * stride + (kernel_size - padding_total)
    return ideal_length - length


def conv_geometry(T, K, s, d, causal, pad_mode='reflect'):
    """SConv1d.forward's padding (modules/conv.py:195-209) + pad1d's short-input zero
    extension (:86-91). Returns (pad_left, pad_right, short_ext, T_out)."""
    pt = (K - 1) * d - (s - 1)
    extra = extra_padding_for_conv1d(T, K, s, pt)
    if causal:
        pl, pr = pt, extra
    else:
        r = pt // 2
        pl, pr = pt - r, r + extra
    e = 0
    if pad_mode == 'reflect' and T <= max(pl, pr):
        e = max(pl, pr) - T + 1
    tout = (pl + T + pr - (K - 1) * d - 1) // s + 1
    return pl, pr, e, tout


def convtr_geometry(T, K, s, causal, trim_right_ratio=1.0):
    """SConvTranspose1d.forward trimming (modules/conv.py:230-252) -> (trim_left, T_out)."""
    pt = K - s
    if causal:
        pr = math.ceil(pt * trim_right_ratio)
        pl = pt - pr
    else:
        pr = pt // 2
        pl = pt - pr
    return pl, (T - 1) * s + K - pl - pr


# ---------------------------------------------------------------------------- batched weight norm
class WnBatch:
    """Weight norm (conv.py:25-34) of every layer of the models a Trainer steps, as ONE launch
    per forward group and one per flushed backward set (encx_weightnorm_{fwd,bwd}_batch) instead
    of a launch per layer.

    Forward: inside `forward(group)` every weight prep (Conv1d / ConvTranspose1d / Conv2d) is
    looked up by (parameter, layout); the group's batched launch at scope entry has already
    written the current weights into the layer's persistent operand buffers. A layer met for the
    first time is computed on its own into new persistent buffers and joins the group (its
    descriptor table is rebuilt when the scope closes, so a HIP-graph capture of a later step
    sees a stable table and stable pointers).
    Backward: with `backward()` active, a layer whose grads go straight into flat-buffer grad
    views writes its weight grad dw into a persistent per-layer buffer and is queued; flush()
    (run by the decoder-bucket all-reduce hook and when the backward scope closes, on the
    stream the step is launched / captured on) turns the queued dw into dv/dg in one launch.
    Per row the arithmetic is the single-layer kernels'."""

    FWD_FIELDS = 9  # encx_wn_fwd_desc: v, g, wf, wp, A0, A1, K, stride, row0 (8 bytes each)
    BWD_FIELDS = 9  # encx_wn_bwd_desc: v, g, dw, dv, dg, rows, cols, row0, accumulate

    def __init__(self):
        self.groups = {}      # group -> {'entries': {key: entry}, 'desc': tensor|None, 'rows': int, 'dirty'}
        self.active = None    # group whose forward scope is open
        self.dw = {}          # id(v) -> persistent dw buffer
        self.pending = []     # [(v, g)] queued for the batched backward
        self.bwd_tables = {}  # tuple of ids -> (desc tensor, rows, keep-alive refs)
        self.in_bwd = False

    # ---- forward
    @contextlib.contextmanager
    def forward(self, group):
        grp = self.groups.setdefault(group, {'entries': {}, 'desc': None, 'rows': 0, 'dirty': False})
        if grp['desc'] is not None:
            call('encx_weightnorm_fwd_batch', ptr(grp['desc']), len(grp['entries']), grp['rows'], stream())
        global _WN
        prev, _WN = _WN, self
        self.active = grp
        try:
            yield
        finally:
            _WN = prev
            self.active = None
            if grp['dirty']:
                self._build_fwd(grp)

    def prep(self, v, g, A0, A1, K, s, want_f, want_p, like):
        grp = self.active
        key = (id(v), A0, A1, K, s, want_f, want_p)
        e = grp['entries'].get(key)
        if e is None:
            J = -(-K // s)
            wf = _f32(A1 * K * A0, like) if want_f else None
            wp = _f32(A0 * J * A1 * s, like) if want_p else None
            call('encx_weightnorm_fwd', ptr(v), ptr(g), ptr(wf), ptr(wp), A0, A1, K, s, stream())
            e = grp['entries'][key] = (v, g, wf, wp, A0, A1, K, s)
            grp['dirty'] = True
        return e[2], e[3]

    def _build_fwd(self, grp):
        rows, tab = 0, []
        for v, g, wf, wp, A0, A1, K, s in grp['entries'].values():
            tab.append([v.data_ptr(), ptr(g) or 0, ptr(wf) or 0, ptr(wp) or 0, A0, A1, K, s, rows])
            rows += A0
        grp['desc'] = torch.tensor(np.array(tab, dtype=np.int64)).to(next(iter(grp['entries'].values()))[0].device)
        grp['rows'], grp['dirty'] = rows, False

    # ---- backward
    @contextlib.contextmanager
    def backward(self):
        global _WNB
        prev, _WNB = _WNB, self
        self.in_bwd = True
        try:
            yield
        finally:
            _WNB = prev
            self.in_bwd = False
            self.flush()

    def dw_buffer(self, v):
        """-> (persistent dw buffer of v, accumulate). A layer met twice before a flush (the
        discriminator's real and fake graphs share its weights) adds its second weight grad into
        the queued one: the batched backward then runs once on the summed dw, which is the
        order of the reference's autograd (grad of w summed over its uses, then weight norm)."""
        b = self.dw.get(id(v))
        if b is None:
            b = self.dw[id(v)] = torch.empty(v.shape, device=v.device, dtype=torch.float32)
        return b, any(p is v for p, _ in self.pending)

    def queue(self, v, g):
        if any(p is v for p, _ in self.pending):
            return
        self.pending.append((v, g))

    def flush(self):
        if not self.pending:
            return
        key = tuple(id(v) for v, _ in self.pending)
        ent = self.bwd_tables.get(key)
        if ent is None:
            rows, tab = 0, []
            for v, g in self.pending:
                cols = v[0].numel()
                tab.append([v.data_ptr(), g.data_ptr(), self.dw[id(v)].data_ptr(), v.grad.data_ptr(),
                            g.grad.data_ptr(), v.shape[0], cols, rows, 1])
                rows += v.shape[0]
            desc = torch.tensor(np.array(tab, dtype=np.int64)).to(self.pending[0][0].device)
            ent = self.bwd_tables[key] = (desc, rows, [(v, g, v.grad, g.grad) for v, g in self.pending])
        else:
            for (v, g), (v0, g0, vg, gg) in zip(self.pending, ent[2]):
                if v.grad is not vg or g.grad is not gg:
                    raise RuntimeError('encx: a flat grad view moved; rebuild the WnBatch')
        call('encx_weightnorm_bwd_batch', ptr(ent[0]), len(self.pending), ent[1], stream())
        self.pending = []


_WN = None   # WnBatch with an open forward scope
_WNB = None  # WnBatch collecting weight-norm backwards


def _wn_fwd(v, g, wf_or_none, wp_or_none, A0, A1, K, s):
    call('encx_weightnorm_fwd', ptr(v), ptr(g), ptr(wf_or_none), ptr(wp_or_none), A0, A1, K, s, stream())


def _weight_prep(v, g, K, s, want_f, want_p):
    """w = v*(g/||v||) (weight_norm, conv.py:25-34) written in the kernels' operand layouts."""
    A0, A1 = v.shape[0], v.shape[1]
    if _WN is not None:
        return _WN.prep(v, g, A0, A1, K, s, want_f, want_p, v)
    J = -(-K // s)
    wf = _f32(A1 * K * A0, v) if want_f else None
    wp = _f32(A0 * J * A1 * s, v) if want_p else None
    call('encx_weightnorm_fwd', ptr(v), ptr(g), ptr(wf), ptr(wp), A0, A1, K, s, stream())
    return wf, wp


def _weight_bwd(v, g, dw):
    if g is None:
        return dw.view_as(v), None
    dv = torch.empty_like(v)
    dg = torch.empty_like(g)
    call('encx_weightnorm_bwd', ptr(v), ptr(g), ptr(dw), ptr(dv), ptr(dg), v.shape[0],
         v[0].numel(), 0, stream())
    return dv, dg


def _direct(p):
    return p is None or (getattr(p, '_encx_flat', False) and p.grad is not None)


def _dw_buffer(v, g, b, shape, like):
    """Weight-grad output of a conv backward -> (buffer, accumulate): the WnBatch's persistent
    per-layer buffer when a batched weight-norm backward will consume it, else a fresh tensor."""
    if _WNB is not None and g is not None and _direct(v) and _direct(g) and _direct(b):
        return _WNB.dw_buffer(v)
    return torch.empty(shape, device=like.device, dtype=torch.float32), 0


def _param_grads(v, g, b, dw, bias_src, Bn, C, T):
    """dw (natural layout) + the bias-grad source -> grads of (v, g, b). For parameters that
    live in a FlatAdam buffer the kernels accumulate straight into the (pre-zeroed) flat grad
    views and autograd gets None: no separate accumulation pass over the weights."""
    st = stream()
    if _direct(v) and _direct(g) and _direct(b):
        if g is None:
            call('encx_axpby', ptr(dw), ptr(v.grad), dw.numel(), 1.0, None, 1.0, st)
        elif _WNB is not None and dw is _WNB.dw.get(id(v)):
            _WNB.queue(v, g)  # dv/dg in the batched launch (a second use of v added into dw)
        else:
            call('encx_weightnorm_bwd', ptr(v), ptr(g), ptr(dw), ptr(v.grad), ptr(g.grad),
                 v.shape[0], v[0].numel(), 1, st)
        if b is not None:
            ws = _f32(lib.encx_channel_sum_workspace(C) // 4, dw)
            call('encx_channel_sum', ptr(bias_src), ptr(b.grad), ptr(ws), Bn, C, T, 1, st)
        return None, None, None
    dv, dg = _weight_bwd(v, g, dw)
    db = None
    if b is not None:
        db = torch.empty(C, device=dw.device, dtype=torch.float32)
        ws = _f32(lib.encx_channel_sum_workspace(C) // 4, dw)
        call('encx_channel_sum', ptr(bias_src), ptr(db), ptr(ws), Bn, C, T, 0, st)
    return dv, dg, db


# ---------------------------------------------------------------------------- Conv1d
class Conv1dFn(torch.autograd.Function):
    """SConv1d.forward (modules/conv.py:195-210) incl. weight_norm and a fused pre-ELU."""

    @staticmethod
    def forward(ctx, x, v, g, b, res, K, s, d, causal, pad_mode, act, link=None, link_role=None):
        _check(x)
        x = x.contiguous()
        B, Cin, T = x.shape
        Cout = v.shape[0]
        pl, pr, e, tout = conv_geometry(T, K, s, d, causal, pad_mode)
        need_dx = ctx.needs_input_grad[0]
        # a dilated conv's backward-data reads the forward layout (encx_conv1d_bwd_data_dilated)
        wf, wp = _weight_prep(v, g, K, s, True, need_dx and d == 1)
        if need_dx and d != 1:
            wp = wf
        y = torch.empty(B, Cout, tout, device=x.device, dtype=torch.float32)
        if res is not None:
            res = res.contiguous()
            assert res.shape == y.shape
        ws = _ws(lib.encx_conv1d_fwd_workspace(B, Cin, Cout, tout, K, s, d), x)
        call('encx_conv1d_fwd', ptr(x), ptr(wf), ptr(b), ptr(res), ptr(y), ptr(ws), B, Cin, T, Cout,
             tout, K, s, d, pl, e, PAD[pad_mode], ACT[act], stream())
        ctx.save_for_backward(x, wp)
        ctx.params = (v, g, b)
        ctx.cfg = (K, s, d, pl, pr, e, tout, PAD[pad_mode], ACT[act], res is not None, b is not None)
        ctx.link, ctx.link_role = link, link_role
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp = ctx.saved_tensors
        v, g, b = ctx.params
        K, s, d, pl, pr, e, tout, mode, act, has_res, has_b = ctx.cfg
        dy = dy.contiguous()
        link, role = ctx.link, ctx.link_role
        B, Cin, T = x.shape
        Cout = v.shape[0]
        st = stream()
        dx = dv = dg = db = None
        park = False
        if ctx.needs_input_grad[0]:
            acc = 0
            if role == 'head' and link.grad is not None:
                # the block's skip gradient, handed over by its tail conv: accumulate into it
                # in the bwd-data epilogue instead of a separate add (see residual_block)
                dx, acc, link.grad = link.grad, 1, None
            elif role == 'join' and link.grad is not None:
                # the second of a conv-shortcut block's two convs that read the block input:
                # add into the first one's parked input grad; autograd gets the sum
                dx, acc, link.grad = link.grad, 1, None
            else:
                dx = torch.empty_like(x)
                park = role == 'join'  # the first of the two: park it, hand autograd nothing
            if d == 1:
                ws = _ws(lib.encx_conv1d_bwd_data_workspace(B, Cin, T, Cout, tout, K, s, pl, pr), x)
                call('encx_conv1d_bwd_data', ptr(dy), ptr(wp), ptr(x), ptr(dx), ptr(ws), B, Cin, T,
                     Cout, tout, K, s, pl, pr, e, mode, act, acc, st)
            else:  # wp holds the forward layout here
                ws = _f32(B * Cin * (pl + pr) + 1, x)
                call('encx_conv1d_bwd_data_dilated', ptr(dy), ptr(wp), ptr(x), ptr(dx), ptr(ws), B, Cin,
                     T, Cout, tout, K, s, d, pl, pr, e, mode, act, acc, st)
            if park:
                link.grad, dx = dx, None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            dw, acc_w = _dw_buffer(v, g, b, (Cout, Cin, K), x)
            ws = _f32(lib.encx_conv1d_bwd_weight_workspace(B, Cin, Cout, tout, K) // 4 + 1, x)
            # the bias grad comes out of the same launch (the GEMM's ones column): straight into
            # the flat grad view (accumulate) or into a fresh tensor
            direct_b = b is not None and _direct(v) and _direct(g) and _direct(b)
            db = None
            if b is not None and not direct_b:
                db = torch.empty(Cout, device=x.device, dtype=torch.float32)
            dbp = ptr(b.grad) if direct_b else ptr(db)
            call('encx_conv1d_bwd_weight_bias', ptr(dy), ptr(x), ptr(dw), dbp, ptr(ws), B, Cin, T,
                 Cout, tout, K, s, d, pl, e, mode, act, acc_w, int(direct_b), st)
            dv, dg, _ = _param_grads(v, g, None, dw, dy, B, Cout, tout)
            if direct_b and dv is not None:
                raise RuntimeError('encx: bias grad went to the flat view but the weight grads did not')
        dres = dy if has_res else None
        if role == 'tail' and has_res:
            # skip gradient of an identity-shortcut residual block: the head conv of the same
            # block adds its bwd-data result into this buffer (accumulate=1), so autograd sees
            # no second path into the block input and launches no elementwise add
            link.grad, dres = dy, None
        return dx, dv, dg, db, dres, None, None, None, None, None, None, None, None


def conv1d(x, v, g, b, K, stride=1, dilation=1, causal=True, pad_mode='reflect', act=None, res=None,
           link=None, link_role=None):
    return Conv1dFn.apply(x, v, g, b, res, K, stride, dilation, causal, pad_mode, act, link, link_role)


# ---------------------------------------------------------------------------- fused residual block
class ResBlockFn(torch.autograd.Function):
    """SEANetResnetBlock.forward (modules/seanet.py:46-63) with the EnCodec defaults -- ELU, k3
    causal reflect-padded conv (C -> C/2), ELU, 1x1 conv (C/2 -> C), plus the 1x1 shortcut conv
    -- as one kernel per direction (csrc/resblock.hip): the hidden tensor and the shortcut never
    make a round trip through HBM between three convs. (x, then (v, g, b) of the k3 conv, the
    second conv and the shortcut.) Saves x and the pre-ELU hidden h for the backward."""

    @staticmethod
    def forward(ctx, x, v1, g1, b1, v2, g2, b2, vs, gs, bs):
        _check(x)
        x = x.contiguous()
        B, C, T = x.shape
        w1, _ = _weight_prep(v1, g1, 3, 1, True, False)
        w2, _ = _weight_prep(v2, g2, 1, 1, True, False)
        ws, _ = _weight_prep(vs, gs, 1, 1, True, False)
        # the pre-ELU hidden tensor is written only for a backward (no_grad / eval: NULL)
        h = torch.empty(B, C // 2, T, device=x.device, dtype=torch.float32) if any(ctx.needs_input_grad) else None
        y = torch.empty_like(x)
        call('encx_resblock_fwd', ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(ws), ptr(bs), ptr(h), ptr(y),
             B, C, T, stream())
        ctx.save_for_backward(x, h, w1, w2, ws)
        ctx.params = ((v1, g1, b1), (v2, g2, b2), (vs, gs, bs))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, h, w1, w2, ws = ctx.saved_tensors
        (v1, g1, b1), (v2, g2, b2), (vs, gs, bs) = ctx.params
        dy = dy.contiguous()
        B, C, T = x.shape
        HD = C // 2
        dx = torch.empty_like(x)  # the data-grad kernel writes dx and dh together
        bufs = [_dw_buffer(v1, g1, b1, (HD, C, 3), x), _dw_buffer(v2, g2, b2, (C, HD, 1), x),
                _dw_buffer(vs, gs, bs, (C, C, 1), x)]
        accs = {a for _, a in bufs}
        if len(accs) != 1:  # a layer met twice before a flush (never in SEANet): fresh buffers
            bufs = [(torch.empty(sh, device=x.device, dtype=torch.float32), 0)
                    for sh in ((HD, C, 3), (C, HD, 1), (C, C, 1))]
        acc_w = bufs[0][1]
        direct_b = all(_direct(v) and _direct(g) and _direct(b) for v, g, b in ctx.params)
        if direct_b:
            dbs_ = [b1.grad, b2.grad, bs.grad]
        else:
            dbs_ = [torch.empty_like(b1), torch.empty_like(b2), torch.empty_like(bs)]
        wsp = _ws(lib.encx_resblock_bwd_workspace(B, C, T), x)
        call('encx_resblock_bwd', ptr(dy), ptr(x), ptr(h), ptr(w1), ptr(w2), ptr(ws), ptr(dx),
             ptr(bufs[0][0]), ptr(dbs_[0]), ptr(bufs[1][0]), ptr(dbs_[1]), ptr(bufs[2][0]), ptr(dbs_[2]),
             int(acc_w), int(direct_b), ptr(wsp), B, C, T, stream())
        out = []
        for (v, g, b), (dw, _), db in zip(ctx.params, bufs, dbs_):
            dv, dg, _ = _param_grads(v, g, None, dw, None, B, 0, T)
            out += [dv, dg, None if direct_b else db]
        return (dx, *out)


def resblock(x, p1, p2, ps):
    """p1 / p2 / ps: (v, g, b) of the block's k3 conv, 1x1 conv and 1x1 shortcut."""
    return ResBlockFn.apply(x, *p1, *p2, *ps)


RESBLOCK_TMIN = 2048  # fused residual block from this many samples up (the HBM-bound stages)


# ---------------------------------------------------------------------------- ConvTranspose1d
class ConvTr1dFn(torch.autograd.Function):
    """SConvTranspose1d.forward (modules/conv.py:230-252) incl. weight_norm (dim 0 = in
    channels, conv.py:149) and a fused pre-ELU."""

    @staticmethod
    def forward(ctx, x, v, g, b, K, s, causal, trim_right_ratio, act, untrimmed=False):
        _check(x)
        x = x.contiguous()
        B, Cin, T = x.shape
        Cout = v.shape[1]
        if untrimmed:  # full (T - 1) * s + K output; the caller trims after its norm
            trim_left, tout = 0, (T - 1) * s + K
        else:
            trim_left, tout = convtr_geometry(T, K, s, causal, trim_right_ratio)
        need_dx = ctx.needs_input_grad[0]
        wf, wp = _weight_prep(v, g, K, s, need_dx, True)
        y = torch.empty(B, Cout, tout, device=x.device, dtype=torch.float32)
        ws = _ws(lib.encx_convtr1d_fwd_workspace(B, Cin, Cout, tout, K, s, trim_left), x)
        call('encx_convtr1d_fwd', ptr(x), ptr(wp), ptr(b), ptr(y), ptr(ws), B, Cin, T, Cout, tout, K,
             s, trim_left, ACT[act], stream())
        ctx.save_for_backward(x, wf)
        ctx.params = (v, g, b)
        ctx.cfg = (K, s, trim_left, tout, ACT[act], b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wf = ctx.saved_tensors
        v, g, b = ctx.params
        K, s, trim_left, tout, act, has_b = ctx.cfg
        dy = dy.contiguous()
        B, Cin, T = x.shape
        Cout = v.shape[1]
        st = stream()
        dx = dv = dg = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            ws = _ws(lib.encx_convtr1d_bwd_data_workspace(B, Cin, T, Cout, K, s), x)
            call('encx_convtr1d_bwd_data', ptr(dy), ptr(wf), ptr(x), ptr(dx), ptr(ws), B, Cin, T,
                 Cout, tout, K, s, trim_left, act, 0, st)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            dw, acc_w = _dw_buffer(v, g, b, (Cin, Cout, K), x)
            ws = _f32(lib.encx_convtr1d_bwd_weight_workspace(B, Cin, Cout, T, K) // 4 + 1, x)
            call('encx_convtr1d_bwd_weight', ptr(x), ptr(dy), ptr(dw), None, ptr(ws), B, Cin, T,
                 Cout, tout, K, s, trim_left, act, acc_w, st)
            dv, dg, db = _param_grads(v, g, b, dw, dy, B, Cout, tout)
        return dx, dv, dg, db, None, None, None, None, None, None


def convtr1d(x, v, g, b, K, stride, causal=True, trim_right_ratio=1.0, act=None, untrimmed=False):
    return ConvTr1dFn.apply(x, v, g, b, K, stride, causal, trim_right_ratio, act, untrimmed)


# ---------------------------------------------------------------------------- normalisation
def normalize(x):
    """model.py:152-157 -> (x / scale, scale [B,1]). The input wave never needs a grad."""
    _check(x)
    x = x.contiguous()
    B, C, T = x.shape
    xn = torch.empty_like(x)
    scale = torch.empty(B, device=x.device, dtype=torch.float32)
    call('encx_normalize_fwd', ptr(x), ptr(xn), ptr(scale), B, C, T, stream())
    return xn, scale.view(-1, 1)


class ScaleRowsFn(torch.autograd.Function):
    """out * scale.view(-1, 1, 1) (model.py:191-192); scale carries no grad."""

    @staticmethod
    def forward(ctx, x, scale):
        x = x.contiguous()
        y = torch.empty_like(x)
        call('encx_scale_rows', ptr(x), ptr(scale), ptr(y), x.shape[0], x[0].numel(), stream())
        ctx.save_for_backward(scale)
        return y

    @staticmethod
    def backward(ctx, dy):
        scale, = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call('encx_scale_rows', ptr(dy), ptr(scale), ptr(dx), dy.shape[0], dy[0].numel(), stream())
        return dx, None


# ---------------------------------------------------------------------------- losses
class L1LossFn(torch.autograd.Function):
    """losses.py:37 l_t = L1Loss(input_wav, output_wav); grad w.r.t. the output only."""

    @staticmethod
    def forward(ctx, x, y):
        _check(y, 'output')
        x, y = x.contiguous(), y.contiguous()
        loss = torch.empty(1, device=y.device, dtype=torch.float32)
        grad = torch.empty_like(y) if ctx.needs_input_grad[1] else None
        ws = _f32(1024, y)
        call('encx_l1_loss', ptr(x), ptr(y), ptr(loss), ptr(grad), ptr(ws), y.numel(), stream())
        ctx.save_for_backward(grad)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        grad, = ctx.saved_tensors
        out = torch.empty_like(grad)
        call('encx_axpby', ptr(grad), ptr(out), grad.numel(), 1.0, ptr(g.contiguous().view(1)), 0.0,
             stream())
        return None, out


_MEL_CACHE = {}


def mel_tables(device, n_fft, n_mels, sr, fmin=0.0, fmax=None):
    """Device DFT (window*cos / -window*sin) + mel-basis tables for one scale, built once."""
    key = (str(device), n_fft, n_mels, sr, float(fmin), fmax)
    t = _MEL_CACHE.get(key)
    if t is None:
        from .audio_to_mel import mel_filterbank
        basis = torch.from_numpy(mel_filterbank(sr, n_fft, n_mels, fmin, fmax)).to(device)
        t = torch.empty(lib.encx_mel_tables_floats(n_fft, n_mels), device=device, dtype=torch.float32)
        call('encx_mel_tables_init', ptr(t), ptr(basis), n_fft, n_mels, stream())
        _MEL_CACHE[key] = (t, basis)
        t = _MEL_CACHE[key]
    return t[0]


_FRAMED_CACHE = {}


def logmel_framed(x, n_fft, hop, win, n_mels, sr, fmin=0.0, fmax=None):
    """Audio2Mel.forward (audio_to_mel.py:34-55) with any hop and win_length <= n_fft ->
    [B, C, n_mels * F] (encx_mel_logmel_framed: reflect pad, the windowed spectrogram, mel, log)."""
    _check(x)
    x = x.contiguous()
    shape = x.shape
    B = shape[0] * (shape[1] if x.dim() > 2 else 1)
    T = shape[-1]
    key = (str(x.device), n_fft, hop, win, n_mels, sr, float(fmin), fmax)
    ent = _FRAMED_CACHE.get(key)
    if ent is None:
        from .audio_to_mel import mel_filterbank
        basis = torch.from_numpy(mel_filterbank(sr, n_fft, n_mels, fmin, fmax)).to(x.device).contiguous()
        tab, _ = spec_window_tables(torch.hann_window(win).to(x.device), n_fft, False)
        ent = _FRAMED_CACHE[key] = (basis, tab)
    basis, tab = ent
    p = (n_fft - hop) // 2
    F = (T + 2 * p - n_fft) // hop + 1
    out = torch.empty(B, n_mels, F, device=x.device, dtype=torch.float32)
    ws = _f32(lib.encx_mel_logmel_framed_workspace_floats(B, T, n_fft, hop), x)
    call('encx_mel_logmel_framed', ptr(x), ptr(tab), ptr(basis), ptr(ws), ptr(out), B, T, n_fft, hop, n_mels,
         stream())
    if x.dim() > 2:
        return out.reshape(shape[0], shape[1], -1)
    return out


# the fused multi-scale mel loss (encx_mel_loss_multi: one launch per scale + one overlap-add +
# one finish, round 6); False: the per-scale calls of encx_mel_loss (nine launches each)
MEL_FUSED = os.environ.get('ENCX_MEL_FUSED', '1') != '0'


class MelLossFn(torch.autograd.Function):
    """l_f of total_loss (losses.py:40-42): sum over n_fft = 2^5..2^11 (hop n/4, 64 mels) of
    L1 + MSE between Audio2Mel(x) and Audio2Mel(y) (audio_to_mel.py:34-55). The gradient
    w.r.t. y is produced by the same pass (the balancer always asks for it)."""

    @staticmethod
    def forward(ctx, x, y, sr, n_mels, scales):
        _check(y, 'output')
        x, y = x.contiguous(), y.contiguous()
        B = y.shape[0] * y.shape[1]
        T = y.shape[-1]
        loss = torch.zeros(1, device=y.device, dtype=torch.float32)
        grad = torch.zeros_like(y) if ctx.needs_input_grad[1] else None
        if MEL_FUSED and n_mels == 64 and all(32 <= n <= 2048 and n & (n - 1) == 0 for n in scales):
            ns = (ctypes.c_int64 * len(scales))(*scales)
            tabs = (ctypes.c_void_p * len(scales))(*[mel_tables(y.device, n, n_mels, sr).data_ptr() for n in scales])
            ws = _f32(lib.encx_mel_loss_multi_workspace_floats(B, T, ns, len(scales)), y)
            call('encx_mel_loss_multi', ptr(x), ptr(y), tabs, ns, len(scales), ptr(ws), ptr(loss), ptr(grad), B, T,
                 stream())
            ctx.save_for_backward(grad)
            return loss
        wsn = max(lib.encx_mel_workspace_floats(B, T, n, n_mels) for n in scales)
        ws = _f32(wsn, y)
        for n in scales:
            tab = mel_tables(y.device, n, n_mels, sr)
            call('encx_mel_loss', ptr(x), ptr(y), ptr(tab), ptr(ws), ptr(loss), ptr(grad), B, T, n,
                 n_mels, stream())
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        grad, = ctx.saved_tensors
        out = torch.empty_like(grad)
        call('encx_axpby', ptr(grad), ptr(out), grad.numel(), 1.0, ptr(g.contiguous().view(1)), 0.0,
             stream())
        return None, out, None, None, None


def logmel(x, n_fft, n_mels, sr, fmin=0.0, fmax=None):
    """Audio2Mel.forward (audio_to_mel.py:34-55) -> [B, C, n_mels * F]; fmin / fmax: the mel
    filters' band (librosa.filters.mel's, audio_to_mel.py:24)."""
    _check(x)
    x = x.contiguous()
    shape = x.shape
    B = shape[0] * (shape[1] if x.dim() > 2 else 1)
    T = shape[-1]
    F = lib.encx_mel_frames(T, n_fft)
    out = torch.empty(B, n_mels, F, device=x.device, dtype=torch.float32)
    ws = _f32(lib.encx_mel_workspace_floats(B, T, n_fft, n_mels), x)
    call('encx_mel_logmel', ptr(x), ptr(mel_tables(x.device, n_fft, n_mels, sr, fmin, fmax)), ptr(ws), ptr(out),
         B, T, n_fft, n_mels, stream())
    if x.dim() > 2:
        return out.reshape(shape[0], shape[1], -1)
    return out


# ---------------------------------------------------------------------------- RVQ
def rvq_argmin(res, embed, direct=False):
    """EuclideanCodebook.quantize (core_vq.py:181-189) over res [B, D, T] -> int64 [B*T]."""
    B, D, T = res.shape
    N = B * T
    idx = torch.empty(N, device=res.device, dtype=torch.int64)
    keys = torch.empty(N, device=res.device, dtype=torch.int64)
    call('encx_rvq_argmin', ptr(res), ptr(embed), ptr(idx), ptr(keys), B, D, T, embed.shape[0],
         int(direct), stream())
    return idx


def kmeans(samples, num_clusters, num_iters, seed):
    """kmeans (core_vq.py:80-102) on the device: samples [N, D] -> (means, bins)."""
    N, D = samples.shape
    means = torch.empty(num_clusters, D, device=samples.device, dtype=torch.float32)
    call('encx_sample_rows', ptr(samples), ptr(means), N, D, num_clusters, seed & (2 ** 64 - 1), stream())
    bins = torch.zeros(num_clusters, device=samples.device, dtype=torch.int64)
    idx = torch.empty(N, device=samples.device, dtype=torch.int64)
    keys = torch.empty(N, device=samples.device, dtype=torch.int64)
    ws = _ws(lib.encx_rvq_bucket_workspace(N, D, num_clusters), samples)
    for _ in range(num_iters):
        call('encx_kmeans_step', ptr(samples), ptr(means), ptr(bins), ptr(idx), ptr(keys), ptr(ws),
             N, D, num_clusters, stream())
    return means, bins


def rvq_to_rows(res):
    B, D, T = res.shape
    out = torch.empty(B * T, D, device=res.device, dtype=torch.float32)
    call('encx_bdt_to_nd', ptr(res), ptr(out), B, D, T, stream())
    return out


_CB_DEFER = None  # list collecting CodebookSync entries while defer_codebook_sync is active


class CodebookSync:
    """The data-parallel EMA codebook sync of one RVQ forward: `sums` [n_q, K, D+1] holds each
    layer's per-code sums (sum of x over the rows assigned to a code, and their count); after
    an all-reduce (SUM) of `sums` over the ranks, apply() runs each layer's EMA update from them
    (core_vq.py:227-235), so every rank applies the same update."""

    def __init__(self, sums, codebooks, decay, eps):
        self.sums, self.codebooks, self.decay, self.eps = sums, codebooks, decay, eps

    def apply(self):
        n_q, Kc, D1 = self.sums.shape
        for i, cb in enumerate(self.codebooks):
            call('encx_rvq_ema_from_sums', ptr(self.sums[i]), ptr(cb.cluster_size), ptr(cb.embed_avg),
                 ptr(cb.embed), D1 - 1, Kc, self.decay, self.eps, stream())


@contextlib.contextmanager
def defer_codebook_sync(pending: list):
    """Inside this scope a synced RVQ forward leaves its CodebookSync in `pending` instead of
    all-reducing and applying it, so a HIP-graph trainer can run the collective eagerly between
    two captured segments and apply() it in a later one."""
    global _CB_DEFER
    prev, _CB_DEFER = _CB_DEFER, pending
    try:
        yield pending
    finally:
        _CB_DEFER = prev


class RVQTrainFn(torch.autograd.Function):
    """ResidualVectorQuantization.forward in train mode (core_vq.py:337-355) over
    VectorQuantization.forward (:301-324) + the EMA codebook update (:212-237), one fused
    pass per layer. Returns (quantized [B,D,T], codes [n_q,B,T], penalty [1]).
    Backward: d emb = n_q * d quantized + d penalty * 2/(n_q*numel) * sum_i (x_i - q_ste_i)
    (per-layer straight-through, Appendix A quirk 1)."""

    @staticmethod
    def forward(ctx, emb, codebooks, decay, eps, sync=False, cw=1.0):
        """cw: the layers' commitment_weight (core_vq.py:267: loss += commit_loss * w; the
        penalty is their mean, vq.py:99). sync: all-reduce (SUM) each layer's per-code sums over the data-parallel ranks
        before its EMA, so every rank applies the same update (the reference never
        syncs, core_vq.py:157,175 / train_multi_gpu.py:318 -- off by default)."""
        _check(emb, 'emb')
        emb = emb.contiguous()
        B, D, T = emb.shape
        n_q = len(codebooks)
        numel = emb.numel()
        st = stream()
        res = [emb.clone(), torch.empty_like(emb)]
        out = torch.empty_like(emb)
        cdir = torch.empty_like(emb)
        P = lib.encx_rvq_apply_parts(B, D, T)
        parts = torch.empty(n_q, P, device=emb.device, dtype=torch.float32)
        commits = torch.empty(n_q, device=emb.device, dtype=torch.float32)
        codes = torch.empty(n_q, B * T, device=emb.device, dtype=torch.int64)
        keys = torch.empty(B * T, device=emb.device, dtype=torch.int64)
        Kc = codebooks[0].embed.shape[0]
        bws = _ws(lib.encx_rvq_bucket_workspace(B * T, D, Kc), emb)
        sums = None
        if sync and codebooks[0].training and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1:
            # every layer's sums, all-reduced in ONE collective after the layer loop: layer i's
            # EMA update is read by no later layer of this forward (each quantizes with its own
            # codebook), so deferring it is value-identical to updating inside the loop
            sums = torch.empty(n_q, Kc, D + 1, device=emb.device, dtype=torch.float32)
        for i, cb in enumerate(codebooks):
            x = res[i % 2]
            cb.init_embed_(x)
            call('encx_rvq_argmin', ptr(x), ptr(cb.embed), ptr(codes[i]), ptr(keys), B, D, T,
                 cb.embed.shape[0], 0, st)
            # dequantize with the pre-update codebook (core_vq.py:221), then update it (:223-235)
            call('encx_rvq_apply', ptr(x), ptr(res[(i + 1) % 2]), ptr(cb.embed), ptr(codes[i]),
                 ptr(out), ptr(cdir), ptr(parts[i]), B, D, T, int(i == 0), 1, st)
            if cb.training and sums is not None:
                call('encx_rvq_code_sums', ptr(x), ptr(codes[i]), ptr(sums[i]), ptr(bws), B, D, T, Kc, st)
            elif cb.training:
                call('encx_rvq_ema', ptr(x), ptr(codes[i]), ptr(cb.cluster_size), ptr(cb.embed_avg),
                     ptr(cb.embed), ptr(bws), B, D, T, cb.embed.shape[0], float(decay), float(eps), st)
            call('encx_reduce_sum', ptr(parts[i]), P, 1.0 / numel, ptr(commits[i:i + 1]), 0, st)
        if sums is not None:
            sync_ent = CodebookSync(sums, list(codebooks), float(decay), float(eps))
            if _CB_DEFER is not None:  # the Trainer runs the collective between graph segments
                _CB_DEFER.append(sync_ent)
            else:
                torch.distributed.all_reduce(sums)  # n_q x 1024 x 129 fp32 = 528 KB per layer
                sync_ent.apply()
        penalty = torch.empty(1, device=emb.device, dtype=torch.float32)
        call('encx_reduce_sum', ptr(commits), n_q, float(cw) / n_q, ptr(penalty), 0, st)
        ctx.save_for_backward(cdir)
        ctx.n_q, ctx.numel, ctx.cw = n_q, numel, float(cw)
        ctx.mark_non_differentiable(codes)
        return out, codes.view(n_q, B, T), penalty.view(())

    @staticmethod
    def backward(ctx, dq, dcodes, dpen):
        cdir, = ctx.saved_tensors
        n_q, numel = ctx.n_q, ctx.numel
        if dq is None:
            dq = torch.zeros_like(cdir)
        dq = dq.contiguous()
        demb = torch.empty_like(cdir)
        if dpen is None:
            call('encx_lincomb', ptr(dq), ptr(cdir), ptr(demb), demb.numel(), float(n_q), None, 0.0,
                 stream())
        else:
            call('encx_lincomb', ptr(dq), ptr(cdir), ptr(demb), demb.numel(), float(n_q),
                 ptr(dpen.contiguous().view(1)), 2.0 * ctx.cw / (n_q * numel), stream())
        return demb, None, None, None, None, None


def rvq_encode(emb, embeds):
    """ResidualVectorQuantization.encode (core_vq.py:357-367): residual -= exact q."""
    _check(emb, 'emb')
    emb = emb.contiguous()
    B, D, T = emb.shape
    res = emb.clone()
    codes = torch.empty(len(embeds), B * T, device=emb.device, dtype=torch.int64)
    keys = torch.empty(B * T, device=emb.device, dtype=torch.int64)
    for i, E in enumerate(embeds):
        call('encx_rvq_argmin', ptr(res), ptr(E), ptr(codes[i]), ptr(keys), B, D, T, E.shape[0], 0,
             stream())
        call('encx_rvq_apply', ptr(res), ptr(res), ptr(E), ptr(codes[i]), None, None, None, B, D, T,
             0, 0, stream())
    return codes.view(len(embeds), B, T)


def rvq_decode(codes, embeds):
    """ResidualVectorQuantization.decode (core_vq.py:369-375)."""
    n_q, B, T = codes.shape
    D = embeds[0].shape[1]
    out = torch.empty(B, D, T, device=codes.device, dtype=torch.float32)
    codes = codes.contiguous()
    for i in range(n_q):
        call('encx_rvq_gather', ptr(embeds[i]), ptr(codes[i]), ptr(out), B, D, T, int(i > 0), stream())
    return out


# ---------------------------------------------------------------------------- LSTM
class LSTMFn(torch.autograd.Function):
    """SLSTM.forward (modules/lstm.py:22-28): torch.nn.LSTM(H, H, L) over [T, B, H] + skip.

    Takes x in the conv layout [B][H][T] and returns the same layout. All L layers run as one
    diagonal wavefront (csrc/lstm.hip); the sequences live as [L][B][T][.] on the device.
    Weights per layer: (w_ih, w_hh, b_ih, b_hh), packed per call into [W_ih | W_hh]."""

    @staticmethod
    def forward(ctx, x, skip, *weights):
        _check(x)
        x = x.contiguous()
        B, H, T = x.shape
        L = len(weights) // 4
        if B > LSTM_MAX_BATCH or H % 16 or H > 1024:
            raise NotImplementedError('encx LSTM: hidden % 16 == 0 and <= 1024 (lstm() splits the batch)')
        st = stream()
        wcat = _f32(L * 8 * H * H, x)
        wcatT = _f32(L * 8 * H * H, x)
        bsum = _f32(L * 4 * H, x)
        for l in range(L):
            w_ih, w_hh, b_ih, b_hh = (w.contiguous() for w in weights[4 * l:4 * l + 4])
            call('encx_lstm_pack', ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh), ptr(wcat), ptr(wcatT),
                 ptr(bsum), H, l, st)
        xt = _f32(B * T * H, x)
        Y = _f32(L * B * T * H, x)
        Cs = _f32(L * B * T * H, x)
        Gs = _f32(L * B * T * 4 * H, x)
        out = torch.empty_like(x)
        call('encx_lstm_fwd', ptr(x), ptr(wcat), ptr(bsum), ptr(xt), ptr(Y), ptr(Cs), ptr(Gs), ptr(out),
             int(bool(skip)), B, T, H, L, st)
        # saved (not ctx attributes) so autograd frees them after the backward unless the
        # graph is retained (a second backward through the same LSTM, e.g. the commit loss)
        ctx.save_for_backward(xt, Y, Cs, Gs, wcatT)
        ctx.weights = weights
        ctx.skip = skip
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        B, H, T = dout.shape
        weights = ctx.weights
        xt, Y, Cs, Gs, wcatT = ctx.saved_tensors
        L = len(weights) // 4
        st = stream()
        if ctx.needs_input_grad[0]:  # the skip passes dout through; the kernels add the rest
            dx, acc_x = (dout.clone(), 1) if ctx.skip else (torch.empty_like(dout), 0)
        else:
            dx, acc_x = None, 0
        DA = _f32(L * B * T * 4 * H, dout)
        ws = _ws(lib.encx_lstm_bwd_workspace(B, T, H, L), dout)
        call('encx_lstm_bwd', ptr(dout), ptr(wcatT), ptr(Cs), ptr(Gs), ptr(DA), ptr(dx), acc_x, ptr(ws),
             B, T, H, L, st)
        grads = [None] * len(weights)
        wsw = None
        for l in range(L):
            w4 = weights[4 * l:4 * l + 4]
            if not any(ctx.needs_input_grad[2 + 4 * l + i] for i in range(4)):
                continue
            if all(_direct(w) for w in w4):
                dws, acc_w = [w.grad for w in w4], 1
            else:
                dws, acc_w = [torch.empty_like(w) for w in w4], 0
                grads[4 * l:4 * l + 4] = dws
            if wsw is None:
                wsw = _ws(lib.encx_lstm_bwd_weight_workspace(B, T, H), dout)
            call('encx_lstm_bwd_weight', ptr(DA), ptr(xt), ptr(Y), ptr(dws[0]), ptr(dws[1]), ptr(dws[2]),
                 ptr(dws[3]), acc_w, ptr(wsw), B, T, H, L, l, st)
        return (dx, None, *grads)


LSTM_MAX_BATCH = 64  # batch rows one launch of the recurrence kernels takes (csrc/lstm.hip)


def lstm(x, weights, skip=True):
    """nn.LSTM takes any batch (modules/lstm.py:20-27); the batch items' recurrences are
    independent, so a batch above LSTM_MAX_BATCH runs as near-equal chunks of at most that many
    (the weight grads summed over the chunks by autograd)."""
    B = x.shape[0]
    if B <= LSTM_MAX_BATCH:
        return LSTMFn.apply(x, skip, *weights)
    n = -(-B // LSTM_MAX_BATCH)
    sizes = [B // n + (i < B % n) for i in range(n)]
    return torch.cat([LSTMFn.apply(xc, skip, *weights) for xc in torch.split(x, sizes)], dim=0)


# ---------------------------------------------------------------------------- MS-STFT disc
def conv2d_geometry(Fi, kernel, stride, dilation, padding):
    (KT, KF), (st, sf), (dt, df), (pt, pf) = kernel, stride, dilation, padding
    if st != 1 or df != 1 or 2 * pt != dt * (KT - 1):
        raise NotImplementedError('encx conv2d: the DiscriminatorSTFT geometry (time stride 1, '
                                  'freq dilation 1, time-preserving padding)')
    Fo = (Fi + 2 * pf - KF) // sf + 1
    return KT, KF, sf, dt, pt, pf, Fo


class DiscGradMode:
    """Which gradients a discriminator graph's backward produces. One forward graph of the
    discriminator serves both phases of a GAN step (encx.train.Trainer): the generator phase
    differentiates it w.r.t. the audio only (params=False: no weight-gradient kernels), the
    discriminator phase w.r.t. its weights only (input=False: no gradient into the
    spectrogram, as the reference's disc(output.detach()), train_multi_gpu.py:114-116)."""

    def __init__(self, params=True, input=True, premask=False):
        self.params, self.input = params, input
        # premask: the graph's owner guarantees that the feature maps are read only by the next
        # Conv2d and by FeatFn (no other autograd consumer). Each Conv2d then hands its input's
        # producer the grad of that producer's pre-activation (the LeakyReLU' mask applied in the
        # bwd-data epilogue), so the producer's bwd-data and bwd-weight never read its output map.
        self.premask = premask

    def set(self, params, input):
        self.params, self.input = params, input

    def reuse_weights(self, on=True):
        """Within one train step the discriminator runs forward twice (real, fake) with the same
        weights: while on, each Conv2d derives its weight-normed and polyphase weights once and
        shares them between the two graphs. Turning it off (or on again) drops the cache; the
        owner must do so before the weights change."""
        self.reuse = bool(on)
        self.cache = {}

    reuse = False
    cache = None


_ALL_GRADS = DiscGradMode()


class Conv2dFn(torch.autograd.Function):
    """NormConv2d.forward (modules/conv.py:136-139) + the LeakyReLU(0.2) that follows it in
    DiscriminatorSTFT.forward (msstftd.py:100-103) when act. Returns the post-activation map
    (the fmap entry); its sign is the pre-activation's, so it also serves as the LeakyReLU'
    mask in the backward. mode (DiscGradMode) gates the weight grads, and the input grad of
    the layer that reads the spectrogram (first=True)."""

    @staticmethod
    def forward(ctx, x, v, g, b, geo, act, mode=_ALL_GRADS, first=False, feat_slot=None, out_slot=None):
        _check(x)
        x = x.contiguous()
        B, Ci, T2, Fi = x.shape
        Co = v.shape[0]
        KT, KF, sf, dt, pt, pf, Fo = geo
        st = stream()
        ent = mode.cache.get(id(v)) if mode.reuse else None
        if ent is None:
            if _WN is not None:
                wf = _WN.prep(v, g, Co, Ci * KT, KF, 1, True, False, x)[0]
            else:
                wf = _f32(Co * Ci * KT * KF, x)
                call('encx_weightnorm_fwd', ptr(v), ptr(g), ptr(wf), None, Co, Ci * KT, KF, 1, st)
            wp = None
            if mode.reuse:
                wp = _wpoly(wf, Co, Ci, KT, KF, sf, x)
                mode.cache[id(v)] = (wf, wp)
        else:
            wf, wp = ent
        y = torch.empty(B, Co, T2, Fo, device=x.device, dtype=torch.float32)
        call('encx_conv2d_fwd', ptr(x), ptr(wf), ptr(b), ptr(y), B, Ci, T2, Fi, Co, Fo, KT, KF, sf, dt, pt,
             pf, int(act), st)
        ctx.save_for_backward(x, y, wf)
        ctx.wp = wp
        ctx.feat_slot = feat_slot
        ctx.out_slot = out_slot
        ctx.params = (v, g, b)
        ctx.geo, ctx.act = geo, act
        ctx.mode, ctx.first = mode, first
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return (None,) * 10
        x, y, wf = ctx.saved_tensors
        slot = ctx.feat_slot
        feat = slot.pending if slot is not None else None
        if feat is not None:
            slot.pending = None
        v, g, b = ctx.params
        KT, KF, sf, dt, pt, pf, Fo = ctx.geo
        dy = dy.contiguous()
        B, Ci, T2, Fi = x.shape
        Co = v.shape[0]
        st = stream()
        # dy arrives already multiplied by LeakyReLU'(y) when the one layer reading y applied it
        # in its bwd-data epilogue (FeatSlot.premasked); the flag is consumed here
        out = ctx.out_slot
        premasked = out is not None and out.premasked
        if out is not None:
            out.premasked = False
        yact = y if ctx.act and not premasked else None
        dims = (B, Ci, T2, Fi, Co, Fo, KT, KF, sf, dt, pt, pf)
        dx = dv = dg = db = None
        mode = ctx.mode
        if ctx.needs_input_grad[0] and (mode.input or not ctx.first):
            wp = ctx.wp if ctx.wp is not None else _wpoly(wf, Co, Ci, KT, KF, sf, x)
            dx = torch.empty_like(x)
            # hand the producer of x the grad of its pre-activation when this layer is the only
            # path by which x receives a gradient
            xact = None
            if slot is not None:
                # only where the epilogue reads x anyway (the feature term): elsewhere the
                # extra read of x costs more than the producer saves by not reading its map
                slot.premasked = (mode.premask and feat is not None and slot.act and slot.readers == 1
                                  and not slot.autograd_feat)
                xact = x if slot.premasked else None
            if feat is None:
                call('encx_conv2d_bwd_data', ptr(dy), ptr(yact), ptr(wp), ptr(xact), ptr(dx), 0, *dims, st)
            else:  # + FeatFn's grad of this input map, in the epilogue
                fr, den, fg, fscale, code = feat
                call('encx_conv2d_bwd_data_feat', ptr(dy), ptr(yact), ptr(wp), ptr(xact), ptr(dx), 0, ptr(fr),
                     ptr(x), ptr(den), ptr(fg), float(fscale), ptr(code), *dims, st)
        elif feat is not None:
            raise RuntimeError('encx: a feature-matching grad was handed to a Conv2d whose input grad '
                               'is not computed')
        if any(ctx.needs_input_grad[1:4]) and mode.params:
            ws = _ws(lib.encx_conv2d_bwd_weight_workspace(*dims), x)
            direct = _direct(v) and _direct(g) and _direct(b)
            if direct and g is None:   # plain weight: straight into the flat grad views
                call('encx_conv2d_bwd_weight', ptr(dy), ptr(yact), ptr(x), ptr(v.grad), ptr(b.grad), 1, 1,
                     ptr(ws), *dims, st)
            elif direct and _WNB is not None:  # dv/dg in the batched weight-norm backward
                dw, acc_w = _WNB.dw_buffer(v)
                call('encx_conv2d_bwd_weight', ptr(dy), ptr(yact), ptr(x), ptr(dw), ptr(b.grad), acc_w, 1,
                     ptr(ws), *dims, st)
                _WNB.queue(v, g)
            elif direct:
                dw = torch.empty(v.shape, device=x.device, dtype=torch.float32)
                call('encx_conv2d_bwd_weight', ptr(dy), ptr(yact), ptr(x), ptr(dw), ptr(b.grad), 0, 1,
                     ptr(ws), *dims, st)
                call('encx_weightnorm_bwd', ptr(v), ptr(g), ptr(dw), ptr(v.grad), ptr(g.grad), Co,
                     v[0].numel(), 1, st)
            else:
                dw = torch.empty(v.shape, device=x.device, dtype=torch.float32)
                db = torch.empty(Co, device=x.device, dtype=torch.float32) if b is not None else None
                call('encx_conv2d_bwd_weight', ptr(dy), ptr(yact), ptr(x), ptr(dw), ptr(db), 0, 0,
                     ptr(ws), *dims, st)
                dv, dg = _weight_bwd(v, g, dw)
        return dx, dv, dg, db, None, None, None, None, None, None


class FeatSlot:
    """Attached to every Conv2d output map: FeatFn.backward parks its grad of the map here
    (the real map, the pair's mean |fr|, the upstream grad, the scale) and the Conv2d that reads
    the map adds it in its bwd-data epilogue (encx_conv2d_bwd_data_feat), so the map's grad is
    never materialised twice and autograd does no add. FeatFn runs before every Conv2d of its
    graph in a traversal (it is the loss node), and the consumer clears the slot."""
    __slots__ = ('pending', 'consumer_out', 'act', 'readers', 'autograd_feat', 'premasked')

    def __init__(self, act=False):
        self.pending = None
        self.consumer_out = None  # the slot of the map the reading Conv2d produces
        self.act = act            # the map is a LeakyReLU output (its sign is the pre-activation's)
        self.readers = 0          # Conv2d layers reading the map
        self.autograd_feat = False  # FeatFn returns this map's grad through autograd
        # set by the reading Conv2d's backward when its dx is already the grad of the producing
        # layer's pre-activation (dy * LeakyReLU'(map)); read and cleared by the producer
        self.premasked = False


def _wpoly(wf, Co, Ci, KT, KF, sf, like):
    """Polyphase (along f) weight layout of the bwd-data kernel."""
    J = -(-KF // sf)
    wp = _f32(Co * KT * J * Ci * sf, like)
    call('encx_conv2d_wpoly', ptr(wf), ptr(wp), Co, Ci, KT, KF, sf, stream())
    return wp


def conv2d(x, v, g, b, kernel, stride=(1, 1), dilation=(1, 1), padding=(0, 0), act=False, mode=_ALL_GRADS,
           first=False):
    geo = conv2d_geometry(x.shape[-1], kernel, stride, dilation, padding)
    in_slot = getattr(x, '_encx_feat_slot', None)
    out_slot = FeatSlot(act=bool(act))
    y = Conv2dFn.apply(x, v, g, b, geo, act, mode, first, in_slot, out_slot)
    y._encx_feat_slot = out_slot
    if in_slot is not None:
        in_slot.consumer_out = out_slot
        in_slot.readers += 1
    return y


class DiscSpecFn(torch.autograd.Function):
    """torchaudio Spectrogram(normalized=True, center=False, power=None) + cat([re, im], 1) +
    'b c w t -> b c t w' of DiscriminatorSTFT.forward (msstftd.py:62-64, 97-99)."""

    @staticmethod
    def forward(ctx, x, n_fft, hop, sr, window=None):
        """window: None = hann(n_fft), normalized (the reference's configuration); else
        (tables, scale) from spec_window_tables."""
        _check(x)
        x = x.contiguous()
        B, C, T = x.shape
        tab, scale = window if window is not None else (mel_tables(x.device, n_fft, 64, sr), None)
        Fr = (T - n_fft) // hop + 1
        z = torch.empty(B, 2 * C, Fr, n_fft // 2 + 1, device=x.device, dtype=torch.float32)
        if scale is None:
            call('encx_disc_spec_fwd', ptr(x), ptr(tab), ptr(z), B, C, T, n_fft, hop, stream())
        else:
            call('encx_disc_spec_fwd_scaled', ptr(x), ptr(tab), ptr(z), B, C, T, n_fft, hop, float(scale), stream())
        ctx.cfg = (B, C, T, n_fft, hop, scale)
        ctx.tab = tab
        ctx.set_materialize_grads(False)
        return z

    @staticmethod
    def backward(ctx, dz):
        if dz is None:  # the first conv produced no input grad (DiscGradMode.input False)
            return None, None, None, None, None
        B, C, T, n_fft, hop, scale = ctx.cfg
        dz = dz.contiguous()
        dx = torch.empty(B, C, T, device=dz.device, dtype=torch.float32)
        ws = _ws(lib.encx_disc_spec_bwd_workspace(B, C, T, n_fft, hop), dz)
        if scale is None:
            call('encx_disc_spec_bwd', ptr(dz), ptr(ctx.tab), ptr(dx), ptr(ws), 0, B, C, T, n_fft, hop, stream())
        else:
            call('encx_disc_spec_bwd_scaled', ptr(dz), ptr(ctx.tab), ptr(dx), ptr(ws), 0, B, C, T, n_fft, hop,
                 float(scale), stream())
        return dx, None, None, None, None


def spec_window_tables(window, n_fft, normalized):
    """Tables + scale of torchaudio Spectrogram(n_fft, win_length=len(window), window,
    normalized, center=False, power=None) (msstftd.py:62-64): torch.stft centres a shorter window
    in n_fft zeros; normalized divides by sqrt(sum window^2) (torchaudio's 'window' norm)."""
    wl = window.numel()
    if wl > n_fft:
        raise ValueError(f'win_length {wl} > n_fft {n_fft}')
    w = torch.zeros(n_fft, device=window.device, dtype=torch.float32)
    left = (n_fft - wl) // 2
    w[left:left + wl] = window.float()
    tab = torch.empty(lib.encx_mel_tables_floats(n_fft, 1), device=window.device, dtype=torch.float32)
    basis = torch.zeros(1, n_fft // 2 + 1, device=window.device, dtype=torch.float32)
    call('encx_mel_tables_init', ptr(tab), ptr(basis), n_fft, 1, stream())  # (mel part unused)
    call('encx_spec_tables_window', ptr(tab), ptr(w), n_fft, stream())
    scale = 1.0 / float(window.double().pow(2).sum().sqrt()) if normalized else 1.0
    return tab, scale


class HingeFn(torch.autograd.Function):
    """scale * sum_i mean(relu(1 + s_i * x_i)) over a list of logits (losses.py:48, 78-79)."""

    @staticmethod
    def forward(ctx, signs, scale, *xs):
        out = torch.zeros(1, device=xs[0].device, dtype=torch.float32)
        ws = _ws(lib.encx_disc_loss_workspace(), out)
        xs = [x.contiguous() for x in xs]
        for s, x in zip(signs, xs):
            _check(x)
            call('encx_hinge_loss', ptr(x), x.numel(), float(s), float(scale), ptr(out), 1, ptr(ws), stream())
        ctx.save_for_backward(*xs)
        ctx.signs, ctx.scale = signs, scale
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        grads = []
        for i, (s, x) in enumerate(zip(ctx.signs, ctx.saved_tensors)):
            if not ctx.needs_input_grad[2 + i]:
                grads.append(None)
                continue
            dx = torch.empty_like(x)
            call('encx_hinge_loss_bwd', ptr(x), x.numel(), float(s), float(ctx.scale), ptr(g), ptr(dx), stream())
            grads.append(dx)
        return (None, None, *grads)


class FeatFn(torch.autograd.Function):
    """scale * sum_i l1(fr_i, ff_i) / mean|fr_i| (losses.py:53): the relative feature-matching
    loss. Gradients flow to the fake maps; the real maps are treated as constants (in the
    reference they only reach the discriminator's parameters, which the generator step's
    balancer never differentiates)."""

    @staticmethod
    def forward(ctx, scale, n_pairs, *maps):
        frs, ffs = maps[:n_pairs], maps[n_pairs:]
        out = torch.zeros(1, device=ffs[0].device, dtype=torch.float32)
        denom = torch.empty(n_pairs, device=out.device, dtype=torch.float32)
        ws = _ws(lib.encx_disc_loss_workspace(), out)
        frs = [f.contiguous() for f in frs]
        ffs = [f.contiguous() for f in ffs]
        # park a map's grad only when the Conv2d reading it produces another map of this loss:
        # that Conv2d is then on every traversal from this loss and is sure to collect it
        slots = [getattr(f, '_encx_feat_slot', None) for f in maps[n_pairs:]]
        live = {id(sl) for sl in slots if sl is not None}
        ctx.slots = [sl if sl is not None and id(sl.consumer_out) in live else None for sl in slots]
        # a parked pair also gets its 1-byte-per-element code (sign(ff - fr), ff > 0), which the
        # reading Conv2d's bwd-data epilogue reads instead of both maps (encx_feat_loss_code)
        ctx.codes = [None] * n_pairs
        for i, (fr, ff) in enumerate(zip(frs, ffs)):
            _check(ff)
            if ctx.slots[i] is not None and ctx.needs_input_grad[2 + n_pairs + i]:
                code = torch.empty(ff.numel(), device=ff.device, dtype=torch.uint8)
                call('encx_feat_loss_code', ptr(fr), ptr(ff), ff.numel(), float(scale), ptr(out),
                     ptr(denom[i:i + 1]), 1, ptr(ws), ptr(code), stream())
                ctx.codes[i] = code
            else:
                call('encx_feat_loss', ptr(fr), ptr(ff), ff.numel(), float(scale), ptr(out), ptr(denom[i:i + 1]),
                     1, ptr(ws), stream())
        ctx.save_for_backward(denom, *frs, *ffs)
        ctx.scale, ctx.n = scale, n_pairs
        for sl, parked in zip(slots, ctx.slots):
            if sl is not None and parked is None:
                sl.autograd_feat = True  # a second gradient path into the map: its reader must not premask
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        denom, *maps = ctx.saved_tensors
        n = ctx.n
        frs, ffs = maps[:n], maps[n:]
        grads = [None] * (2 * n)
        for i, (fr, ff) in enumerate(zip(frs, ffs)):
            if ctx.needs_input_grad[2 + n + i] and ctx.slots[i] is not None:
                ctx.slots[i].pending = (fr, denom[i:i + 1], g, ctx.scale, ctx.codes[i])  # the reading Conv2d adds it
            elif ctx.needs_input_grad[2 + n + i]:
                d = torch.empty_like(ff)
                call('encx_feat_loss_bwd', ptr(fr), ptr(ff), ff.numel(), float(ctx.scale), ptr(denom[i:i + 1]),
                     ptr(g), ptr(d), stream())
                grads[n + i] = d
        return (None, None, *grads)


# ---------------------------------------------------------------------------- 48 kHz model
class AddFn(torch.autograd.Function):
    """x + y (SEANetResnetBlock's shortcut sum, seanet.py:63, where it cannot ride in a conv
    epilogue)."""

    @staticmethod
    def forward(ctx, x, y):
        _check(x)
        x, y = x.contiguous(), y.contiguous()
        out = torch.empty_like(x)
        call('encx_lincomb', ptr(x), ptr(y), ptr(out), x.numel(), 1.0, None, 1.0, stream())
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(x, y):
    return AddFn.apply(x, y)


class GroupNormFn(torch.autograd.Function):
    """nn.GroupNorm(1, C) of norm='time_group_norm' (modules/conv.py:45-49). With a trim the
    statistics cover the whole input and only x[..., trim_left : T - trim_right] is returned:
    NormConvTranspose1d normalises before SConvTranspose1d trims (conv.py:153-156, 248-252)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, trim_left=0, trim_right=0):
        _check(x)
        x = x.contiguous()
        B, C, T = x.shape
        Ty = T - trim_left - trim_right
        y = torch.empty(B, C, Ty, device=x.device, dtype=torch.float32)
        stats = _f32(2 * B, x)
        ws = _ws(lib.encx_groupnorm_workspace(B, C), x)
        call('encx_groupnorm_fwd', ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(stats), ptr(ws), B, C, T,
             trim_left, Ty, float(eps), stream())
        ctx.save_for_backward(x, stats)
        ctx.params = (gamma, beta)
        ctx.win = (trim_left, Ty)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stats = ctx.saved_tensors
        gamma, beta = ctx.params
        dy = dy.contiguous()
        B, C, T = x.shape
        ws = _ws(lib.encx_groupnorm_workspace(B, C), x)
        coef = _f32(2 * B, x)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        want_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        if want_p and _direct(gamma) and _direct(beta):
            dg, db, acc, ret = (gamma.grad if gamma is not None else None,
                                beta.grad if beta is not None else None, 1, False)
        elif want_p:
            dg = torch.empty_like(gamma) if gamma is not None else None
            db = torch.empty_like(beta) if beta is not None else None
            acc, ret = 0, True
        else:
            dg = db = None
            acc, ret = 0, False
        tl, Ty = ctx.win
        call('encx_groupnorm_bwd', ptr(dy), ptr(x), ptr(gamma), ptr(stats), ptr(dx), ptr(dg), ptr(db), 0, acc,
             ptr(ws), ptr(coef), B, C, T, tl, Ty, stream())
        return dx, (dg if ret else None), (db if ret else None), None, None, None


def group_norm(x, gamma, beta, eps=1e-5, trim_left=0, trim_right=0):
    return GroupNormFn.apply(x, gamma, beta, eps, trim_left, trim_right)


class OverlapAddFn(torch.autograd.Function):
    """_linear_overlap_add (utils.py:22-61): triangle-weighted sum of decoded segments."""

    @staticmethod
    def forward(ctx, stride, *frames):
        import ctypes
        frames = [f.contiguous() for f in frames]
        for f in frames:
            _check(f)
        shape = frames[0].shape[:-1]
        BC = int(np.prod(shape))
        lens = [f.shape[-1] for f in frames]
        total = stride * (len(frames) - 1) + lens[-1]
        out = torch.empty(*shape, total, device=frames[0].device, dtype=torch.float32)
        parr = (ctypes.c_void_p * len(frames))(*[f.data_ptr() for f in frames])
        larr = (ctypes.c_int64 * len(frames))(*lens)
        call('encx_overlap_add', parr, larr, len(frames), stride, BC, ptr(out), stream())
        ctx.cfg = (stride, lens, BC, total, shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        stride, lens, BC, total, shape = ctx.cfg
        dout = dout.contiguous()
        grads = []
        for k, L in enumerate(lens):
            d = torch.empty(*shape, L, device=dout.device, dtype=torch.float32)
            call('encx_overlap_add_bwd', ptr(dout), len(lens), stride, lens[0], BC, total, k, L, ptr(d), stream())
            grads.append(d)
        return (None, *grads)


def linear_overlap_add(frames, stride):
    if len(frames) == 1:
        return frames[0]
    return OverlapAddFn.apply(stride, *frames)


# ---------------------------------------------------------------------------- .ecdc payload
def pack_codes(codes, bits):
    """BitPacker over whole frames (binary.py:55-88, push order compress.py:88-98): codes
    [F][K][T] int64 on the GPU (any strides) -> uint8 [F][ceil(K*T*bits/8)] on the GPU, each
    frame its own byte-aligned stream. Raises ValueError if a code does not fit in `bits`."""
    if not codes.is_cuda or codes.dtype != torch.int64 or codes.dim() != 3:
        raise RuntimeError('encx: pack_codes takes int64 [F][K][T] codes on the GPU (no CPU fallback)')
    ensure_device(codes.device)
    Fn, K, T = codes.shape
    nbytes = int(lib.encx_bitpack_bytes(K * T, int(bits)))
    if nbytes < 0:
        raise ValueError(f'encx: bits must be in 1..32 (got {bits})')
    out = torch.empty(Fn, nbytes, device=codes.device, dtype=torch.uint8)
    err = torch.zeros(1, device=codes.device, dtype=torch.int32)
    s_f, s_k, s_t = codes.stride()
    call('encx_bitpack', codes.data_ptr(), s_f, s_k, s_t, Fn, K, T, int(bits), out.data_ptr(), nbytes,
         err.data_ptr(), stream())
    return out, err


def unpack_codes(data, K, T, bits):
    """BitUnpacker.pull (binary.py:105-123) of F frames: data uint8 [F][>= ceil(K*T*bits/8)]
    on the GPU -> int64 codes [F][K][T]."""
    if not data.is_cuda or data.dtype != torch.uint8 or data.dim() != 2 or not data.is_contiguous():
        raise RuntimeError('encx: unpack_codes takes contiguous uint8 [F][bytes] on the GPU (no CPU fallback)')
    ensure_device(data.device)
    Fn = data.shape[0]
    need = int(lib.encx_bitpack_bytes(K * T, int(bits)))
    if need < 0:
        raise ValueError(f'encx: bits must be in 1..32 (got {bits})')
    if data.shape[1] < need:
        raise EOFError('The stream ended sooner than expected.')
    codes = torch.empty(Fn, K, T, device=data.device, dtype=torch.int64)
    call('encx_bitunpack', data.data_ptr(), data.shape[1], Fn, K, T, int(bits), codes.data_ptr(),
         K * T, T, 1, stream())
    return codes
