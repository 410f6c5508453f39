"""Convolution wrappers mirroring modules/conv.py of the reference, on the encx HIP kernels.

Same class names, constructor arguments and state-dict keys (`conv.conv.weight_g/weight_v/
bias`, `convtr.convtr.*`), so reference checkpoints load unchanged. forward() takes two
optional fusion hooks the reference does not have: `act='elu'` applies the preceding nn.ELU
inside the conv's input staging, and `res=` adds a residual in the conv's epilogue.
"""
import math
import typing as tp

import torch
from torch import nn

from .. import ops

CONV_NORMALIZATIONS = frozenset(['none', 'weight_norm', 'spectral_norm',
                                 'time_layer_norm', 'layer_norm', 'time_group_norm'])

get_extra_padding_for_conv1d = None  # bound below (kept as the reference's public name)


def _extra(x: torch.Tensor, kernel_size: int, stride: int, padding_total: int = 0) -> int:
    """modules/conv.py:54-61 (takes the tensor like the reference)."""
    return ops.extra_padding_for_conv1d(x.shape[-1], kernel_size, stride, padding_total)


get_extra_padding_for_conv1d = _extra


class _ConvParams(nn.Module):
    """Parameter holder named like torch's weight-normed conv (weight_g, weight_v, bias)."""

    def __init__(self, wshape, out_channels, norm, bias=True, g_rows=None):
        super().__init__()
        self.norm_type = norm
        fan_in = wshape[1] * math.prod(wshape[2:])
        bound = 1.0 / math.sqrt(fan_in)
        v = torch.empty(wshape).uniform_(-bound, bound)
        if norm == 'weight_norm':
            self.weight_v = nn.Parameter(v)
            self.weight_g = nn.Parameter(v.reshape(v.shape[0], -1).norm(dim=1).reshape(
                (v.shape[0],) + (1,) * (v.dim() - 1)).clone())
        elif norm in ('none', 'time_group_norm'):
            self.weight = nn.Parameter(v)
        else:
            raise NotImplementedError(f'encx: conv norm {norm!r} is not on the hot path')
        self.bias = nn.Parameter(torch.empty(out_channels).uniform_(-bound, bound)) if bias else None

    def wv(self):
        if self.norm_type == 'weight_norm':
            return self.weight_v, self.weight_g
        return self.weight, None


class NormConv1d(nn.Module):
    """modules/conv.py:108-122 (`conv` holds the params; `norm` the optional GroupNorm)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1, groups=1,
                 bias=True, causal=False, norm='none', norm_kwargs={}):
        super().__init__()
        assert norm in CONV_NORMALIZATIONS
        if groups != 1:
            raise NotImplementedError('encx: grouped convs are not used by EnCodec')
        self.conv = _ConvParams((out_channels, in_channels, kernel_size), out_channels, norm, bias)
        if norm == 'time_group_norm':
            if causal:
                raise ValueError("GroupNorm doesn't support causal evaluation.")
            self.norm = nn.GroupNorm(1, out_channels, **norm_kwargs)  # conv.py:45-49 (params only)
        else:
            self.norm = nn.Identity()
        self.norm_type = norm
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.dilation = kernel_size, stride, dilation


class NormConvTranspose1d(nn.Module):
    """modules/conv.py:142-156 (weight [Cin, Cout, K]; weight_norm over dim 0 = Cin)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, causal=False,
                 norm='none', norm_kwargs={}):
        super().__init__()
        assert norm in CONV_NORMALIZATIONS
        self.convtr = _ConvParams((in_channels, out_channels, kernel_size), out_channels, norm)
        if norm == 'time_group_norm':
            if causal:
                raise ValueError("GroupNorm doesn't support causal evaluation.")
            self.norm = nn.GroupNorm(1, out_channels, **norm_kwargs)
        else:
            self.norm = nn.Identity()
        self.norm_type = norm
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride = kernel_size, stride


class NormConv2d(nn.Module):
    """modules/conv.py:125-139: Conv2d with weight norm (or none), the DiscriminatorSTFT layer.
    forward(x, act) also applies the LeakyReLU(0.2) that follows every inner layer of the
    discriminator (msstftd.py:100-103); param_grads=False runs the layer as a function of its
    input only (the generator step differentiates the discriminator w.r.t. audio, never its
    weights)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1, padding=0,
                 bias=True, norm='none', norm_kwargs={}):
        super().__init__()
        assert norm in CONV_NORMALIZATIONS
        pair = lambda v: tuple(v) if isinstance(v, (tuple, list)) else (v, v)
        self.kernel_size, self.stride = pair(kernel_size), pair(stride)
        self.dilation, self.padding = pair(dilation), pair(padding)
        self.conv = _ConvParams((out_channels, in_channels) + self.kernel_size, out_channels, norm, bias)
        self.norm = nn.Identity()
        self.norm_type = norm

    def forward(self, x, act=False, param_grads=True, mode=None, first=False):
        v, g = self.conv.wv()
        b = self.conv.bias
        if not param_grads:
            v = v.detach()
            g = g.detach() if g is not None else None
            b = b.detach() if b is not None else None
        return ops.conv2d(x, v, g, b, self.kernel_size, self.stride, self.dilation, self.padding, act,
                          mode if mode is not None else ops.DiscGradMode(), first)


class SConv1d(nn.Module):
    """modules/conv.py:175-210: causal / asymmetric reflect padding + conv, one HIP launch."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 dilation: int = 1, groups: int = 1, bias: bool = True, causal: bool = False,
                 norm: str = 'none', norm_kwargs: tp.Dict[str, tp.Any] = {},
                 pad_mode: str = 'reflect'):
        super().__init__()
        self.conv = NormConv1d(in_channels, out_channels, kernel_size, stride, dilation=dilation,
                               groups=groups, bias=bias, causal=causal, norm=norm,
                               norm_kwargs=norm_kwargs)
        self.causal = causal
        self.pad_mode = pad_mode

    def forward(self, x, act=None, res=None, link=None, link_role=None):
        c = self.conv
        v, g = c.conv.wv()
        if c.norm_type != 'time_group_norm':
            return ops.conv1d(x, v, g, c.conv.bias, c.kernel_size, c.stride, c.dilation, self.causal,
                              self.pad_mode, act, res, link, link_role)
        # conv -> GroupNorm(1, C) (NormConv1d.forward, conv.py:119-122); a residual is added
        # after the norm, so it is not fused into the conv epilogue here
        y = ops.conv1d(x, v, g, c.conv.bias, c.kernel_size, c.stride, c.dilation, self.causal,
                       self.pad_mode, act, None)
        y = ops.group_norm(y, c.norm.weight, c.norm.bias, c.norm.eps)
        return y if res is None else ops.add(y, res)


class SConvTranspose1d(nn.Module):
    """modules/conv.py:213-252: ConvTranspose1d + causal/asymmetric trim, one HIP launch."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 causal: bool = False, norm: str = 'none', trim_right_ratio: float = 1.,
                 norm_kwargs: tp.Dict[str, tp.Any] = {}):
        super().__init__()
        self.convtr = NormConvTranspose1d(in_channels, out_channels, kernel_size, stride,
                                          causal=causal, norm=norm, norm_kwargs=norm_kwargs)
        self.causal = causal
        self.trim_right_ratio = trim_right_ratio
        assert self.causal or self.trim_right_ratio == 1., \
            "`trim_right_ratio` != 1.0 only makes sense for causal convolutions"
        assert 0. <= self.trim_right_ratio <= 1.

    def forward(self, x, act=None):
        c = self.convtr
        v, g = c.convtr.wv()
        if c.norm_type != 'time_group_norm':
            return ops.convtr1d(x, v, g, c.convtr.bias, c.kernel_size, c.stride, self.causal,
                                self.trim_right_ratio, act)
        # NormConvTranspose1d.forward normalises the FULL transposed-conv output (conv.py:153-156)
        # and only then does SConvTranspose1d trim it (:248-252): the GroupNorm statistics include
        # the trimmed edge samples, so the conv runs untrimmed and the norm writes the window
        y = ops.convtr1d(x, v, g, c.convtr.bias, c.kernel_size, c.stride, self.causal,
                         self.trim_right_ratio, act, untrimmed=True)
        tl, tout = ops.convtr_geometry(x.shape[-1], c.kernel_size, c.stride, self.causal, self.trim_right_ratio)
        return ops.group_norm(y, c.norm.weight, c.norm.bias, c.norm.eps, tl, y.shape[-1] - tl - tout)
