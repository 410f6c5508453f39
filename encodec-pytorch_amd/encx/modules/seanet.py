"""SEANet encoder / decoder (modules/seanet.py of the reference) on the encx kernels.

The layer lists and indices are the reference's (nn.Sequential with the nn.ELU entries kept as
parameter-free placeholders), so state-dict keys match. forward() walks the list and folds
every ELU into the conv that consumes it, and each resblock's residual sum into its second
conv's epilogue: the SEANet stack never materialises an activation tensor on its own.
"""
import os
import types
import typing as tp

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .conv import SConv1d, SConvTranspose1d
from .lstm import SLSTM


def _act_name(activation):
    if activation != 'ELU':
        raise NotImplementedError(f'encx fuses nn.ELU only (got {activation})')
    return 'elu'


class SEANetResnetBlock(nn.Module):
    """modules/seanet.py:21-63: shortcut(x) + conv1x1(ELU(conv_k(ELU(x))))."""

    def __init__(self, dim: int, kernel_sizes: tp.List[int] = [3, 1], dilations: tp.List[int] = [1, 1],
                 activation: str = 'ELU', activation_params: dict = {'alpha': 1.0},
                 norm: str = 'weight_norm', norm_params: tp.Dict[str, tp.Any] = {}, causal: bool = False,
                 pad_mode: str = 'reflect', compress: int = 2, true_skip: bool = True):
        super().__init__()
        assert len(kernel_sizes) == len(dilations), 'Number of kernel sizes should match number of dilations'
        assert activation_params.get('alpha', 1.0) == 1.0
        self.act = _act_name(activation)
        hidden = dim // compress
        block = []
        for i, (kernel_size, dilation) in enumerate(zip(kernel_sizes, dilations)):
            in_chs = dim if i == 0 else hidden
            out_chs = dim if i == len(kernel_sizes) - 1 else hidden
            block += [nn.ELU(**activation_params),
                      SConv1d(in_chs, out_chs, kernel_size=kernel_size, dilation=dilation, norm=norm,
                              norm_kwargs=norm_params, causal=causal, pad_mode=pad_mode)]
        self.block = nn.Sequential(*block)
        self.shortcut: nn.Module
        if true_skip:
            self.shortcut = nn.Identity()
        else:
            self.shortcut = SConv1d(dim, dim, kernel_size=1, norm=norm, norm_kwargs=norm_params,
                                    causal=causal, pad_mode=pad_mode)
        self._fuse = (not true_skip and list(kernel_sizes) == [3, 1] and list(dilations) == [1, 1]
                      and compress == 2 and dim in (32, 64) and causal and pad_mode == 'reflect'
                      and norm == 'weight_norm')

    def _fusable(self, x):
        """The EnCodec block (k3 + 1x1, compress 2, 1x1 shortcut, causal reflect weight_norm
        convs) at a high rate: one fused kernel per direction (ops.ResBlockFn)."""
        if not self._fuse or x.dim() != 3 or x.shape[-1] < ops.RESBLOCK_TMIN:
            return False
        return os.environ.get('ENCX_RESBLOCK', '1') != '0'

    def forward(self, x):
        if self._fusable(x):
            c1, c2 = [m for m in self.block if isinstance(m, SConv1d)]
            ps = [(c.conv.conv.weight_v, c.conv.conv.weight_g, c.conv.conv.bias) for c in (c1, c2, self.shortcut)]
            return ops.resblock(x, *ps)
        convs = [m for m in self.block if isinstance(m, SConv1d)]
        linkable = (len(convs) > 1 and torch.is_grad_enabled() and x.requires_grad
                    and all(c.conv.norm_type != 'time_group_norm' for c in convs))
        # conv shortcut (true_skip False, the EnCodec default): the shortcut conv and the head
        # conv both read x; whichever backward runs second adds its bwd-data result into the
        # other's (ops.Conv1dFn 'join'), so autograd sees one grad for x and launches no add
        join = None
        if linkable and isinstance(self.shortcut, SConv1d) and self.shortcut.conv.norm_type != 'time_group_norm':
            join = types.SimpleNamespace(grad=None)
            sc = self.shortcut(x, link=join, link_role='join')
        else:
            sc = self.shortcut(x)
        # identity shortcut: the skip gradient is summed into the head conv's bwd-data output
        # (ops.Conv1dFn 'head' / 'tail' link) instead of by autograd's elementwise add
        link = None
        if linkable and isinstance(self.shortcut, nn.Identity):
            link = types.SimpleNamespace(grad=None)
        h = x
        for i, c in enumerate(convs):
            last = i == len(convs) - 1
            if join is not None:
                h = c(h, act=self.act, res=sc if last else None, link=join if i == 0 else None,
                      link_role='join' if i == 0 else None)
                continue
            role = None if link is None else ('tail' if last else 'head' if i == 0 else None)
            h = c(h, act=self.act, res=sc if last else None, link=link, link_role=role)
        return h


def _run(seq, x):
    pending = None
    for m in seq:
        if isinstance(m, nn.ELU):
            assert pending is None
            pending = 'elu'
        elif isinstance(m, (SConv1d, SConvTranspose1d)):
            x = m(x, act=pending)
            pending = None
        else:
            assert pending is None, 'ELU must precede a conv'
            x = m(x)
    assert pending is None
    return x


class SEANetEncoder(nn.Module):
    """modules/seanet.py:66-144."""

    def __init__(self, channels: int = 1, dimension: int = 128, n_filters: int = 32, n_residual_layers: int = 1,
                 ratios: tp.List[int] = [8, 5, 4, 2], activation: str = 'ELU', activation_params: dict = {'alpha': 1.0},
                 norm: str = 'weight_norm', norm_params: tp.Dict[str, tp.Any] = {}, kernel_size: int = 7,
                 last_kernel_size: int = 7, residual_kernel_size: int = 3, dilation_base: int = 2, causal: bool = False,
                 pad_mode: str = 'reflect', true_skip: bool = False, compress: int = 2, lstm: int = 2):
        super().__init__()
        self.channels = channels
        self.dimension = dimension
        self.n_filters = n_filters
        self.ratios = list(reversed(ratios))
        del ratios
        self.n_residual_layers = n_residual_layers
        self.hop_length = np.prod(self.ratios)
        _act_name(activation)
        mult = 1
        model: tp.List[nn.Module] = [
            SConv1d(channels, mult * n_filters, kernel_size, norm=norm, norm_kwargs=norm_params,
                    causal=causal, pad_mode=pad_mode)]
        for ratio in self.ratios:
            for j in range(n_residual_layers):
                model += [SEANetResnetBlock(mult * n_filters, kernel_sizes=[residual_kernel_size, 1],
                                            dilations=[dilation_base ** j, 1], norm=norm, norm_params=norm_params,
                                            activation=activation, activation_params=activation_params,
                                            causal=causal, pad_mode=pad_mode, compress=compress,
                                            true_skip=true_skip)]
            model += [nn.ELU(**activation_params),
                      SConv1d(mult * n_filters, mult * n_filters * 2, kernel_size=ratio * 2, stride=ratio,
                              norm=norm, norm_kwargs=norm_params, causal=causal, pad_mode=pad_mode)]
            mult *= 2
        if lstm:
            model += [SLSTM(mult * n_filters, num_layers=lstm)]
        model += [nn.ELU(**activation_params),
                  SConv1d(mult * n_filters, dimension, last_kernel_size, norm=norm, norm_kwargs=norm_params,
                          causal=causal, pad_mode=pad_mode)]
        self.model = nn.Sequential(*model)

    def forward(self, x):
        return _run(self.model, x)


class SEANetDecoder(nn.Module):
    """modules/seanet.py:147-238."""

    def __init__(self, channels: int = 1, dimension: int = 128, n_filters: int = 32, n_residual_layers: int = 1,
                 ratios: tp.List[int] = [8, 5, 4, 2], activation: str = 'ELU', activation_params: dict = {'alpha': 1.0},
                 final_activation: tp.Optional[str] = None, final_activation_params: tp.Optional[dict] = None,
                 norm: str = 'weight_norm', norm_params: tp.Dict[str, tp.Any] = {}, kernel_size: int = 7,
                 last_kernel_size: int = 7, residual_kernel_size: int = 3, dilation_base: int = 2, causal: bool = False,
                 pad_mode: str = 'reflect', true_skip: bool = False, compress: int = 2, lstm: int = 2,
                 trim_right_ratio: float = 1.0):
        super().__init__()
        self.dimension = dimension
        self.channels = channels
        self.n_filters = n_filters
        self.ratios = ratios
        del ratios
        self.n_residual_layers = n_residual_layers
        self.hop_length = np.prod(self.ratios)
        _act_name(activation)
        if final_activation is not None:
            raise NotImplementedError('encx: final_activation is unused by EnCodec configs')
        mult = int(2 ** len(self.ratios))
        model: tp.List[nn.Module] = [
            SConv1d(dimension, mult * n_filters, kernel_size, norm=norm, norm_kwargs=norm_params,
                    causal=causal, pad_mode=pad_mode)]
        if lstm:
            model += [SLSTM(mult * n_filters, num_layers=lstm)]
        for ratio in self.ratios:
            model += [nn.ELU(**activation_params),
                      SConvTranspose1d(mult * n_filters, mult * n_filters // 2, kernel_size=ratio * 2,
                                       stride=ratio, norm=norm, norm_kwargs=norm_params, causal=causal,
                                       trim_right_ratio=trim_right_ratio)]
            for j in range(n_residual_layers):
                model += [SEANetResnetBlock(mult * n_filters // 2, kernel_sizes=[residual_kernel_size, 1],
                                            dilations=[dilation_base ** j, 1], activation=activation,
                                            activation_params=activation_params, norm=norm,
                                            norm_params=norm_params, causal=causal, pad_mode=pad_mode,
                                            compress=compress, true_skip=true_skip)]
            mult //= 2
        model += [nn.ELU(**activation_params),
                  SConv1d(n_filters, channels, last_kernel_size, norm=norm, norm_kwargs=norm_params,
                          causal=causal, pad_mode=pad_mode)]
        self.model = nn.Sequential(*model)

    def forward(self, z):
        return _run(self.model, z)
