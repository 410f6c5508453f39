"""MS-STFT discriminator (msstftd.py of the reference) and its losses on the encx kernels.

Same classes, constructor arguments and state-dict keys (`discriminators.{k}.convs.{i}.conv.*`,
`discriminators.{k}.conv_post.conv.*`). forward(x, param_grads=True, mode=None) takes two
arguments the reference does not have: param_grads=False evaluates the discriminator as a
function of its input only; mode (ops.DiscGradMode) lets one forward graph serve both phases
of a GAN step (Trainer.step), so no weight-gradient kernel runs in the generator phase and the
discriminator phase reuses the generator phase's activations.
"""
import typing as tp

import torch
from torch import nn

from . import ops
from .modules.conv import NormConv2d

FeatureMapType = tp.List[torch.Tensor]
LogitsType = torch.Tensor
DiscriminatorOutput = tp.Tuple[tp.List[LogitsType], tp.List[FeatureMapType]]


def get_2d_padding(kernel_size: tp.Tuple[int, int], dilation: tp.Tuple[int, int] = (1, 1)):
    """msstftd.py:24-25."""
    return (((kernel_size[0] - 1) * dilation[0]) // 2, ((kernel_size[1] - 1) * dilation[1]) // 2)


class _SpecTransform(nn.Module):
    """Holds the `window` buffer torchaudio's Spectrogram registers (msstftd.py:62-64), so the
    state dict matches the reference's key for key; the transform itself is ops.DiscSpecFn."""

    def __init__(self, win_length):
        super().__init__()
        self.register_buffer('window', torch.hann_window(win_length))


class DiscriminatorSTFT(nn.Module):
    """msstftd.py:28-105."""

    def __init__(self, filters: int, in_channels: int = 1, out_channels: int = 1,
                 n_fft: int = 1024, hop_length: int = 256, win_length: int = 1024, max_filters: int = 1024,
                 filters_scale: int = 1, kernel_size: tp.Tuple[int, int] = (3, 9), dilations: tp.List = [1, 2, 4],
                 stride: tp.Tuple[int, int] = (1, 2), normalized: bool = True, norm: str = 'weight_norm',
                 activation: str = 'LeakyReLU', activation_params: dict = {'negative_slope': 0.2},
                 sample_rate: int = 24000):
        super().__init__()
        assert len(kernel_size) == 2 and len(stride) == 2
        if activation != 'LeakyReLU' or activation_params.get('negative_slope', 0.01) != 0.2:
            raise NotImplementedError('encx DiscriminatorSTFT: LeakyReLU(0.2) is fused into the convs')
        self.filters = filters
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.win_length = win_length
        self.normalized = normalized
        self.sample_rate = sample_rate
        self.spec_transform = _SpecTransform(win_length)
        self._win_tables = None  # (device / window key, (tables, scale)) when win_length != n_fft or not normalized
        spec_channels = 2 * in_channels
        self.convs = nn.ModuleList()
        self.convs.append(NormConv2d(spec_channels, filters, kernel_size=kernel_size,
                                     padding=get_2d_padding(kernel_size)))
        in_chs = min(filters_scale * filters, max_filters)
        for i, dilation in enumerate(dilations):
            out_chs = min((filters_scale ** (i + 1)) * filters, max_filters)
            self.convs.append(NormConv2d(in_chs, out_chs, kernel_size=kernel_size, stride=stride,
                                         dilation=(dilation, 1),
                                         padding=get_2d_padding(kernel_size, (dilation, 1)), norm=norm))
            in_chs = out_chs
        out_chs = min((filters_scale ** (len(dilations) + 1)) * filters, max_filters)
        k2 = (kernel_size[0], kernel_size[0])
        self.convs.append(NormConv2d(in_chs, out_chs, kernel_size=k2, padding=get_2d_padding(k2), norm=norm))
        self.conv_post = NormConv2d(out_chs, out_channels, kernel_size=k2, padding=get_2d_padding(k2), norm=norm)

    def forward(self, x: torch.Tensor, param_grads: bool = True, mode=None):
        """msstftd.py:86-105: x [B, C, T] -> (logits [B, out, frames, bins'], 5 feature maps)."""
        fmap = []
        window = None  # the reference's configuration: hann(n_fft), normalized (precomputed tables)
        if self.win_length != self.n_fft or not self.normalized:
            key = (str(x.device), self.spec_transform.window.data_ptr())
            if self._win_tables is None or self._win_tables[0] != key:
                self._win_tables = (key, ops.spec_window_tables(self.spec_transform.window, self.n_fft,
                                                                self.normalized))
            window = self._win_tables[1]
        z = ops.DiscSpecFn.apply(x, self.n_fft, self.hop_length, self.sample_rate, window)
        for i, layer in enumerate(self.convs):
            z = layer(z, act=True, param_grads=param_grads, mode=mode, first=i == 0)
            fmap.append(z)
        z = self.conv_post(z, act=False, param_grads=param_grads, mode=mode)
        return z, fmap


class MultiScaleSTFTDiscriminator(nn.Module):
    """msstftd.py:108-149."""

    def __init__(self, filters: int, in_channels: int = 1, out_channels: int = 1,
                 n_ffts: tp.List[int] = [1024, 2048, 512], hop_lengths: tp.List[int] = [256, 512, 128],
                 win_lengths: tp.List[int] = [1024, 2048, 512], **kwargs):
        super().__init__()
        assert len(n_ffts) == len(hop_lengths) == len(win_lengths)
        self.discriminators = nn.ModuleList([
            DiscriminatorSTFT(filters, in_channels=in_channels, out_channels=out_channels,
                              n_fft=n_ffts[i], win_length=win_lengths[i], hop_length=hop_lengths[i], **kwargs)
            for i in range(len(n_ffts))
        ])
        self.num_discriminators = len(self.discriminators)

    def forward(self, x: torch.Tensor, param_grads: bool = True, mode=None) -> DiscriminatorOutput:
        """mode: an ops.DiscGradMode shared by every layer of this forward's graph (Trainer
        flips it between the generator and the discriminator phase of one step)."""
        logits, fmaps = [], []
        for disc in self.discriminators:
            logit, fmap = disc(x, param_grads=param_grads, mode=mode)
            logits.append(logit)
            fmaps.append(fmap)
        return logits, fmaps


def adversarial_losses(fmap_real, logits_fake, fmap_fake):
    """l_g and l_feat of total_loss (losses.py:44-56): l_g = sum_k mean(relu(1 - D_k(y))) / K,
    divided by K again at :56 (reproduced); l_feat = sum_{k,l} l1(fr, ff) / mean|fr| / (K L)."""
    K = len(logits_fake)
    l_g = ops.HingeFn.apply([-1.0] * K, 1.0 / (K * K), *logits_fake)
    frs = [f for fm in fmap_real for f in fm]
    ffs = [f for fm in fmap_fake for f in fm]
    KL = len(fmap_real) * len(fmap_real[0])
    l_feat = ops.FeatFn.apply(1.0 / KL, len(frs), *frs, *ffs)
    return l_g, l_feat


def hinge_disc_loss(logits_real, logits_fake):
    """disc_loss (losses.py:65-80): sum_k mean(relu(1 - D_k(x))) + mean(relu(1 + D_k(y))), / K."""
    K = len(logits_real)
    return ops.HingeFn.apply([-1.0] * K + [1.0] * K, 1.0 / K, *logits_real, *logits_fake)
