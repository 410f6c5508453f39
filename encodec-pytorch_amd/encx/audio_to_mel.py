"""Audio2Mel (audio_to_mel.py of the reference) on the encx DFT/mel kernels.

`mel_filterbank` restates librosa.filters.mel(htk=False, norm='slaney') (the reference's
audio_to_mel.py:24 call; librosa is not in this image). It is host setup, run once per scale;
the per-step STFT, power, mel projection and log run in HIP (csrc/mel.hip).
"""
import numpy as np
import torch
import torch.nn as nn

from . import ops


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    lin = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    safe = np.maximum(f, min_log_hz)
    return np.where(f >= min_log_hz, min_log_mel + np.log(safe / min_log_hz) / logstep, lin)


def _mel_to_hz(mm):
    mm = np.asanyarray(mm, dtype=np.float64)
    f_sp = 200.0 / 3
    lin = f_sp * mm
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(mm >= min_log_mel, min_log_hz * np.exp(logstep * (mm - min_log_mel)), lin)


def mel_filterbank(sr, n_fft, n_mels=128, fmin=0.0, fmax=None):
    """Triangular slaney-normalised mel filters, float32 [n_mels, 1 + n_fft // 2]."""
    fmax = float(sr) / 2 if fmax is None else fmax
    freqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    edges = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    widths = np.diff(edges)
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    for i in range(n_mels):
        rise = (freqs - edges[i]) / widths[i]
        fall = (edges[i + 2] - freqs) / widths[i + 1]
        w[i] = np.maximum(0, np.minimum(rise, fall))
    w *= (2.0 / (edges[2:n_mels + 2] - edges[:n_mels]))[:, None]
    return w


class Audio2Mel(nn.Module):
    """audio_to_mel.py:7-55: log10(clamp(mel_basis @ |STFT(reflect_pad(x))|^2, 1e-5))."""

    def __init__(self, n_fft=1024, hop_length=256, win_length=1024, sampling_rate=22050,
                 n_mel_channels=80, mel_fmin=0.0, mel_fmax=None, device='cuda'):
        super().__init__()
        if win_length > n_fft or hop_length > n_fft:
            raise ValueError('Audio2Mel: win_length and hop_length must not exceed n_fft (torch.stft)')
        # the loss configuration (hop n/4, win n) runs the fused mel kernels; any other framing the
        # windowed-spectrogram path (ops.logmel_framed)
        self._loss_framing = hop_length * 4 == n_fft and win_length == n_fft
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.win_length = win_length
        self.sampling_rate = sampling_rate
        self.n_mel_channels = n_mel_channels
        self.mel_fmin, self.mel_fmax = float(mel_fmin), mel_fmax
        self.register_buffer('mel_basis', torch.from_numpy(
            mel_filterbank(sampling_rate, n_fft, n_mel_channels, mel_fmin, mel_fmax)))
        self.register_buffer('window', torch.hann_window(win_length).float())

    def forward(self, audioin):
        if self._loss_framing:
            return ops.logmel(audioin, self.n_fft, self.n_mel_channels, self.sampling_rate, self.mel_fmin,
                              self.mel_fmax)
        return ops.logmel_framed(audioin, self.n_fft, self.hop_length, self.win_length, self.n_mel_channels,
                                 self.sampling_rate, self.mel_fmin, self.mel_fmax)
