"""Import shims that let the reference (`/root/reference`) run in THIS container only.

Test infrastructure for `make_goldens.py`; never used on the GPU box and never by the
product. The reference needs three packages this image lacks:

* `torchaudio.transforms.Spectrogram` (used by `msstftd.py:62-64`): restated as
  `torch.stft(center=False, onesided=True, return_complex=True)` followed by the
  `normalized=True` window norm `/ sqrt(sum(window**2))` (torchaudio's `spectrogram`).
* `librosa.filters.mel` (used by `audio_to_mel.py:24`): slaney mel scale + slaney area
  norm, from `oracle.encodec_oracle.mel_filterbank` (itself cross-checked against
  `transformers.audio_utils.mel_filter_bank` in tests/test_oracle.py).
* `soundfile` (imported by `utils.py:16`, unused on the path): empty stub.

`audio_to_mel.py:23,25` and `losses.py:31-34,76` hard-code CUDA; the shim maps
`device='cuda'` to the CPU and `Tensor.cuda()` to identity while the reference is imported.
"""
import sys
import types

import numpy as np
import torch

REF = '/root/reference'


def _install():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from oracle.encodec_oracle import mel_filterbank

    sf = types.ModuleType('soundfile')
    sys.modules.setdefault('soundfile', sf)

    ta = types.ModuleType('torchaudio')
    ta_t = types.ModuleType('torchaudio.transforms')

    class Spectrogram(torch.nn.Module):
        def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0,
                     window_fn=torch.hann_window, power=2.0, normalized=False,
                     wkwargs=None, center=True, pad_mode='reflect', onesided=True):
            super().__init__()
            assert pad == 0 and power is None
            self.n_fft = n_fft
            self.win_length = win_length or n_fft
            self.hop_length = hop_length or self.win_length // 2
            self.register_buffer('window', window_fn(self.win_length))
            self.normalized = normalized
            self.center = center
            self.pad_mode = pad_mode or 'reflect'

        def forward(self, x):
            shape = x.shape
            x = x.reshape(-1, shape[-1])
            s = torch.stft(x, n_fft=self.n_fft, hop_length=self.hop_length,
                           win_length=self.win_length, window=self.window,
                           center=self.center, pad_mode=self.pad_mode, normalized=False,
                           onesided=True, return_complex=True)
            s = s.reshape(shape[:-1] + s.shape[-2:])
            if self.normalized:
                s = s / self.window.pow(2.).sum().sqrt()
            return s

    ta_t.Spectrogram = Spectrogram
    ta.transforms = ta_t
    ta.load = None
    ta.save = None
    sys.modules.setdefault('torchaudio', ta)
    sys.modules.setdefault('torchaudio.transforms', ta_t)

    lb = types.ModuleType('librosa')
    lb_f = types.ModuleType('librosa.filters')

    def mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, **kw):
        return mel_filterbank(sr, n_fft, n_mels, fmin, fmax)

    lb_f.mel = mel
    lb.filters = lb_f
    sys.modules.setdefault('librosa', lb)
    sys.modules.setdefault('librosa.filters', lb_f)

    # 'cuda' -> cpu while the reference runs here (no GPU in this container)
    _tensor, _hann = torch.tensor, torch.hann_window

    def _fix(kw):
        if str(kw.get('device', '')).startswith('cuda'):
            kw['device'] = 'cpu'
        return kw

    torch.tensor = lambda *a, **kw: _tensor(*a, **_fix(kw))
    torch.hann_window = lambda *a, **kw: _hann(*a, **_fix(kw))
    torch.Tensor.cuda = lambda self, *a, **kw: self


def import_reference():
    _install()
    import model as ref_model  # noqa: E402
    import losses as ref_losses
    import msstftd as ref_msstftd
    import balancer as ref_balancer
    import audio_to_mel as ref_mel
    import scheduler as ref_sched
    import modules as ref_modules
    import quantization as ref_q
    return types.SimpleNamespace(model=ref_model, losses=ref_losses, msstftd=ref_msstftd,
                                 balancer=ref_balancer, audio_to_mel=ref_mel,
                                 scheduler=ref_sched, modules=ref_modules, quantization=ref_q,
                                 np=np)
