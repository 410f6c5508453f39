"""Training batches from clips resident in HBM (customAudioDataset.py of the reference).

The reference decodes every file per item on the host (librosa.load), crops a random
`tensor_cut` window, expands mono to `channels` and zero-pads the batch (collate_fn).
`CustomAudioDataset` keeps the same configuration fields, `__len__`, and random-crop rule,
but decodes each file once into an `AudioPool` in HBM (288 GB holds ~1000 h of 24 kHz
fp32 audio). `make_batch` then draws the crop starts on the host with Python's `random`, in the
reference's call order (so the same seed gives the same windows), and builds the
[B][C][Tmax] batch with one `encx_crop_collate` launch. There is no CPU batch path.

File decoding: PCM WAV through the standard library `wave` module (the image has no librosa
or soundfile). It needs the model's sample rate (no resampler) and downmixes to mono by
channel mean, as librosa.load(mono=True) does.
"""
import random
import typing as tp
import wave

import numpy as np
import torch

from ._lib import call, stream, ensure_device


def load_wav(path: str, sample_rate: int, mono: bool) -> np.ndarray:
    """-> float32 [C][T] in [-1, 1). customAudioDataset.py:38-42 (librosa.load(sr, mono))."""
    with wave.open(path, 'rb') as w:
        sr, ch, width, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    if sr != sample_rate:
        raise ValueError(f'{path}: sample rate {sr} != {sample_rate} (no resampler in encx)')
    if width == 2:
        x = np.frombuffer(raw, '<i2').astype(np.float32) / 32768.0
    elif width == 4:
        x = np.frombuffer(raw, '<i4').astype(np.float32) / 2147483648.0
    elif width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f'{path}: unsupported sample width {width}')
    x = x.reshape(-1, ch).T
    if mono:
        x = x.mean(0, keepdims=True)
    return np.ascontiguousarray(x, np.float32)


class AudioPool:
    """Decoded clips packed back to back in one device buffer; clip i is
    [channels[i]][lengths[i]] at offsets[i]."""

    def __init__(self, clips: tp.Sequence[np.ndarray], device='cuda'):
        self.device = torch.device(device)
        arrs = [a[None] if a.ndim == 1 else a for a in (np.asarray(c, np.float32) for c in clips)]
        self.channels = np.array([a.shape[0] for a in arrs], np.int64)
        self.lengths = np.array([a.shape[1] for a in arrs], np.int64)
        sizes = self.channels * self.lengths
        self.offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        flat = np.concatenate([a.reshape(-1) for a in arrs]) if arrs else np.zeros(0, np.float32)
        self.data = torch.from_numpy(flat).to(self.device)

    def __len__(self):
        return len(self.lengths)

    def gather(self, idx: tp.Sequence[int], starts: tp.Sequence[int], out_len: tp.Sequence[int],
               channels: int) -> torch.Tensor:
        """One encx_crop_collate launch -> [B][channels][max(out_len)] on the device."""
        ensure_device(self.device)
        idx = np.asarray(idx, np.int64)
        starts = np.asarray(starts, np.int64)
        out_len = np.asarray(out_len, np.int64)
        src = self.channels[idx]
        if not np.all((src == 1) | (src == channels)):
            raise ValueError('clip channel count must be 1 or the model channel count')
        if np.any(starts < 0) or np.any(starts + out_len > self.lengths[idx]):
            raise ValueError('crop window outside the clip')
        B, Tmax = len(idx), int(out_len.max()) if len(idx) else 0
        # pinned + non_blocking: a pageable H2D copy would block the host until the stream has
        # drained (the previous train step), leaving the GPU idle while the next step is enqueued
        meta = torch.from_numpy(np.stack([self.offsets[idx], self.lengths[idx], src, starts, out_len])
                                ).pin_memory().to(self.device, non_blocking=True)
        out = torch.empty(B, channels, Tmax, device=self.device, dtype=torch.float32)
        call('encx_crop_collate', self.data.data_ptr(), meta[0].data_ptr(), meta[1].data_ptr(),
             meta[2].data_ptr(), meta[3].data_ptr(), meta[4].data_ptr(), out.data_ptr(), B, channels,
             Tmax, stream())
        return out


class CustomAudioDataset:
    """customAudioDataset.py:15-69 over an AudioPool. `config` carries the reference's fields
    (datasets.train_csv_path / test_csv_path, fixed_length, tensor_cut, model.sample_rate,
    model.channels); `clips` may be given directly instead of reading the csv's files."""

    def __init__(self, config, transform=None, mode='train', clips=None, device='cuda'):
        assert mode in ['train', 'test'], 'dataset mode must be train or test'
        self.transform = transform
        self.fixed_length = config.datasets.fixed_length
        self.tensor_cut = config.datasets.tensor_cut
        self.sample_rate = config.model.sample_rate
        self.channels = config.model.channels
        if clips is None:
            import pandas as pd
            csv = config.datasets.train_csv_path if mode == 'train' else config.datasets.test_csv_path
            files = pd.read_csv(csv, on_bad_lines='skip').iloc[:, 0].tolist()
            clips = [load_wav(f, self.sample_rate, self.channels == 1) for f in files]
        self.pool = AudioPool(clips, device=device)

    def __len__(self):
        n = len(self.pool)
        return self.fixed_length if self.fixed_length and n > self.fixed_length else n

    def _window(self, i):
        L = int(self.pool.lengths[i])
        if self.tensor_cut > 0 and L > self.tensor_cut:
            start = random.randint(0, L - self.tensor_cut - 1)  # customAudioDataset.py:66
            return start, self.tensor_cut
        return 0, L

    def make_batch(self, indices: tp.Sequence[int]) -> torch.Tensor:
        """[dataset[i] for i in indices] + collate_fn (customAudioDataset.py:58-91) as one
        launch; crop starts drawn in item order like the reference's DataLoader does."""
        wins = [self._window(int(i)) for i in indices]
        out = self.pool.gather(indices, [w[0] for w in wins], [w[1] for w in wins], self.channels)
        if self.transform is not None:
            out = self.transform(out)
        return out

    def batches(self, batch_size: int, shuffle: bool = True, drop_last: bool = True):
        """DataLoader(shuffle) order over __len__ (train_multi_gpu.py:277-282)."""
        order = list(range(len(self)))
        if shuffle:
            random.shuffle(order)
        stop = len(order) - (len(order) % batch_size if drop_last else 0)
        for s in range(0, stop, batch_size):
            yield self.make_batch(order[s:s + batch_size])
