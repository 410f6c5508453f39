"""Batch assembly: the oracle against the reference-generated g11
fixture (CPU) and encx.data's HIP crop/collate against both (GPU, through the C ABI)."""
import random
import types

import numpy as np
import pytest
import torch

from oracle import data_oracle as D
from fixtures import load

DEV = 'cuda:0'
SETS = ['mono', 'stereo']


def clips_of(d, name):
    lens, mono, ch = d[f'{name}/lens'], d[f'{name}/mono'], int(d[f'{name}/channels'])
    sizes = [int(L) if m else int(L) * ch for L, m in zip(lens, mono)]
    flat = np.split(d[f'{name}/clips'], np.cumsum(sizes)[:-1])
    return [f if m else f.reshape(ch, -1) for f, m in zip(flat, mono)]


def cfg(cut, channels):
    return types.SimpleNamespace(
        datasets=types.SimpleNamespace(fixed_length=0, tensor_cut=cut, train_csv_path=None,
                                       test_csv_path=None),
        model=types.SimpleNamespace(sample_rate=24000, channels=channels))


@pytest.mark.parametrize('name', SETS)
def test_oracle_crop_collate_matches_reference(name):
    d = load('g11_data.npz')
    clips = clips_of(d, name)
    cut, ch = int(d[f'{name}/cut']), int(d[f'{name}/channels'])
    random.seed(1212)
    items = [D.crop(D.expand(clips[i], ch), cut)[0] for i in d[f'{name}/order']]
    np.testing.assert_array_equal(D.collate(items), d[f'{name}/batch'])


def test_load_wav_pcm16(tmp_path):
    import wave
    from encx.data import load_wav
    x = (np.arange(-300, 300, dtype=np.int16) * 50).reshape(-1, 2)
    p = str(tmp_path / 'a.wav')
    with wave.open(p, 'wb') as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(24000)
        w.writeframes(x.tobytes())
    st = load_wav(p, 24000, mono=False)
    np.testing.assert_array_equal(st, x.T.astype(np.float32) / 32768.0)
    mo = load_wav(p, 24000, mono=True)
    np.testing.assert_allclose(mo[0], x.astype(np.float32).mean(1) / 32768.0, rtol=1e-6)
    with pytest.raises(ValueError):
        load_wav(p, 48000, mono=True)


@pytest.mark.gpu
@pytest.mark.parametrize('name', SETS)
def test_gpu_make_batch_matches_reference(name):
    from encx.data import CustomAudioDataset
    d = load('g11_data.npz')
    cut, ch = int(d[f'{name}/cut']), int(d[f'{name}/channels'])
    ds = CustomAudioDataset(cfg(cut, ch), clips=clips_of(d, name), device=DEV)
    random.seed(1212)
    out = ds.make_batch([int(i) for i in d[f'{name}/order']])
    assert out.is_cuda
    np.testing.assert_array_equal(out.cpu().numpy(), d[f'{name}/batch'])


@pytest.mark.gpu
def test_gpu_make_batch_bench_size_vs_oracle():
    """Config-2 batch: 32 clips of 1-5 s cropped to tensor_cut 24000, ragged short clips padded."""
    from encx.data import CustomAudioDataset
    g = np.random.default_rng(7)
    lens = list(g.integers(20000, 120000, size=40))
    clips = [g.standard_normal(int(L)).astype(np.float32) for L in lens]
    ds = CustomAudioDataset(cfg(24000, 1), clips=clips, device=DEV)
    order = [int(i) for i in g.permutation(40)[:32]]
    random.seed(5)
    out = ds.make_batch(order).cpu().numpy()
    random.seed(5)
    ref = D.collate([D.crop(D.expand(clips[i], 1), 24000)[0] for i in order])
    np.testing.assert_array_equal(out, ref)
    with pytest.raises(ValueError):
        ds.pool.gather([0], [lens[0] - 10], [24000], 1)
