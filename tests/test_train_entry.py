"""train_multi_gpu.py mirror (encx.train_multi_gpu): config loading, the loader's sharding
against torch's own samplers (CPU), and one tiny epoch from WAV files with a checkpoint that
the reference-format loaders accept (GPU)."""
import os
import wave

import numpy as np
import pytest
import torch

CFG = {
    'common': {'save_interval': 1, 'test_interval': 5, 'log_interval': 1, 'max_epoch': 1, 'seed': 3401,
               'amp': False},
    'datasets': {'train_csv_path': None, 'test_csv_path': None, 'batch_size': 2, 'tensor_cut': 4800,
                 'num_workers': 0, 'fixed_length': 0, 'pin_memory': True},
    'checkpoint': {'resume': False, 'checkpoint_path': '', 'disc_checkpoint_path': '',
                   'save_folder': None,
                   'save_location': '${checkpoint.save_folder}/bs${datasets.batch_size}_cut${datasets.tensor_cut}_'},
    'optimization': {'lr': 3e-4, 'disc_lr': 3e-4},
    'lr_scheduler': {'warmup_epoch': 0},
    'model': {'target_bandwidths': [1.5, 3., 6., 12., 24.], 'sample_rate': 24000, 'channels': 1,
              'train_discriminator': True, 'audio_normalize': True, 'filters': 32, 'ratios': [8, 5, 4, 2],
              'disc_win_lengths': [1024, 2048, 512], 'disc_hop_lengths': [256, 512, 128],
              'disc_n_ffts': [1024, 2048, 512], 'causal': False, 'norm': 'time_group_norm',
              'segment': 'None', 'name': 'my_encodec'},
    'distributed': {'data_parallel': False, 'world_size': 1, 'find_unused_parameters': False,
                    'torch_distributed_debug': False, 'init_method': 'tcp'},
    'balancer': {'weights': {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}},
}


def test_config_interpolation():
    from encx.train_multi_gpu import load_config
    d = dict(CFG)
    d['checkpoint'] = dict(CFG['checkpoint'], save_folder='/tmp/ck')
    c = load_config(d)
    assert c.checkpoint.save_location == '/tmp/ck/bs2_cut4800_'
    assert c.balancer.weights.l_g == 3 and c.model.ratios == [8, 5, 4, 2]


@pytest.mark.parametrize('n,world', [(10, 1), (10, 2), (7, 4), (3, 4)])
def test_shard_order_matches_torch_samplers(n, world):
    from torch.utils.data import DistributedSampler, RandomSampler, BatchSampler
    from encx.train_multi_gpu import shard_order
    ds = list(range(n))
    for rank in range(world):
        ref = list(BatchSampler(DistributedSampler(ds, num_replicas=world, rank=rank), 3, False))
        assert shard_order(n, rank, world, 3, True) == ref
    torch.manual_seed(11)
    ref = list(BatchSampler(RandomSampler(ds), 3, False))
    torch.manual_seed(11)
    assert shard_order(n, 0, 1, 3, False) == ref


def _write_wavs(folder, n):
    g = np.random.default_rng(0)
    paths = []
    for i in range(n):
        x = (0.1 * g.standard_normal(6000 + 1000 * i) * 32767).astype(np.int16)
        p = os.path.join(folder, f'c{i}.wav')
        with wave.open(p, 'wb') as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(24000)
            w.writeframes(x.tobytes())
        paths.append(p)
    csv = os.path.join(folder, 'train.csv')
    with open(csv, 'w') as fh:
        fh.write('path\n' + '\n'.join(paths) + '\n')
    return csv


@pytest.mark.gpu
def test_gpu_one_epoch_from_wav_files(tmp_path):
    from encx.train_multi_gpu import load_config, train
    from encx.model import EncodecModel
    d = {k: dict(v) for k, v in CFG.items()}
    d['datasets']['train_csv_path'] = _write_wavs(str(tmp_path), 4)
    d['checkpoint']['save_folder'] = str(tmp_path / 'ck')
    tr = train(0, 1, load_config(d))
    assert tr.sched.last_epoch == 2                       # 4 clips / batch 2
    ck = str(tmp_path / 'ck') + '/bs2_cut4800_epoch1_lr0.0003.pt'
    assert os.path.exists(ck) and os.path.exists(ck.replace('_lr', '_disc_lr'))
    m = EncodecModel.my_encodec_model(ck).to('cuda:0')   # the reference's loader for this file
    for k, v in tr.model.state_dict().items():
        assert torch.equal(m.state_dict()[k].cpu(), v.cpu()), k
