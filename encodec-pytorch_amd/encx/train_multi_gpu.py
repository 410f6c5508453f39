"""train_multi_gpu.py of the reference on the encx path.

Same structure: `train_one_step` (one epoch over the loader), `train(local_rank, world_size,
config)`, `main`, `save_master_checkpoint`, `set_seed`. Differences, by design:
  * the config is the reference's YAML (config/config.yaml) read with yaml.safe_load, with
    `${a.b}` interpolation; hydra is not in the image;
  * one process per GPU launched by torchrun (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the
    env) instead of mp.spawn; the group is `nccl` (RCCL). Each rank takes its DistributedSampler
    shard of a shuffled order that every rank shares (seed + epoch), and the step all-reduces the
    flat gradient buffer (encx.optim.FlatAdam), as DDP's bucketed all-reduce does;
  * batches come from encx.data.CustomAudioDataset (clips decoded once into HBM, one
    crop/collate launch per batch) instead of a host DataLoader;
  * AMP is absent (the reference's AMP branch is broken), and so are
    tensorboard and the test-set wav dumps (logging goes to the python logger).

python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
    encodec-pytorch_amd/encx/train_multi_gpu.py config/config.yaml
"""
import logging
import math
import os
import random
import re
import sys
import types

import numpy as np
import torch

if __package__ in (None, ''):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    __package__ = 'encx'

from . import distrib  # noqa: E402
from .data import CustomAudioDataset  # noqa: E402
from .model import EncodecModel  # noqa: E402
from .msstftd import MultiScaleSTFTDiscriminator  # noqa: E402
from .train import Trainer  # noqa: E402

logger = logging.getLogger('encx.train')


def _ns(d):
    return types.SimpleNamespace(**{k: _ns(v) if isinstance(v, dict) else v for k, v in d.items()})


def load_config(path_or_dict):
    """YAML (or dict) -> nested namespace; resolves `${section.key}` references."""
    import yaml
    if isinstance(path_or_dict, dict):
        raw = path_or_dict
    else:
        with open(path_or_dict) as fh:
            raw = yaml.safe_load(fh)

    def look(ref):
        v = raw
        for k in ref.split('.'):
            v = v[k]
        return str(v)

    def res(v):
        if isinstance(v, dict):
            return {k: res(x) for k, x in v.items()}
        if isinstance(v, str):
            return re.sub(r'\$\{([^}]+)\}', lambda m: look(m.group(1)), v)
        return v
    return _ns(res(raw))


def set_seed(seed):
    """utils.py:118-130."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


def save_master_checkpoint(epoch, model, optimizer, scheduler, ckpt_name):
    """utils.py:132-148: the same keys, so my_encodec_model / encodec_model_bw load it."""
    state = {'epoch': epoch, 'model_state_dict': model.state_dict(),
             'optimizer_state_dict': optimizer.state_dict()}
    if scheduler is not None:
        state['scheduler_state_dict'] = scheduler.state_dict()
    torch.save(state, ckpt_name)


def shard_order(n, rank, world, batch_size, dp):
    """The reference loader's batches of item indices (train_multi_gpu.py:271-282).
    dp: DistributedSampler(trainset) with its defaults (seed 0, shuffle, no drop_last) and no
    set_epoch call anywhere in the reference, so every epoch repeats epoch 0's order; padded to
    a multiple of world, rank r takes r::world. Otherwise RandomSampler (shuffle=True): a seed
    drawn from torch's global generator, then randperm. DataLoader keeps the last partial batch."""
    if dp:
        g = torch.Generator()
        g.manual_seed(0)
        order = torch.randperm(n, generator=g).tolist()
        total = -(-n // world) * world
        while len(order) < total:
            order += order[:total - len(order)]
        order = order[rank:total:world]
    else:
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        order = torch.randperm(n, generator=g).tolist()
    return [order[i:i + batch_size] for i in range(0, len(order), batch_size)]


def build(config, device):
    m = config.model
    seg = m.segment
    segment = None if seg in (None, 'None') else float(seg)
    model = EncodecModel._get_model(list(m.target_bandwidths), int(m.sample_rate), m.channels,
                                    causal=m.causal, model_norm=m.norm, audio_normalize=m.audio_normalize,
                                    segment=segment, name=m.name, ratios=list(m.ratios)).to(device)
    disc = MultiScaleSTFTDiscriminator(filters=m.filters, in_channels=m.channels, out_channels=m.channels,
                                       hop_lengths=list(m.disc_hop_lengths), win_lengths=list(m.disc_win_lengths),
                                       n_ffts=list(m.disc_n_ffts)).to(device)
    return model, disc


def train_one_step(epoch, trainer, dataset, config, rank=0, world=1):
    """train_multi_gpu.py:32-143: one epoch; the discriminator trains from warmup_epoch on, with
    probability eval(train_discriminator) per step (:105-107)."""
    td = config.model.train_discriminator
    if td and epoch >= config.lr_scheduler.warmup_epoch:
        trainer.disc_prob = float(td) if isinstance(td, (bool, int, float)) else float(eval(str(td)))
    else:
        trainer.disc_prob = None  # the reference's `and` short-circuits before random.random()
    batches = shard_order(len(dataset), rank, world, config.datasets.batch_size, world > 1)
    last = {}
    for idx, ids in enumerate(batches, 1):
        out = trainer.step(dataset.make_batch(ids))
        if rank == 0 and (idx % config.common.log_interval == 0 or idx == len(batches)):
            last = {k: float(v.detach().reshape(-1)[0]) for k, v in out.items()}
            logger.info(f'Epoch {epoch} {idx}/{len(batches)} ' +
                        ' '.join(f'{k} {v:.4f}' for k, v in last.items()))
    return last


def train(local_rank, world_size, config):
    """train_multi_gpu.py:172-352."""
    if world_size > 1 and not config.distributed.data_parallel:
        # the reference would run W independent copies that all log and write the same
        # checkpoint paths; refuse instead of racing on the files
        raise ValueError(f'WORLD_SIZE={world_size} but distributed.data_parallel is off')
    dp = bool(config.distributed.data_parallel) and world_size > 1
    device = torch.device('cuda', local_rank)
    torch.cuda.set_device(device)
    if dp and not torch.distributed.is_initialized():
        torch.distributed.init_process_group('nccl', device_id=device)
    rank = torch.distributed.get_rank() if dp else 0
    if config.common.seed is not None:
        set_seed(config.common.seed)
    os.makedirs(config.checkpoint.save_folder, exist_ok=True)
    model, disc = build(config, device)
    dataset = CustomAudioDataset(config, mode='train', device=device)
    per_rank = math.ceil(len(dataset) / (world_size if dp else 1))     # DistributedSampler pads
    steps = max(1, math.ceil(per_rank / config.datasets.batch_size))  # no drop_last
    if getattr(config.distributed, 'sync_codebooks', False):  # opt-in, not a reference key
        model.quantizer.set_sync_codebooks(True)
    # the discriminator always takes part in the generator loss (train_multi_gpu.py:61-71); the
    # train_discriminator flag only gates its update (train_one_step sets disc_prob)
    trainer = Trainer(model, disc, lr=float(config.optimization.lr), disc_lr=float(config.optimization.disc_lr),
                      weights=dict(vars(config.balancer.weights)), sample_rate=int(config.model.sample_rate),
                      max_iter=config.common.max_epoch * steps,
                      warmup_iter=config.lr_scheduler.warmup_epoch * steps,
                      # opt-in, not a reference key: replay each step from HIP graphs
                      graphs=bool(getattr(config.common, 'hip_graphs', False)))
    start_epoch = 1
    if config.checkpoint.resume:
        # train_multi_gpu.py:226-238 + :303-308; weights_only loads (no unpickling)
        ck = torch.load(config.checkpoint.checkpoint_path, map_location='cpu', weights_only=True)
        dk = torch.load(config.checkpoint.disc_checkpoint_path, map_location='cpu', weights_only=True)
        model.load_state_dict(ck['model_state_dict'])
        disc.load_state_dict(dk['model_state_dict'])
        start_epoch = max(1, ck['epoch'] + 1)
        if start_epoch > config.common.max_epoch:
            raise ValueError(f'resume epoch {ck["epoch"]} is larger than total epochs {config.common.max_epoch}')
        if 'scheduler_state_dict' in ck and 'scheduler_state_dict' in dk:
            trainer.load_state_dicts(ck['optimizer_state_dict'], ck['scheduler_state_dict'],
                                     dk['optimizer_state_dict'], dk['scheduler_state_dict'])
    for epoch in range(start_epoch, config.common.max_epoch + 1):
        train_one_step(epoch, trainer, dataset, config, rank, world_size if dp else 1)
        if epoch % config.common.save_interval == 0 and rank == 0:
            base = f'{config.checkpoint.save_location}epoch{epoch}_lr{config.optimization.lr}'
            save_master_checkpoint(epoch, model, trainer.opt, trainer.sched, base + '.pt')
            save_master_checkpoint(epoch, disc, trainer.opt_d, trainer.sched_d,
                                   f'{config.checkpoint.save_location}epoch{epoch}_disc_lr{config.optimization.lr}.pt')
    if dp:
        torch.distributed.destroy_process_group()
    return trainer


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    logging.basicConfig(level=logging.INFO)
    config = load_config(argv[0])
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    train(local, world, config)


if __name__ == '__main__':
    main()
