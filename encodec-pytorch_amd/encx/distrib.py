"""The torch.distributed helpers of distrib.py (the reference) that the training step calls:
rank / world size and the parameter broadcast at Trainer start (distrib.py:14-29, 55-72). The
reference's sync_buffer / sync_grad are never called on its path (their calls are commented out,
core_vq.py:157,175) and average_metrics runs on the device inside encx.balancer, so they are not
restated here. Backend 'nccl' is RCCL on ROCm."""
import os
import typing as tp

import torch

# ENCX_DIST_FORCE=1: take the N > 1 code path (the Trainer's segments with their collectives, the
# balancer's statistics all-reduce, the grad buckets' async all-reduces) even when the process
# group has ONE rank -- a one-GPU rehearsal of the multi-GPU step over the real RCCL backend
# (bench.py, tests/test_gpu_rccl.py). At world 1 every collective is an identity.
FORCE = os.environ.get('ENCX_DIST_FORCE', '0') == '1'


def rank():
    return torch.distributed.get_rank() if torch.distributed.is_initialized() else 0


def world_size():
    return torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1


def is_distributed():
    return world_size() > 1 or (FORCE and torch.distributed.is_initialized())


def broadcast_tensors(tensors: tp.Iterable[torch.Tensor], src: int = 0):
    """distrib.py:55-72."""
    if not is_distributed():
        return
    tensors = [t for t in tensors if torch.is_floating_point(t) or torch.is_complex(t)]
    handles = [torch.distributed.broadcast(t.data, src=src, async_op=True) for t in tensors]
    for h in handles:
        h.wait()
