"""The torch.distributed helpers of distrib.py (the reference) that the training step calls:
rank / world size and the parameter broadcast at Trainer start (distrib.py:14-29, 55-72). The
reference's sync_buffer / sync_grad are never called on its path (their calls are commented out,
core_vq.py:157,175) and average_metrics runs on the device inside encx.balancer, so they are not
restated here. Backend 'nccl' is RCCL on ROCm."""
import typing as tp

import torch


def rank():
    return torch.distributed.get_rank() if torch.distributed.is_initialized() else 0


def world_size():
    return torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1


def is_distributed():
    return world_size() > 1


def broadcast_tensors(tensors: tp.Iterable[torch.Tensor], src: int = 0):
    """distrib.py:55-72."""
    if not is_distributed():
        return
    tensors = [t for t in tensors if torch.is_floating_point(t) or torch.is_complex(t)]
    handles = [torch.distributed.broadcast(t.data, src=src, async_op=True) for t in tensors]
    for h in handles:
        h.wait()
