"""torch.distributed helpers (distrib.py of the reference); backend 'nccl' is RCCL on ROCm."""
import typing as tp

import torch


def rank():
    return torch.distributed.get_rank() if torch.distributed.is_initialized() else 0


def world_size():
    return torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1


def is_distributed():
    return world_size() > 1


def all_reduce(tensor: torch.Tensor, op=torch.distributed.ReduceOp.SUM):
    if is_distributed():
        return torch.distributed.all_reduce(tensor, op)


def broadcast_tensors(tensors: tp.Iterable[torch.Tensor], src: int = 0):
    """distrib.py:55-72."""
    if not is_distributed():
        return
    tensors = [t for t in tensors if torch.is_floating_point(t) or torch.is_complex(t)]
    handles = [torch.distributed.broadcast(t.data, src=src, async_op=True) for t in tensors]
    for h in handles:
        h.wait()


def sync_buffer(buffers, average=True):
    """distrib.py:75-93 (the reference divides by the function `world_size`; fixed here)."""
    if not is_distributed():
        return
    handles = []
    for b in buffers:
        if torch.is_floating_point(b.data):
            if average:
                handles.append((b, torch.distributed.all_reduce(b.data, async_op=True)))
            else:
                handles.append((b, torch.distributed.broadcast(b.data, src=0, async_op=True)))
    for b, h in handles:
        h.wait()
        if average:
            b.data /= world_size()


def sync_grad(params):
    """distrib.py:96-109."""
    if not is_distributed():
        return
    handles = []
    for p in params:
        if p.grad is not None:
            handles.append((p, torch.distributed.all_reduce(p.grad.data, async_op=True)))
    for p, h in handles:
        h.wait()
        p.grad.data /= world_size()


def average_metrics(metrics: tp.Dict[str, float], count=1.):
    """distrib.py:112-124 (host version; the Balancer uses its device twin)."""
    if not is_distributed():
        return metrics
    keys, values = zip(*metrics.items())
    device = 'cuda' if torch.cuda.is_available() else 'cpu'
    tensor = torch.tensor(list(values) + [1], device=device, dtype=torch.float32)
    tensor *= count
    all_reduce(tensor)
    averaged = (tensor[:-1] / tensor[-1]).cpu().tolist()
    return dict(zip(keys, averaged))
