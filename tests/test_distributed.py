"""world_size-2 `gloo` tests of the data-parallel plumbing (CPU; the GPU run uses RCCL through
the same calls): parameter broadcast at Trainer start, the flat-grad all-reduce of FlatAdam,
the bucketed async reduction of the training step, distrib.py's broadcast (distrib.py:55-72)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        q.put((rank, globals()[fn_name](rank, world)))
    except Exception as e:  # report, do not hang the peer
        q.put((rank, f'ERROR {type(e).__name__}: {e}'))
    finally:
        dist.destroy_process_group()


def _run(fn_name, world=2):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith('ERROR')), v
    return out


# ---- per-rank bodies (module-level so spawn can pickle them by name)
def _body_flat_grad(rank, world):
    from encx.optim import FlatAdam
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7))]
    opt = FlatAdam(params, lr=1e-3)
    # each rank fills its grads through the views, as the conv kernels do in place
    params[0].grad.fill_(float(rank + 1))
    params[1].grad.copy_(torch.arange(7, dtype=torch.float32) * (rank + 1))
    opt.all_reduce_grads()
    mean = sum(r + 1 for r in range(world)) / world
    ok0 = torch.allclose(params[0].grad, torch.full((5, 3), mean))
    ok1 = torch.allclose(params[1].grad, torch.arange(7, dtype=torch.float32) * mean)
    same_storage = params[0].grad.data_ptr() == opt.flat_grad.data_ptr()
    return ok0 and ok1 and same_storage


def _body_broadcast(rank, world):
    from encx import distrib
    ts = [torch.full((4,), float(rank)), torch.full((2, 2), 10.0 + rank),
          torch.tensor([rank], dtype=torch.int64)]
    distrib.broadcast_tensors(ts)
    # floating tensors follow rank 0; integer tensors are skipped (distrib.py:63-64)
    return (ts[0].tolist(), ts[1].flatten().tolist(), int(ts[2]))


def _body_buckets(rank, world):
    """The Trainer's bucketed exchange: the decoder span reduced async first, the rest (the
    encoder span) async second, both waited for together -- equals one all-reduce."""
    from encx.optim import FlatAdam
    from encx import distrib
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(6)), torch.nn.Parameter(torch.randn(4, 2)),
              torch.nn.Parameter(torch.randn(3))]
    opt = FlatAdam(params, lr=1e-3)
    g = torch.arange(opt.flat_grad.numel(), dtype=torch.float32) * (rank + 1)
    opt.flat_grad.copy_(g)
    a, b = opt.span(params[1:])
    works = [opt.reduce_async(a, b), opt.reduce_async(0, a)]
    for w in works:
        w.wait()
    want = torch.arange(opt.flat_grad.numel(), dtype=torch.float32) * sum(r + 1 for r in range(world))
    return bool(torch.equal(opt.flat_grad, want)), (a, b), distrib.rank(), distrib.world_size()


def test_flat_grad_all_reduce_mean():
    out = _run('_body_flat_grad')
    assert all(out.values()), out


def test_broadcast_tensors_from_rank0():
    out = _run('_body_broadcast')
    for r in range(2):
        assert out[r][0] == [0.0] * 4
        assert out[r][1] == [10.0] * 4
        assert out[r][2] == r


def test_bucketed_async_reduce():
    out = _run('_body_buckets')
    for r in range(2):
        ok, span, rk, ws = out[r]
        assert ok and span == (6, 17) and rk == r and ws == 2
