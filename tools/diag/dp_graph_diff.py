"""Two ranks on one GPU over gloo: Trainer.step eager vs HIP-graph mode, per step, on the
test_gpu_dp 'gan_eager3' case; prints where the generator grads / params first differ.
ENCX_DP_GRAPHS=1 python tools/diag/dp_graph_diff.py (GPU box; the variable lets the Trainer
capture at world > 1)."""
import os
import socket
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, 'encodec-pytorch_amd'), os.path.join(ROOT, 'tests', 'golden'),
          os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)


def rank_main(rank, port, outdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo', rank=rank, world_size=2)
    import test_gpu_dp as T
    from encx.train import Trainer
    x = T._batch()[rank * T.B:(rank + 1) * T.B]
    if os.environ.get('DP_TRACE') and rank == 0:  # report host->device table builds inside a capture
        from encx import ops as _ops
        _orig_flush = _ops.WnBatch.flush

        def flush(self, _o=_orig_flush):
            key = tuple(id(v) for v, _ in self.pending)
            if self.pending:
                print(f'flush: {len(self.pending)} layers, capturing={torch.cuda.is_current_stream_capturing()}, '
                      f'new table={key not in self.bwd_tables}', flush=True)
            return _o(self)
        _ops.WnBatch.flush = flush
        _orig_build = _ops.WnBatch._build_fwd

        def build(self, grp, _o=_orig_build):
            print(f'build_fwd: capturing={torch.cuda.is_current_stream_capturing()}', flush=True)
            return _o(self, grp)
        _ops.WnBatch._build_fwd = build
    if os.environ.get('DP_RSYNC'):  # a device sync after every graph replay
        _rep = torch.cuda.CUDAGraph.replay

        def replay(self, _r=_rep):
            _r(self)
            torch.cuda.synchronize()
        torch.cuda.CUDAGraph.replay = replay
    res = {}
    for graphs in (False, True):
        torch.manual_seed(0)
        m, disc = T._build(True, False)
        tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False,
                     weights={'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, graphs=graphs)
        if os.environ.get('DP_NOSPLIT'):  # one backward segment (no decoder / encoder split)
            tr._dec_span = None
        if os.environ.get('DP_NORESCALE'):  # balancer without the norm statistics all-reduce
            tr.balancer.rescale_grads = False
        if os.environ.get('DP_NOCOLL'):  # the same segments, every collective dropped (ranks local)
            segs1 = tr._segments

            def segs_nocoll(*a, _s=segs1):
                segs, c = _s(*a)
                return [(s_, None) for s_, _ in segs], c
            tr._segments = segs_nocoll
        if os.environ.get('DP_MERGE'):  # e.g. "01,2,3,45": segments merged into one graph per group
            groups = [[int(c) for c in g] for g in os.environ['DP_MERGE'].split(',')]
            segs2 = tr._segments

            def segs_merge(*a, _s=segs2):
                segs, c = _s(*a)
                out = []
                tail = bool(os.environ.get('DP_TAIL'))  # a trivial kernel closing every graph
                for g in groups:
                    fs = [segs[i][0] for i in g]
                    out.append(((lambda fs=fs: ([f() for f in fs],
                                                torch.zeros(1, device='cuda').add_(1) if tail else None)), None))
                return out, c
            tr._segments = segs_merge
        if os.environ.get('DP_POOLS'):  # a fresh graph pool for every captured segment
            class _Fresh:
                def __bool__(self):
                    return True
            orig_cap = tr._capture

            def cap(key, x, _o=orig_cap):
                import torch as _t
                real = _t.cuda.graph

                class G(real):
                    def __init__(self, g, pool=None, **kw):
                        super().__init__(g, pool=_t.cuda.graph_pool_handle(), **kw)
                _t.cuda.graph = G
                try:
                    return _o(key, x)
                finally:
                    _t.cuda.graph = real
            tr._capture = cap
        if os.environ.get('DP_SYNC'):  # every bucket all-reduce waited for at once (no overlap)
            orig = tr.opt.reduce_async

            def sync_reduce(*a, _o=orig):
                w = _o(*a)
                w.wait()
                return w
            tr.opt.reduce_async = sync_reduce
        if os.environ.get('DP_DEVSYNC'):  # a device-wide sync after every collective
            segs0 = tr._segments

            def segs_sync(*a, _s=segs0):
                segs, c = _s(*a)
                wrap = lambda f: None if f is None else (lambda: (f(), torch.cuda.synchronize()))
                return [(s, wrap(cl)) for s, cl in segs], c
            tr._segments = segs_sync
        steps = []
        for i in range(3):
            out = tr.step(x.to('cuda') * (1.0 + 0.1 * i))
            torch.cuda.synchronize()
            steps.append({'grad': tr.opt.flat_grad.cpu().clone(), 'param': tr.opt.flat.cpu().clone(),
                          'dgrad': tr.opt_d.flat_grad.cpu().clone(),
                          'loss': {k: float(v) for k, v in out.items()}})
        res[graphs] = (steps, tr._dec_span, tr.opt.flat_grad.numel())
    torch.save(res, os.path.join(outdir, f'r{rank}.pt'))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    outdir = tempfile.mkdtemp()
    ctx = mp.get_context('spawn')
    ps = [ctx.Process(target=rank_main, args=(r, port, outdir)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=240)
    assert [p.exitcode for p in ps] == [0, 0], [p.exitcode for p in ps]
    for r in range(2):
        res = torch.load(os.path.join(outdir, f'r{r}.pt'))
        (se, span, n), (sg, _, _) = res[False], res[True]
        a, b = span if span is not None else (n, n)
        for i in range(3):
            e, g = se[i], sg[i]
            def d(t, lo, hi):
                return float((e[t][lo:hi] - g[t][lo:hi]).abs().max()) if hi > lo else 0.0
            print(f'rank {r} step {i}: grad diff enc [0,{a}) {d("grad", 0, a):.2e} dec [{a},{b}) '
                  f'{d("grad", a, b):.2e} rest [{b},{n}) {d("grad", b, n):.2e}; param diff {d("param", 0, n):.2e}; '
                  f'disc grad diff {float((e["dgrad"] - g["dgrad"]).abs().max()):.2e}; '
                  f'losses eager {e["loss"]} graph {g["loss"]}')


if __name__ == '__main__':
    main()
