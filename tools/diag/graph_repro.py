"""Single-process repro of the HIP-graph replay drift of the segmented (data-parallel) step.

World 1, the test_gpu_dp 'gan_eager3' model (B=16, all four losses balanced). An eager trainer
and a graph trainer run the same steps; after every segment (eager steps and replays) the
persistent buffers are snapshotted and compared bit for bit, so the first segment whose replay
diverges is named.

python tools/diag/graph_repro.py [--seg] [--merge 012,345] [--steps 4] [--hold] [--tail]
  --seg     the data-parallel segment list (split backward, one graph per segment)
  --merge   groups of segments captured into one graph each (implies --seg)
  --hold    keep a reference to every tensor the captured step's state dict held after each
            segment's capture (no pool block is reused across segments)
  --tail    a one-element torch kernel closing every captured graph
"""
import argparse
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, 'encodec-pytorch_amd'), os.path.join(ROOT, 'tests', 'golden'),
          os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)

W = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}


def snap(tr):
    torch.cuda.synchronize()
    out = {'gen': tr.opt.flat, 'gen_grad': tr.opt.flat_grad, 'gen_m': tr.opt.exp_avg,
           'gen_v': tr.opt.exp_avg_sq, 'disc': tr.opt_d.flat, 'disc_grad': tr.opt_d.flat_grad,
           'disc_m': tr.opt_d.exp_avg}
    for k, v in tr.model.state_dict().items():
        if '_codebook' in k and 'inited' not in k:
            out[k] = v
    st = tr.balancer._state or {}
    for k in ('total', 'fix', 'avg', 'red', 'norms', 'scales'):
        if k in st:
            out['bal.' + k] = st[k]
    return {k: v.detach().clone() for k, v in out.items()}


def run(args, graphs, x):
    import test_gpu_dp as T
    from encx.train import Trainer
    torch.manual_seed(0)
    random.seed(0)
    m, disc = T._build(True, False)
    seg = args.seg or bool(args.merge)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=W, graphs=graphs,
                 segmented=seg)
    groups = [[int(c) for c in g] for g in args.merge.split(',')] if (args.merge and graphs) else None
    if groups or args.tail or args.hold:
        base = tr._segments
        held = []

        def segs_patched(*a, _s=base):
            segs, c = _s(*a)
            if groups is None:
                gs = [[i] for i in range(len(segs))]
            else:
                gs = groups

            def mk(fs):
                def f():
                    for fn in fs:
                        fn()
                    if args.tail and torch.cuda.is_current_stream_capturing():
                        torch.zeros(1, device='cuda').add_(1)
                    if args.hold and torch.cuda.is_current_stream_capturing():
                        held.append([v for v in _tensors(c)])
                return f
            return [(mk([segs[i][0] for i in g]), None) for g in gs], c
        tr._segments = segs_patched
        tr._held = held
    rec = []
    for s in range(args.steps):
        cur = []
        tr._seg_hook = lambda i, c, cur=cur: cur.append((i, snap(tr)))
        out = tr.step(x * (1.0 + 0.1 * s))
        torch.cuda.synchronize()
        rec.append((cur, {k: float(v) for k, v in out.items()}, snap(tr)))
    return rec, groups


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, dict):
        for v in obj.values():
            yield from _tensors(v)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            yield from _tensors(v)


def diff(a, b):
    rows = []
    for k in a:
        if not torch.equal(a[k], b[k]):
            rows.append(f'{k} {float((a[k].double() - b[k].double()).abs().max()):.2e}')
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seg', action='store_true')
    ap.add_argument('--merge', default='')
    ap.add_argument('--steps', type=int, default=4)
    ap.add_argument('--hold', action='store_true')
    ap.add_argument('--tail', action='store_true')
    args = ap.parse_args()
    import test_gpu_dp as T
    x = T._batch()[:T.B].to('cuda')
    eager, _ = run(args, False, x)
    graph, groups = run(args, True, x)
    print(f'args {vars(args)}')
    for s in range(args.steps):
        (ce, le, fe), (cg, lg, fg) = eager[s], graph[s]
        kind = ['eager', 'capture'][s] if s < 2 else 'replay'
        d = diff(fe, fg)
        print(f'step {s} ({kind}): losses equal {le == lg}; end-of-step diffs: {d[:8] if d else "none"}')
        if le != lg:
            print(f'   eager {le}\n   graph {lg}')
        emap = dict(ce)
        for i, sn in cg:
            j = groups[i][-1] if groups else i
            d = diff(emap[j], sn)
            print(f'   after segment {j}: {"; ".join(d[:8]) if d else "equal"}')


if __name__ == '__main__':
    main()
