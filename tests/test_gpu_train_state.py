"""Run-twice determinism of a full GAN step and checkpoint / resume parity
(train_multi_gpu.py:224-238, 303-308; utils.py:132-148) on the HIP path.

Determinism: the kernels use no floating-point atomics and fixed-order reductions, so two
identical trainers fed the same clips must produce bit-identical parameters, Adam moments,
codebooks and losses after several GAN steps.

Resume: the reference checkpoints {epoch, model_state_dict, optimizer_state_dict,
scheduler_state_dict} per model. A trainer rebuilt from those four state dicts and stepped once
must match the uninterrupted run bit for bit. The reference's Balancer keeps its EMA
statistics outside every state dict (balancer.py:31-118), so a resumed reference run restarts
them; the uninterrupted run here resets its balancer at the same step to compare like with
like.
"""
import io

import numpy as np
import pytest
import torch

from fixtures import model_state, codebooks_from_stats, disc_state
from synth import synth_wave

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def make_trainer(B=4, graphs=False, disc_on=True, disc_prob=1.0):
    from oracle import encodec_oracle as O
    from encx.model import EncodecModel
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from encx.train import Trainer
    cfg = O.Config(target_bandwidths=(6.0,), audio_normalize=True)
    m = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    sd = dict(model_state(cfg, 3))
    stats = np.zeros((cfg.n_q, 2, 128), np.float32)
    stats[:, 1] = 0.05
    for i, cb in enumerate(codebooks_from_stats(stats, 4, cfg.n_q, cfg.n_q)):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    disc = None
    if disc_on:
        disc = MultiScaleSTFTDiscriminator(filters=32)
        disc.load_state_dict(disc_state(5), strict=False)
        disc = disc.to(DEV)
    tr = Trainer(m.to(DEV), disc, lr=3e-4, disc_lr=3e-4, max_iter=100, warmup_iter=3,
                 graphs=graphs, disc_prob=disc_prob)
    return tr


def batches(n, B=4):
    return [torch.from_numpy(synth_wave((B, 1, 24000), 200 + i)).to(DEV) for i in range(n)]


def snapshot(tr):
    out = {'gen': tr.opt.flat.clone(), 'gen_m': tr.opt.exp_avg.clone(), 'gen_v': tr.opt.exp_avg_sq.clone()}
    if tr.opt_d is not None:
        out.update({'disc': tr.opt_d.flat.clone(), 'disc_m': tr.opt_d.exp_avg.clone()})
    for k, v in tr.model.state_dict().items():
        if '_codebook' in k:
            out[k] = v.clone()
    return out


def assert_same(a, b):
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_gan_step_run_twice_bit_identical():
    xs = batches(3)
    outs, snaps = [], []
    for _ in range(2):
        tr = make_trainer()
        losses = [tr.step(x) for x in xs]
        torch.cuda.synchronize()
        outs.append([{k: float(v) for k, v in o.items()} for o in losses])
        snaps.append(snapshot(tr))
    assert outs[0] == outs[1]
    assert_same(snaps[0], snaps[1])


def _roundtrip(obj):
    """torch.save -> torch.load(weights_only=True): what a checkpoint file goes through."""
    buf = io.BytesIO()
    torch.save(obj, buf)
    buf.seek(0)
    return torch.load(buf, map_location='cpu', weights_only=True)


def test_resume_matches_uninterrupted_run():
    from encx.balancer import Balancer
    xs = batches(4)
    # uninterrupted: 3 steps, (balancer restart as a resume has it), 1 more step
    tr = make_trainer()
    for x in xs[:3]:
        tr.step(x)
    ck = _roundtrip({'model_state_dict': tr.model.state_dict(), **tr.state_dicts(),
                     'disc_state_dict': tr.disc.state_dict()})
    assert set(ck['optimizer']['state'][0]) == {'step', 'exp_avg', 'exp_avg_sq'}
    assert float(ck['optimizer']['state'][0]['step']) == 3.0
    assert ck['scheduler']['last_epoch'] == 3
    tr.balancer = Balancer(tr.balancer.weights)
    tr.step(xs[3])
    torch.cuda.synchronize()
    want = snapshot(tr)
    # resumed: a fresh trainer from the checkpoint's state dicts, then the same step
    tr2 = make_trainer()
    tr2.model.load_state_dict(ck['model_state_dict'])
    tr2.disc.load_state_dict(ck['disc_state_dict'])
    tr2.load_state_dicts(ck['optimizer'], ck['scheduler'], ck['disc_optimizer'], ck['disc_scheduler'])
    assert tr2.opt.n_step == 3 and tr2.sched.last_epoch == 3
    tr2.step(xs[3])
    torch.cuda.synchronize()
    assert_same(want, snapshot(tr2))


@pytest.mark.parametrize('case', ['gan', 'gen', 'gan_coin'])
def test_hip_graph_steps_match_eager(case):
    """Trainer(graphs=True): step 1 eager, step 2 captured + replayed, steps 3.. replayed, with
    the LR changing every step (warmup) and a new batch each step. Every step's losses and the
    final parameters, Adam moments and codebooks must equal the eager trainer's bit for bit.
    gan_coin trains the discriminator with probability 0.5: two graph keys."""
    import random
    xs = batches(6)
    kw = dict(disc_on=case != 'gen', disc_prob=0.5 if case == 'gan_coin' else 1.0)
    runs = []
    for graphs in (False, True):
        random.seed(11)
        tr = make_trainer(graphs=graphs, **kw)
        losses = []
        for x in xs:
            o = tr.step(x)
            losses.append({k: float(v) for k, v in o.items()})
        torch.cuda.synchronize()
        runs.append((losses, snapshot(tr), tr))
    assert runs[0][0] == runs[1][0]
    assert_same(runs[0][1], runs[1][1])
    g = runs[1][2]._graphs
    assert any(isinstance(v, tuple) for v in g.values())


def test_graph_pool_memory_bounded_across_keys():
    """Every (bandwidth, coin, shape) key is captured into ONE shared graph pool (steps never
    overlap; only each key's returned losses stay alive), so capturing three bandwidths reserves
    little beyond what the first key's capture did; one pool per key would add a whole step's
    activations per key. Also: past max_graph_keys, keys run eagerly."""
    tr = make_trainer(graphs=True)
    x = batches(1)[0]
    marks, act = [], None
    for bw in (6.0, 3.0, 1.5):
        tr.model.target_bandwidths = [bw]
        for i in range(3):  # eager, capture, replay
            if act is None:  # one step's activations: the peak of the first eager step
                torch.cuda.synchronize()
                a0 = torch.cuda.memory_allocated()
                torch.cuda.reset_peak_memory_stats()
            tr.step(x)
            if act is None:
                torch.cuda.synchronize()
                act = torch.cuda.max_memory_allocated() - a0
        torch.cuda.synchronize()
        marks.append(torch.cuda.memory_reserved())
    extra = marks[-1] - marks[0]
    print(f'one step peaks at +{act / 2**20:.0f} MiB; two more captured keys reserve +{extra / 2**20:.0f} MiB')
    assert sum(isinstance(v, tuple) for v in tr._graphs.values()) == 3
    assert extra <= 0.5 * act, (act, extra)
    tr.max_graph_keys = 3
    assert not tr._graph_ok((0.75, True, tuple(x.shape)))


def test_weight_norm_batch_matches_per_layer():
    """ops.WnBatch (every weight norm of a step as one launch per model forward / backward)
    against the per-layer launches: generator grads bit-identical (the same per-row arithmetic);
    discriminator grads within fp32 rounding (its layers serve the real and the fake graph, and
    the batched backward normalises the summed weight grad once, as the reference's autograd
    does, instead of each use's grad separately)."""
    import encx.ops as ops
    x = batches(1)[0]
    grads = []
    for batched in (False, True):
        tr = make_trainer()
        if not batched:
            tr.wn = None
        tr.step(x)
        grads.append((tr.opt.flat_grad.clone(), tr.opt_d.flat_grad.clone(), tr.opt.flat.clone()))
        assert ops._WN is None and ops._WNB is None
    (g0, d0, p0), (g1, d1, p1) = grads
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
    assert float((d0 - d1).abs().max()) <= 1e-5 * float(d0.abs().max())


@pytest.mark.parametrize('segmented', [False, True])
def test_two_graph_keys_back_to_back_match_eager(segmented):
    """Two graph keys (bandwidths 6 and 3 kbps: n_q 8 and 4) alternating step by step, so every
    replay of one key follows a replay of the other in the shared graph pool: the generator and
    discriminator flat grads and parameters after EVERY step equal the eager trainer's bit for
    bit; segmented=True captures the data-parallel segment list (one graph per segment) at world 1."""
    xs = batches(8)
    runs = []
    for graphs in (False, True):
        tr = make_trainer(graphs=graphs)
        tr.segmented = segmented
        per_step = []
        for i, x in enumerate(xs):
            tr.model.target_bandwidths = [6.0 if i % 2 == 0 else 3.0]
            tr.step(x)
            torch.cuda.synchronize()
            per_step.append([t.clone() for t in (tr.opt.flat_grad, tr.opt.flat, tr.opt_d.flat_grad, tr.opt_d.flat)])
        runs.append(per_step)
        if graphs:
            assert sum(isinstance(v, tuple) for v in tr._graphs.values()) == 2
    for i, (a, b) in enumerate(zip(*runs)):
        for k, (ta, tb) in enumerate(zip(a, b)):
            assert torch.equal(ta, tb), (i, k, float((ta - tb).abs().max()))
