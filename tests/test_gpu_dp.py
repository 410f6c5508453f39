"""Multi-rank data parallelism on ONE GPU (SURVEY §8e, config 4's logic): two child processes
share cuda:0 and talk over `gloo` (which takes CUDA tensors), running encx.train.Trainer.step on
half a batch each; the parent runs the same step on the whole batch in one process.

What must hold (all with the reference's step semantics, train_multi_gpu.py:56-129):
  * ranks stay in sync: after the step both ranks hold bit-identical parameters, Adam moments
    and (with sync_codebooks) codebook buffers;
  * sync_codebooks: the EMA sums are all-reduced (SUM), so 2 x B16 gives the codebook buffers of
    1 x B32, and every code equals the single-process code;
  * sync off (the reference, core_vq.py:157,175): each rank's codebooks follow its own half;
  * kmeans init with sync_codebooks: every rank ends with rank 0's initial codebook;
  * gradients: without the balancer's rescaling every loss is a batch mean, so the averaged
    grads of 2 x B16 equal 1 x B32 (generator and discriminator). With the balancer (its
    per-item norm statistics all-reduced, balancer.py:99) the balanced gradient is invariant
    to the batch split per ITEM, so DDP's mean over ranks halves it: the 2 x B16 generator
    grad = 1/2 balanced + commit grad of 1 x B32 (checked component-wise).
The feature-matching loss (losses.py:53) is a ratio of per-rank means (l1 / mean|fr|), which
does not decompose over ranks; the GAN comparison gives it weight 0.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
B = 16  # per rank


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _build(gan, sync, seed_cb=4, inited=True):
    from oracle import encodec_oracle as O
    from fixtures import model_state, codebooks_from_stats, disc_state
    from encx.model import EncodecModel
    from encx.msstftd import MultiScaleSTFTDiscriminator
    cfg = O.Config(target_bandwidths=(6.0,), audio_normalize=True)
    m = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                audio_normalize=True, sync_codebooks=sync)
    sd = dict(model_state(cfg, 3))
    stats = np.zeros((cfg.n_q, 2, 128), np.float32)
    stats[:, 1] = 0.05
    if inited:
        for i, cb in enumerate(codebooks_from_stats(stats, seed_cb, cfg.n_q, cfg.n_q)):
            for k, v in cb.items():
                sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
        m.load_state_dict(sd)
    else:
        m.load_state_dict(sd, strict=False)
    m = m.to(DEV)
    disc = None
    if gan:
        disc = MultiScaleSTFTDiscriminator(filters=32)
        disc.load_state_dict(disc_state(5), strict=False)
        disc = disc.to(DEV)
    return m, disc


def _batch():
    from synth import synth_wave
    return torch.from_numpy(synth_wave((2 * B, 1, 24000), 99))


CASES = {
    # name: (gan, sync, rescale, weights, inited)
    'gen_sync': (False, True, True, {'l_t': 0.1, 'l_f': 1}, True),
    'gen_sync_plain': (False, True, False, {'l_t': 0.1, 'l_f': 1}, True),
    'gen_nosync': (False, False, True, {'l_t': 0.1, 'l_f': 1}, True),
    'gan_sync_plain': (True, True, False, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 0}, True),
    'kmeans_sync': (False, True, True, {'l_t': 0.1, 'l_f': 1}, False),
    # 3 GAN steps, all four losses balanced, eager (decoder-grad bucket all-reduce overlapping the
    # encoder backward) vs HIP graphs (segments captured between the eager collectives)
    # (5 steps: eager, capture, 3 replays)
    'gan_eager3': (True, False, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 5, False),
    'gan_graph3': (True, False, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 5, True),
    # the same with the codebook sums all-reduced (deferred to one collective between segments)
    'gan_sync_eager3': (True, True, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 5, False),
    'gan_sync_graph3': (True, True, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 5, True),
}
MULTI_STEP = ('gan_eager3', 'gan_graph3', 'gan_sync_eager3', 'gan_sync_graph3')
# config 4's partition count: 8 ranks x B/8 against 1 rank x B (the same cases as the 2-rank run)
CASES8 = ('gen_sync', 'gan_sync_plain')


def _run_case(name, x):
    """One Trainer.step on x; returns everything the comparisons need (CPU tensors)."""
    from encx.train import Trainer
    gan, sync, rescale, weights, inited, steps, graphs = (CASES[name] + (1, False))[:7]
    torch.manual_seed(0)
    m, disc = _build(gan, sync, inited=inited)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=weights,
                 balancer_kwargs={'rescale_grads': rescale}, graphs=graphs)
    losses = []
    # graphs at world > 1 are opt-in (ENCX_DP_GRAPHS=1, encx/train.py)
    os.environ['ENCX_DP_GRAPHS'] = '1' if graphs else '0'
    try:
        for i in range(steps):
            o = tr.step(x.to(DEV) * (1.0 + 0.1 * i))
            losses.append(torch.stack([o[k].reshape(()) for k in sorted(o)]).cpu())
        torch.cuda.synchronize()
    finally:
        os.environ.pop('ENCX_DP_GRAPHS', None)
    captured = any(isinstance(v, tuple) for v in tr._graphs.values())
    assert captured == (graphs and steps >= 2), (name, captured)
    out = {'gen_grad': tr.opt.flat_grad.cpu(), 'gen_param': tr.opt.flat.cpu(), 'losses': torch.stack(losses),
           'gen_m': tr.opt.exp_avg.cpu(), 'codes': m.last_codes[0].cpu()}
    for i, layer in enumerate(m.quantizer.vq.layers):
        cb = layer._codebook
        for k in ('cluster_size', 'embed', 'embed_avg', 'inited'):
            out[f'cb{i}.{k}'] = getattr(cb, k).detach().cpu().clone()
    if disc is not None:
        out['disc_grad'] = tr.opt_d.flat_grad.cpu()
        out['disc_param'] = tr.opt_d.flat.cpu()
    return out


def _run_g13(rank, local):
    """The G13 step (tests/golden/make_goldens.py:g13): the reference's train_one_step under DDP,
    2 ranks x 2 clips of 4800 samples, n_q 2, all four losses balanced, the discriminator trained,
    warm-cosine LR at its first step. local: Trainer(ddp_commit_local=True), the reference's
    rank-local commit grads."""
    from oracle import encodec_oracle as O
    from fixtures import model_state, codebooks_from_stats, disc_state, load
    from synth import synth_wave
    from encx.model import EncodecModel
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from encx.train import Trainer
    d = load('g13_ddp.npz')
    cfg = O.Config(target_bandwidths=(1.5,), audio_normalize=True)
    m = EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    sd = dict(model_state(cfg, 71))
    for i, cb in enumerate(codebooks_from_stats(d['stats'], 73, 2, cfg.n_q)):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m = m.to(DEV)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(74), strict=False)
    disc = disc.to(DEV)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, max_iter=100, warmup_iter=0, ddp_commit_local=local)
    x = torch.from_numpy(synth_wave((4, 1, 4800), 131))[2 * rank:2 * rank + 2].to(DEV)
    out = tr.step(x)
    torch.cuda.synchronize()
    res = {'loss/' + k: float(v) for k, v in out.items()}
    names = [k for k, p in m.named_parameters() if p.requires_grad]
    for (p, g), k in zip(tr.opt._views, names):
        res['grad/' + k] = g.detach().cpu().clone()
        res['param/' + k] = p.detach().cpu().clone()
    res['disc_grad'] = tr.opt_d.flat_grad.cpu()
    dn = [k for k, p in disc.named_parameters() if p.requires_grad]
    for (p, _), k in zip(tr.opt_d._views, dn):
        res['dparam/' + k] = p.detach().cpu().clone()
    for i in range(2):
        cb = m.quantizer.vq.layers[i]._codebook
        for k in ('cluster_size', 'embed', 'embed_avg'):
            res[f'cb{i}/{k}'] = getattr(cb, k).detach().cpu().clone()
    return res


def _rank_main(rank, world, port, outdir, cases, g13):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    try:
        b = 2 * B // world
        x = _batch()[rank * b:(rank + 1) * b]
        for name in cases:
            torch.save(_run_case(name, x), os.path.join(outdir, f'{name}_r{rank}.pt'))
        if g13:
            for local in (False, True):
                torch.save(_run_g13(rank, local), os.path.join(outdir, f'g13_{int(local)}_r{rank}.pt'))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def _spawn(world, cases, g13=False):
    import torch.multiprocessing as mp
    outdir = tempfile.mkdtemp(prefix='encx_dp_')
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, outdir, cases, g13)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, f'rank processes exited with {codes}'
    return outdir


@pytest.fixture(scope='module')
def runs():
    outdir = _spawn(2, list(CASES), g13=True)
    two = {n: [torch.load(os.path.join(outdir, f'{n}_r{r}.pt'), weights_only=True) for r in range(2)]
           for n in CASES}
    for local in (0, 1):
        two[f'g13_{local}'] = [torch.load(os.path.join(outdir, f'g13_{local}_r{r}.pt'), weights_only=True)
                               for r in range(2)]
    x = _batch()
    one = {n: _run_case(n, x) for n in CASES if n != 'gen_nosync' and n not in MULTI_STEP}
    halves = [_run_case('gen_nosync', x[r * B:(r + 1) * B]) for r in range(2)]
    return two, one, halves


@pytest.fixture(scope='module')
def runs8(runs):
    outdir = _spawn(8, list(CASES8))
    return {n: [torch.load(os.path.join(outdir, f'{n}_r{r}.pt'), weights_only=True) for r in range(8)]
            for n in CASES8}


def close(a, b, rtol):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30)) <= rtol


def test_ranks_identical(runs):
    two, _, _ = runs
    for name in CASES:
        r0, r1 = two[name]
        assert torch.equal(r0['gen_param'], r1['gen_param']), name
        assert torch.equal(r0['gen_m'], r1['gen_m']), name
        if 'disc_param' in r0:
            assert torch.equal(r0['disc_param'], r1['disc_param']), name


def test_sync_codebooks_match_single_process(runs):
    two, one, _ = runs
    for name in ('gen_sync', 'gen_sync_plain', 'gan_sync_plain'):
        r0, r1 = two[name]
        ref = one[name]
        # every code of each half equals the single-process code of the same clips
        codes = torch.cat([r0['codes'], r1['codes']], dim=1)
        assert torch.equal(codes, ref['codes']), (name, int((codes != ref['codes']).sum()))
        for i in range(8):
            for k in ('cluster_size', 'embed', 'embed_avg'):
                key = f'cb{i}.{k}'
                assert torch.equal(r0[key], r1[key]), (name, key)
                assert close(r0[key], ref[key], 1e-5), (name, key)


def test_nosync_codebooks_follow_local_half(runs):
    two, _, halves = runs
    r = two['gen_nosync']
    for i in range(8):
        for k in ('cluster_size', 'embed_avg'):
            key = f'cb{i}.{k}'
            assert not torch.equal(r[0][key], r[1][key]), key
            for rank in range(2):
                assert close(r[rank][key], halves[rank][key], 1e-5), (rank, key)


def test_kmeans_init_broadcast(runs):
    two, _, _ = runs
    r0, r1 = two['kmeans_sync']
    for i in range(8):
        assert float(r0[f'cb{i}.inited']) == 1.0
        for k in ('cluster_size', 'embed', 'embed_avg'):
            assert torch.equal(r0[f'cb{i}.{k}'], r1[f'cb{i}.{k}']), (i, k)


def test_plain_grads_match_single_process(runs):
    two, one, _ = runs
    for name in ('gen_sync_plain', 'gan_sync_plain'):
        r0 = two[name][0]
        ref = one[name]
        assert close(r0['gen_grad'], ref['gen_grad'], 1e-4), name
        if 'disc_grad' in r0:
            assert close(r0['disc_grad'], ref['disc_grad'], 1e-4), name


def _split_grads(x):
    """Single-process generator grads of one step, split into the balanced part (y.backward
    of the balancer's out_grad) and the commit part (loss_w.backward)."""
    from encx.train import Trainer
    from encx.losses import total_loss
    torch.manual_seed(0)
    m, _ = _build(False, True)
    tr = Trainer(m, None, lr=3e-4, scheduler=False, weights={'l_t': 0.1, 'l_f': 1})
    m.train()
    tr.opt.zero_grad()
    y, loss_w, _ = m(x.to(DEV))
    out_grad = tr.balancer.compute(total_loss(None, None, None, x.to(DEV), y, 24000), y)
    torch.autograd.backward([y], [out_grad], retain_graph=True)
    g_bal = tr.opt.flat_grad.clone()
    tr.opt.flat_grad.zero_()
    loss_w.backward()
    return g_bal.cpu(), tr.opt.flat_grad.cpu()


def test_balanced_grads_half_plus_commit(runs):
    """1 x B32 split into its balanced and commit parts, against the 2 x B16 run's grads."""
    two, _, _ = runs
    g_bal, g_commit = _split_grads(_batch())
    want = 0.5 * g_bal.double() + g_commit.double()
    assert close(two['gen_sync'][0]['gen_grad'], want, 1e-4)


def test_graph_trainer_replays_match_eager_at_two_ranks(runs):
    """Trainer(graphs=True) at world 2: one HIP graph per segment between the collectives (the
    decoder's grad bucket all-reduced under the encoder backward, the encoder's under the
    discriminator phase), captured at step 2 and replayed at steps 3-5. Every step's losses and
    the final grads, parameters, Adam moments and codebooks equal the eager trainer's bit for
    bit, with and without the codebook sums all-reduced, and both ranks stay identical."""
    two, _, _ = runs
    for eager, graph in (('gan_eager3', 'gan_graph3'), ('gan_sync_eager3', 'gan_sync_graph3')):
        for r in range(2):
            a, b = two[eager][r], two[graph][r]
            for k in a:
                assert torch.equal(a[k], b[k]), (eager, r, k)
        # the ranks' codebooks agree only when their sums are all-reduced (sync_codebooks)
        for k in (('cb0.embed', 'cb7.cluster_size', 'gen_param') if 'sync' in graph else ('gen_param',)):
            assert torch.equal(two[graph][0][k], two[graph][1][k]), (graph, k)


# ---------------------------------------------------------------- G13: the reference's DDP step
def _g13_stats(v):
    v = v.double().reshape(-1)
    return np.array([v.sum().item(), v.abs().sum().item(), v.pow(2).sum().item()])


def _g13_close(mine, want, what, rtol):
    """per tensor: the sampled elements within rtol of the tensor's sampled scale, and the
    abs-sum / squared sum of the whole tensor within rtol."""
    from fixtures import g13_samples
    worst = 0.0
    for k, (ws, wsum) in want.items():
        t = mine[k].double().reshape(-1)
        s = t[torch.from_numpy(g13_samples(t.numel()))].numpy()
        scale = max(np.abs(ws).max(), 1e-30)
        e = float(np.abs(s - ws).max() / scale)
        ms = _g13_stats(t)
        e = max(e, abs(ms[1] - wsum[1]) / max(wsum[1], 1e-30), abs(ms[2] - wsum[2]) / max(wsum[2], 1e-30))
        worst = max(worst, e)
        assert e <= rtol, (what, k, e)
    return worst


def _g13_want(d, tag, rank=None):
    pre = '' if rank is None else f'r{rank}/'
    names = [k[len(pre + tag + '/'):] for k in d.files if k.startswith(pre + tag + '/')]
    return {k: (d[f'{pre}{tag}/{k}'], d[f'{pre}{tag}_sum/{k}']) for k in names}


def test_g13_reference_ddp_exact(runs):
    """Trainer(ddp_commit_local=True) on 2 ranks against the reference's own DDP step (G13,
    train_multi_gpu.py:56-124 under DDP :310-325): per rank, the generator grads Adam sees (the
    DDP-averaged balanced grads + that rank's own commit grads), the post-Adam parameters (which
    differ between the ranks, as the reference's do), the losses, each rank's codebook EMA
    buffers, and the DDP-averaged discriminator grads."""
    from fixtures import load
    d = load('g13_ddp.npz')
    two, _, _ = runs
    r = two['g13_1']
    for rank in range(2):
        mine = {k[5:]: v for k, v in r[rank].items() if k.startswith('grad/')}
        _g13_close(mine, _g13_want(d, 'total', rank), f'grad r{rank}', 2e-4)
        for k in ('l_t', 'l_f', 'l_g', 'l_feat'):
            want = float(d[f'r{rank}/loss/{k}'])
            assert abs(r[rank]['loss/' + k] - want) <= 2e-5 * abs(want), (rank, k, r[rank]['loss/' + k], want)
        for i in range(2):
            assert close(r[rank][f'cb{i}/cluster_size'], torch.from_numpy(d[f'r{rank}/cb{i}/cluster_size']), 1e-6)
            assert close(r[rank][f'cb{i}/embed_avg'][::16], torch.from_numpy(d[f'r{rank}/cb{i}/embed_avg_rows']), 1e-5)
            assert close(r[rank][f'cb{i}/embed'][::16], torch.from_numpy(d[f'r{rank}/cb{i}/embed_rows']), 1e-5)
        _g13_params(r[rank], d, rank)
    # the commit grads stay rank-local: the ranks' encoder weights differ after the step
    k = 'encoder.model.0.conv.conv.weight_v'
    assert not torch.equal(r[0]['param/' + k], r[1]['param/' + k])
    _g13_disc_close(r[0], d)


def _g13_disc_close(res, d, rtol=2e-4):
    """The DDP-averaged discriminator grads, per named tensor: within rtol of the tensor's
    largest magnitude, or, for a tensor whose exact value is zero (conv_post's bias: with every
    logit inside the hinge the real and fake terms cancel exactly, so the reference holds fp32
    noise, ~1e-6), within 1e-3 of the whole discriminator grad's largest magnitude. The
    fixture's flat vector is in the reference's parameter order (torch weight_norm registers
    bias, weight_g, weight_v), ours in this build's; both are cut by name."""
    names = [k[len('dparam/'):] for k in d.files if k.startswith('dparam/')]
    numel = {k[len('dparam/'):]: v.numel() for k, v in res.items() if k.startswith('dparam/')}
    assert sorted(names) == sorted(numel)

    def cut(flat, order):
        out, o = {}, 0
        for k in order:
            out[k] = flat[o:o + numel[k]]
            o += numel[k]
        assert o == flat.numel()
        return out

    mine = cut(res['disc_grad'].double(), list(numel))
    want = cut(torch.from_numpy(d['disc_grad']).double(), names)
    floor = 1e-3 * max(float(v.abs().max()) for v in want.values())
    rows = []
    for k in names:
        a, b = mine[k], want[k]
        err, scale = float((a - b).abs().max()), float(b.abs().max())
        rows.append((k, err / max(scale, 1e-30)))
        assert err <= max(rtol * scale, floor), (k, err, scale, floor)
    print('G13 disc grads: worst rel ' + ', '.join(f'{k} {e:.1e}' for k, e in sorted(rows, key=lambda r: -r[1])[:4]))


def _g13_params(res, d, rank):
    """Post-Adam parameters (first Adam step: p - lr * g / (|g| + eps) up to bias correction)
    at the sampled elements, element-wise; where the grad is so small that fp32 rounding can flip
    its sign (|g| below 1e-3 of the tensor's largest sampled grad), Adam's step direction is
    rounding, and the element is skipped."""
    from fixtures import g13_samples
    for k, want in _g13_want(d, 'param', rank).items():
        p = res['param/' + k].double().reshape(-1)
        idx = torch.from_numpy(g13_samples(p.numel()))
        g = d[f'r{rank}/total/{k}']
        live = np.abs(g) > 1e-3 * max(np.abs(g).max(), 1e-30)
        diff = np.abs(p[idx].numpy() - want[0])
        assert float(diff[live].max(initial=0.0)) <= 2e-6, (rank, k, float(diff[live].max()))


def test_g13_true_data_parallel(runs):
    """The default Trainer (one combined backward, deviation #7) on the G13 step: both ranks
    hold the same grads = the reference's DDP-averaged balanced grads + the MEAN of the two ranks'
    commit grads, and the same parameters."""
    from fixtures import load
    d = load('g13_ddp.npz')
    two, _, _ = runs
    r = two['g13_0']
    bal = _g13_want(d, 'bal')
    c0, c1 = _g13_want(d, 'commit', 0), _g13_want(d, 'commit', 1)
    for rank in range(2):
        mine = {k[5:]: v.double() for k, v in r[rank].items() if k.startswith('grad/')}
        worst = 0.0
        for k, (bs, _) in bal.items():
            from fixtures import g13_samples
            t = mine[k].reshape(-1)
            s = t[torch.from_numpy(g13_samples(t.numel()))].numpy()
            ws = bs + 0.5 * (c0[k][0] + c1[k][0])
            e = float(np.abs(s - ws).max() / max(np.abs(ws).max(), 1e-30))
            worst = max(worst, e)
            assert e <= 2e-4, (rank, k, e)
    for k in r[0]:
        if k.startswith(('grad/', 'param/')):
            assert torch.equal(r[0][k], r[1][k]), k


# ---------------------------------------------------------------- config 4's partition count
def test_eight_ranks_identical(runs8):
    for name in CASES8:
        r0 = runs8[name][0]
        for r in range(1, 8):
            assert torch.equal(r0['gen_param'], runs8[name][r]['gen_param']), (name, r)
            if 'disc_param' in r0:
                assert torch.equal(r0['disc_param'], runs8[name][r]['disc_param']), (name, r)


def test_eight_ranks_match_single_process(runs8, runs):
    """8 ranks x B4 over gloo (config 4's partition of a batch) against 1 rank x B32: codes,
    synced codebooks, and (balancer off) the averaged grads; with the balancer, 1/8 of the
    balanced grad + the commit grad."""
    _, one, _ = runs
    r8 = runs8['gan_sync_plain']
    ref = one['gan_sync_plain']
    codes = torch.cat([r8[r]['codes'] for r in range(8)], dim=1)
    assert torch.equal(codes, ref['codes'])
    for i in range(8):
        for k in ('cluster_size', 'embed', 'embed_avg'):
            assert close(r8[0][f'cb{i}.{k}'], ref[f'cb{i}.{k}'], 1e-5), (i, k)
    assert close(r8[0]['gen_grad'], ref['gen_grad'], 1e-4)
    assert close(r8[0]['disc_grad'], ref['disc_grad'], 1e-4)
    g_bal, g_commit = _split_grads(_batch())
    want = g_bal.double() / 8 + g_commit.double()
    assert close(runs8['gen_sync'][0]['gen_grad'], want, 1e-4)
