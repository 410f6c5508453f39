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
    'gan_eager3': (True, False, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 3, False),
    'gan_graph3': (True, False, True, {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}, True, 3, True),
}
MULTI_STEP = ('gan_eager3', 'gan_graph3')


def _run_case(name, x):
    """One Trainer.step on x; returns everything the comparisons need (CPU tensors)."""
    from encx.train import Trainer
    gan, sync, rescale, weights, inited, steps, graphs = (CASES[name] + (1, False))[:7]
    torch.manual_seed(0)
    m, disc = _build(gan, sync, inited=inited)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=weights,
                 balancer_kwargs={'rescale_grads': rescale}, graphs=graphs)
    for i in range(steps):
        tr.step(x.to(DEV) * (1.0 + 0.1 * i))
    torch.cuda.synchronize()
    assert not graphs or any(isinstance(v, tuple) for v in tr._graphs.values())
    out = {'gen_grad': tr.opt.flat_grad.cpu(), 'gen_param': tr.opt.flat.cpu(),
           'gen_m': tr.opt.exp_avg.cpu(), 'codes': m.last_codes[0].cpu()}
    for i, layer in enumerate(m.quantizer.vq.layers):
        cb = layer._codebook
        for k in ('cluster_size', 'embed', 'embed_avg', 'inited'):
            out[f'cb{i}.{k}'] = getattr(cb, k).detach().cpu().clone()
    if disc is not None:
        out['disc_grad'] = tr.opt_d.flat_grad.cpu()
        out['disc_param'] = tr.opt_d.flat.cpu()
    return out


def _rank_main(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    try:
        x = _batch()[rank * B:(rank + 1) * B]
        for name in CASES:
            torch.save(_run_case(name, x), os.path.join(outdir, f'{name}_r{rank}.pt'))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.fixture(scope='module')
def runs():
    import torch.multiprocessing as mp
    outdir = tempfile.mkdtemp(prefix='encx_dp_')
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, outdir)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], f'rank processes exited with {codes}'
    two = {n: [torch.load(os.path.join(outdir, f'{n}_r{r}.pt'), weights_only=True) for r in range(2)]
           for n in CASES}
    x = _batch()
    one = {n: _run_case(n, x) for n in CASES if n != 'gen_nosync' and n not in MULTI_STEP}
    halves = [_run_case('gen_nosync', x[r * B:(r + 1) * B]) for r in range(2)]
    return two, one, halves


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


def test_graph_steps_match_eager_two_ranks(runs):
    """3 data-parallel GAN steps replayed from HIP graphs (collectives eager between the captured
    segments) equal the eager run with the overlapped decoder-bucket all-reduce, bit for bit."""
    two, _, _ = runs
    for r in range(2):
        a, b = two['gan_eager3'][r], two['gan_graph3'][r]
        for k in a:
            assert torch.equal(a[k], b[k]), (r, k)
