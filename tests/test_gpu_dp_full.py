"""Configs 4 and 5's data-parallel step at real size, rehearsed on ONE GPU over gloo (SURVEY §8e;
train_multi_gpu.py:277-282 per-rank batch, DDP :310-325; scripts/train.sbatch:12-35 for the
48 kHz stereo model). Child processes share cuda:0, one per rank; the parent checks them against
single-process runs of the same HIP path.

Config 4: 8 ranks x B32 config-3 GAN steps, all four losses balanced (l_t .1, l_f 1, l_g 3,
l_feat 3, config.yaml:55-60), codebook sums all-reduced (sync_codebooks):
  * ranks identical after the step (parameters, Adam moments, codebooks, discriminator);
  * G13-style grad decomposition, at full size and with every loss on: rank 0's generator grad
    equals (1/W) sum_r sum_k s_k G_k^r + (1/W) sum_r C^r, where G_k^r is loss k's backward through
    the generator on rank r's clips alone (computed here, in one process, one loss at a time),
    C^r the commit loss's, and s_k = (w_k / sum w) / (1e-12 + mean_r n_k^r) the balancer scale
    from the ranks' averaged per-item grad norms n_k^r (balancer.py:83-118 + distrib.py:112-124
    at the first step); the discriminator grad is the mean of the ranks' hinge-loss grads;
  * the synced codebooks: cluster_size = 0.99 cs0 + 0.01 * bincount(codes of ALL ranks).
Config 4 against one process: 2 ranks x B32 vs 1 x B64 (8 x B32 = B256 in one process would hold
eight ranks' activations on one GPU; since round 6 the LSTM takes it, in chunks of 64 rows): every
code bit-identical, codebooks within 1e-5.
Config 5: 2 ranks x B16 of the 48 kHz stereo model (n_q 16, 1 s = two segments, GroupNorm,
sync_codebooks, l_g = l_feat = 4 as train.sbatch:32-33) vs 1 x B32: codes bit-identical (the
second segment quantises with the codebooks synced after the first), codebooks within 1e-5,
ranks identical; and, with rank-local codebooks, the same grad decomposition.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
W24 = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}
W48 = {'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4}
# name: (48 kHz, world, clips per rank, sync_codebooks)
CASES = {'c4_8x32': (False, 8, 32, True), 'c4_2x32': (False, 2, 32, True), 'c5_2x16': (True, 2, 16, True),
         'c5_2x16_local': (True, 2, 16, False)}


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _build(k48, sync=True):
    """Synthetic PCG64 weights (fixtures.model_state) and inited codebooks; the discriminator of
    the model's channel count."""
    from oracle import encodec_oracle as O
    from fixtures import model_state, codebooks_from_stats, disc_state, cfg48k
    from encx.model import EncodecModel
    from encx.msstftd import MultiScaleSTFTDiscriminator
    if k48:
        cfg = cfg48k(target_bandwidths=(24.0,), segment=1.0)
        m = EncodecModel._get_model([24.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                    audio_normalize=True, segment=1.0, sync_codebooks=sync)
        sd, cbseed, dseed, ch = dict(model_state(cfg, 91)), 93, 94, 2
    else:
        cfg = O.Config(target_bandwidths=(6.0,), audio_normalize=True)
        m = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True, sync_codebooks=sync)
        sd, cbseed, dseed, ch = dict(model_state(cfg, 3)), 4, 5, 1
    stats = np.zeros((cfg.n_q, 2, 128), np.float32)
    stats[:, 1] = 0.05
    for i, cb in enumerate(codebooks_from_stats(stats, cbseed, cfg.n_q, cfg.n_q)):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    disc = MultiScaleSTFTDiscriminator(filters=32, in_channels=ch, out_channels=ch)
    disc.load_state_dict(disc_state(dseed, ch, ch), strict=False)
    return m.to(DEV), disc.to(DEV)


def _batch(k48, n):
    from synth import synth_wave
    shape = (n, 2, 48000) if k48 else (n, 1, 24000)
    return torch.from_numpy(synth_wave(shape, 808 if k48 else 707))


def _trainer(m, disc, k48):
    from encx.train import Trainer
    return Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=W48 if k48 else W24,
                   sample_rate=48000 if k48 else 24000)


def _state(tr, m):
    out = {'gen_grad': tr.opt.flat_grad.cpu(), 'gen_param': tr.opt.flat.cpu(), 'gen_m': tr.opt.exp_avg.cpu(),
           'disc_grad': tr.opt_d.flat_grad.cpu(), 'disc_param': tr.opt_d.flat.cpu(),
           'codes': m.last_codes[0].cpu()}
    for i, layer in enumerate(m.quantizer.vq.layers):
        for k in ('cluster_size', 'embed', 'embed_avg'):
            out[f'cb{i}.{k}'] = getattr(layer._codebook, k).detach().cpu().clone()
    return out


def _rank_main(rank, world, port, outdir, name):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    try:
        k48, _, b, sync = CASES[name]
        x = _batch(k48, world * b)[rank * b:(rank + 1) * b].to(DEV)
        torch.manual_seed(0)
        m, disc = _build(k48, sync)
        tr = _trainer(m, disc, k48)
        # every segment's codes (48 kHz: the last segment's are model.last_codes)
        codes = []
        q_fwd = m.quantizer.forward

        def qf(*a, _f=q_fwd, **k):
            r = _f(*a, **k)
            codes.append(r.codes)
            return r
        m.quantizer.forward = qf
        tr.step(x)
        torch.cuda.synchronize()
        res = _state(tr, m)
        res['codes_all'] = [c.cpu() for c in codes]
        res['max_mem_gib'] = torch.cuda.max_memory_allocated() / 2 ** 30
        torch.save(res, os.path.join(outdir, f'{name}_r{rank}.pt'))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def _spawn(name):
    import torch.multiprocessing as mp
    world = CASES[name][1]
    outdir = tempfile.mkdtemp(prefix='encx_dpf_')
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, outdir, name)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    rc = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert rc == [0] * world, f'rank processes exited with {rc}'
    return [torch.load(os.path.join(outdir, f'{name}_r{r}.pt'), weights_only=True) for r in range(world)]


def _single(name, n):
    """One process, one step on the first n clips of the case's batch (sync has no peer)."""
    k48 = CASES[name][0]
    torch.manual_seed(0)
    m, disc = _build(k48)
    tr = _trainer(m, disc, k48)
    codes = []
    q_fwd = m.quantizer.forward

    def qf(*a, _f=q_fwd, **k):
        r = _f(*a, **k)
        codes.append(r.codes)
        return r
    m.quantizer.forward = qf
    tr.step(_batch(k48, n).to(DEV))
    torch.cuda.synchronize()
    res = _state(tr, m)
    res['codes_all'] = [c.cpu() for c in codes]
    return res


def _decomposed(name):
    """The expected rank-averaged generator / discriminator grads of the case's first step,
    from per-rank, per-loss backward passes in this one process (see the module docstring)."""
    from encx.losses import total_loss, disc_loss
    from encx.ops import DiscGradMode
    k48, world, b, _ = CASES[name]
    wts = W48 if k48 else W24
    sr = 48000 if k48 else 24000
    x_all = _batch(k48, world * b).to(DEV)
    torch.manual_seed(0)
    m, disc = _build(k48, sync=False)
    tr = _trainer(m, disc, k48)  # for the flat grad buffers only
    cb0 = [{k: getattr(l._codebook, k).detach().clone() for k in ('cluster_size', 'embed', 'embed_avg')}
           for l in m.quantizer.vq.layers]
    m.train()
    disc.train()
    G = {k: torch.zeros_like(tr.opt.flat_grad) for k in wts}
    C = torch.zeros_like(tr.opt.flat_grad)
    D = torch.zeros_like(tr.opt_d.flat_grad)
    norms = {k: [] for k in wts}
    for r in range(world):
        for l, cb in zip(m.quantizer.vq.layers, cb0):  # every rank starts from the same codebooks
            for k, v in cb.items():
                getattr(l._codebook, k).data.copy_(v)
        x = x_all[r * b:(r + 1) * b]
        tr.opt.zero_grad()
        tr.opt_d.zero_grad()
        y, loss_w, _ = m(x, bandwidth=m.target_bandwidths[0])
        yd = y.detach().requires_grad_()
        mode = DiscGradMode(params=False, input=True)
        _, fr = disc(x, mode=mode)
        lf, ff = disc(yd, mode=mode)
        losses = total_loss(fr, lf, ff, x, yd, sr)
        for j, k in enumerate(wts):
            g = torch.autograd.grad(losses[k], [yd], retain_graph=True)[0]
            norms[k].append(g.double().flatten(1).norm(dim=1).mean())
            tr.opt.flat_grad.zero_()
            torch.autograd.backward([y], [g], retain_graph=True)
            G[k] += tr.opt.flat_grad
        tr.opt.flat_grad.zero_()
        loss_w.backward()
        C += tr.opt.flat_grad
        # the discriminator phase: hinge loss on real / detached fake, weight grads only
        mode_d = DiscGradMode(params=True, input=False)
        lr2, _ = disc(x, mode=mode_d)
        lf2, _ = disc(y.detach(), mode=mode_d)
        tr.opt_d.flat_grad.zero_()
        disc_loss(lr2, lf2).backward()
        D += tr.opt_d.flat_grad
    tw = sum(wts.values())
    gen = C.double() / world
    for k in wts:
        avg = torch.stack(norms[k]).mean()
        s = (wts[k] / tw) / (1e-12 + avg)
        gen += s * G[k].double() / world
    return gen.cpu(), (D.double() / world).cpu()


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _identical(runs, name):
    r0 = runs[0]
    for r, res in enumerate(runs[1:], 1):
        for k in r0:
            if k.startswith(('gen_param', 'gen_m', 'disc_param', 'cb', 'gen_grad', 'disc_grad')):
                assert torch.equal(r0[k], res[k]), (name, r, k)


def _check_decomposition(runs, name):
    gen, dg = _decomposed(name)
    e, ed = _rel(runs[0]['gen_grad'], gen), _rel(runs[0]['disc_grad'], dg)
    print(f'{name}: generator grad vs the per-rank, per-loss decomposition {e:.2e}; disc {ed:.2e}; '
          f'peak memory per rank {max(r["max_mem_gib"] for r in runs):.1f} GiB')
    assert e <= 1e-4, (name, e)
    assert ed <= 1e-4, (name, ed)


def _check_cluster_sizes(runs, name):
    """Synced EMA counts: 0.99 cs0 + 0.01 * (codes of every rank, every segment in turn)."""
    k48 = CASES[name][0]
    torch.manual_seed(0)
    m, _ = _build(k48, sync=False)
    n_seg = len(runs[0]['codes_all'])
    for i, layer in enumerate(m.quantizer.vq.layers):
        cs = layer._codebook.cluster_size.detach().double().cpu()
        for s in range(n_seg):
            cnt = sum(torch.bincount(r['codes_all'][s][i].reshape(-1), minlength=1024) for r in runs)
            cs = 0.99 * cs + 0.01 * cnt.double()
        assert _rel(runs[0][f'cb{i}.cluster_size'], cs) <= 1e-6, (name, i)


def _check_vs_single(runs, single, name):
    for s in range(len(single['codes_all'])):
        codes = torch.cat([r['codes_all'][s] for r in runs], dim=1)
        assert torch.equal(codes, single['codes_all'][s]), (name, s, int((codes != single['codes_all'][s]).sum()))
    for k in single:
        if k.startswith('cb'):
            assert _rel(runs[0][k], single[k]) <= 1e-5, (name, k, _rel(runs[0][k], single[k]))


def test_config4_eight_ranks_b32_full_gan():
    runs = _spawn('c4_8x32')
    _identical(runs, 'c4_8x32')
    _check_cluster_sizes(runs, 'c4_8x32')
    _check_decomposition(runs, 'c4_8x32')


def test_config4_two_ranks_b32_vs_one_process_b64():
    runs = _spawn('c4_2x32')
    _identical(runs, 'c4_2x32')
    _check_vs_single(runs, _single('c4_2x32', 64), 'c4_2x32')


def _commit_grad(name, n):
    """The commit loss's generator grad of one forward on the first n clips from the case's initial
    state (the unbalanced part of a step's generator grad)."""
    k48 = CASES[name][0]
    torch.manual_seed(0)
    m, disc = _build(k48)
    tr = _trainer(m, disc, k48)  # for the flat grad buffer only
    m.train()
    tr.opt.zero_grad()
    _, loss_w, _ = m(_batch(k48, n).to(DEV), bandwidth=m.target_bandwidths[0])
    loss_w.backward()
    torch.cuda.synchronize()
    return tr.opt.flat_grad.double().cpu()


def test_config5_two_ranks_48k_stereo_vs_one_process():
    """Synced codebooks at 48 kHz (the in-forward all-reduce between the two segments): codes
    bit-identical to one process on B32, codebooks within 1e-5, and the grads related as the
    reference's DDP step relates them (train_multi_gpu.py:310-325 + balancer.py:83-118): the
    balancer makes each clip's balanced output grad independent of the batch it sits in, so the
    W ranks' averaged generator grad is (1/W) x the one-process balanced part plus the one-process
    commit part C (computed separately): g_dp = (g_1 - C) / W + C; the discriminator's hinge grad
    is the one-process grad. Both up to fp32 summation order (1e-4 of the largest element)."""
    runs = _spawn('c5_2x16')
    single = _single('c5_2x16', 32)
    _identical(runs, 'c5_2x16')
    _check_vs_single(runs, single, 'c5_2x16')
    _check_cluster_sizes(runs, 'c5_2x16')
    world = CASES['c5_2x16'][1]
    C = _commit_grad('c5_2x16', 32)
    want = (single['gen_grad'].double() - C) / world + C
    eg, ed = _rel(runs[0]['gen_grad'], want), _rel(runs[0]['disc_grad'], single['disc_grad'])
    print(f'c5_2x16 synced: generator grad vs (g_1 - C) / W + C of one process {eg:.2e}; discriminator vs '
          f'one process {ed:.2e}')
    assert eg <= 1e-4 and ed <= 1e-4, (eg, ed)


def test_config5_two_ranks_48k_stereo_grad_decomposition():
    """The grad decomposition for the 48 kHz step with rank-local codebooks (the reference's
    default, core_vq.py:157,175): with two segments the second one quantises with codebooks the
    first one updated, so the per-rank restatement matches the trainer only when each rank's
    codebooks follow its own clips."""
    runs = _spawn('c5_2x16_local')
    for r, res in enumerate(runs[1:], 1):
        for k in ('gen_param', 'gen_m', 'disc_param', 'gen_grad', 'disc_grad'):
            assert torch.equal(runs[0][k], res[k]), (r, k)
    _check_decomposition(runs, 'c5_2x16_local')
