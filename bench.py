"""EnCodec 24 kHz training throughput on MI355X (BASELINE.json metric).

python bench.py [--gpus N] [--steps K] [--warmup W] [--config gen|gan]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step = one train_multi_gpu.py:train_one_step iteration on one batch of 32 synthetic 1 s clips
per GPU. Default `--config gan` = BASELINE config 3, the configuration the metric's 1/2/4/8-GPU
series scales (config 4 = config 3 per rank): generator + RVQ (n_q 8) + MS-STFT discriminator,
l_t / l_f / l_g / l_feat through the Balancer, commit loss, Adam, then the discriminator update
(every step). `--config gen` = config 2 (no discriminator), `--config 48k` = config 5. Inputs are
resident in HBM before the timed region. Rank 0 prints one JSON line.

Steps replay HIP graphs at N = 1 (encx.train.Trainer(graphs=True): the step captured once
after one eager step); at N > 1 the steps run eagerly (Trainer.step; ENCX_DP_GRAPHS=1 replays one
graph per segment between the collectives, opt-in: DESIGN.md §6); --no-graphs steps eagerly.
The warmup covers the eager step and the capture. The roofline / whole-step books come from a
second, untimed, profiled pass of K eager steps (identical kernels).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))

MI355X_FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
MI355X_HBM_PEAK_GBS = 8000.0


WORKLOADS = {
    'gen': 'config 2: 24 kHz mono SEANet + RVQ n_q=8, generator-only (l_t, l_f via Balancer, commit loss, Adam)',
    'gan': 'config 3: 24 kHz mono full GAN (MS-STFT disc + Balancer)',
    '48k': 'config 5: 48 kHz stereo, non-causal time_group_norm, 1 s segments, n_q=16, full GAN',
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', choices=['gen', 'gan', '48k'], default='gan')
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--no-graphs', action='store_true', help='eager steps instead of HIP-graph replay')
    ap.add_argument('--sync-codebooks', action='store_true',
                    help='all-reduce the RVQ EMA code sums across ranks (north_star DP; off = reference)')
    return ap.parse_args()


def cpu_baseline(config, threads):
    """The CPU oracle's train step (oracle/encodec_oracle.py, the reference algorithm restated on
    torch-CPU) on a bounded sample: 8 clips (2 stereo clips for 48k) with initialised codebooks, 1 warm-up
    step, then timed steps until at least 12 s of wall time have passed (>= 2 steps)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
    from oracle import encodec_oracle as O
    from fixtures import model_state, codebooks_from_stats, disc_state, cfg48k
    from synth import synth_wave
    torch.set_num_threads(threads)
    if config == '48k':
        cfg = cfg48k(target_bandwidths=(24.0,), segment=1.0)
        bw, B, shape, lr = 24.0, 2, (2, 2, 48000), 1e-4
    else:
        cfg = O.Config(target_bandwidths=(6.0,), audio_normalize=True)
        bw, B, shape, lr = 6.0, 8, (8, 1, 24000), 3e-4
    p = model_state(cfg, 3)
    stats = np.zeros((cfg.n_q, 2, 128), np.float32)
    stats[:, 1] = 0.05
    cbs = codebooks_from_stats(stats, 4, cfg.n_q, cfg.n_q)
    gan = config in ('gan', '48k')
    dp = disc_state(5, cfg.channels, cfg.channels) if gan else None
    lg = 4 if config == '48k' else 3
    w = {'l_t': 0.1, 'l_f': 1, 'l_g': lg, 'l_feat': lg} if gan else {'l_t': 0.1, 'l_f': 1}
    bal = O.Balancer(w)
    st, dst = {}, {}
    x = torch.from_numpy(synth_wave(shape, 99))
    O.train_step(x, p, cbs, cfg, bw, bal, st, lr, dp, dst, lr)
    t0 = time.perf_counter()
    n = 0
    while n < 2 or (time.perf_counter() - t0 < 12.0 and n < 200):
        O.train_step(x, p, cbs, cfg, bw, bal, st, lr, dp, dst, lr)
        n += 1
    dt = time.perf_counter() - t0
    return {'value': B * n / dt, 'unit': 'audio-seconds/sec', 'cores': threads, 'kind': 'port',
            'sample': f'oracle train step ({config}), {B} x 1 s clips, {n} timed steps after 1 warm-up, '
                      f'{dt:.1f} s wall on {threads} threads'}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # ENCX_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- a one-GPU rehearsal of the
    # N-rank path (collectives, barriers, max-over-ranks timing); the real runs use RCCL
    rehearse = os.environ.get('ENCX_BENCH_REHEARSE', '0') == '1'
    if rehearse:
        local = 0
        # the ranks share one GPU: two persistent LSTM launches (each one workgroup per CU,
        # spinning on its own peers) from two processes can hold each other's CUs -- round 5's
        # eager rehearsal paid that in stalls (216 ms/step), round 6's loud-failure check turned
        # the spin timeouts into errors; the step form has no inter-workgroup waits
        os.environ.setdefault('ENCX_LSTM_PERSIST', '0')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    # ENCX_DIST_FORCE=1 at one rank: the N > 1 step (segments, RCCL all-reduces) over a one-rank
    # RCCL group -- the per-rank cost of the data-parallel path on this GPU (encx/distrib.py)
    force = os.environ.get('ENCX_DIST_FORCE', '0') == '1' and world == 1 and not rehearse
    if force:
        for k, v in (('MASTER_ADDR', '127.0.0.1'), ('MASTER_PORT', '29533'), ('RANK', '0'), ('WORLD_SIZE', '1')):
            os.environ.setdefault(k, v)
    if world > 1 or force:
        if rehearse:
            torch.distributed.init_process_group('gloo')
        else:
            torch.distributed.init_process_group('nccl', device_id=dev)
    import encx
    from encx.model import EncodecModel
    from encx.train import Trainer
    from encx._lib import lib

    torch.manual_seed(3401 + rank)
    B = args.batch
    g = np.random.Generator(np.random.PCG64(1234 + rank))
    if args.config == '48k':
        # config 5 (scripts/train.sbatch:18-33): 48 kHz stereo, non-causal, time_group_norm,
        # 1 s segments (48000 + 480 samples per clip), n_q 16, lr 1e-4, l_g = l_feat = 4
        model = EncodecModel._get_model([24.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                        audio_normalize=True, segment=1.0, name='encodec_48khz',
                                        sync_codebooks=args.sync_codebooks).to(dev)
        from encx.msstftd import MultiScaleSTFTDiscriminator
        disc = MultiScaleSTFTDiscriminator(filters=32, in_channels=2, out_channels=2).to(dev)
        trainer = Trainer(model, disc, lr=1e-4, disc_lr=1e-4, max_iter=100000, warmup_iter=500,
                          weights={'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4}, sample_rate=48000,
                          graphs=not args.no_graphs)
        shape = (B, 2, 48000)
    else:
        model = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                        audio_normalize=True, name='my_encodec',
                                        sync_codebooks=args.sync_codebooks).to(dev)
        disc = None
        if args.config == 'gan':
            from encx.msstftd import MultiScaleSTFTDiscriminator
            disc = MultiScaleSTFTDiscriminator(filters=32).to(dev)
        trainer = Trainer(model, disc, lr=3e-4, disc_lr=3e-4, max_iter=100000, warmup_iter=500,
                          graphs=not args.no_graphs)
        shape = (B, 1, 24000)
    batches = [torch.from_numpy((0.1 * g.standard_normal(shape)).astype(np.float32)).to(dev)
               for _ in range(4)]

    for i in range(args.warmup):
        trainer.step(batches[i % 4])
    torch.cuda.synchronize()

    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.step(batches[i % 4])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    trainer.check_sync()  # no persistent-LSTM hand-off failed in the timed steps (raises otherwise)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    prof = not args.no_roofline
    if prof:
        # a second, untimed pass of the same K steps with the encx profiler on (eager: profiler
        # events are not graph-captured) books every kernel's algorithmic FLOPs / bytes and times
        # the conv family with HIP events on the launch stream; whole-step rates use the timed
        # region's wall time above
        lib.encx_prof_enable(1)
        for i in range(args.steps):
            trainer.step(batches[i % 4])
        torch.cuda.synchronize()
    roof = whole = None
    if prof:
        import ctypes
        n = ctypes.c_int64()
        lib.encx_prof_read(None, None, None, ctypes.byref(n))
        # the dominant family: the implicit-GEMM conv kernels, SEANet Conv1d / ConvTranspose1d and
        # the discriminator's Conv2d (fwd + bwd-data + bwd-weight); every other booked scope
        # (LSTM, RVQ, mel, STFT, Adam, elementwise) enters the whole-step totals only
        ms = fl = by = 0.0
        launches = 0
        all_fl = all_by = all_ms = 0.0
        for i in range(n.value):
            m_, f_, b_, tag = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_char_p()
            lib.encx_prof_slot(i, ctypes.byref(m_), ctypes.byref(f_), ctypes.byref(b_), ctypes.byref(tag))
            all_fl += f_.value
            all_by += b_.value
            if m_.value > 0:
                all_ms += m_.value
            if tag.value.decode().startswith(('conv', 'c2_')):
                ms, fl, by, launches = ms + m_.value, fl + f_.value, by + b_.value, launches + 1
        lib.encx_prof_enable(0)
        achieved = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        # traffic: HBM bytes per conv-family ABI call from the committed rocprofv3 PMC passes
        # (FETCH_SIZE x2 + WRITE_SIZE, calibrated: tools/traffic.py); null when no pass exists
        traffic = None
        tpath = next((p for p in (os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', r,
                                               f'traffic_{args.config}.json') for r in ('r06', 'r05', 'r04', 'r03', 'r02'))
                      if os.path.exists(p)), '')
        if os.path.exists(tpath) and launches:
            with open(tpath) as fh:
                tj = json.load(fh)
            traffic = round(tj['hbm_bytes_per_step'] / (launches / args.steps))
        roof = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': MI355X_FP32_PEAK_TFLOPS,
                'unit': 'TFLOP/s', 'frac': round(achieved / MI355X_FP32_PEAK_TFLOPS, 4), 'traffic': traffic,
                'traffic_source': os.path.relpath(tpath) if tpath else None,
                'algorithmic_bytes_per_launch': round(by / launches) if launches else None,
                'kernel': 'encx conv/convtr/conv2d fwd + bwd-data + bwd-weight (implicit-GEMM f32 MFMA)',
                'launches': launches, 'kernel_ms_per_step': round(ms / args.steps, 3),
                'algorithmic_bytes_per_step': by / args.steps,
                'algorithmic_flops_per_step': fl / args.steps}
        # whole step: every booked kernel's algorithmic FLOPs / bytes over the wall
        # time of a step; hbm_frac = bytes / (t * 8 TB/s), max_roofline_frac = max(bytes / 8 TB/s,
        # flops / 157.3 TF/s) / t
        t_step = dt / args.steps
        f_step, b_step = all_fl / args.steps, all_by / args.steps
        whole = {'flops_per_step': f_step, 'bytes_per_step': b_step,
                 'timed_kernel_ms_per_step': round(all_ms / args.steps, 3),
                 'achieved_tflops': round(f_step / t_step / 1e12, 2),
                 'achieved_gbs': round(b_step / t_step / 1e9, 1),
                 'hbm_frac': round(b_step / (t_step * MI355X_HBM_PEAK_GBS * 1e9), 4),
                 'mfma_frac': round(f_step / (t_step * MI355X_FP32_PEAK_TFLOPS * 1e12), 4),
                 'max_roofline_frac': round(max(b_step / (MI355X_HBM_PEAK_GBS * 1e9),
                                                f_step / (MI355X_FP32_PEAK_TFLOPS * 1e12)) / t_step, 4)}

    value = B * world * args.steps * 1.0 / dt
    if rank == 0:
        out = {
            'metric': 'audio-seconds/sec EnCodec24k train step, batch 32x1s',
            'value': round(value, 2), 'unit': 'audio-seconds/sec', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(dt * 1e3 / args.steps, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
            'data': 'synthetic (0.1*N(0,1) clips, random-init weights)',
            'config': {'workload': WORKLOADS[args.config],
                       'global_batch': B * world, 'clip_seconds': 1.0,
                       'sample_rate': 48000 if args.config == '48k' else 24000,
                       'parallelism': f'dp{world}'},
            'roofline': roof,
            'whole_step': whole,
        }
        if args.sync_codebooks:
            out['config']['sync_codebooks'] = True
        if rehearse:
            # every rank shared ONE physical GPU over gloo: a rehearsal of the N-rank code path,
            # not an N-GPU measurement
            out['rehearsal'] = True
            out['n_gpus'] = 1
            out['ranks'] = world
            out['config']['parallelism'] = f'dp{world} rehearsal: {world} ranks on 1 GPU over gloo'
        if force:
            out['config']['parallelism'] = 'dp1, the N > 1 step forced over a one-rank RCCL group (ENCX_DIST_FORCE)'
        if world == 1 and not args.no_cpu_baseline:
            # every host core this job may use: the process's CPU affinity, capped by the CPU share
            # the box grants a one-GPU job (OMP_NUM_THREADS, 16 on the pool's boxes; os.cpu_count()
            # there reports the whole machine, most of it not ours)
            cores = len(os.sched_getaffinity(0))
            share = int(os.environ.get('OMP_NUM_THREADS', '0') or 0)
            out['cpu_baseline'] = cpu_baseline(args.config, min(cores, share) if share > 0 else cores)
        print(json.dumps(out), flush=True)
    if world > 1 or force:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
