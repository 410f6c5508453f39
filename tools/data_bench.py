"""Batch assembly throughput: encx.data.make_batch from 2000 resident 5 s
clips into [32][1][24000] batches (config 2). Prints one JSON line: batches/s and audio-s/s of
the whole call (host crop draws + one metadata copy + one launch), the crop/collate kernel's
own GB/s (HIP events on its stream; 8 B per output sample) against HBM peak, and the oracle's
numpy crop+collate on the host as the CPU baseline.

python tools/data_bench.py [--iters N]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    args = ap.parse_args()
    import types
    from encx.data import CustomAudioDataset
    cfg = types.SimpleNamespace(datasets=types.SimpleNamespace(fixed_length=0, tensor_cut=24000),
                                model=types.SimpleNamespace(sample_rate=24000, channels=1))
    g = np.random.default_rng(3)
    clips = [(0.1 * g.standard_normal(120000)).astype(np.float32) for _ in range(2000)]
    ds = CustomAudioDataset(cfg, clips=clips, device='cuda')
    random.seed(0)
    order = list(range(2000))
    for _ in range(5):
        ds.make_batch(order[:32])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.iters):
        s = (i * 32) % 1984
        ds.make_batch(order[s:s + 32])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters

    # kernel alone, large batch (4096 crops) so it is not launch bound
    idx = [i % 2000 for i in range(4096)]
    starts = [random.randint(0, 120000 - 24000 - 1) for _ in idx]
    lens = [24000] * len(idx)
    st = torch.cuda.current_stream()
    out = ds.pool.gather(idx, starts, lens, 1)   # checked path once; then the bare launch
    from encx._lib import call, stream
    pool = ds.pool
    ii = np.asarray(idx)
    meta = torch.from_numpy(np.stack([pool.offsets[ii], pool.lengths[ii], pool.channels[ii],
                                      np.asarray(starts), np.asarray(lens)])).cuda()
    ref = out.clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(20):
        call('encx_crop_collate', pool.data.data_ptr(), meta[0].data_ptr(), meta[1].data_ptr(),
             meta[2].data_ptr(), meta[3].data_ptr(), meta[4].data_ptr(), out.data_ptr(), len(idx), 1,
             24000, stream())
    e1.record(st)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    k_s = e0.elapsed_time(e1) / 20 * 1e-3
    gbs = out.numel() * 8 / k_s / 1e9

    from oracle import data_oracle as D
    t0 = time.perf_counter()
    n = 0
    while n < 3 or time.perf_counter() - t0 < 2.0:
        D.collate([D.crop(D.expand(clips[i], 1), 24000)[0] for i in order[:32]])
        n += 1
    cpu = (time.perf_counter() - t0) / n
    print(json.dumps({
        'metric': 'training batches/s, [32][1][24000] crops from resident clips',
        'value': round(1 / dt, 1), 'audio_seconds_per_sec': round(32 / dt, 1), 'unit': 'batches/s',
        'ms_per_batch': round(dt * 1e3, 4),
        'kernel': {'crops': 4096, 'us': round(k_s * 1e6, 2), 'GBs': round(gbs, 1), 'peak_GBs': 8000.0,
                   'frac': round(gbs / 8000.0, 4), 'bytes_per_sample': 8},
        'cpu_baseline': {'ms_per_batch': round(cpu * 1e3, 3), 'kind': 'port', 'cores': 1,
                         'sample': 'oracle numpy crop + collate of the same 32 clips'},
        'data': 'synthetic 5 s clips (0.1*N(0,1)), 2000 resident in HBM'}), flush=True)


if __name__ == '__main__':
    main()
