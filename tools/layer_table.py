"""Per-launch-group table of one training step from the library's own HIP-event profiler
(encx_prof_slot): op, shape, time, achieved TFLOP/s and algorithmic GB/s, aggregated over the
timed steps. Usage (GPU box): python tools/layer_table.py [--config gen|gan] [--steps 3]."""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='gen')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--batch', type=int, default=32)
    args = ap.parse_args()
    from encx.model import EncodecModel
    from encx.train import Trainer
    from encx._lib import lib
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True, name='my_encodec').to(dev)
    disc = None
    if args.config == 'gan':
        from encx.msstftd import MultiScaleSTFTDiscriminator
        disc = MultiScaleSTFTDiscriminator(filters=32).to(dev)
    tr = Trainer(model, disc, lr=3e-4, disc_lr=3e-4, max_iter=100000, warmup_iter=500)
    g = np.random.Generator(np.random.PCG64(1234))
    x = torch.from_numpy((0.1 * g.standard_normal((args.batch, 1, 24000))).astype(np.float32)).to(dev)
    for _ in range(3):
        tr.step(x)
    torch.cuda.synchronize()
    lib.encx_prof_enable(1)
    for _ in range(args.steps):
        tr.step(x)
    torch.cuda.synchronize()
    n = ctypes.c_int64()
    ms_, fl_, by_ = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    lib.encx_prof_read(ctypes.byref(ms_), ctypes.byref(fl_), ctypes.byref(by_), ctypes.byref(n))
    agg = collections.OrderedDict()
    for i in range(n.value):
        ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        tag = ctypes.c_char_p()
        lib.encx_prof_slot(i, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by), ctypes.byref(tag))
        k = tag.value.decode()
        a = agg.setdefault(k, [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += max(ms.value, 0.0)  # booked-only (untimed) scopes report -1
        a[2] += fl.value
        a[3] += by.value
    lib.encx_prof_enable(0)
    S = args.steps
    tot = sum(a[1] for a in agg.values()) / S
    print(f'| op shape | calls/step | us/step | TFLOP/s | GB/s | % |\n|---|---|---|---|---|---|')
    for k, (c, ms, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if ms <= 0:
            continue
        print(f'| {k} | {c // S} | {1e3 * ms / S:.1f} | {fl / ms / 1e9:.1f} | {by / ms / 1e6:.0f} | '
              f'{100 * ms / S / tot:.1f} |')
    print(f'\ntotal {tot:.3f} ms/step over {n.value // S} scopes; '
          f'{fl_.value / S / 1e9:.1f} GFLOP/step -> {fl_.value / ms_.value / 1e9:.1f} TFLOP/s')


if __name__ == '__main__':
    main()
