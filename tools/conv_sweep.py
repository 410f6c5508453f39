"""Per-layer time of the SEANet conv layers (conv_* / convtr_* / pw tags of the library's HIP-event
profiler) under several settings of the kernel-selection options, in ONE process: the generator
train step (config 2) is warmed, then profiled for --steps steps per setting.
Usage (GPU box): python tools/conv_sweep.py "CONV_SPLIT=1024" "CONV_SPLIT=2048" "CONV_CK=128" ...
Each argument is a comma-separated list of NAME=VALUE; "-" is the defaults. Prints a markdown table
of us per step per layer and setting, and each setting's total."""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))


def profile(tr, x, steps, lib):
    torch.cuda.synchronize()
    lib.encx_prof_enable(1)
    for _ in range(steps):
        tr.step(x)
    torch.cuda.synchronize()
    n = ctypes.c_int64()
    lib.encx_prof_read(None, None, None, ctypes.byref(n))
    agg = collections.OrderedDict()
    for i in range(n.value):
        ms, tag = ctypes.c_double(), ctypes.c_char_p()
        lib.encx_prof_slot(i, ctypes.byref(ms), None, None, ctypes.byref(tag))
        t = tag.value.decode()
        if t.startswith(('conv_', 'convtr_')) and not t.startswith('conv_rb'):
            agg[t] = agg.get(t, 0.0) + max(ms.value, 0.0) * 1e3 / steps
    lib.encx_prof_enable(0)
    return agg


def main():
    settings = sys.argv[1:] or ['-']
    steps = int(os.environ.get('SWEEP_STEPS', '3'))
    from encx.model import EncodecModel
    from encx.train import Trainer
    from encx._lib import lib, set_option
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True, name='my_encodec').to(dev)
    tr = Trainer(model, None, lr=3e-4, max_iter=100000, warmup_iter=500)
    g = np.random.Generator(np.random.PCG64(1234))
    x = torch.from_numpy((0.1 * g.standard_normal((32, 1, 24000))).astype(np.float32)).to(dev)
    for _ in range(3):
        tr.step(x)
    cols, defaults = [], {}
    for st in settings:
        kv = [] if st == '-' else [p.split('=') for p in st.split(',')]
        for k, v in kv:
            defaults.setdefault(k, set_option(k, int(v)))
        for _ in range(2):
            tr.step(x)
        cols.append((st, profile(tr, x, steps, lib)))
        for k, _ in kv:
            set_option(k, defaults[k])
        print(f'# {st}: {sum(cols[-1][1].values()):.1f} us per step', flush=True)
    rows = list(cols[0][1])
    print('| layer | ' + ' | '.join(c for c, _ in cols) + ' |')
    print('|---|' + '---|' * len(cols))
    for r in rows:
        print(f'| {r} | ' + ' | '.join(f'{c.get(r, float("nan")):.1f}' for _, c in cols) + ' |')
    print('| total | ' + ' | '.join(f'{sum(c.values()):.1f}' for _, c in cols) + ' |')


if __name__ == '__main__':
    main()
