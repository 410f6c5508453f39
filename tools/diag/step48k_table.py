"""Diagnostic: the per-tensor error table of the 48 kHz GAN fixture step (tests/steputil.py),
written to gpurun_out/step48k_table.txt, all tensors, both steps (no assertion)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', '..', 'tests'),
                os.path.join(os.path.dirname(__file__), '..', '..', 'tests', 'golden'),
                os.path.join(os.path.dirname(__file__), '..', '..', 'encodec-pytorch_amd'),
                os.path.join(os.path.dirname(__file__), '..', '..')]
import torch  # noqa: E402

import steputil  # noqa: E402
from test_gpu_48k import build48k, load, T, DEV, disc_state  # noqa: E402



def table_step(tr, x, cfg, bw, weights):
    snap = steputil.snapshot(tr)
    tr.step(x)
    torch.cuda.synchronize()
    o64 = steputil.oracle_step(snap, x, cfg, bw, weights, torch.float64)[0]
    o32 = steputil.oracle_step(snap, x, cfg, bw, weights, torch.float32)[0]
    rows = []
    for tag, mod, opt, key in (('gen', tr.model, tr.opt, 'grads'), ('disc', tr.disc, tr.opt_d, 'disc_grads')):
        names = [k for k, q in mod.named_parameters() if q.requires_grad]
        for k, (q, g, _, _) in steputil._flat_views(opt, names).items():
            if k in o64[key]:
                rows.append((f'{tag}:{k}', steputil._rel(g, o64[key][k]), steputil._rel(o32[key][k], o64[key][k]), 0))
    return rows
from encx.train import Trainer  # noqa: E402
from encx.msstftd import MultiScaleSTFTDiscriminator  # noqa: E402

d = load('g9_step48k.npz')
m, p, cbs, cfg = build48k(d, 'gan/')
disc = MultiScaleSTFTDiscriminator(filters=32, in_channels=2, out_channels=2)
disc.load_state_dict(disc_state(94, 2, 2), strict=False)
disc = disc.to(DEV)
weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 4, 'l_feat': 4}
tr = Trainer(m, disc, lr=1e-4, disc_lr=1e-4, scheduler=False, weights=weights, sample_rate=48000)
x = T(d['gan/x']).to(DEV)
os.makedirs('gpurun_out', exist_ok=True)
with open('gpurun_out/step48k_table.txt', 'w') as f:
    for it in range(2):
        table = table_step(tr, x, cfg, 3.0, weights)
        f.write(f'# step {it}\n')
        for n, e, e32, b in sorted(table, key=lambda r: -r[1]):
            f.write(f'{n:60s} {e:.3e} {e32:.3e} {e / max(e32, 1e-30):7.2f}\n')
print(open('gpurun_out/step48k_table.txt').read()[:6000])
