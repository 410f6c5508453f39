"""The multi-GPU step over the real RCCL backend, on the one GPU the pool gives this build.

A one-rank `nccl` (= RCCL) process group with ENCX_DIST_FORCE (encx/distrib.py) makes
encx.train.Trainer take its N > 1 path (train_multi_gpu.py:245-266 rendezvous, :310-325 DDP
all-reduce): the step cut into segments, the balancer's statistics all-reduce (balancer.py:99),
the decoder / encoder / discriminator grad buckets all-reduced asynchronously underneath the
following segments -- so RCCL kernels run while the persistent LSTM recurrences (one workgroup
per CU, spinning on their peers) are in flight. What must hold after 3 GAN steps:
  * the process group is RCCL and no LSTM hand-off spin timed out (Trainer.check_sync);
  * the first step's generator and discriminator grads and all three steps' losses equal the
    non-distributed step's within fp32 rounding (at world 1 every collective is an identity; the
    balancer takes its averages from the all-reduced fp32 buffer, red[k] / red[nl], instead of the
    fp64 EMA, and the backward runs split at the decoder input: rounding-level differences), and
    the parameters within Adam's per-step bound of 2 lr per element.
Runs in a child process (its own process group, under a time limit)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.join(sys.argv[1], 'encodec-pytorch_amd'))
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
torch.distributed.init_process_group('nccl', device_id=dev, rank=0, world_size=1)
from encx import distrib
from encx.model import EncodecModel
from encx.msstftd import MultiScaleSTFTDiscriminator
from encx.train import Trainer

def run(force):
    distrib.FORCE = force
    torch.manual_seed(11)
    model = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True, name='my_encodec').to(dev)
    disc = MultiScaleSTFTDiscriminator(filters=32).to(dev)
    tr = Trainer(model, disc, lr=3e-4, disc_lr=3e-4, max_iter=1000, warmup_iter=0, graphs=False)
    assert distrib.is_distributed() == force
    g = np.random.Generator(np.random.PCG64(5))
    losses, grads = [], None
    for i in range(3):
        x = torch.from_numpy((0.1 * g.standard_normal((32, 1, 24000))).astype(np.float32)).to(dev)
        out = tr.step(x)
        losses.append({k: float(v) for k, v in out.items()})
        if i == 0:  # the first step's gradients (the flat buffers Adam read; / world = 1)
            torch.cuda.synchronize()
            grads = [tr.opt.flat_grad.clone(), tr.opt_d.flat_grad.clone()]
    torch.cuda.synchronize()
    tr.check_sync()
    return losses, grads, [p.detach().clone() for p in model.parameters()] + [p.detach().clone() for p in disc.parameters()]

lf, gf, pf = run(True)
lp, gp, pp = run(False)
grad_rel = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(gf, gp))
dl = max(abs(a[k] - b[k]) / (abs(b[k]) + 1e-12) for a, b in zip(lf, lp) for k in b)
# Adam moves every element by at most ~lr per step whatever its gradient, so near-zero grads whose
# rounding differs may move differently: parameters agree to 2 * lr * steps in the worst element
dp = max(float((a - b).abs().max()) for a, b in zip(pf, pp))
print(json.dumps({'backend': torch.distributed.get_backend(), 'grad_rel': grad_rel, 'loss_rel': dl,
                  'param_abs': dp, 'losses_forced': lf[-1]}))
torch.distributed.destroy_process_group()
'''


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_rccl_one_rank_dp_step_matches_plain_step():
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()), ENCX_DIST_FORCE='0')
    r = subprocess.run([sys.executable, '-c', SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res['backend'] == 'nccl'
    assert res['grad_rel'] < 1e-5, res
    assert res['loss_rel'] < 1e-5, res
    assert res['param_abs'] <= 2 * 3e-4 * 3, res
