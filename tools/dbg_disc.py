import sys, os
sys.path[:0] = ['.', 'tests', 'tests/golden', 'encodec-pytorch_amd']
import torch, numpy as np
from oracle import encodec_oracle as O
from fixtures import disc_state
from encx.msstftd import MultiScaleSTFTDiscriminator
from encx.losses import total_loss
DEV = 'cuda:0'
def rel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))
disc = MultiScaleSTFTDiscriminator(filters=32)
p = disc_state(9)
disc.load_state_dict(p, strict=False)
disc = disc.to(DEV)
g = torch.Generator().manual_seed(5)
x64 = 0.1 * torch.randn(2, 1, 24000, generator=g, dtype=torch.float64)
y64 = (x64 + 0.05 * torch.randn(2, 1, 24000, generator=g, dtype=torch.float64)).requires_grad_(True)
p64 = {k: v.double() for k, v in p.items()}
lr64, fr64 = O.msstft_forward(x64, p64)
lf64, ff64 = O.msstft_forward(y64, p64)
print('logit range', [ (float(l.min()), float(l.max())) for l in lf64])
ref = O.total_loss(fr64, lf64, ff64, x64, y64)
gg64, = torch.autograd.grad(ref['l_g'].sum(), [y64], retain_graph=True)
gf64, = torch.autograd.grad(ref['l_feat'].sum(), [y64], retain_graph=True)
x = x64.float().to(DEV)
y = y64.detach().float().to(DEV).requires_grad_(True)
lr, fr = disc(x, param_grads=False)
lf, ff = disc(y, param_grads=False)
for a, b in zip(lf, lf64): print('logit rel', rel(a, b))
out = total_loss(fr, lf, ff, x, y)
print({k: (out[k].item(), ref[k].item()) for k in ('l_g', 'l_feat')})
gg, = torch.autograd.grad(out['l_g'], [y], retain_graph=True)
gf, = torch.autograd.grad(out['l_feat'], [y], retain_graph=True)
print('gg rel', rel(gg, gg64), 'gf rel', rel(gf, gf64))
e = (gg.double().cpu() - gg64.detach()).abs().reshape(-1)
i = int(e.argmax()); print('worst idx', i, 'of', e.numel(), 'val', float(gg.reshape(-1)[i]), float(gg64.reshape(-1)[i]), 'max', float(gg64.abs().max()))
print('err quantiles', [float(q) for q in torch.quantile(e[:100000], torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.float64))])
# per-scale grad: one discriminator at a time through hinge
for k in range(3):
    g64k, = torch.autograd.grad(torch.relu(1 - lf64[k]).mean(), [y64], retain_graph=True)
    gk, = torch.autograd.grad(torch.relu(1 - lf[k]).mean(), [y], retain_graph=True)
    print('scale', k, 'rel', rel(gk, g64k))
