"""Diagnostic: where the discriminator's input grad of l_g (the hinge generator loss) loses
precision. Config-3 disc at B 32 x 1 s: our grads of every feature map and of the audio against
the fp64 oracle (slope masks from our maps), beside the fp32 oracle's. GPU box, repo root."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), ROOT,
                os.path.join(ROOT, 'encodec-pytorch_amd')]
import steputil as S  # noqa: E402
from oracle import encodec_oracle as O  # noqa: E402
from synth import synth_wave  # noqa: E402
from fixtures import disc_state  # noqa: E402

DEV = 'cuda:0'


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def main():
    from encx.msstftd import MultiScaleSTFTDiscriminator, adversarial_losses
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.to(DEV)
    y = torch.as_tensor(synth_wave((32, 1, 24000), 608)).to(DEV).requires_grad_(True)
    store = []
    hooks = S.disc_mask_hooks(disc, store, DEV)
    logits, fmaps = disc(y)
    for h in hooks:
        h.remove()
    for fm in fmaps:
        for f in fm:
            f.retain_grad()
    l_g, _ = adversarial_losses(fmaps, logits, fmaps)
    l_g.backward()
    torch.cuda.synchronize()
    masks = [[m > 0 for m in store[k * 5:(k + 1) * 5]] for k in range(3)]
    res = {}
    for dt in (torch.float64, torch.float32):
        p = {k: v.detach().to(dt).requires_grad_(True) for k, v in disc.named_parameters()}
        yy = y.detach().to(dt).requires_grad_(True)
        with torch.backends.cudnn.flags(enabled=False):
            lg, fm = O.msstft_forward(yy, p, masks=masks)
            for f in fm:
                for z in f:
                    z.retain_grad()
            K = len(lg)
            l = sum(torch.mean(torch.relu(1 - lg[k])) for k in range(K)) / K / K
            l.backward()
        res[dt] = (yy, fm)
    y64, fm64 = res[torch.float64]
    y32, fm32 = res[torch.float32]
    print(f'd l_g / d y: ours {rel(y.grad, y64.grad):.3e}  fp32 oracle (GPU torch) {rel(y32.grad, y64.grad):.3e}')
    for k in range(3):
        for j in range(5):
            print(f'  disc {k} map {j} grad: ours {rel(fmaps[k][j].grad, fm64[k][j].grad):.3e}  fp32 oracle '
                  f'{rel(fm32[k][j].grad, fm64[k][j].grad):.3e}')


if __name__ == '__main__':
    main()
