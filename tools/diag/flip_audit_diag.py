"""Diagnostic for tests/steputil.check_flips: runs the G7 GAN fixture's two checked steps
(tests/test_gpu_disc.py::test_train_step_gan_fixture) with check_flips wrapped; when it fails,
prints for the failing map the whole-map fp64 recompute (F.conv2d of the captured HIP input with
the snapshot weights, and with the trainer's current weights), whether the captured input equals
the previous layer's captured output, and the element's neighbourhood. Run on a GPU box from the
repo root."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden'), ROOT,
                os.path.join(ROOT, 'encodec-pytorch_amd')]
import steputil as S  # noqa: E402
from oracle import encodec_oracle as O  # noqa: E402
from fixtures import load, T, model_state, codebooks_from_stats  # noqa: E402
from test_gpu_disc import make_disc  # noqa: E402

DEV = 'cuda:0'


def full_conv(layer, prm, x):
    g = prm.get('weight_g')
    w = prm['weight_v' if g is not None else 'weight'].double().to(x.device)
    if g is not None:
        w = O.weight_norm(w, g.double().to(x.device))
    b = prm['bias'].double().to(x.device)
    return F.conv2d(x.double(), w, b, stride=layer.stride, dilation=layer.dilation, padding=layer.padding)


def main():
    from encx.train import Trainer
    from encx.model import EncodecModel
    d = load('g7_step.npz')
    cfg = O.Config(target_bandwidths=(1.5,), audio_normalize=True)
    m = EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    p = model_state(cfg, 71)
    cbs = codebooks_from_stats(d['gan/stats'], 73, 2, cfg.n_q)
    sd = dict(p)
    for i, cb in enumerate(cbs):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m = m.to(DEV)
    disc, _ = make_disc(74)
    weights = {'l_t': 0.1, 'l_f': 1, 'l_g': 3, 'l_feat': 3}
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False, weights=weights)
    x = T(d['gan/x']).to(DEV)
    orig = S.check_flips

    def wrapped(disc_, params, maps_in, maps_out, a64, f64, what):
        try:
            return orig(disc_, params, maps_in, maps_out, a64, f64, what)
        except AssertionError as e:
            print('AUDIT FAILED:', e, flush=True)
            msg = str(e)
            i = int(msg.split("'map ")[1].split(':')[0])
            half, per = 15, 5
            layer = disc_.discriminators[(i % half) // per].convs[i % per]
            pre = f'discriminators.{(i % half) // per}.convs.{i % per}.conv.'
            prm = {k[len(pre):]: v for k, v in params.items() if k.startswith(pre)}
            cur = {k[len(pre):]: v.detach().cpu() for k, v in disc_.named_parameters() if k.startswith(pre)}
            y = maps_out[i].double()
            zh = torch.where(y > 0, y, y / 0.2)
            for tag, pr in (('snapshot', prm), ('current', cur)):
                z64 = full_conv(layer, pr, maps_in[i])
                r = (zh - z64).abs()
                print(f'  {tag} weights: max |z_hip - z64| {float(r.max()):.3e}, median {float(r.median()):.3e}', flush=True)
            zo = a64[i][0].double().cpu()
            z64s = full_conv(layer, prm, maps_in[i])
            print(f'  HIP vs oracle (whole map): max {float((zh - zo).abs().max()):.3e}; recompute vs oracle: max '
                  f'{float((z64s - zo).abs().max()):.3e}; shapes hip {tuple(zh.shape)} oracle {tuple(zo.shape)}', flush=True)
            if i % per:
                yo = a64[i - 1][0].double().cpu()
                xo = torch.where(a64[i - 1][1].cpu(), yo, 0.2 * yo)
                print(f'  captured input vs the oracle\'s input (lrelu of its previous map): max '
                      f'{float((maps_in[i].double() - xo).abs().max()):.3e}', flush=True)
                z64o = full_conv(layer, prm, xo)
                print(f'  recompute from the oracle input vs oracle: max {float((z64o - zo).abs().max()):.3e}', flush=True)
            if i % per:
                dlt = (maps_in[i].double() - maps_out[i - 1].double()).abs()
                print(f'  input vs previous output: max diff {float(dlt.max()):.3e}', flush=True)
            for k, v in prm.items():
                print(f'  snapshot {k} vs current: max diff {float((v.double() - cur[k].double()).abs().max()):.3e}')
            raise
    S.check_flips = wrapped
    for it in range(2):
        try:
            S.check_step(tr, x, cfg, 1.5, weights)
            print(f'step {it}: ok', flush=True)
        except AssertionError as e:
            print(f'step {it}: {str(e)[:300]}', flush=True)


if __name__ == '__main__':
    main()
