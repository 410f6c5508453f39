"""Config 3 at its real size (B 32, 1 s clips) against fp64: every SEANet conv layer in
isolation (forward, input grad, weight-norm and bias grads), and one whole Trainer step's
generator and discriminator weight grads, post-Adam parameters and codebook buffers.

The conv1d planners pick their split-K and weight-grad slab plans from B and T
(csrc/conv1d.hip plan_split / plan_wgrad), so the plans the bench times are only exercised at
B 32 and the real lengths; the fixture- and oracle-sized tests elsewhere run at B 2. The fp64
side is the oracle's own functions (oracle/encodec_oracle.py: sconv1d, sconvtr1d, resblock,
train_step; reference modules/conv.py:195-252, modules/seanet.py:46-144,
train_multi_gpu.py:56-129) evaluated by torch on the GPU in float64 -- test-only checker, never
on the product path -- from the same fp32 operands."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import encodec_oracle as O
from synth import synth_wave

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
B = 32


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _layer_walk(seq, C, Tn, batch=B):
    """(index, module, act, input shape) of every conv / residual block of a SEANet nn.Sequential
    (the encx stack folds each nn.ELU into the next conv: modules/seanet.py _run)."""
    from encx.modules.conv import SConv1d, SConvTranspose1d
    from encx.modules.seanet import SEANetResnetBlock
    from encx import ops
    out, act = [], None
    for i, m in enumerate(seq):
        if isinstance(m, nn.ELU):
            act = 'elu'
            continue
        if isinstance(m, SEANetResnetBlock):
            out.append((i, m, None, (batch, C, Tn)))
        elif isinstance(m, SConv1d):
            c = m.conv
            out.append((i, m, act, (batch, C, Tn)))
            Tn = ops.conv_geometry(Tn, c.kernel_size, c.stride, c.dilation, m.causal, m.pad_mode)[3]
            C = c.out_channels
        elif isinstance(m, SConvTranspose1d):
            c = m.convtr
            out.append((i, m, act, (batch, C, Tn)))
            Tn = ops.convtr_geometry(Tn, c.kernel_size, c.stride, m.causal, m.trim_right_ratio)[1]
            C = c.out_channels
        act = None
    return out


def _fp64_layer(m, x64, act):
    """The oracle's restatement of one layer on fp64 copies of the module's fp32 parameters."""
    from encx.modules.conv import SConv1d, SConvTranspose1d
    p = {'m.' + k: v.detach().double().requires_grad_(True) for k, v in m.named_parameters()}
    xin = F.elu(x64) if act == 'elu' else x64
    if isinstance(m, SConv1d):
        c = m.conv
        y = O.sconv1d(xin, p, 'm', c.kernel_size, c.stride, c.dilation, m.causal, m.pad_mode, c.norm_type)
    elif isinstance(m, SConvTranspose1d):
        c = m.convtr
        y = O.sconvtr1d(xin, p, 'm', c.kernel_size, c.stride, m.causal, m.trim_right_ratio, c.norm_type)
    else:
        c1 = m.block[1]
        hidden = c1.conv.out_channels
        dim = c1.conv.in_channels
        y = O.resblock(xin, p, 'm', dim, c1.conv.kernel_size, dim // hidden, c1.causal, c1.conv.norm_type)
    return y, p


@pytest.mark.parametrize('stack', ['encoder', 'decoder'])
def test_seanet_layers_b32_vs_fp64(stack):
    """Every Conv1d / ConvTranspose1d / residual block of the config-3 SEANet stack (24 kHz,
    causal, weight norm, the preceding ELU fused) at B 32 and its real length -- T 24000 down to
    75 -- through the encx module the model runs (the fused block kernels at T >= 2048, the
    linked convs with the shortcut-join and residual epilogue below): output, input grad and
    every parameter grad within 2e-5 of the fp64 restatement, relative to the tensor's largest
    magnitude (fp32 accumulation over up to 768 k positions per weight-grad element)."""
    from encx.model import EncodecModel
    from encx.modules.seanet import SEANetResnetBlock
    torch.manual_seed(11)
    model = EncodecModel._get_model([6.0], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=True)
    seq = getattr(model, stack).model
    # weight-norm gains away from ||v|| so the norm's scale and its grad are exercised
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for k, prm in seq.named_parameters():
            if k.endswith('weight_g'):
                prm.mul_(0.5 + torch.rand(prm.shape, generator=g))
    seq = seq.to(DEV)
    walk = _layer_walk(seq, 1, 24000) if stack == 'encoder' else _layer_walk(seq, 128, 75)
    assert len(walk) == 10, len(walk)
    bad = []
    for idx, m, act, shape in walk:
        torch.cuda.empty_cache()
        gen = torch.Generator(device=DEV).manual_seed(1000 + idx)
        x = torch.randn(shape, generator=gen, device=DEV).requires_grad_(True)
        for prm in m.parameters():
            prm.grad = None
        y = m(x) if isinstance(m, SEANetResnetBlock) else m(x, act=act)
        dy = torch.randn(y.shape, generator=gen, device=DEV)
        y.backward(dy)
        x64 = x.detach().double().requires_grad_(True)
        with torch.backends.cudnn.flags(enabled=False):
            y64, p64 = _fp64_layer(m, x64, act)
            y64.backward(dy.double())
        errs = {'y': _rel(y, y64), 'dx': _rel(x.grad, x64.grad)}
        for k, prm in m.named_parameters():
            errs['d' + k] = _rel(prm.grad, p64['m.' + k].grad)
        name = f'{stack}.model.{idx} {type(m).__name__} {tuple(shape)}'
        print(name + ': ' + ' '.join(f'{k} {e:.1e}' for k, e in errs.items()))
        bad += [(name, k, e) for k, e in errs.items() if not e < 2e-5]
        del x, y, dy, x64, y64, p64
    assert not bad, bad


@pytest.mark.parametrize('seg', [48000, 4800, 320])
@pytest.mark.parametrize('stack', ['encoder', 'decoder'])
def test_seanet_layers_48k_vs_fp64(stack, seg):
    """The config-5 SEANet stack (48 kHz stereo: non-causal, symmetric reflect padding,
    time_group_norm convs with plain weights) layer by layer at B 2 and the 1 s segment's lengths
    (48000 samples down to 150 frames; the 0.1 s segments of the g9 fixture's model; and its
    one-frame tail segment, whose decoder runs the linked convs at 160 and 320 samples): output, input grad and parameter grads within 2e-5 of the
    fp64 restatement, relative to the tensor's largest magnitude."""
    from encx.model import EncodecModel
    from encx.modules.seanet import SEANetResnetBlock
    torch.manual_seed(12)
    model = EncodecModel._get_model([24.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                    audio_normalize=True, segment=seg / 48000)
    seq = getattr(model, stack).model.to(DEV)
    walk = _layer_walk(seq, 2, seg, 2) if stack == 'encoder' else _layer_walk(seq, 128, seg // 320, 2)
    bad = []
    for idx, m, act, shape in walk:
        gen = torch.Generator(device=DEV).manual_seed(2000 + idx)
        x = torch.randn(shape, generator=gen, device=DEV).requires_grad_(True)
        for prm in m.parameters():
            prm.grad = None
        y = m(x) if isinstance(m, SEANetResnetBlock) else m(x, act=act)
        dy = torch.randn(y.shape, generator=gen, device=DEV)
        y.backward(dy)
        x64 = x.detach().double().requires_grad_(True)
        with torch.backends.cudnn.flags(enabled=False):
            y64, p64 = _fp64_layer(m, x64, act)
            y64.backward(dy.double())
        errs = {'y': _rel(y, y64), 'dx': _rel(x.grad, x64.grad)}
        for k, prm in m.named_parameters():
            errs['d' + k] = _rel(prm.grad, p64['m.' + k].grad)
        name = f'48k {stack}.model.{idx} {type(m).__name__} {tuple(shape)}'
        print(name + ': ' + ' '.join(f'{k} {e:.1e}' for k, e in errs.items()))
        bad += [(name, k, e) for k, e in errs.items() if not e < 2e-5]
    assert not bad, bad


def test_config3_b32_step_vs_oracle_fp64():
    """One config-3 Trainer step at its real size (B 32 x 1 s, n_q 8, the MS-STFT
    discriminator, all four losses through the balancer, both Adams) against the oracle's step
    from the same state, run on the GPU in fp64 and in fp32 (tests/steputil.check_step): every
    generator and discriminator weight grad within 4x the plain fp32 oracle's error, post-Adam
    parameters per element, the codebook EMA buffers, the losses, and the slope-mask /
    feature-sign audit. The second of two steps, so the balancer's averages and the Adam moments
    are warm. The balanced output grad is checked on its own and the generator backward from it
    (check_step isolate: the decoder's last bias grads sum 768 k output-grad elements)."""
    from encx.train import Trainer, DEFAULT_WEIGHTS
    from encx.msstftd import MultiScaleSTFTDiscriminator
    from fixtures import disc_state
    from steputil import check_step
    from test_gpu_model import build
    m, p, cbs, cfg = build((6.0,), True, 3, np.stack([np.zeros((2, 128)), np.full((2, 128), 0.05)], 1)
                           .astype(np.float32)[[0] * 8], 4, 8)
    disc = MultiScaleSTFTDiscriminator(filters=32)
    disc.load_state_dict(disc_state(5), strict=False)
    disc = disc.to(DEV)
    tr = Trainer(m, disc, lr=3e-4, disc_lr=3e-4, scheduler=False)
    x = torch.as_tensor(synth_wave((B, 1, 24000), 607)).to(DEV)
    tr.step(x)
    torch.cuda.synchronize()
    out, table = check_step(tr, x, cfg, 6.0, DEFAULT_WEIGHTS, device=DEV, isolate=True)
    assert any(r[0] == 'out_grad' for r in table)
    n_gen = sum(1 for r in table if r[0].startswith('gen:'))
    n_disc = sum(1 for r in table if r[0].startswith('disc:'))
    assert n_gen == sum(1 for q in m.parameters() if q.requires_grad), n_gen
    assert n_disc == sum(1 for q in disc.parameters() if q.requires_grad), n_disc
