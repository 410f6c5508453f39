"""CPU checks of the C-ABI boundary and the host layer (no GPU compute)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    from encx._lib import lib
    return lib.load()


def test_library_exports_every_header_symbol():
    from encx._lib import parse_header, LIB_PATH
    assert os.path.exists(LIB_PATH), 'build first: __graft_entry__.build()'
    sigs = parse_header()
    src = open(os.path.join(ROOT, 'include', 'encx.h')).read()
    declared = set(re.findall(r'\b(encx_\w+)\s*\(', re.sub(r'/\*.*?\*/', '', src, flags=re.S)))
    assert declared == set(sigs), declared ^ set(sigs)
    lib = ctypes.CDLL(LIB_PATH)
    missing = [n for n in sigs if not hasattr(lib, n)]
    assert not missing, missing
    assert len(sigs) >= 40


def test_library_build_id_matches_sources():
    """The library carries the hash of the sources it was built from; a stale library is
    refused at load (encx._lib.check_build_id)."""
    from encx import _lib as L
    from buildid import build_id
    lib = _lib()
    assert lib.encx_build_id().decode() == build_id()

    class Stale:
        def encx_build_id(self):
            return b'0' * 32
    env = os.environ.pop('ENCX_LIB', None)
    try:
        with pytest.raises(RuntimeError, match='built from other sources'):
            L.check_build_id(Stale())
    finally:
        if env is not None:
            os.environ['ENCX_LIB'] = env


def test_kernel_options_settable_in_process():
    """encx_set_option / encx_get_option: every kernel-selection option is readable, settable
    (with or without the ENCX_ prefix) and restorable; unknown names are refused."""
    from encx import _lib as L
    opts = L.options()
    assert {'FFT', 'LSTM_FUSE', 'PW', 'FWR', 'DGR', 'WGR'} <= set(opts)
    assert opts['FFT'] == int(os.environ.get('ENCX_FFT', 1))
    with L.option(DGR=7, LSTM_FUSE=1):
        assert L.get_option('DGR') == 7 and L.get_option('ENCX_LSTM_FUSE') == 1
    assert L.options() == opts
    lib = _lib()
    assert lib.encx_set_option(b'NO_SUCH_OPTION', 1, None) == 9001
    assert lib.encx_option_name(lib.encx_option_count()) is None


def test_host_only_queries():
    lib = _lib()
    assert lib.encx_version() == 1
    assert b'invalid' in lib.encx_strerror(9001)
    assert lib.encx_mel_frames(24000, 2048) == 46
    assert lib.encx_mel_frames(24000, 32) == 3000
    assert lib.encx_rvq_apply_parts(32, 128, 75) == 1024
    assert lib.encx_conv1d_bwd_weight_workspace(32, 32, 16, 24000, 3) > 0
    assert lib.encx_mel_tables_floats(32, 64) == 32 * 34 + 2 * 17 * 64 + 2 * 64 + 2 * 17
    # argument validation happens before any device call
    assert lib.encx_conv1d_fwd(*([None] * 6 + [0] * 12 + [None])) == 9001


def test_ops_refuse_cpu_tensors():
    from encx import ops
    x = torch.zeros(1, 1, 100)
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        ops.normalize(x)


def test_geometry_matches_oracle():
    from encx import ops
    from oracle import encodec_oracle as O
    for T in (5, 30, 97, 480, 4800, 24000):
        for K, s in ((7, 1), (3, 1), (1, 1), (4, 2), (8, 4), (10, 5), (16, 8)):
            for causal in (True, False):
                pl, pr, e, tout = ops.conv_geometry(T, K, s, 1, causal)
                assert (pl, pr) == O.conv_padding(T, K, s, 1, causal)
                x = torch.zeros(1, 1, T)
                xp = O.pad1d(x, (pl, pr), 'reflect') if max(pl, pr) < T + e else None
                if xp is not None:
                    assert xp.shape[-1] == pl + T + pr
                    assert tout == (xp.shape[-1] - K) // s + 1


def test_state_dict_keys_and_count_match_reference():
    from encx.model import EncodecModel
    d = np.load(os.path.join(ROOT, 'tests', 'golden', 'g7_step.npz'))
    keys = {k[6:] for k in d.files if k.startswith('gen/p/')}
    m = EncodecModel._get_model([1.5], 24000, 1, causal=True, model_norm='weight_norm', audio_normalize=True)
    assert set(m.state_dict()) == keys
    m = EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True, model_norm='weight_norm')
    assert sum(p.numel() for p in m.parameters()) == 14851810


def test_product_mel_filterbank_matches_fixture():
    from encx.audio_to_mel import mel_filterbank
    d = np.load(os.path.join(ROOT, 'tests', 'golden', 'g4_mel.npz'))
    for i in range(5, 12):
        n = 2 ** i
        np.testing.assert_array_equal(mel_filterbank(24000, n, 64), d[f'melbasis{n}'])


def test_scheduler_matches_fixture():
    from encx.scheduler import WarmupCosineLrScheduler
    d = np.load(os.path.join(ROOT, 'tests', 'golden', 'g8_sched.npz'))
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=3e-4)
    s = WarmupCosineLrScheduler(opt, max_iter=400, eta_ratio=0.1, warmup_iter=50, warmup_ratio=1e-4)
    lrs = []
    for _ in range(400):
        lrs.append(opt.param_groups[0]['lr'])
        opt.step()
        s.step()
    np.testing.assert_allclose(lrs, d['lr'], rtol=1e-12)


def test_bandwidth_rule():
    from encx.quantization import ResidualVectorQuantizer
    q = ResidualVectorQuantizer(dimension=128, n_q=32, bins=1024)
    assert [q.get_num_quantizers_for_bandwidth(75, b) for b in (1.5, 3., 6., 12., 24.)] == [2, 4, 8, 16, 32]


def test_flat_adam_state_dict_is_torch_adam_layout():
    """FlatAdam.state_dict / load_state_dict interchange with torch.optim.Adam (the reference's
    optimizer_state_dict, train_multi_gpu.py:303-308). Host logic only: no step is taken."""
    import torch
    from encx.optim import FlatAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(3, 4)), torch.nn.Parameter(torch.randn(5))]
    opt = FlatAdam(ps, lr=3e-4, betas=(0.5, 0.9))
    assert opt.state_dict()['state'] == {}
    opt.exp_avg.copy_(torch.randn(17))
    opt.exp_avg_sq.copy_(torch.rand(17))
    opt.n_step = 7
    sd = opt.state_dict()
    ref = torch.optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1.0, betas=(0.5, 0.9))
    ref.load_state_dict(sd)
    rsd = ref.state_dict()
    assert set(rsd['param_groups'][0]) >= {'lr', 'betas', 'eps', 'weight_decay', 'amsgrad', 'params'}
    assert rsd['param_groups'][0]['lr'] == 3e-4
    assert torch.equal(rsd['state'][1]['exp_avg'], opt.exp_avg[12:].view(5))
    assert torch.equal(rsd['state'][0]['exp_avg_sq'], opt.exp_avg_sq[:12].view(3, 4))
    assert float(rsd['state'][0]['step']) == 7.0
    # and back: a torch Adam state dict restores FlatAdam's flat moments and step
    opt2 = FlatAdam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1.0, betas=(0.5, 0.9))
    opt2.load_state_dict(rsd)
    assert opt2.n_step == 7 and opt2.param_groups[0]['lr'] == 3e-4
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
