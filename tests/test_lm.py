"""LM entropy coding (quantization/ac.py, modules/transformer.py,
model.py:27-65, compress.py use_lm=True).

CPU: the host layer (state-dict keys, argument checks, capacity queries). GPU, through the C
ABI: the quantized cdf and the arithmetic coder bit-exact against the reference-generated g12
fixture; the LM's probabilities against the fixture and the oracle (tolerance below); the
one-pass encoder and the step-by-step decoder bit-identical; compress / decompress round trips.

Tolerance: LM probabilities within rtol 2e-4 / atol 1e-6 of the reference's (fp32 attention,
LayerNorm and softmax in another reduction order). Everything integer -- cdfs, coding
intervals, coded bytes, decoded codes -- is bit-exact given the same probabilities. Bytes of
OUR LM coded stream are not compared with the reference's: they depend on the probabilities
bit for bit (ac.py:29-30, 220-224), which no two implementations share; the reference's own
stream is decoded instead from the reference's cdfs.
"""
import io

import numpy as np
import pytest
import torch

from fixtures import load, T, g12_ac_rows, g12_lm_config

DEV = 'cuda:0'


def _lm(name, device=DEV):
    from encx.lm import LMModel
    cfg, st = g12_lm_config(name)
    lm = LMModel(cfg.n_q, cfg.card, dim=cfg.dim, num_heads=cfg.num_heads, num_layers=cfg.num_layers,
                 past_context=cfg.past_context)
    lm.load_state_dict(st)
    return lm.to(device).eval(), cfg, st


# ----------------------------------------------------------------------------- CPU
def test_lm_state_dict_keys_match_reference_layout():
    from encx.lm import LMModel
    from oracle.lm_oracle import LMConfig, lm_param_shapes
    lm = LMModel(32, 1024, dim=200, num_layers=5, past_context=262)
    shapes = lm_param_shapes(LMConfig())
    sd = lm.state_dict()
    assert set(sd) == set(shapes)
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in shapes.items())


def test_lm_host_checks():
    from encx._lib import lib
    from encx.lm import LMModel
    with pytest.raises(NotImplementedError):
        LMModel(4, 64, dim=64, num_heads=4, gelu=False)
    lib.load()
    assert lib.encx_ac_encode_capacity(100, 24) >= 100 * 24 // 8
    assert lib.encx_ac_encode_capacity(-1, 24) == -1
    assert lib.encx_lm_layer_workspace(10, 200, 800) == 10 * (5 * 200 + 800) * 4
    # argument validation happens before any device call
    assert lib.encx_ac_cdf(None, 1, 1024, 1024, 10, 1e-8, 2, None, None, None) == 9001   # alpha > 1
    assert lib.encx_lm_layer(*([None] * 2 + [1, 1, None, 4, 0, None, 0, 200, 7, 800] + [None] * 14)) == 9001
    lm = LMModel(4, 64, dim=64, num_heads=4, num_layers=1)
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        lm(torch.zeros(1, 4, 1, dtype=torch.long))


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_quantized_cdf_matches_reference():
    from encx import ac
    from encx._lib import call, stream
    d = load('g12_lm.npz')
    for card, bits, pdf, cdf, sym, data, eof in g12_ac_rows(d):
        for p, c in zip(pdf[:8], cdf[:8]):     # the mirror, one row at a time
            got = ac.build_stable_quantized_cdf(T(p).to(DEV), bits, check=False)
            assert got.dtype == torch.int64
            np.testing.assert_array_equal(got.cpu().numpy(), c)
        # every row of the case in one launch
        P = T(pdf).to(DEV).contiguous()
        out = torch.empty(P.shape, dtype=torch.int32, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        call('encx_ac_cdf', P.data_ptr(), P.shape[0], card, card, bits, 1e-8, 2, out.data_ptr(),
             err.data_ptr(), stream())
        np.testing.assert_array_equal(out.cpu().numpy(), cdf)
        assert int(err.item()) == 0
    o = 0
    for card, bits in zip(d['ac_over_card'], d['ac_over_bits']):
        p, c = d['ac_over_pdf'][o:o + card], d['ac_over_cdf'][o:o + card]
        o += card
        got = ac.build_stable_quantized_cdf(T(p).to(DEV), int(bits), check=False)
        np.testing.assert_array_equal(got.cpu().numpy(), c)
        with pytest.raises(AssertionError):
            ac.build_stable_quantized_cdf(T(p).to(DEV), int(bits), check=True)
    with pytest.raises(AssertionError):
        ac.build_stable_quantized_cdf(torch.full((1024,), 1 / 1024, device=DEV), 10)


def straddle_stream(bits=24, rounds=6, seed=0):
    """Symbols + per-step cdfs that keep the coder's interval straddling the bit-max_bit boundary
    B = 2^max_bit for as long as ac.py:157 allows (each straddling push picks a 2m+1-wide symbol
    around B, so nothing flushes and max_bit grows by ~bits - log2(2m+1) per push), then resolve
    it with the symbol just below B, which flushes the whole carried prefix at once. Returns
    (symbols, cdfs, the largest max_bit reached before a flush). Big-int arithmetic, as ac.py's."""
    g = np.random.default_rng(seed)
    R = 1 << bits
    low = high = 0
    max_bit = -1
    syms, cdfs, peak = [], [], -1
    for _ in range(rounds):
        straddle = True
        while True:
            lo, hi, mb = low, high, max_bit
            while hi - lo + 1 < R:
                lo, hi, mb = 2 * lo, 2 * hi + 1, mb + 1
            delta = hi - lo + 1
            B = 1 << mb
            m = int(g.integers(2, 6))
            if straddle and lo < B <= hi:
                t = ((B - lo) * R) // delta
                rl, rh = max(1, t - m), min(R - 2, t + m)
                cdf = [rl, rh + 1, R]
                el = -((-rl * delta) // R)
                eh = (rh * delta) // R
                nlo, nhi = lo + el, lo + eh
                # keep straddling while the push leaves max_bit <= 61 (nothing flushes: ac.py:157)
                if nlo < B <= nhi and mb <= 61:
                    syms.append(1)
                    cdfs.append(cdf)
                    low, high, max_bit = nlo, nhi, mb
                    peak = max(peak, mb)
                    continue
            # resolve: the symbol whose interval ends just below B (or a random one if none)
            t = ((B - lo) * R) // delta if lo < B <= hi else R // 2
            cut = max(2, min(R - 2, t - 1))
            cdf = [cut, R]
            el, eh = 0, ((cut - 1) * delta) // R
            low, high = lo + el, lo + eh
            max_bit = mb
            peak = max(peak, mb)
            syms.append(0)
            cdfs.append(cdf)
            while max_bit >= 0 and (low >> max_bit) == (high >> max_bit):
                b = low >> max_bit
                low -= b << max_bit
                high -= b << max_bit
                max_bit -= 1
            assert max_bit <= 61
            break
    return syms, [np.array(c, np.int32) for c in cdfs], peak


def test_ac_oracle_long_straddle():
    """The crafted stream carries more than 64 undecided bits through a push (the reference's
    Python ints hold them; a 64-bit coder state would overflow) and round-trips in the oracle."""
    from oracle import ac_oracle as A
    syms, cdfs, peak = straddle_stream()
    assert peak > 64, peak
    data = A.encode(syms, cdfs, 24)
    assert A.decode(data, cdfs, 24) == syms


@pytest.mark.gpu
def test_gpu_ac_long_straddle_matches_oracle():
    """encx_ac_encode / encx_ac_decode on the long-straddle stream: bytes and symbols equal the
    big-int oracle's (the coder state is 128 bits wide)."""
    from oracle import ac_oracle as A
    from encx import ac
    for seed in range(3):
        syms, cdfs, peak = straddle_stream(seed=seed)
        want = A.encode(syms, cdfs, 24)
        fo = io.BytesIO()
        enc = ac.ArithmeticCoder(fo, total_range_bits=24)
        dc = [torch.from_numpy(c).to(DEV) for c in cdfs]
        for sy, c in zip(syms, dc):
            enc.push(sy, c)
        enc.flush()
        assert fo.getvalue() == want, (seed, peak)
        dec = ac.ArithmeticDecoder(io.BytesIO(want), total_range_bits=24)
        assert [dec.pull(c) for c in dc] == syms


@pytest.mark.gpu
def test_gpu_arithmetic_coder_matches_reference_bytes():
    from encx import ac
    d = load('g12_lm.npz')
    for card, bits, pdf, cdf, sym, data, eof in g12_ac_rows(d):
        fo = io.BytesIO()
        enc = ac.ArithmeticCoder(fo, total_range_bits=bits)
        cdfs = [T(c).to(DEV) for c in cdf]
        for s, c in zip(sym.tolist(), cdfs):
            enc.push(s, c)
        enc.flush()
        assert fo.getvalue() == data, (card, bits)
        fo = io.BytesIO(data + b'trailing')
        dec = ac.ArithmeticDecoder(fo, total_range_bits=bits)
        assert [dec.pull(c) for c in cdfs] == sym.tolist()
        assert fo.tell() == len(data)                  # where BitUnpacker(bits=1) stopped
        if eof == 1:
            dec = ac.ArithmeticDecoder(io.BytesIO(data), total_range_bits=bits)
            for c in cdfs:
                dec.pull(c)
            assert dec.pull(torch.zeros(1, device=DEV)) is None
        else:
            with pytest.raises(RuntimeError, match='Binary search failed'):
                dec.pull(torch.zeros(1, device=DEV))
    # a cdf whose total exceeds 2^bits: the reference's coder asserts (ac.py:116)
    o0 = int(d['ac_over_card'][0])
    c = T(d['ac_over_cdf'][:o0]).to(DEV)
    enc = ac.ArithmeticCoder(io.BytesIO(), 24)
    enc.push(o0 - 1, c)
    with pytest.raises(AssertionError):
        enc.flush()


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['a', 'b'])
def test_gpu_lm_streaming_probs_match_reference(name):
    """lm(input_, states, offset) step by step, as compress.py:76-78 calls it, against the
    reference's probabilities; the one-pass form bit-identical to the steps."""
    lm, cfg, _ = _lm(name)
    d = load('g12_lm.npz')
    codes = T(d[f'lm_{name}/codes']).to(DEV)
    ref = d[f'lm_{name}/probs']                         # [B][T][K][card]
    B, K, Tn = codes.shape
    states, offset = None, 0
    inp = torch.zeros(B, K, 1, dtype=torch.long, device=DEV)
    steps = []
    for t in range(Tn):
        p, states, offset = lm(inp, states, offset)
        assert p.shape == (B, cfg.card, K, 1)
        inp = (1 + codes[:, :, t:t + 1]).contiguous()
        steps.append(p[:, :, :, 0].permute(0, 2, 1))
    got = torch.stack(steps, 1).cpu()
    np.testing.assert_allclose(got.numpy(), ref, rtol=2e-4, atol=1e-6)
    # all T steps in one call (teacher-forced inputs) == the steps, bit for bit
    full = torch.zeros_like(codes)
    full[:, :, 1:] = codes[:, :, :-1] + 1
    p_all, _, off = lm(full)
    assert off == Tn
    assert torch.equal(p_all.permute(0, 3, 2, 1).cpu(), got)


@pytest.mark.gpu
def test_gpu_lm_window_truncation_vs_oracle():
    """past_context = 262 at T = 300 (the 24 kHz LM's 3.5 s window closes within the
    sequence): one pass against the oracle's, and the last steps streamed bit-identically."""
    from oracle import lm_oracle as L
    lm, cfg, st = _lm('a')
    g = np.random.default_rng(5)
    B, K, Tn = 2, 4, 300
    codes = torch.from_numpy(g.integers(0, 1024, size=(B, K, Tn))).to(DEV)
    full = torch.zeros_like(codes)
    full[:, :, 1:] = codes[:, :, :-1] + 1
    p_all, _, _ = lm(full)
    ref = L.lm_all(st, codes.cpu(), cfg)
    np.testing.assert_allclose(p_all.cpu().numpy(), ref.numpy(), rtol=2e-4, atol=1e-6)
    # stream: 295 steps in one call, then 5 single steps
    p0, states, off = lm(full[:, :, :295].contiguous())
    for t in range(295, 300):
        p1, states, off = lm(full[:, :, t:t + 1].contiguous(), states, off)
        assert torch.equal(p1[..., 0], p_all[..., t])
    assert torch.equal(p0, p_all[..., :295])


@pytest.mark.gpu
def test_gpu_lm_coder_round_trip_and_oracle_bytes():
    """encode_streams (one pass + one coder thread per stream) -> decode_streams (step by step)
    gives back every code of 3 streams; the GPU cdfs equal the oracle's build of the GPU
    probabilities, and the oracle coder over them reproduces the GPU bytes."""
    from oracle import ac_oracle as A
    lm, cfg, _ = _lm('a')
    g = np.random.default_rng(7)
    B, K, Tn = 3, 8, 40
    codes = torch.from_numpy(g.integers(0, 1024, size=(B, K, Tn))).to(DEV)
    codes[1] = codes[0]                     # two identical streams code identically
    datas = lm.encode_streams(codes)
    assert datas[0] == datas[1] and datas[0] != datas[2]
    back, used = lm.decode_streams(datas, K, Tn)              # HIP-graph replayed steps
    assert torch.equal(back, codes)
    assert used == [len(x) for x in datas]
    back_e, used_e = lm.decode_streams(datas, K, Tn, graph=False)   # eager steps
    assert torch.equal(back_e, codes) and used_e == used
    # the integer path against the oracle, on the GPU's own probabilities
    full = torch.zeros_like(codes)
    full[:, :, 1:] = codes[:, :, :-1] + 1
    x = lm._body(full, full.stride(), B, K, Tn, False, lm.new_state(B, Tn + 1))
    probas = torch.empty(B, Tn, K, cfg.card, device=DEV)
    cdf = torch.empty(B, Tn, K, cfg.card, device=DEV, dtype=torch.int32)
    lm._heads(x, B, Tn, K, probas=probas, cdf=cdf)
    probas, cdf = probas.cpu().numpy(), cdf.cpu().numpy().astype(np.int64)
    for b in range(B):
        rows = [(b, t, k) for t in range(Tn) for k in range(K)]
        for (bb, t, k) in rows[::37]:
            np.testing.assert_array_equal(A.quantized_cdf(probas[bb, t, k], 24, check=False), cdf[bb, t, k])
        syms = [int(codes[b, k, t]) for (_, t, k) in rows]
        assert A.encode(syms, [cdf[b, t, k] for (_, t, k) in rows]) == datas[b]
    # a truncated stream: the decoder runs dry (EOFError, compress.py:147-148)
    with pytest.raises(EOFError):
        lm.decode_streams([datas[0][:len(datas[0]) // 2]], K, Tn)


@pytest.mark.gpu
def test_gpu_compress_use_lm_fixture():
    """compress(use_lm=True) / decompress with the g12 LM on the g1 model (1.5 kbps): header as
    the reference's, codes and wave identical to the use_lm=False path; the reference's own
    LM-coded stream decodes (from the reference's cdfs) to the reference's codes; our LM's
    probabilities for those codes match the reference's pdfs."""
    from test_ecdc import _model24
    from encx import compress as C, ac
    from oracle import ecdc_oracle as E
    d = load('g12_lm.npz')
    m, _ = _model24()
    lm, cfg, _ = _lm('a')
    m.set_lm_model(lm)
    x = T(d['e2e_x'])
    ref = d['e2e_bytes'].tobytes()
    mine = C.compress(m, x, use_lm=True)
    meta, off = E.parse_header(mine)
    rmeta, roff = E.parse_header(ref)
    assert meta == rmeta and mine[:off] == ref[:roff]
    plain = C.compress(m, x, use_lm=False)
    _, frames = E.decompress_codes(plain, 10, 1, False)
    y_lm, sr = C.decompress(m, mine)
    y_plain, _ = C.decompress(m, plain)
    assert sr == 24000 and torch.equal(y_lm, y_plain)
    # our codes = the reference's where fp32 encoders agree (fp64-certified elsewhere, g1 tests)
    assert (frames[0][0] == d['e2e_codes'][0]).mean() > 0.95
    # the reference's LM-coded payload, decoded on the GPU from the reference's cdfs
    dec = ac.ArithmeticDecoder(io.BytesIO(ref[roff:]))
    K, Tn = d['e2e_codes'].shape[1:]
    cdfs = T(d['e2e_cdf']).to(DEV)
    got = [dec.pull(cdfs[i]) for i in range(K * Tn)]
    assert got == d['e2e_codes'][0].T.reshape(-1).tolist()
    # our LM on the reference's codes against the reference's pdfs
    codes = T(d['e2e_codes']).to(DEV)
    full = torch.zeros_like(codes)
    full[:, :, 1:] = codes[:, :, :-1] + 1
    p, _, _ = lm(full)
    np.testing.assert_allclose(p[0].permute(2, 1, 0).reshape(-1, cfg.card).cpu().numpy(), d['e2e_pdf'],
                               rtol=2e-4, atol=1e-6)


@pytest.mark.gpu
def test_gpu_compress_use_lm_48k_segments():
    """48 kHz stereo, normalised, 0.1 s segments (the g9/g10 model, n_q 2), use_lm=True: every
    segment is its own scale + arithmetic coded stream (compress.py:67-89) and the decoder stops
    where the reference's does, so the next segment's scale is read from the right offset; the
    decoded wave equals the use_lm=False one bit for bit. Two segments hit the reference's
    short-last-segment quirk (every segment decoded with the first's frame count,
    compress.py:126): the decoder runs dry -> EOFError, as for use_lm=False."""
    from test_ecdc import _model48
    from encx import compress as C
    from encx.lm import LMModel
    from oracle.lm_oracle import LMConfig, lm_param_shapes
    from synth import synth_lm_state
    m = _model48()
    cfg = LMConfig(n_q=m.quantizer.n_q, past_context=int(3.5 * m.frame_rate))
    lm = LMModel(cfg.n_q, 1024, dim=200, num_layers=5, past_context=cfg.past_context)
    lm.load_state_dict({k: T(v) for k, v in synth_lm_state(lm_param_shapes(cfg), 131).items()})
    m.set_lm_model(lm.to(DEV).eval())
    d = load('g10_ecdc.npz')
    w = T(d['c48_x'])
    one = C.compress(m, w[:, :4752], use_lm=True)
    y_lm, _ = C.decompress(m, one)
    y_plain, _ = C.decompress(m, C.compress(m, w[:, :4752], use_lm=False))
    assert torch.equal(y_lm, y_plain)
    two = C.compress(m, w, use_lm=True)
    with pytest.raises(EOFError):
        C.decompress(m, two)
    # the same two segments, each decoded with its own length: the first stream ends exactly
    # where the second segment's scale begins
    import io as _io
    from encx import binary
    fo = _io.BytesIO(two)
    meta = binary.read_ecdc_header(fo)
    K = meta['nc']
    lengths = [f.shape[-1] for f, _ in m.encode(w[None].to(DEV))]
    codes = []
    for Tn in lengths:
        fo.read(4)                                   # the segment's '!f' scale
        start = fo.tell()
        c, used = lm.decode_streams([fo.read()], K, Tn)
        fo.seek(start + used[0])
        codes.append(c)
    assert fo.tell() == len(two)
    ref = [f for f, _ in m.encode(w[None].to(DEV))]
    for a, b in zip(codes, ref):
        assert torch.equal(a, b)
