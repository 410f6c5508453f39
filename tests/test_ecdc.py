"""`.ecdc` bitstream: the oracle against the reference-generated g10
fixture (CPU), and the HIP pack/unpack kernels, BitPacker/BitUnpacker and
compress()/decompress() against the oracle and the fixture (GPU, through the C ABI)."""
import io
import struct

import numpy as np
import pytest
import torch

from oracle import ecdc_oracle as E
from fixtures import load, T, codebooks_from_stats

DEV = 'cuda:0'


def bp_cases():
    d = load('g10_ecdc.npz')
    toks = np.split(d['bp_tokens'], np.cumsum(d['bp_cases'][:, 1])[:-1])
    byts = np.split(d['bp_bytes'], np.cumsum(d['bp_nbytes'])[:-1])
    return [(int(b), tok, by.tobytes(), int(gh))
            for (b, _), tok, by, gh in zip(d['bp_cases'], toks, byts, d['bp_ghosts'])]


def rel(a, b):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


# ------------------------------------------------------------------------------ CPU: oracle
def test_oracle_bitpack_matches_reference_vectors():
    for bits, tok, ref, ghosts in bp_cases():
        assert E.bitpack(tok, bits) == ref, (bits, len(tok))
        back = E.bitunpack(ref, bits)
        assert len(back) - len(tok) == ghosts           # flush ghosts (binary.py:144-146)
        np.testing.assert_array_equal(back[:len(tok)], tok)
        if len(ref):
            with pytest.raises(EOFError):
                E.bitunpack(ref[:-1], bits, len(tok))


def test_oracle_header_and_compress_bytes_match_reference():
    d = load('g10_ecdc.npz')
    meta = {'m': 'encodec_24khz', 'al': 24000, 'nc': 2, 'lm': False, 'fr': 75}
    assert E.header_bytes(meta) == d['header'].tobytes()
    assert E.parse_header(d['header'].tobytes()) == (meta, len(d['header']))
    codes = load('g1_eval24k.npz')['codes'].astype(np.int64)[0]     # [K=2][T=75]
    assert E.compress_bytes('encodec_24khz', 24000, [(codes, None)], 10) == d['c24_bytes'].tobytes()
    # 48 kHz, one normalised segment: scale + codes
    b48 = d['c48_bytes'].tobytes()
    meta48, frames = E.decompress_codes(b48, 10, 1, True)
    assert meta48 == {'m': 'encodec_48khz', 'al': 4752, 'nc': 2, 'lm': False, 'fr': 15}
    np.testing.assert_array_equal(frames[0][0], d['c48_codes'][0])
    assert E.compress_bytes('encodec_48khz', 4752, frames, 10) == b48
    # two segments (4800 + 48 samples): the short one is read with fr = 15 frames -> EOF
    assert int(d['c48s_eof']) == 1
    with pytest.raises(EOFError):
        E.decompress_codes(d['c48s_bytes'].tobytes(), 10, 2, True)


def test_product_header_io_matches_reference():
    """encx.binary's header writer/reader (host bytes, no GPU) against the fixture."""
    from encx import binary
    d = load('g10_ecdc.npz')
    meta = {'m': 'encodec_24khz', 'al': 24000, 'nc': 2, 'lm': False, 'fr': 75}
    fo = io.BytesIO()
    binary.write_ecdc_header(fo, meta)
    assert fo.getvalue() == d['header'].tobytes()
    fo.seek(0)
    assert binary.read_ecdc_header(fo) == meta
    with pytest.raises(ValueError):
        binary.read_ecdc_header(io.BytesIO(b'XXXX' + fo.getvalue()[4:]))
    with pytest.raises(ValueError):
        binary.read_ecdc_header(io.BytesIO(fo.getvalue()[:4] + b'\x01' + fo.getvalue()[5:]))
    with pytest.raises(EOFError):
        binary.read_ecdc_header(io.BytesIO(fo.getvalue()[:20]))


def test_pack_refuses_cpu_tensors():
    from encx import ops
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        ops.pack_codes(torch.zeros(1, 2, 3, dtype=torch.int64), 10)
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        ops.unpack_codes(torch.zeros(1, 4, dtype=torch.uint8), 1, 3, 10)


def test_bitpack_bytes_query():
    from encx._lib import lib
    assert lib.encx_bitpack_bytes(600, 10) == 750
    assert lib.encx_bitpack_bytes(0, 10) == 0
    assert lib.encx_bitpack_bytes(13, 1) == 2
    assert lib.encx_bitpack_bytes(5, 0) == -1 and lib.encx_bitpack_bytes(5, 33) == -1


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_pack_unpack_reference_vectors():
    from encx import ops
    for bits, tok, ref, _ in bp_cases():
        codes = torch.from_numpy(tok).to(DEV).view(1, 1, -1)
        data, err = ops.pack_codes(codes, bits)
        assert int(err.item()) == 0
        assert data.cpu().numpy().tobytes() == ref, (bits, len(tok))
        if len(tok):
            back = ops.unpack_codes(data, 1, len(tok), bits)
            np.testing.assert_array_equal(back.cpu().numpy().reshape(-1), tok)


@pytest.mark.gpu
@pytest.mark.parametrize('bits', [1, 3, 8, 10, 13, 16, 24, 32])
def test_gpu_pack_strided_frames_vs_oracle(bits):
    """Several frames in one launch from the transposed view EncodecModel.encode returns
    ([n_q][F][T] storage seen as [F][K][T]); ragged T; unpack back to [F][K][T]."""
    from encx import ops
    g = np.random.default_rng(bits)
    for F, K, Tn in [(5, 8, 75), (3, 2, 1), (1, 32, 150), (7, 3, 13)]:
        base = torch.from_numpy(g.integers(0, 1 << bits, size=(K, F, Tn), dtype=np.int64)).to(DEV)
        codes = base.transpose(0, 1)
        data, err = ops.pack_codes(codes, bits)
        assert int(err.item()) == 0
        host = codes.cpu().numpy()
        for f in range(F):
            assert data[f].cpu().numpy().tobytes() == E.bitpack(host[f].T.reshape(-1), bits)
        back = ops.unpack_codes(data, K, Tn, bits)
        assert torch.equal(back, codes)


@pytest.mark.gpu
def test_gpu_pack_full_batch_roundtrip_and_range_check():
    """bench size: 32 clips x n_q 8 x 75 frames (and 32 x 32 x 750), round trip bit-exact;
    a code >= 2^bits raises instead of corrupting its neighbours."""
    from encx import ops
    g = torch.Generator(device=DEV).manual_seed(5)
    for F, K, Tn in [(32, 8, 75), (32, 32, 750)]:
        codes = torch.randint(0, 1024, (F, K, Tn), device=DEV, generator=g)
        data, err = ops.pack_codes(codes, 10)
        assert data.shape == (F, (K * Tn * 10 + 7) // 8) and int(err.item()) == 0
        assert torch.equal(ops.unpack_codes(data, K, Tn, 10), codes)
    codes[3, 1, 7] = 1024
    _, err = ops.pack_codes(codes, 10)
    assert int(err.item()) == 1


@pytest.mark.gpu
def test_gpu_bitpacker_stream_api():
    from encx import binary
    for bits, tok, ref, ghosts in bp_cases()[:6]:
        fo = io.BytesIO()
        pk = binary.BitPacker(bits, fo, device=DEV)
        for v in tok.tolist():
            pk.push(v)
        pk.flush()
        assert fo.getvalue() == ref
        fo.seek(0)
        up = binary.BitUnpacker(bits, fo, device=DEV)
        pulled = []
        while (v := up.pull()) is not None:
            pulled.append(v)
        assert pulled[:len(tok)] == tok.tolist() and len(pulled) - len(tok) <= 8 // bits
        fo.seek(0)
        if len(tok):
            fr = binary.BitUnpacker(bits, fo, device=DEV).pull_frame(1, len(tok))
            np.testing.assert_array_equal(fr.cpu().numpy()[0], tok)


def _model24():
    from encx.model import EncodecModel
    from oracle import encodec_oracle as O
    from fixtures import model_state
    d = load('g1_eval24k.npz')
    m = EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True, model_norm='weight_norm',
                                audio_normalize=False, name='encodec_24khz')
    cfg = O.Config(target_bandwidths=(1.5, 3., 6., 12., 24.), audio_normalize=False)
    sd = dict(model_state(cfg, 1))
    for i, cb in enumerate(codebooks_from_stats(d['stats'], 77, 2, cfg.n_q)):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m.eval()
    m.set_target_bandwidth(1.5)
    return m.to(DEV), d


def _model48():
    from encx.model import EncodecModel
    from fixtures import model_state, cfg48k
    d9 = load('g9_step48k.npz')
    cfg = cfg48k()
    m = EncodecModel._get_model([3.0], 48000, 2, causal=False, model_norm='time_group_norm',
                                audio_normalize=True, segment=0.1, name='encodec_48khz')
    sd = dict(model_state(cfg, 91))
    for i, cb in enumerate(codebooks_from_stats(d9['gen/stats'], 93, 2, cfg.n_q)):
        for k, v in cb.items():
            sd[f'quantizer.vq.layers.{i}._codebook.{k}'] = v
    m.load_state_dict(sd)
    m.eval()
    m.set_target_bandwidth(3.0)
    return m.to(DEV)


@pytest.mark.gpu
def test_gpu_compress_decompress_24k_fixture():
    from encx import compress as C
    m, d1 = _model24()
    d = load('g10_ecdc.npz')
    x = T(d1['x'])[0]
    mine = C.compress(m, x, use_lm=False)
    meta, frames = E.decompress_codes(mine, 10, 1, False)
    ref_codes = d1['codes'].astype(np.int64)[0]
    if (frames[0][0] == ref_codes).all():
        assert mine == d['c24_bytes'].tobytes()
    else:  # a code may differ only where the fp64 top-2 gap is below fp32 rounding
        assert (frames[0][0] != ref_codes).mean() < 0.02
    y, sr = C.decompress(m, d['c24_bytes'].tobytes())
    assert sr == 24000 and y.shape == (1, 24000) and not y.is_cuda
    assert rel(y, d['c24_y']) < 1e-3, rel(y, d['c24_y'])
    m.name = 'unset'
    with pytest.raises(ValueError):
        C.compress(m, x)


@pytest.mark.gpu
def test_gpu_compress_decompress_48k_fixture():
    from encx import compress as C
    m = _model48()
    d = load('g10_ecdc.npz')
    w = T(d['c48_x'])
    mine = C.compress(m, w[:, :4752])
    ref = d['c48_bytes'].tobytes()
    _, fm = E.decompress_codes(mine, 10, 1, True)
    _, fr = E.decompress_codes(ref, 10, 1, True)
    np.testing.assert_array_equal(fm[0][0], fr[0][0])
    assert abs(fm[0][1] - fr[0][1]) <= 1e-6 * abs(fr[0][1])
    hdr = E.parse_header(ref)[1]
    assert mine[:hdr] == ref[:hdr] and mine[hdr + 4:] == ref[hdr + 4:]   # all but the fp32 scale
    y, _ = C.decompress(m, ref)
    assert y.shape == (2, 4752)
    assert rel(y, d['c48_y']) < 1e-3, rel(y, d['c48_y'])
    # two segments: both ends of the reference quirk (compress.py:126) -> EOFError
    mine_s = C.compress(m, w)
    assert len(mine_s) == len(d['c48s_bytes'])
    with pytest.raises(EOFError):
        C.decompress(m, d['c48s_bytes'].tobytes())


@pytest.mark.gpu
def test_gpu_compress_batch_matches_per_clip_compress():
    """compress_batch's B files == compress() of each clip (same header, payload layout and
    scale handling); codes may differ only where fp reassociation across batch shapes can
    move a near-tie argmin."""
    from encx import compress as C
    m = _model48()
    d = load('g10_ecdc.npz')
    w = T(d['c48_x'])[:, :4752]
    batch = torch.stack([w, 0.5 * w.flip(-1), -w])
    blobs = C.compress_batch(m, batch)
    for b in range(3):
        single = C.compress(m, batch[b])
        assert len(blobs[b]) == len(single)
        meta_b, fb = E.decompress_codes(blobs[b], 10, 1, True)
        meta_s, fs = E.decompress_codes(single, 10, 1, True)
        assert meta_b == meta_s
        assert (fb[0][0] != fs[0][0]).mean() < 0.05
        assert abs(fb[0][1] - fs[0][1]) <= 1e-6 * abs(fs[0][1])
