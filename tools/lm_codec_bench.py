"""LM entropy coding throughput on one MI355X (compress.py use_lm=True).

The 24 kHz LM at its real size (n_q 32, card 1024, dim 200, 8 heads, 5 layers, past_context
262 = 3.5 s of frames, model.py:221-226) with random-init weights (the pretrained LM is
remote-only), K = 8 codebooks (6 kbps), random codes. Times, with inputs resident in HBM:
  * encode: LMModel.encode_streams over B streams x T steps (one LM pass over all rows, fused
    softmax + quantized cdf + coding intervals, one coder thread per stream, bytes to host);
  * decode: LMModel.decode_streams (T graph-replayed steps of LM + cdf + arithmetic decode);
and reports audio-seconds per second (75 steps = 1 s). CPU baseline: the reference's own loop
restated by the oracle (torch-CPU streaming LM step + quantized cdf + integer coder,
compress.py:74-89) on one stream.

python tools/lm_codec_bench.py [--streams B] [--seconds S] [--iters N] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'encodec-pytorch_amd'))
sys.path.insert(0, ROOT)

FRAME_RATE = 75


def timed(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters, out


def cpu_baseline(lm_cpu, cfg, K, steps):
    from oracle import lm_oracle as L, ac_oracle as A
    st = {k: v.detach().float() for k, v in lm_cpu.state_dict().items()}
    g = np.random.default_rng(3)
    codes = torch.from_numpy(g.integers(0, cfg.card, size=(1, K, steps)))
    t0 = time.perf_counter()
    syms, cdfs = L.compress_lm_symbols(st, codes, cfg)
    A.encode(syms, cdfs)
    dt = time.perf_counter() - t0
    return {'value': round(steps / FRAME_RATE / dt, 4), 'unit': 'audio-seconds/sec',
            'cores': torch.get_num_threads(), 'kind': 'port',
            'sample': f'oracle streaming LM + quantized cdf + coder, 1 stream x {steps} steps (K={K}), '
                      f'{dt:.1f} s wall'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--streams', type=int, default=32)
    ap.add_argument('--seconds', type=float, default=10.0)
    ap.add_argument('--dec-seconds', type=float, default=5.0)
    ap.add_argument('--iters', type=int, default=3)
    ap.add_argument('--K', type=int, default=8)
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()
    from encx.lm import LMModel
    from oracle.lm_oracle import LMConfig
    torch.manual_seed(0)
    lm_cpu = LMModel(32, 1024, dim=200, num_layers=5, past_context=int(3.5 * FRAME_RATE))
    dev = torch.device('cuda', 0)
    lm = LMModel(32, 1024, dim=200, num_layers=5, past_context=int(3.5 * FRAME_RATE))
    lm.load_state_dict(lm_cpu.state_dict())
    lm = lm.to(dev).eval()
    B, K = args.streams, args.K
    Te = int(args.seconds * FRAME_RATE)
    Td = int(args.dec_seconds * FRAME_RATE)
    g = np.random.default_rng(1)
    codes = torch.from_numpy(g.integers(0, 1024, size=(B, K, Te))).to(dev)
    lm.encode_streams(codes[:, :, :8].contiguous())                      # warm-up
    t_enc, datas = timed(lambda: lm.encode_streams(codes), args.iters)
    bits_per_code = 8 * sum(len(d) for d in datas) / (B * K * Te)
    dcodes = codes[:, :, :Td].contiguous()
    ddatas = lm.encode_streams(dcodes)
    lm.decode_streams([d[:64] for d in ddatas], K, 4)                   # warm-up (graph path)
    t_dec, (back, _) = timed(lambda: lm.decode_streams(ddatas, K, Td), args.iters)
    assert torch.equal(back, dcodes), 'round trip failed'
    t_dec_eager, _ = timed(lambda: lm.decode_streams(ddatas, K, Td, graph=False), 1)
    # LM-only one-pass time (no coder, no host copy)
    full = torch.zeros_like(codes)
    full[:, :, 1:] = codes[:, :, :-1] + 1

    def lm_pass():
        x = lm._body(full, full.stride(), B, K, Te, False, lm.new_state(B, Te + 1))
        cdf = torch.empty(B, Te, K, 1024, device=dev, dtype=torch.int32)
        lm._heads(x, B, Te, K, cdf=cdf)
    t_lm, _ = timed(lm_pass, args.iters)
    D, Fh, L = 200, 800, 5
    flops_row = L * 2 * (3 * D * D + D * D + 2 * D * Fh) + 2 * K * 1024 * D
    line = {
        'metric': 'LM entropy coding throughput (use_lm=True), 24 kHz LM, 6 kbps (K=8)',
        'unit': 'audio-seconds/sec', 'streams': B,
        'encode': {'value': round(B * Te / FRAME_RATE / t_enc, 2), 'ms': round(1e3 * t_enc, 2),
                   'seconds_per_stream': args.seconds, 'bits_per_code': round(bits_per_code, 3)},
        'decode': {'value': round(B * Td / FRAME_RATE / t_dec, 2), 'ms': round(1e3 * t_dec, 2),
                   'seconds_per_stream': args.dec_seconds, 'us_per_step': round(1e6 * t_dec / Td, 1),
                   'eager_us_per_step': round(1e6 * t_dec_eager / Td, 1)},
        'lm_pass': {'ms': round(1e3 * t_lm, 3), 'rows': B * Te,
                    'tflops': round(flops_row * B * Te / t_lm / 1e12, 3)},
        'data': 'synthetic (random codes, random-init LM weights)', 'dtype': 'f32',
    }
    if not args.no_cpu:
        torch.set_num_threads(16)
        line['cpu_baseline'] = cpu_baseline(lm_cpu, LMConfig(), K, FRAME_RATE)
        line['encode']['vs_cpu'] = round(line['encode']['value'] / line['cpu_baseline']['value'], 1)
    print(json.dumps(line))


if __name__ == '__main__':
    main()
