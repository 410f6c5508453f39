"""`.ecdc` codec throughput on one MI355X: 32 synthetic 1 s clips through
encx.compress.compress_batch (SEANet encoder + RVQ n_q 8 + GPU bit packing, bytes to host) and
back through the GPU unpack + RVQ gather + SEANet decoder. Prints one JSON line with audio-s/s
for each direction and the bit-pack kernels' own time (HIP events on the launch stream) against
the HBM roofline. CPU baseline: the oracle's numpy bit packer on the same codes.

python tools/codec_bench.py [--steps K] [--warmup W]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=32)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    from encx.model import EncodecModel
    from encx import compress as C, ops
    B = args.batch
    model = EncodecModel._get_model([1.5, 3., 6., 12., 24.], 24000, 1, causal=True, model_norm='weight_norm',
                                    audio_normalize=False, name='encodec_24khz').to(dev)
    model.eval()
    model.set_target_bandwidth(6.0)
    g = np.random.Generator(np.random.PCG64(1234))
    x = torch.from_numpy((0.1 * g.standard_normal((B, 1, 24000))).astype(np.float32)).to(dev)

    def compress_step():
        return C.compress_batch(model, x)

    def decompress_step(blobs):
        # parse all B files, one H2D copy, one unpack launch, one batched decode
        import io
        from encx import binary
        metas, payload = [], []
        for bl in blobs:
            fo = io.BytesIO(bl)
            metas.append(binary.read_ecdc_header(fo))
            payload.append(np.frombuffer(fo.read(), np.uint8))
        K, Tf = metas[0]['nc'], metas[0]['fr']
        data = torch.from_numpy(np.stack(payload)).to(dev)
        codes = ops.unpack_codes(data, K, Tf, model.bits_per_codebook)
        with torch.no_grad():
            return model.decode([(codes, None)])

    for _ in range(args.warmup):
        blobs = compress_step()
        decompress_step(blobs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        blobs = compress_step()
    torch.cuda.synchronize()
    t_c = (time.perf_counter() - t0) / args.steps
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = decompress_step(blobs)
    torch.cuda.synchronize()
    t_d = (time.perf_counter() - t0) / args.steps

    # the pack / unpack kernels alone, on the stream they are launched on
    with torch.no_grad():
        frames = model.encode(x)
    codes = frames[0][0]
    Kq, Tf = codes.shape[1], codes.shape[2]
    st = torch.cuda.current_stream()
    reps = 200
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    data, _ = ops.pack_codes(codes, 10)
    e0.record(st)
    for _ in range(reps):
        data, _ = ops.pack_codes(codes, 10)
    e1.record(st)
    for _ in range(reps):
        back = ops.unpack_codes(data, Kq, Tf, 10)
    e2.record(st)
    torch.cuda.synchronize()
    assert torch.equal(back, codes.contiguous())
    pack_us = e0.elapsed_time(e1) * 1e3 / reps
    unpack_us = e1.elapsed_time(e2) * 1e3 / reps
    n = codes.numel()
    alg_bytes = n * 8 + data.numel()   # int64 codes in, packed bytes out (and the reverse)
    # large-batch pack: 32768 clips' codes in one launch, where the kernel is not launch bound
    big = torch.randint(0, 1024, (32768, Kq, Tf), device=dev)
    bd, _ = ops.pack_codes(big, 10)
    e0.record(st)
    for _ in range(20):
        bd, _ = ops.pack_codes(big, 10)
    e1.record(st)
    for _ in range(20):
        ops.unpack_codes(bd, Kq, Tf, 10)
    e2.record(st)
    torch.cuda.synchronize()
    big_bytes = big.numel() * 8 + bd.numel()
    big_pack_gbs = big_bytes / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e9
    big_unpack_gbs = big_bytes / (e1.elapsed_time(e2) / 20 * 1e-3) / 1e9

    from oracle import ecdc_oracle as E
    host = codes.cpu().numpy()
    t0 = time.perf_counter()
    nrep = 0
    while nrep < 3 or time.perf_counter() - t0 < 2.0:
        for b in range(B):
            E.bitpack(host[b].T.reshape(-1), 10)
        nrep += 1
    cpu_pack_s = (time.perf_counter() - t0) / nrep

    print(json.dumps({
        'metric': 'audio-seconds/sec .ecdc codec (24 kHz, n_q 8, 1 s clips)',
        'compress_value': round(B / t_c, 1), 'decompress_value': round(B / t_d, 1),
        'unit': 'audio-seconds/sec', 'batch': B, 'steps': args.steps, 'n_gpus': 1,
        'ms_compress': round(t_c * 1e3, 3), 'ms_decompress': round(t_d * 1e3, 3),
        'bytes_per_clip': len(blobs[0]), 'decoded_shape': list(y.shape),
        'pack_kernel': {'us': round(pack_us, 2), 'unpack_us': round(unpack_us, 2), 'codes': n,
                        'algorithmic_bytes': alg_bytes,
                        'big_batch': {'clips': 32768, 'pack_GBs': round(big_pack_gbs, 1),
                                      'unpack_GBs': round(big_unpack_gbs, 1), 'peak_GBs': 8000.0,
                                      'pack_frac': round(big_pack_gbs / 8000.0, 4),
                                      'unpack_frac': round(big_unpack_gbs / 8000.0, 4)}},
        'cpu_baseline': {'pack_ms': round(cpu_pack_s * 1e3, 3), 'kind': 'port', 'cores': 1,
                         'sample': f'oracle numpy bitpack of the same {B} frames'},
        'data': 'synthetic (0.1*N(0,1) clips, random-init weights)',
    }), flush=True)


if __name__ == '__main__':
    main()
