"""Background GPU load for concurrency experiments: elementwise + GEMM kernels in a loop on
cuda:0 for at most --seconds (then exits by itself). python tools/diag/gpu_noise.py --seconds 120"""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument('--seconds', type=float, default=120)
args = ap.parse_args()
a = torch.randn(4096, 4096, device='cuda')
b = torch.randn(64 * 2 ** 20, device='cuda')
t0 = time.time()
n = 0
while time.time() - t0 < args.seconds:
    for _ in range(20):
        a = torch.tanh(a @ a * 1e-3)
        b.mul_(0.999).add_(1e-3)
    torch.cuda.synchronize()
    n += 1
print(f'noise: {n} rounds in {time.time() - t0:.1f} s')
