"""fp32 GEMM rate of the vendor BLAS (torch.mm -> hipBLASLt / rocBLAS) at the LSTM weight-grad
shape ([2H+1] x [B*T] x [4H] = 1025 x 2400 x 2048) and the LSTM input projection shape, to decide
whether handing those GEMMs to the library pays. Usage (GPU box): python tools/diag/blas_rate.py"""
import torch


def rate(m, k, n, reps=20):
    a = torch.randn(m, k, device='cuda')
    b = torch.randn(k, n, device='cuda')
    for _ in range(3):
        torch.mm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(f'{m} x {k} x {n}: {us:.1f} us, {2 * m * k * n / us / 1e6:.1f} TFLOP/s', flush=True)


torch.backends.cuda.matmul.allow_tf32 = False
rate(1025, 2400, 2048)
rate(2048, 2400, 1025)
rate(2400, 512, 2048)
rate(4096, 4096, 4096)
