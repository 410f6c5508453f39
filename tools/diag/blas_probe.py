"""How fast is the vendor fp32 GEMM (torch.mm -> hipBLASLt / rocBLAS, TF32 off) at the shapes of
the short-T conv layers and the LSTM weight grad? Informs whether an im2col + library GEMM beats
the flattened implicit GEMMs. Run on a GPU box."""
import torch

torch.backends.cuda.matmul.allow_tf32 = False
dev = 'cuda:0'
shapes = [('k16s8 T75 fwd (512 x 2400 x 4096)', 512, 2400, 4096),
          ('k16s8 T75 wgrad (512 x 4096 x 2400)', 512, 4096, 2400),
          ('k7 T75 fwd (128 x 2400 x 3584)', 128, 2400, 3584),
          ('lstm wgrad (2048 x 1025 x 2400)', 2048, 1025, 2400),
          ('lstm wgrad (2048 x 1024 x 2400)', 2048, 1024, 2400),
          ('k10s5 T600 fwd (256 x 19200 x 1280)', 256, 19200, 1280),
          ('k10s5 T600 wgrad (1280 x 256 x 19200)', 1280, 256, 19200),
          ('k10s5 T600 poly (640 x 19200 x 512)', 640, 19200, 512),
          ('k8s4 T3000 fwd (128 x 96000 x 512)', 128, 96000, 512),
          ('k3 T600 fwd (128 x 19200 x 768)', 128, 19200, 768),
          ('square 4096', 4096, 4096, 4096)]
for name, M, N, K in shapes:
    for ta in (False,):
        a = torch.randn(K, M, device=dev).t() if ta else torch.randn(M, K, device=dev)
        b = torch.randn(K, N, device=dev)
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f'{name:40s} A^T={ta}: {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:6.1f} TF/s', flush=True)
