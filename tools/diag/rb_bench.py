"""Fused residual block alone (csrc/resblock.hip) at the config-3 shapes (B 32: C 32 x T 24000,
C 64 x T 12000): forward + backward N times, for rocprofv3 --kernel-trace --stats."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'encodec-pytorch_amd'))
from encx.modules.seanet import SEANetResnetBlock  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for C, T in ((32, 24000), (64, 12000)):
    blk = SEANetResnetBlock(C, norm='weight_norm', causal=True, true_skip=False).cuda()
    x = (0.5 * torch.randn(32, C, T, device='cuda')).requires_grad_(True)
    dy = torch.randn(32, C, T, device='cuda')
    for _ in range(n):
        y = blk(x)
        torch.autograd.grad(y, [x] + list(blk.parameters()), dy)
    torch.cuda.synchronize()
print('ok')
