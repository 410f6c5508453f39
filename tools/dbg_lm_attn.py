import sys, torch
sys.path.insert(0, 'encodec-pytorch_amd')
from encx._lib import call, lib, stream
from encx.lm import LMModel
torch.manual_seed(0)
dev = 'cuda:0'
lm = LMModel(32, 1024, dim=200, num_layers=1, past_context=262).to(dev)
layer = lm.transformer.layers[0]; a = layer.self_attn
D, F, H, P = 200, 800, 8, 262
def run(x, T, kv, seq0, B=1):
    y = torch.empty(B * T, D, device=dev)
    work = torch.empty((int(lib.encx_lm_layer_workspace(B * T, D, F)) + 3) // 4, device=dev)
    call('encx_lm_layer', x.data_ptr(), y.data_ptr(), B, T, kv.data_ptr(), kv.shape[1], seq0, None, P, D, H, F,
         a.in_proj_weight.data_ptr(), a.in_proj_bias.data_ptr(), a.out_proj.weight.data_ptr(), a.out_proj.bias.data_ptr(),
         layer.linear1.weight.data_ptr(), layer.linear1.bias.data_ptr(), layer.linear2.weight.data_ptr(), layer.linear2.bias.data_ptr(),
         layer.norm1.weight.data_ptr(), layer.norm1.bias.data_ptr(), layer.norm2.weight.data_ptr(), layer.norm2.bias.data_ptr(),
         work.data_ptr(), stream())
    N = B * T
    q = work[:N * D].view(N, D).clone(); ctx = work[N * D:2 * N * D].view(N, D).clone()
    return y, q, ctx
Tn = 300
B = 2
x = torch.randn(B, Tn, D, device=dev)
kv1 = torch.zeros(B, Tn + 1, 2 * D, device=dev)
y1, q1, c1 = run(x, Tn, kv1, 1, B)
y1, q1, c1 = y1.view(B, Tn, D), q1.view(B, Tn, D), c1.view(B, Tn, D)
kv2 = torch.zeros(B, Tn + 1, 2 * D, device=dev)
y2, q2, c2 = run(x[:, :295].contiguous(), 295, kv2, 1, B)
print('prefix y equal', torch.equal(y2.view(B, 295, D), y1[:, :295]), 'kv prefix equal', torch.equal(kv2[:, 1:296], kv1[:, 1:296]))
for t in range(295, 300):
    y3, q3, c3 = run(x[:, t:t + 1].contiguous(), 1, kv2, t + 1, B)
    print(t, 'q', torch.equal(q3, q1[:, t]), 'ctx', torch.equal(c3, c1[:, t]), (c3 - c1[:, t]).abs().max().item(),
          'kv', torch.equal(kv2[:, t + 1], kv1[:, t + 1]), 'y', torch.equal(y3, y1[:, t]))
# small T: both kernels = row kernel? compare block vs row at T=100 (N*H=800 -> row) vs T=600
