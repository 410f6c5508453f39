"""Residual vector quantization (quantization/core_vq.py of the reference) on encx kernels.

Module / buffer names match the reference (`layers.{i}._codebook.{inited,cluster_size,embed,
embed_avg}`). Train mode runs each layer as argmin (MFMA) -> dequantize/STE/residual/commit
-> EMA update, all on the device; dead-code expiry (core_vq.py:165-175) is omitted because
core_vq.py:235 overwrites the expired rows before anything reads them (no effect on outputs).
"""
import typing as tp

import torch
from torch import nn

from .. import ops


def default(val, d):
    return val if val is not None else d


class EuclideanCodebook(nn.Module):
    """core_vq.py:105-237."""

    def __init__(self, dim: int, codebook_size: int, kmeans_init: int = False, kmeans_iters: int = 10,
                 decay: float = 0.99, epsilon: float = 1e-5, threshold_ema_dead_code: int = 2):
        super().__init__()
        self.decay = decay
        if kmeans_init:
            embed = torch.zeros(codebook_size, dim)
        else:
            embed = torch.empty(codebook_size, dim)
            nn.init.kaiming_uniform_(embed)
        self.codebook_size = codebook_size
        self.kmeans_iters = kmeans_iters
        self.epsilon = epsilon
        self.threshold_ema_dead_code = threshold_ema_dead_code
        self.register_buffer('inited', torch.Tensor([not kmeans_init]))
        self.register_buffer('cluster_size', torch.zeros(codebook_size))
        self.register_buffer('embed', embed)
        self.register_buffer('embed_avg', embed.clone())
        self._inited_host = None  # host mirror of `inited` (read once, then trusted)
        # opt-in data-parallel codebook sync: rank 0's kmeans init is broadcast and
        # the EMA sums are all-reduced before every update. Off = the reference (core_vq.py:157,
        # 175 keep their broadcasts commented out; train_multi_gpu.py:318 broadcast_buffers=False)
        self.sync_codebooks = False

    def _load_from_state_dict(self, *args, **kwargs):
        self._inited_host = None
        return super()._load_from_state_dict(*args, **kwargs)

    @torch.no_grad()
    def init_embed_(self, data):
        """core_vq.py:146-157: kmeans on the first batch. data: [B, D, T] residual."""
        if self._inited_host is None:
            self._inited_host = bool(self.inited.item())
        if self._inited_host:
            return
        samples = ops.rvq_to_rows(data)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        embed, bins = ops.kmeans(samples, self.codebook_size, self.kmeans_iters, seed)
        self.embed.data.copy_(embed)
        self.embed_avg.data.copy_(embed)
        self.cluster_size.data.copy_(bins)
        self.inited.data.fill_(1.0)
        self._inited_host = True
        if self.sync_codebooks and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1:
            # the broadcast core_vq.py:157 intends: every rank starts from rank 0's codebook
            for b in (self.embed, self.embed_avg, self.cluster_size, self.inited):
                torch.distributed.broadcast(b.data, src=0)

    def quantize(self, x):
        """core_vq.py:181-189 on [N, D] rows."""
        return ops.rvq_argmin(x.t().contiguous().unsqueeze(0), self.embed)

    def encode(self, x):
        """x: [B, N, D] -> [B, N]."""
        return ops.rvq_argmin(x.permute(0, 2, 1).contiguous(), self.embed).view(x.shape[:-1])

    def decode(self, embed_ind):
        return ops.rvq_decode(embed_ind.unsqueeze(0), [self.embed]).permute(0, 2, 1)


class VectorQuantization(nn.Module):
    """core_vq.py:240-324 (codebook_dim == dim: no projections)."""

    def __init__(self, dim: int, codebook_size: int, codebook_dim: tp.Optional[int] = None,
                 decay: float = 0.99, epsilon: float = 1e-5, kmeans_init: bool = True,
                 kmeans_iters: int = 50, threshold_ema_dead_code: int = 2, commitment_weight: float = 1.):
        super().__init__()
        _codebook_dim: int = default(codebook_dim, dim)
        if _codebook_dim != dim:
            raise NotImplementedError('encx: codebook projections are unused by EnCodec')
        self.project_in = nn.Identity()
        self.project_out = nn.Identity()
        self.epsilon = epsilon
        self.commitment_weight = float(commitment_weight)  # core_vq.py:267, in RVQTrainFn's penalty
        self._codebook = EuclideanCodebook(dim=_codebook_dim, codebook_size=codebook_size,
                                           kmeans_init=kmeans_init, kmeans_iters=kmeans_iters,
                                           decay=decay, epsilon=epsilon,
                                           threshold_ema_dead_code=threshold_ema_dead_code)
        self.codebook_size = codebook_size

    @property
    def codebook(self):
        return self._codebook.embed

    def encode(self, x):
        """x [B, D, N] -> codes [B, N] (core_vq.py:289-293)."""
        return ops.rvq_argmin(x.contiguous(), self._codebook.embed).view(x.shape[0], x.shape[2])

    def decode(self, embed_ind):
        return ops.rvq_decode(embed_ind.unsqueeze(0), [self._codebook.embed])

    def forward(self, x):
        q, codes, loss = ResidualVectorQuantization.run([self], x)
        return q, codes[0], loss


class ResidualVectorQuantization(nn.Module):
    """core_vq.py:327-375."""

    def __init__(self, *, num_quantizers, **kwargs):
        super().__init__()
        self.layers = nn.ModuleList([VectorQuantization(**kwargs) for _ in range(num_quantizers)])

    def set_sync_codebooks(self, on: bool = True):
        for layer in self.layers:
            layer._codebook.sync_codebooks = bool(on)

    @staticmethod
    def run(layers, x):
        cbs = [layer._codebook for layer in layers]
        if layers[0].training:
            cw = layers[0].commitment_weight
            if any(layer.commitment_weight != cw for layer in layers):
                raise ValueError('encx RVQ: one commitment_weight for all layers (the kwargs every layer gets)')
            return ops.RVQTrainFn.apply(x, cbs, cbs[0].decay, cbs[0].epsilon, cbs[0].sync_codebooks, cw)
        # eval forward (no STE, no commit loss, no EMA)
        codes = ops.rvq_encode(x, [c.embed for c in cbs])
        q = ops.rvq_decode(codes, [c.embed for c in cbs])
        return q, codes, torch.zeros(1, device=x.device)

    def forward(self, x, n_q: tp.Optional[int] = None):
        n_q = n_q or len(self.layers)
        q, codes, penalty = self.run(self.layers[:n_q], x)
        # the reference stacks one [1] loss per layer; penalty == their mean (vq.py:99)
        return q, codes, penalty

    def encode(self, x: torch.Tensor, n_q: tp.Optional[int] = None) -> torch.Tensor:
        n_q = n_q or len(self.layers)
        return ops.rvq_encode(x, [layer._codebook.embed for layer in self.layers[:n_q]])

    def decode(self, q_indices: torch.Tensor) -> torch.Tensor:
        return ops.rvq_decode(q_indices, [layer._codebook.embed for layer in self.layers[:len(q_indices)]])
