"""ResidualVectorQuantizer (quantization/vq.py of the reference)."""
from dataclasses import dataclass, field
import math
import typing as tp

import torch
from torch import nn

from .core_vq import ResidualVectorQuantization


@dataclass
class QuantizedResult:
    """vq.py:19-25."""
    quantized: torch.Tensor
    codes: torch.Tensor
    bandwidth: torch.Tensor
    penalty: tp.Optional[torch.Tensor] = None
    metrics: dict = field(default_factory=dict)


class ResidualVectorQuantizer(nn.Module):
    """vq.py:28-128."""

    def __init__(self, dimension: int = 256, n_q: int = 8, bins: int = 1024, decay: float = 0.99,
                 kmeans_init: bool = True, kmeans_iters: int = 50, threshold_ema_dead_code: int = 2,
                 sync_codebooks: bool = False):
        super().__init__()
        self.n_q = n_q
        self.dimension = dimension
        self.bins = bins
        self.decay = decay
        self.kmeans_init = kmeans_init
        self.kmeans_iters = kmeans_iters
        self.threshold_ema_dead_code = threshold_ema_dead_code
        self._bw_cache = {}
        self.vq = ResidualVectorQuantization(dim=self.dimension, codebook_size=self.bins,
                                             num_quantizers=self.n_q, decay=self.decay,
                                             kmeans_init=self.kmeans_init, kmeans_iters=self.kmeans_iters,
                                             threshold_ema_dead_code=self.threshold_ema_dead_code)
        self.set_sync_codebooks(sync_codebooks)

    def set_sync_codebooks(self, on: bool = True):
        """Opt-in cross-rank codebook sync (not in the reference; see core_vq.EuclideanCodebook)."""
        self.sync_codebooks = bool(on)
        self.vq.set_sync_codebooks(on)

    def forward(self, x: torch.Tensor, sample_rate: int, bandwidth: tp.Optional[float] = None) -> QuantizedResult:
        bw_per_q = self.get_bandwidth_per_quantizer(sample_rate)
        n_q = self.get_num_quantizers_for_bandwidth(sample_rate, bandwidth)
        quantized, codes, penalty = self.vq(x, n_q=n_q)
        # the reported bandwidth is a constant per (n_q, device): built once, because a tensor
        # from a host scalar is a pageable H2D copy that stalls the host until the stream drains
        key = (n_q, str(x.device), x.dtype)
        bw = self._bw_cache.get(key)
        if bw is None:
            bw = self._bw_cache[key] = torch.tensor(n_q * bw_per_q, device=x.device, dtype=x.dtype)
        return QuantizedResult(quantized, codes, bw, penalty=penalty)

    def get_num_quantizers_for_bandwidth(self, sample_rate: int, bandwidth: tp.Optional[float] = None) -> int:
        bw_per_q = self.get_bandwidth_per_quantizer(sample_rate)
        n_q = self.n_q
        if bandwidth and bandwidth > 0.:
            n_q = int(max(1, math.floor(bandwidth / bw_per_q)))
        return n_q

    def get_bandwidth_per_quantizer(self, sample_rate: int):
        return math.log2(self.bins) * sample_rate / 1000

    def encode(self, x: torch.Tensor, sample_rate: int, bandwidth: tp.Optional[float] = None) -> torch.Tensor:
        n_q = self.get_num_quantizers_for_bandwidth(sample_rate, bandwidth)
        return self.vq.encode(x, n_q=n_q)

    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        return self.vq.decode(codes)
