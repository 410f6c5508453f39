"""EncodecModel (model.py of the reference) on the encx HIP path.

Same constructor, `_get_model` factory, `encode / decode / forward / set_target_bandwidth`
and state-dict layout, plus `get_lm_model` (model.py:221-240) for the LM entropy coder
(encx.lm). Pretrained checkpoints are fetched as the reference fetches them (torch.hub, which
finds a pre-populated hub cache offline); `set_lm_model` installs an LM directly.
"""
import math
import random
import typing as tp

import numpy as np
import torch
from torch import nn

from . import modules as m
from . import quantization as qt
from . import ops

EncodedFrame = tp.Tuple[torch.Tensor, tp.Optional[torch.Tensor]]


class EncodecModel(nn.Module):
    """model.py:68-369."""

    def __init__(self, encoder: m.SEANetEncoder, decoder: m.SEANetDecoder,
                 quantizer: qt.ResidualVectorQuantizer, target_bandwidths: tp.List[float],
                 sample_rate: int, channels: int, normalize: bool = False,
                 segment: tp.Optional[float] = None, overlap: float = 0.01, name: str = 'unset'):
        super().__init__()
        self.bandwidth: tp.Optional[float] = None
        self.target_bandwidths = target_bandwidths
        self.encoder = encoder
        self.quantizer = quantizer
        self.decoder = decoder
        self.sample_rate = sample_rate
        self.channels = channels
        self.normalize = normalize
        self.segment = segment
        self.overlap = overlap
        self.frame_rate = math.ceil(self.sample_rate / np.prod(self.encoder.ratios))
        self.name = name
        self.bits_per_codebook = int(math.log2(self.quantizer.bins))
        assert 2 ** self.bits_per_codebook == self.quantizer.bins, "quantizer bins must be a power of 2."

    @property
    def segment_length(self) -> tp.Optional[int]:
        if self.segment is None:
            return None
        return int(self.segment * self.sample_rate)

    @property
    def segment_stride(self) -> tp.Optional[int]:
        segment_length = self.segment_length
        if segment_length is None:
            return None
        return max(1, int((1 - self.overlap) * segment_length))

    def encode(self, x: torch.Tensor) -> tp.List[EncodedFrame]:
        """model.py:122-145."""
        assert x.dim() == 3
        _, channels, length = x.shape
        assert 0 < channels <= 2
        segment_length = self.segment_length
        if segment_length is None:
            segment_length = length
            stride = length
        else:
            stride = self.segment_stride
        return [self._encode_frame(x[:, :, offset: offset + segment_length])
                for offset in range(0, length, stride)]

    def _encode_frame(self, x: torch.Tensor) -> EncodedFrame:
        """model.py:147-168: normalise, encode; train mode returns (emb, scale)."""
        length = x.shape[-1]
        duration = length / self.sample_rate
        assert self.segment is None or duration <= 1e-5 + self.segment
        if self.normalize:
            x, scale = ops.normalize(x)
        else:
            scale = None
        emb = self.encoder(x)
        if self.training:
            return emb, scale
        codes = self.quantizer.encode(emb, self.frame_rate, self.bandwidth)
        return codes.transpose(0, 1), scale

    def decode(self, encoded_frames: tp.List[EncodedFrame]) -> torch.Tensor:
        """model.py:170-181: per-segment decode, then the triangle-weighted overlap-add."""
        if self.segment_length is None:
            assert len(encoded_frames) == 1
            return self._decode_frame(encoded_frames[0])
        frames = [self._decode_frame(frame) for frame in encoded_frames]
        return ops.linear_overlap_add(frames, self.segment_stride or 1)  # utils.py:22-61

    def _decode_frame(self, encoded_frame: EncodedFrame) -> torch.Tensor:
        """model.py:183-193."""
        codes, scale = encoded_frame
        if self.training:
            emb = codes
        else:
            emb = self.quantizer.decode(codes.transpose(0, 1))
        out = self.decoder(emb)
        if scale is not None:
            out = ops.ScaleRowsFn.apply(out, scale.contiguous().view(-1))
        return out

    def _pick_bandwidth(self, device):
        """model.py:202-205: random target bandwidth, broadcast from rank 0."""
        index = random.randint(0, len(self.target_bandwidths) - 1)
        if len(self.target_bandwidths) > 1 and torch.distributed.is_initialized():
            t = torch.tensor(index, device=device)
            torch.distributed.broadcast(t, src=0)
            index = int(t.item())
        return self.target_bandwidths[index]

    def forward(self, x: torch.Tensor, bandwidth: tp.Optional[float] = None, split: bool = False):
        """model.py:195-213. Train mode -> (output, loss_w, frames); eval -> output.
        `bandwidth` (train mode, not in the reference) fixes the step's target bandwidth instead
        of drawing it here: the HIP-graph trainer draws it on the host before replaying.
        `split` (train mode, one segment; not in the reference): the decoder reads a detached leaf
        copy of the quantized latent, so the backward runs as two calls -- output -> decoder
        weights + the leaf's grad, then (quantized, loss_w) -> encoder -- and the data-parallel
        trainer all-reduces the decoder's grads between them (self.last_split = (quantized, leaf))."""
        frames = self.encode(x)
        if self.training:
            bw = self._pick_bandwidth(x.device) if bandwidth is None else bandwidth
            codes, seg_codes = [], []
            loss_w = None
            for emb, scale in frames:
                qv = self.quantizer(emb, self.frame_rate, bw)
                seg_codes.append((qv.codes, emb.detach()))
                pen = qv.penalty.reshape(1)  # loss_w = tensor([0.]) + penalty (model.py:199,208)
                loss_w = pen if loss_w is None else loss_w + pen
                codes.append((qv.quantized, scale))
            self.last_codes = [qv.codes]
            # every segment's (codes [n_q, B*T], latent [B, D, T]): the tests' nearest-code audit
            self.seg_codes = seg_codes
            self.last_split = None
            if split and len(codes) == 1:
                q, scale = codes[0]
                leaf = q.detach().requires_grad_()
                self.last_split = (q, leaf)
                codes = [(leaf, scale)]
            return self.decode(codes)[:, :, :x.shape[-1]], loss_w, frames
        return self.decode(frames)[:, :, :x.shape[-1]]

    def set_lm_model(self, lm):
        """Use `lm` (an encx.lm.LMModel) for use_lm=True instead of the pretrained one."""
        self._lm_model = lm

    def get_lm_model(self):
        """model.py:221-240: LMModel(n_q, bins, num_layers=5, dim=200, past_context=3.5 s of
        frames) with the pretrained weights of this model."""
        from .lm import LMModel
        lm = getattr(self, '_lm_model', None)
        if lm is not None:
            return lm
        device = next(self.parameters()).device
        lm = LMModel(self.quantizer.n_q, self.quantizer.bins, num_layers=5, dim=200,
                     past_context=int(3.5 * self.frame_rate)).to(device)
        checkpoints = {
            'encodec_24khz': 'encodec_lm_24khz-1608e3c0.th',
            'encodec_48khz': 'encodec_lm_48khz-7add9fc3.th',
        }
        try:
            checkpoint_name = checkpoints[self.name]
        except KeyError:
            raise RuntimeError("No LM pre-trained for the current Encodec model.")
        url = 'https://dl.fbaipublicfiles.com/encodec/v0/' + checkpoint_name
        state = torch.hub.load_state_dict_from_url(url, map_location='cpu', check_hash=True)
        lm.load_state_dict(state)
        lm.eval()
        return lm

    def set_target_bandwidth(self, bandwidth: float):
        if bandwidth not in self.target_bandwidths:
            raise ValueError(f"This model doesn't support the bandwidth {bandwidth}. "
                             f"Select one of {self.target_bandwidths}.")
        self.bandwidth = bandwidth

    @staticmethod
    def _get_model(target_bandwidths: tp.List[float], sample_rate: int = 24_000, channels: int = 1,
                   causal: bool = True, model_norm: str = 'weight_norm', audio_normalize: bool = False,
                   segment: tp.Optional[float] = None, name: str = 'unset', ratios=[8, 5, 4, 2],
                   n_q: tp.Optional[int] = None, sync_codebooks: bool = False):
        """model.py:242-276. sync_codebooks (not in the reference): all-reduce the RVQ EMA sums and
        broadcast rank 0's kmeans init across data-parallel ranks."""
        encoder = m.SEANetEncoder(channels=channels, norm=model_norm, causal=causal, ratios=ratios)
        decoder = m.SEANetDecoder(channels=channels, norm=model_norm, causal=causal, ratios=ratios)
        if n_q is None:
            n_q = int(1000 * target_bandwidths[-1] // (math.ceil(sample_rate / encoder.hop_length) * 10))
        quantizer = qt.ResidualVectorQuantizer(dimension=encoder.dimension, n_q=n_q, bins=1024,
                                               sync_codebooks=sync_codebooks)
        return EncodecModel(encoder, decoder, quantizer, target_bandwidths, sample_rate, channels,
                            normalize=audio_normalize, segment=segment, name=name)

    @staticmethod
    def encodec_model_24khz(pretrained: bool = False, repository=None):
        """model.py:291-309 architecture (pretrained weights are remote-only: out of scope)."""
        if pretrained:
            raise RuntimeError('encx: pretrained checkpoints are remote-only; load a state dict instead')
        model = EncodecModel._get_model([1.5, 3., 6, 12., 24.], 24_000, 1, causal=True,
                                        model_norm='weight_norm', audio_normalize=False, name='unset')
        model.eval()
        return model

    @staticmethod
    def _load_checkpoint(model, checkpoint):
        """model.py:346-349: a trainer checkpoint's 'model_state_dict', with the old
        'quantizer.model' prefix renamed. Loaded with weights_only=True (no unpickling)."""
        import os
        assert os.path.exists(checkpoint), "checkpoint not exists"
        pre_dic = torch.load(checkpoint, map_location='cpu', weights_only=True)['model_state_dict']
        model.load_state_dict({k.replace('quantizer.model', 'quantizer.vq'): v for k, v in pre_dic.items()})
        model.eval()
        return model

    @staticmethod
    def my_encodec_model(checkpoint: str, ratios=[8, 5, 4, 2]):
        """model.py:332-349: 24 kHz mono, non-causal, time_group_norm, normalised, no segments."""
        model = EncodecModel._get_model([1.5, 3., 6, 12., 24.], 24_000, 1, causal=False,
                                        model_norm='time_group_norm', audio_normalize=True,
                                        segment=None, name='my_encodec', ratios=ratios)
        return EncodecModel._load_checkpoint(model, checkpoint)

    @staticmethod
    def encodec_model_bw(checkpoint: str, bandwidth: float):
        """model.py:351-369: as my_encodec_model with 1 s segments and target_bandwidths =
        `bandwidth` (the reference passes it through unwrapped; a list is expected)."""
        model = EncodecModel._get_model(bandwidth, 24_000, 1, causal=False,
                                        model_norm='time_group_norm', audio_normalize=True,
                                        segment=1., name='my_encodec')
        return EncodecModel._load_checkpoint(model, checkpoint)

    @staticmethod
    def encodec_model_48khz(pretrained: bool = False, repository=None):
        """model.py:311-329 architecture: 48 kHz stereo, non-causal, time_group_norm, 1 s
        segments (pretrained weights are remote-only: out of scope)."""
        if pretrained:
            raise RuntimeError('encx: pretrained checkpoints are remote-only; load a state dict instead')
        model = EncodecModel._get_model([3., 6., 12., 24.], 48_000, 2, causal=False,
                                        model_norm='time_group_norm', audio_normalize=True,
                                        segment=1., name='unset')
        model.eval()
        return model
