"""quantization/ac.py of the reference on the encx HIP kernels (csrc/ac.hip).

Same names, arguments and error behaviour:
  * build_stable_quantized_cdf (ac.py:18-53): a GPU float32 pdf -> int64 cdf (the reference's
    dtype) on the same device; AssertionError / ValueError where the reference raises;
  * ArithmeticCoder (ac.py:56-167): push(symbol, quantized_cdf) records the symbol's coding
    interval on the GPU, flush() runs the coder kernel over the whole stream and writes its
    bytes to `fo` (the reference writes bytes as they complete; the file content is the same);
  * ArithmeticDecoder (ac.py:170-260): pull(quantized_cdf) -> symbol, or None when the stream
    runs dry. It reads the rest of `fo` once and leaves `fo` positioned after the bytes the
    reference's BitUnpacker would have consumed, so containers with data after the coded
    stream (compress.py's multi-segment files) read the same way.
The batched coder of whole frames (compress.py) is encx.lm.LMModel.encode_streams /
decode_streams; these per-symbol classes keep the reference's streaming API.
"""
import io
import typing as tp

import torch

from ._lib import call, lib, stream, ensure_device, ENCX_AC_STATE, ENCX_AC_MAXBIT, ENCX_AC_POS


def _dev_tensor(x, dtype):
    if not torch.is_tensor(x) or not x.is_cuda:
        raise RuntimeError('encx: the arithmetic coder takes GPU tensors (no CPU fallback)')
    ensure_device(x.device)
    return x.to(dtype).contiguous()


def build_stable_quantized_cdf(pdf: torch.Tensor, total_range_bits: int,
                               roundoff: float = 1e-8, min_range: int = 2,
                               check: bool = True) -> torch.Tensor:
    """ac.py:18-53 on the GPU (csrc/ac.hip softmax_cdf_kernel, pdf mode)."""
    pdf = _dev_tensor(pdf.detach(), torch.float32).reshape(-1)
    total_range = 2 ** total_range_bits
    cardinality = len(pdf)
    alpha = min_range * cardinality / total_range
    assert alpha <= 1, "you must reduce min_range"
    if min_range < 2:
        raise ValueError("min_range must be at least 2.")
    cdf = torch.empty(cardinality, device=pdf.device, dtype=torch.int32)
    err = torch.zeros(1, device=pdf.device, dtype=torch.int32)
    call('encx_ac_cdf', pdf.data_ptr(), 1, cardinality, cardinality, int(total_range_bits),
         float(roundoff or 0.0), int(min_range), cdf.data_ptr(), err.data_ptr(), stream())
    cdf = cdf.long()
    if check and int(err.item()) & 1:
        raise AssertionError(int(cdf[-1]))   # ac.py:50
    return cdf


class ArithmeticCoder:
    """ac.py:56-167."""

    def __init__(self, fo: tp.IO[bytes], total_range_bits: int = 24):
        assert total_range_bits <= 30
        self.total_range_bits = total_range_bits
        self.fo = fo
        self._lohi: tp.List[torch.Tensor] = []
        self._err = None

    def push(self, symbol: int, quantized_cdf: torch.Tensor):
        """ac.py:130-158 (the interval is taken now; the bits come out at flush)."""
        cdf = _dev_tensor(quantized_cdf, torch.int32).reshape(-1)
        if self._err is None:
            self._err = torch.zeros(1, device=cdf.device, dtype=torch.int32)
        lohi = torch.empty(1, 2, device=cdf.device, dtype=torch.int32)
        sym = torch.tensor([int(symbol)], dtype=torch.int64).to(cdf.device)
        call('encx_ac_lohi', cdf.data_ptr(), cdf.numel(), sym.data_ptr(), 1, cdf.numel(), lohi.data_ptr(),
             self._err.data_ptr(), stream())
        self._lohi.append(lohi)

    def flush(self):
        """ac.py:160-167: code every pushed symbol, write the bytes."""
        n = len(self._lohi)
        bits = self.total_range_bits
        if n == 0:
            self.fo.flush()
            return
        lohi = torch.cat(self._lohi)
        dev = lohi.device
        cap = int(lib.encx_ac_encode_capacity(n, bits))
        out = torch.empty(cap, device=dev, dtype=torch.uint8)
        nbytes = torch.empty(1, device=dev, dtype=torch.int64)
        err = torch.empty(1, device=dev, dtype=torch.int32)
        call('encx_ac_encode', lohi.data_ptr(), 1, n, bits, out.data_ptr(), cap, nbytes.data_ptr(),
             err.data_ptr(), stream())
        e, e0 = int(err.item()), int(self._err.item())
        if e0 & 2:
            raise IndexError('symbol outside the quantized cdf')
        if e == 1:
            raise AssertionError('quantized cdf total above 2^total_range_bits (ac.py:116)')
        if e == 3:
            raise AssertionError('coder max_bit above 61 after a flush (ac.py:157)')
        if e:
            raise RuntimeError(f'encx arithmetic coder failed ({e})')
        self.fo.write(out[:int(nbytes.item())].cpu().numpy().tobytes())
        self.fo.flush()
        self._lohi = []


def new_decoder_state(streams, dev):
    """Zeroed arithmetic-decoder states [streams][ENCX_AC_STATE] (max_bit = -1), encx_ac_decode."""
    st = torch.zeros(streams, ENCX_AC_STATE, dtype=torch.int64, device=dev)
    st[:, ENCX_AC_MAXBIT] = -1
    return st


class ArithmeticDecoder:
    """ac.py:170-260."""

    def __init__(self, fo: tp.IO[bytes], total_range_bits: int = 24):
        self.total_range_bits = total_range_bits
        self.fo = fo
        self._start = fo.tell() if hasattr(fo, 'tell') else 0
        self._data = fo.read()
        self._dev = None
        self._state = None

    def _init(self, dev):
        ensure_device(dev)
        self._dev = dev
        buf = torch.frombuffer(bytearray(self._data or b'\0'), dtype=torch.uint8)
        self._buf = buf.to(dev)
        self._nbytes = torch.tensor([len(self._data)], dtype=torch.int64).to(dev)
        self._state = new_decoder_state(1, dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._sym = torch.zeros(1, dtype=torch.int64, device=dev)

    def pull(self, quantized_cdf: torch.Tensor) -> tp.Optional[int]:
        """ac.py:217-260."""
        cdf = _dev_tensor(quantized_cdf, torch.int32).reshape(-1)
        if self._state is None:
            self._init(cdf.device)
        self._err.zero_()
        call('encx_ac_decode', self._buf.data_ptr(), self._buf.numel(), self._nbytes.data_ptr(), 1,
             self._state.data_ptr(), cdf.data_ptr(), 1, cdf.numel(), self.total_range_bits,
             self._sym.data_ptr(), 0, 0, 0, 0, None, None, self._err.data_ptr(), stream())
        e = int(self._err.item())
        used = (int(self._state[0, ENCX_AC_POS].item()) + 7) // 8
        if hasattr(self.fo, 'seek'):
            self.fo.seek(self._start + used)
        if e == 1:
            return None
        if e == 2:
            raise RuntimeError("Binary search failed")
        if e:
            raise RuntimeError(f'encx arithmetic decoder failed ({e}): the stream is not one the '
                               'reference coder can have written')
        return int(self._sym.item())
