"""Raw `.ecdc` container (binary.py of the reference) with the payload packed on the GPU.

Header: `ECDC` magic, uint8 version 0, uint32 json length (struct '!4sBI'), then the json
metadata (binary.py:13-52) -- a few host bytes, written and parsed here. The code payload is
where the work is: `BitPacker` / `BitUnpacker` keep the reference's names and stream semantics
(binary.py:55-123) but pack and unpack through the HIP kernels of csrc/bitstream.hip
(encx.ops.pack_codes / unpack_codes); there is no CPU packer in the product.
"""
import json
import struct
import typing as tp

import torch

from . import ops

_encodec_header_struct = struct.Struct('!4sBI')  # binary.py:19
_ENCODEC_MAGIC = b'ECDC'


def write_ecdc_header(fo: tp.IO[bytes], metadata: tp.Any):
    """binary.py:23-29."""
    meta_dumped = json.dumps(metadata).encode('utf-8')
    fo.write(_encodec_header_struct.pack(_ENCODEC_MAGIC, 0, len(meta_dumped)))
    fo.write(meta_dumped)
    fo.flush()


def _read_exactly(fo: tp.IO[bytes], size: int) -> bytes:
    """binary.py:32-41: EOFError when the stream ends first."""
    chunks = []
    while size > 0:
        buf = fo.read(size)
        if not buf:
            raise EOFError('Impossible to read enough data from the stream, '
                           f'{size} bytes remaining.')
        chunks.append(buf)
        size -= len(buf)
    return b''.join(chunks)


def read_ecdc_header(fo: tp.IO[bytes]):
    """binary.py:44-52."""
    magic, version, meta_size = _encodec_header_struct.unpack(
        _read_exactly(fo, _encodec_header_struct.size))
    if magic != _ENCODEC_MAGIC:
        raise ValueError('File is not in ECDC format.')
    if version != 0:
        raise ValueError('Version not supported.')
    return json.loads(_read_exactly(fo, meta_size).decode('utf-8'))


class BitPacker:
    """binary.py:55-88. Values pushed (ints or int64 tensors, in stream order) are gathered on
    the device; flush() packs them in one HIP launch and writes ceil(n*bits/8) bytes, the
    reference's exact byte stream (its push writes whole bytes eagerly, which only matters to
    a reader of `fo` before flush)."""

    def __init__(self, bits: int, fo: tp.IO[bytes], device='cuda'):
        self.bits = bits
        self.fo = fo
        self.device = torch.device(device)
        self._pending: tp.List[torch.Tensor] = []

    def push(self, value):
        if torch.is_tensor(value):
            self._pending.append(value.reshape(-1).to(self.device, torch.int64))
        else:
            self._pending.append(torch.tensor([int(value)], dtype=torch.int64, device=self.device))

    def push_frame(self, frame: torch.Tensor):
        """All codes of one frame [K][T] in the reference's order (t-major, compress.py:88-98)."""
        self._pending.append(frame.to(self.device, torch.int64).t().reshape(-1))

    def flush(self):
        if self._pending:
            vals = torch.cat(self._pending).view(1, 1, -1)
            self._pending = []
            data, err = ops.pack_codes(vals, self.bits)
            host = data.cpu()
            if int(err.item()):
                raise ValueError(f'BitPacker: a value does not fit in {self.bits} bits')
            self.fo.write(host.numpy().tobytes())
        self.fo.flush()


class BitUnpacker:
    """binary.py:91-123. pull_frame(K, T) reads exactly the bytes a flushed frame of K*T codes
    occupies and unpacks them in one HIP launch; pull() serves single values from the same
    path and returns None at the end of the stream. pull() reads ahead by whole blocks of
    lcm(bits, 8) bits (e.g. 5 bytes = 4 codes at 10 bits), so a caller mixing pull() with other
    reads of `fo` uses pull_frame instead, which consumes exactly the reference's bytes."""

    def __init__(self, bits: int, fo: tp.IO[bytes], device='cuda'):
        self.bits = bits
        self.fo = fo
        self.device = torch.device(device)
        self._buf: tp.List[int] = []

    def pull_frame(self, K: int, T: int) -> torch.Tensor:
        """-> int64 [K][T] on the device; EOFError if the stream is shorter (compress.py:137)."""
        nbytes = (K * T * self.bits + 7) // 8
        raw = self.fo.read(nbytes) if nbytes else b''
        if len(raw) < nbytes:
            raise EOFError('The stream ended sooner than expected.')
        if nbytes == 0:
            return torch.zeros(K, T, dtype=torch.int64, device=self.device)
        data = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device).view(1, -1)
        return ops.unpack_codes(data, K, T, self.bits)[0]

    def pull(self) -> tp.Optional[int]:
        if not self._buf:
            # the smallest whole-byte block that holds a whole number of values
            lcm_bits = self.bits * 8 // _gcd(self.bits, 8)
            raw = self.fo.read(lcm_bits // 8)
            n = len(raw) * 8 // self.bits
            if n == 0:
                return None
            data = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device).view(1, -1)
            self._buf = ops.unpack_codes(data, 1, n, self.bits).view(-1).tolist()[::-1]
        return self._buf.pop()


def _gcd(a, b):
    while b:
        a, b = b, a % b
    return a
