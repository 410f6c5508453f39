"""compress.py of the reference: waveform <-> `.ecdc` bytes through the encx HIP path.

Encode (SEANet encoder + RVQ argmin) and decode (RVQ gather + SEANet decoder) run the encx
kernels; each frame's codes are packed / unpacked on the GPU (csrc/bitstream.hip) and only the
packed bytes cross PCIe. With use_lm=True the codes are arithmetic coded under the LM's
probabilities instead (compress.py:67-89, 128-155): encx.lm runs the LM and the coder on the
GPU (csrc/lm.hip, csrc/ac.hip). Byte format, metadata keys and error behaviour follow
compress.py:30-191.
"""
import io
import struct
import typing as tp

import torch

from . import binary, ops
from .model import EncodecModel, EncodedFrame

MODELS = {  # compress.py:21-26
    'encodec_24khz': EncodecModel.encodec_model_24khz,
    'encodec_48khz': EncodecModel.encodec_model_48khz,
    'my_encodec': EncodecModel.my_encodec_model,
    'encodec_bw': EncodecModel.encodec_model_bw,
}


def _model_device(model):
    return next(model.parameters()).device


def compress_to_file(model: EncodecModel, wav: torch.Tensor, fo: tp.IO[bytes], use_lm: bool = True):
    """compress.py:30-101: header, then per frame the '!f' scale (normalising models) and the
    frame's codes bit-packed t-major at model.bits_per_codebook bits, flushed per frame."""
    assert wav.dim() == 2, "Only single waveform can be encoded."
    if model.name not in MODELS:
        raise ValueError(f"The provided model {model.name} is not supported.")
    if use_lm:
        lm = model.get_lm_model()
    with torch.no_grad():
        frames = model.encode(wav[None].to(_model_device(model), torch.float32))
    metadata = {
        'm': model.name,
        'al': wav.shape[-1],
        'nc': frames[0][0].shape[1],
        'lm': use_lm,
        'fr': frames[0][0].shape[2],
    }
    binary.write_ecdc_header(fo, metadata)
    if use_lm:
        # compress.py:67-89: one arithmetic coded stream per frame, flushed per frame
        for frame, scale in frames:
            if scale is not None:
                fo.write(struct.pack('!f', scale.cpu().item()))
            fo.write(lm.encode_streams(frame.contiguous())[0])
        fo.flush()
        return
    # pack every frame on the device, then one copy of all payloads (and scales) to the host
    packed = [ops.pack_codes(frame, model.bits_per_codebook) for frame, _ in frames]
    scales = [s.reshape(-1)[:1] for _, s in frames if s is not None]
    host = [d.cpu() for d, _ in packed]
    if any(int(err.item()) for _, err in packed):
        raise ValueError(f'codes do not fit in {model.bits_per_codebook} bits')
    scales = torch.cat(scales).cpu().tolist() if scales else []
    si = 0
    for (frame, scale), data in zip(frames, host):
        if scale is not None:
            fo.write(struct.pack('!f', scales[si]))
            si += 1
        fo.write(data.numpy().tobytes())
    fo.flush()


def decompress_from_file(model: EncodecModel, fo: tp.IO[bytes], device='cpu') -> tp.Tuple[torch.Tensor, int]:
    """compress.py:104-162. Decoding runs on the model's GPU; the waveform comes back on the
    host, as the reference returns it for both of its devices (compress.py:158-161). As in the
    reference, every segment is read with the header's frame count `fr` (compress.py:126) and
    the model check looks at `model.name` (compress.py:118)."""
    metadata = binary.read_ecdc_header(fo)
    model_name = metadata['m']
    audio_length = metadata['al']
    num_codebooks = metadata['nc']
    use_lm = metadata['lm']
    assert isinstance(audio_length, int)
    assert isinstance(num_codebooks, int)
    if model.name not in MODELS:
        raise ValueError(f"The audio was compressed with an unsupported model {model_name}.")
    if use_lm:
        lm = model.get_lm_model()
    dev = _model_device(model)
    frames: tp.List[EncodedFrame] = []
    segment_stride = model.segment_stride or audio_length
    if use_lm:
        # compress.py:129-155: the rest of the file is read and uploaded ONCE; each segment's
        # decoder starts where the previous one stopped (the reference's decoder reads lazily
        # and stops there too), and a seekable file is left at that position at the end
        start = fo.tell() if hasattr(fo, 'tell') else 0
        rest = fo.read()
        rest_dev = torch.frombuffer(bytearray(rest or b'\0'), dtype=torch.uint8).to(dev)
        pos = 0
    for offset in range(0, audio_length, segment_stride):
        frame_length = metadata['fr']
        if model.normalize:
            if use_lm:
                if pos + 4 > len(rest):
                    raise EOFError('Impossible to read enough data from the stream, '
                                   f'{pos + 4 - len(rest)} bytes remaining.')
                scale_f, = struct.unpack('!f', rest[pos:pos + 4])
                pos += 4
            else:
                scale_f, = struct.unpack('!f', binary._read_exactly(fo, struct.calcsize('!f')))
            scale = torch.tensor(scale_f, device=dev).view(1)
        else:
            scale = None
        if use_lm:
            codes, used = lm.decode_streams(None, num_codebooks, frame_length,
                                            dev_span=(rest_dev, pos, len(rest) - pos))
            pos += used[0]
            frames.append((codes, scale))
            continue
        unpacker = binary.BitUnpacker(model.bits_per_codebook, fo, device=dev)
        frames.append((unpacker.pull_frame(num_codebooks, frame_length)[None], scale))
    if use_lm and hasattr(fo, 'seek'):
        fo.seek(start + pos)
    with torch.no_grad():
        wav = model.decode(frames)
    return wav[0, :, :audio_length].cpu(), model.sample_rate


def compress(model: EncodecModel, wav: torch.Tensor, use_lm: bool = False) -> bytes:
    """compress.py:165-179."""
    fo = io.BytesIO()
    compress_to_file(model, wav, fo, use_lm=use_lm)
    return fo.getvalue()


def decompress(model: EncodecModel, compressed: bytes, device='cuda') -> tp.Tuple[torch.Tensor, int]:
    """compress.py:182-191."""
    return decompress_from_file(model, io.BytesIO(compressed), device=device)


def compress_batch(model: EncodecModel, wavs: torch.Tensor) -> tp.List[bytes]:
    """Serving form of `compress(model, wavs[i], use_lm=False)` for a batch [B][C][T] of
    equal-length clips: one encode over the batch, one pack launch per segment for all B
    streams, one device->host copy; each element is a complete `.ecdc` file."""
    assert wavs.dim() == 3, "expects [B, C, T]"
    if model.name not in MODELS:
        raise ValueError(f"The provided model {model.name} is not supported.")
    B = wavs.shape[0]
    with torch.no_grad():
        frames = model.encode(wavs.to(_model_device(model), torch.float32))
    bits = model.bits_per_codebook
    packed = [ops.pack_codes(frame, bits) for frame, _ in frames]
    datas = [d.cpu().numpy() for d, _ in packed]
    if any(int(err.item()) for _, err in packed):
        raise ValueError(f'codes do not fit in {bits} bits')
    scales = [s.reshape(B).cpu().tolist() if s is not None else None for _, s in frames]
    out = []
    for b in range(B):
        fo = io.BytesIO()
        binary.write_ecdc_header(fo, {'m': model.name, 'al': wavs.shape[-1],
                                      'nc': frames[0][0].shape[1], 'lm': False,
                                      'fr': frames[0][0].shape[2]})
        for data, sc in zip(datas, scales):
            if sc is not None:
                fo.write(struct.pack('!f', sc[b]))
            fo.write(data[b].tobytes())
        out.append(fo.getvalue())
    return out
