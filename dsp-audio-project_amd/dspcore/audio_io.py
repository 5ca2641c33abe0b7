"""Audio I/O edges of the hot path on the GPU.

Loader (reference modules/dsp_core.py:10-35, cargar_senal_audio): the host
parses the header only (dsp_audio_parse: RIFF/WAVE with PCM, IEEE float and
G.711 A-law/mu-law, FORM/AIFF and AIFF-C with big- or little-endian PCM,
'fl32'/'fl64' and G.711); the raw sample bytes go to the device as they are
and libdspcore decodes, averages the channels and peak-normalises there
(dsp_pcm_to_mono_f32, dsp_peak_normalize_f32), with the reference's arithmetic
(soundfile's float64 scaling, numpy's channel mean, float32 cast, float32
division by the peak when it exceeds 1e-6).  Other containers (FLAC, Ogg, ...)
are decoded by soundfile on the host when it is installed (it is not in this
image) and take the same device path as float64 samples.

Playback (reference app.py:349-355): dsp_quantize_pcm16 turns the chain's z
into 16-bit PCM on the device (nan_to_num, / max|z|, * 32767, truncation) and
dsp_wav_header_pcm16 writes scipy.io.wavfile.write's 44-byte header.
"""
from __future__ import annotations

import ctypes
import io
import os

import numpy as np
import torch

from . import _lib, ops

NORMALISE_THRESHOLD = 1e-6      # dsp_core.py:31


def read_bytes(source) -> bytes:
    """The whole file behind a path, a file-like object or a bytes object."""
    if isinstance(source, (bytes, bytearray, memoryview)):
        return bytes(source)
    if isinstance(source, (str, os.PathLike)):
        with open(source, "rb") as f:
            return f.read()
    if hasattr(source, "read"):
        if hasattr(source, "seek"):
            try:
                source.seek(0)
            except (OSError, ValueError):
                pass
        return source.read()
    raise TypeError(f"cannot read audio from {type(source).__name__}")


def parse_wav(data: bytes) -> _lib.WavInfo:
    """RIFF/WAVE header of an in-memory file (dsp_wav_parse, host only)."""
    info = _lib.WavInfo()
    rc = _lib.load().dsp_wav_parse(data, len(data), ctypes.byref(info))
    _lib.check(rc, "dsp_wav_parse")
    return info


def parse_audio(data: bytes) -> _lib.WavInfo:
    """RIFF/WAVE or FORM/AIFF(-C) header (dsp_audio_parse, host only)."""
    info = _lib.WavInfo()
    rc = _lib.load().dsp_audio_parse(data, len(data), ctypes.byref(info))
    _lib.check(rc, "dsp_audio_parse")
    return info


def _decode_other(data: bytes) -> tuple[np.ndarray, int]:
    """Other containers: soundfile's host decoder, as the reference (float64)."""
    try:
        import soundfile as sf
    except ImportError as e:
        raise ValueError("not a WAV/AIFF file and soundfile is not installed") from e
    x, fs = sf.read(io.BytesIO(data))
    return np.ascontiguousarray(x, dtype=np.float64), int(fs)


def pcm_to_mono(pcm: torch.Tensor, fmt: int, bits: int, channels: int, frames: int,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """Raw interleaved sample bytes (uint8 device tensor [B, >= frames*channels*bits/8])
    -> float32 mono [B, frames], bit-identical to soundfile + mean + astype."""
    if pcm.dim() == 1:
        pcm = pcm.unsqueeze(0)
    B = pcm.shape[0]
    if out is None:
        out = torch.empty((B, frames), dtype=torch.float32, device=pcm.device)
    lib = _lib.load()
    with torch.cuda.device(pcm.device):
        rc = lib.dsp_pcm_to_mono_f32(pcm.data_ptr(), fmt, bits, channels, B, frames,
                                     pcm.stride(0) if B > 1 else pcm.shape[1], out.data_ptr(),
                                     ops.ld(out), ops._stream(pcm.device))
    _lib.check(rc, "dsp_pcm_to_mono_f32")
    return out


def peak_normalize(x: torch.Tensor, threshold: float = NORMALISE_THRESHOLD,
                   n: int | None = None) -> torch.Tensor:
    """In place, per row: x /= max|x| where (double)max|x| > threshold.  Returns
    the float32 peaks [B] (the values the rows were divided by, or not)."""
    if x.dim() == 1:
        x = x.unsqueeze(0)
    B, width = x.shape
    n = width if n is None else int(n)
    peaks = torch.empty(max(B, 1), dtype=torch.int32, device=x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_peak_normalize_f32(x.data_ptr(), B, n, ops.ld(x), float(threshold),
                                        peaks.data_ptr(), ops._stream(x.device))
    _lib.check(rc, "dsp_peak_normalize_f32")
    return peaks[:B].view(torch.float32)


def load(source, device: torch.device | str | None = None) -> tuple[torch.Tensor, int]:
    """cargar_senal_audio's result as a device tensor: (float32 [n], fs)."""
    ops.require_gpu()
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    data = read_bytes(source)
    try:
        info = parse_audio(data)
    except ValueError:
        host, fs = _decode_other(data)
        ch = 1 if host.ndim == 1 else host.shape[1]
        frames = host.shape[0]
        pcm = torch.from_numpy(host.reshape(-1).view(np.uint8)).to(dev)
        x = pcm_to_mono(pcm, _lib.DSP_WAV_FLOAT, 64, ch, frames)
    else:
        fs = info.sample_rate
        frames = info.frames
        nbytes = frames * info.channels * (info.bits // 8)
        raw = np.frombuffer(data, dtype=np.uint8, count=nbytes, offset=info.data_offset)
        pcm = torch.from_numpy(raw.copy()).to(dev)
        x = pcm_to_mono(pcm, info.format, info.bits, info.channels, frames)
    if x.shape[1] == 0:
        raise ValueError("empty audio")   # np.max of an empty array raises in the reference
    peak_normalize(x)
    return x[0], fs


def _raw_rows(datas):
    """(descriptors, raw byte pieces, rates) of in-memory files: headers parsed
    on the host (dsp_audio_parse), the sample bytes as they are; other
    containers decoded by soundfile to float64 (DSP_WAV_FLOAT, 64 bits)."""
    rows, pieces, rates = [], [], []
    for data in datas:
        try:
            info = parse_audio(data)
        except ValueError:
            host, fs = _decode_other(data)
            ch = 1 if host.ndim == 1 else host.shape[1]
            raw = host.reshape(-1).view(np.uint8)
            rows.append((host.shape[0], _lib.DSP_WAV_FLOAT, 64, ch))
        else:
            fs = info.sample_rate
            nbytes = info.frames * info.channels * (info.bits // 8)
            raw = np.frombuffer(data, dtype=np.uint8, count=nbytes, offset=info.data_offset)
            rows.append((info.frames, info.format, info.bits, info.channels))
        pieces.append(raw)
        rates.append(int(fs))
    return rows, pieces, rates


def load_batch(sources, device: torch.device | str | None = None):
    """Several files -> (float32 [B, max_n] zero-padded device batch, lengths, rates),
    each row exactly what cargar_senal_audio returns for that file.

    Headers are parsed on the host; every file's raw sample bytes go to the
    device in ONE host-to-device copy (concatenated, 16-byte aligned pieces,
    from pinned memory), and dsp_pcm_batch_to_mono_f32 decodes, averages,
    zero-pads and peak-normalises the whole batch in two launches."""
    ops.require_gpu()
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    datas = [read_bytes(s) for s in sources]
    B = len(datas)
    if B == 0:
        return torch.zeros((0, 0), dtype=torch.float32, device=dev), [], []
    rows, pieces, rates = _raw_rows(datas)
    lengths = [r[0] for r in rows]
    if min(lengths) == 0:
        raise ValueError("empty audio")   # np.max of an empty array raises in the reference
    width = max(lengths)
    desc = (_lib.PcmRow * B)()
    off = 0
    for b, ((frames, fmt, bits, ch), raw) in enumerate(zip(rows, pieces)):
        desc[b].offset, desc[b].frames = off, frames
        desc[b].format, desc[b].bits, desc[b].channels = fmt, bits, ch
        off += (raw.size + 15) & ~15
    total = max(off, 16)
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    for b, raw in enumerate(pieces):
        hv[desc[b].offset:desc[b].offset + raw.size] = raw
    lib = _lib.load()
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev)
        pcm = host.to(dev, non_blocking=True)
        out = torch.empty((B, width), dtype=torch.float32, device=dev)
        peaks = torch.empty(B, dtype=torch.int32, device=dev)
        ws = torch.empty(int(lib.dsp_pcm_batch_workspace_bytes(B, width)) + 256,
                         dtype=torch.uint8, device=dev)
        wsp = (ws.data_ptr() + 255) & ~255
        rc = lib.dsp_pcm_batch_to_mono_f32(pcm.data_ptr(), total, ctypes.addressof(desc), B,
                                           width, out.data_ptr(), ops.ld(out),
                                           NORMALISE_THRESHOLD, peaks.data_ptr(), wsp,
                                           ws.numel() - (wsp - ws.data_ptr()),
                                           ops._stream(dev))
        _lib.check(rc, "dsp_pcm_batch_to_mono_f32")
        # the descriptor table (host) and the staging buffer outlive their use
        stream.synchronize()
    return out, lengths, rates


def quantize_pcm16(z: torch.Tensor, precision: int = 64) -> torch.Tensor:
    """app.py:349-355 on the device: int16 [B, n] from float32 z [B, n].

    precision: the dtype the app's z_final has, whose arithmetic the
    quantiser reproduces -- 64 (float64: z_final came out of
    conversion_tasa_muestreo or sistema_ecualizador) or 32 (float32: both were
    bypassed and z_final is the loader's float32 array)."""
    squeeze = z.dim() == 1
    if squeeze:
        z = z.unsqueeze(0)
    if z.dtype != torch.float32:
        z = z.float()
    z = z.contiguous()
    B, n = z.shape
    out = torch.empty((B, n), dtype=torch.int16, device=z.device)
    peaks = torch.empty(max(B, 1), dtype=torch.int32, device=z.device)
    lib = _lib.load()
    with torch.cuda.device(z.device):
        rc = lib.dsp_quantize_pcm16(z.data_ptr(), out.data_ptr(), B, n, ops.ld(z), ops.ld(out),
                                    peaks.data_ptr(), int(precision), ops._stream(z.device))
    _lib.check(rc, "dsp_quantize_pcm16")
    return out[0] if squeeze else out


def wav_bytes_pcm16(z: torch.Tensor, fs: int, precision: int = 64) -> bytes:
    """The WAV file app.py:352 writes for z (scipy.io.wavfile.write of int16);
    precision as in quantize_pcm16."""
    pcm = quantize_pcm16(z if z.dim() == 1 else z[0], precision).cpu().numpy()
    header = ctypes.create_string_buffer(44)
    rc = _lib.load().dsp_wav_header_pcm16(header, int(fs), 1, pcm.size)
    _lib.check(rc, "dsp_wav_header_pcm16")
    return header.raw + pcm.astype("<i2").tobytes()
