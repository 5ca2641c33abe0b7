"""Builders for the loader tests: AIFF / AIFF-C files and G.711 WAV files as
bytes, written field by field from the container specs (Apple AIFF 1.3 /
AIFF-C draft: FORM, COMM with an 80-bit extended rate, SSND with its offset
and block-size words; RIFF/WAVE fmt tags 6 A-law and 7 mu-law)."""
import math
import struct

import numpy as np


def ext80(rate):
    """IEEE 754 80-bit extended encoding of a positive integer rate."""
    e = int(math.floor(math.log2(rate)))
    mant = int(rate) << (63 - e)
    return struct.pack(">HQ", 16383 + e, mant)


def _chunk(cid, body):
    return cid + struct.pack(">I", len(body)) + body + (b"\0" if len(body) & 1 else b"")


def aiff(samples, channels, rate, bits, comp=None, ssnd_offset=0, extra_chunk=False,
         comm_frames=None):
    """FORM/AIFF (comp None) or FORM/AIFC with compression `comp` (bytes).
    `samples` is the already-encoded sample payload (bytes)."""
    width = {b"ulaw": 1, b"ULAW": 1, b"alaw": 1, b"ALAW": 1, b"fl32": 4, b"FL32": 4,
             b"fl64": 8, b"FL64": 8}.get(comp, bits // 8)
    frames = len(samples) // (channels * width) if comm_frames is None else comm_frames
    comm = struct.pack(">hIh", channels, frames, bits) + ext80(rate)
    kind = b"AIFF"
    if comp is not None:
        comm += comp + b"\x04none\x00"          # pascal name, padded to even
        kind = b"AIFC"
    body = kind
    if comp is not None:
        body += _chunk(b"FVER", struct.pack(">I", 0xA2805140))
    body += _chunk(b"COMM", comm)
    if extra_chunk:
        body += _chunk(b"NAME", b"odd")         # odd size: padded
    body += _chunk(b"SSND", struct.pack(">II", ssnd_offset, 0) + bytes(ssnd_offset) + samples)
    return b"FORM" + struct.pack(">I", len(body)) + body


def pcm_be(ints, bits):
    """Signed big-endian two's-complement bytes of `ints` at width bits/8."""
    v = np.asarray(ints, dtype=np.int64).reshape(-1)
    w = bits // 8
    u = v & ((1 << bits) - 1)
    return np.stack([(u >> (8 * (w - 1 - k))) & 0xFF for k in range(w)],
                    axis=1).astype(np.uint8).tobytes()


def pcm_le(ints, bits):
    w = bits // 8
    return np.frombuffer(pcm_be(ints, bits), dtype=np.uint8).reshape(-1, w)[:, ::-1].tobytes()


def wav_g711(codes, channels, rate, tag):
    """RIFF/WAVE with format tag 6 (A-law) or 7 (mu-law), 8 bits per sample."""
    fmt = struct.pack("<HHIIHH", tag, channels, rate, rate * channels, channels, 8)
    fmt += struct.pack("<H", 0)                 # cbSize, as non-PCM fmt chunks carry
    data = bytes(codes)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    body += b"fact" + struct.pack("<I", 4) + struct.pack("<I", len(data) // channels)
    body += b"data" + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")
    return b"RIFF" + struct.pack("<I", len(body)) + body


def cases(rng):
    """name -> (file bytes, frames, channels) covering every AIFF/G.711 layout
    the parser accepts."""
    out = {}
    for bits in (8, 16, 24, 32):
        ints = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (777, 2))
        out[f"aiff s{bits} stereo"] = (aiff(pcm_be(ints, bits), 2, 44100, bits), 777, 2)
        out[f"aifc sowt s{bits}"] = (aiff(pcm_le(ints, bits), 2, 48000, bits, b"sowt"), 777, 2)
    ints = rng.integers(-32768, 32768, 1001)
    out["aifc twos mono offset"] = (aiff(pcm_be(ints, 16), 1, 22050, 16, b"twos", ssnd_offset=6,
                                         extra_chunk=True), 1001, 1)
    out["aifc NONE 3ch"] = (aiff(pcm_be(rng.integers(-32768, 32768, 900), 16), 3, 96000, 16,
                                 b"NONE"), 300, 3)
    f32 = rng.uniform(-1.5, 1.5, (640, 2)).astype(">f4")
    out["aifc fl32"] = (aiff(f32.tobytes(), 2, 44100, 32, b"fl32"), 640, 2)
    f64 = rng.uniform(-0.8, 0.8, (500, 5)).astype(">f8")
    out["aifc FL64 5ch"] = (aiff(f64.tobytes(), 5, 8000, 64, b"FL64"), 500, 5)
    codes = rng.integers(0, 256, 1200, dtype=np.uint8).tobytes()
    for comp in (b"ulaw", b"alaw", b"ULAW", b"ALAW"):
        out[f"aifc {comp.decode()}"] = (aiff(codes, 2, 8000, 16, comp), 600, 2)
    for tag, name in ((6, "alaw"), (7, "ulaw")):
        out[f"wav {name} mono"] = (wav_g711(codes[:999], 1, 8000, tag), 999, 1)
        out[f"wav {name} stereo"] = (wav_g711(codes, 2, 11025, tag), 600, 2)
    # COMM frames below what SSND holds: the COMM count wins
    out["aiff short COMM"] = (aiff(pcm_be(rng.integers(-99, 99, 400), 16), 1, 44100, 16,
                                   comm_frames=350), 350, 1)
    return out
