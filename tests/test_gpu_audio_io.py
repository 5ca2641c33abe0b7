"""Loader and playback edges on the GPU, bitwise
against the oracle's restatement of dsp_core.py:10-35 and app.py:349-355."""
import io
import struct

import numpy as np
import pytest
import torch
from scipy.io import wavfile

pytestmark = pytest.mark.gpu


def _wavfile(x, rate):
    buf = io.BytesIO()
    wavfile.write(buf, rate, x)
    return buf.getvalue()


def _wav24(ints, channels, rate):
    """24-bit PCM (scipy cannot write it): little-endian 3-byte samples."""
    v = np.asarray(ints, dtype=np.int32).reshape(-1)
    b = np.stack([(v >> s) & 0xFF for s in (0, 8, 16)], axis=1).astype(np.uint8).tobytes()
    block = 3 * channels
    fmt = struct.pack("<HHIIHH", 1, channels, rate, rate * block, block, 24)
    body = b"WAVEfmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(b)) + b
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _oracle_24(ints, channels):
    x = np.asarray(ints, dtype=np.float64).reshape(-1, channels) / 8388608.0
    x = x.mean(axis=1) if channels > 1 else x[:, 0]
    x = x.astype(np.float32)
    peak = np.max(np.abs(x))
    return x / peak if peak > 1e-6 else x


def test_loader_matches_reference_bitwise(gpu):
    from modules import dsp_core
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(5)
    cases = {
        "int16 stereo": rng.integers(-32768, 32767, (4001, 2), dtype=np.int16),
        "int16 mono": rng.integers(-9000, 9000, 3000, dtype=np.int16),
        "uint8 stereo": rng.integers(0, 255, (2000, 2), dtype=np.uint8),
        "int32 mono": rng.integers(-2**31, 2**31 - 1, 1500, dtype=np.int32),
        "float32 stereo": rng.uniform(-0.7, 0.7, (2500, 2)).astype(np.float32),
        "float64 5ch": rng.uniform(-2, 2, (1200, 5)),
        "float32 10ch": rng.uniform(-1, 1, (700, 10)).astype(np.float32),
        "silence": np.zeros((500, 2), dtype=np.int16),
        "tiny": (rng.uniform(-1, 1, 600) * 1e-7).astype(np.float32),
    }
    for name, arr in cases.items():
        data = _wavfile(arr, 44100)
        x, fs = dsp_core.cargar_senal_audio(io.BytesIO(data))
        ref, rfs = orc.load_audio(data)
        assert fs == rfs and x.dtype == np.float32 and x.shape == ref.shape, name
        np.testing.assert_array_equal(x, ref, err_msg=name)
    ints = rng.integers(-2**23, 2**23 - 1, (900, 2))
    x, fs = dsp_core.cargar_senal_audio(_wav24(ints, 2, 48000))
    np.testing.assert_array_equal(x, _oracle_24(ints, 2))
    # unreadable input: the reference's fallback
    x, fs = dsp_core.cargar_senal_audio(io.BytesIO(b"not audio at all"))
    assert fs == 44100 and x.dtype == np.float32 and np.array_equal(x, np.zeros(100))


def test_loader_batch_rows_equal_single_loads(gpu):
    from dspcore import audio_io
    rng = np.random.default_rng(6)
    files = [_wavfile(rng.integers(-30000, 30000, (n, 2), dtype=np.int16), 48000)
             for n in (1000, 2500, 1777)]
    batch, lengths, rates = audio_io.load_batch(files, gpu)
    assert lengths == [1000, 2500, 1777] and rates == [48000] * 3
    for i, f in enumerate(files):
        one, _ = audio_io.load(f, gpu)
        assert torch.equal(batch[i, :lengths[i]], one)
        assert not batch[i, lengths[i]:].any()


def _mixed_files(rng):
    """64 files of every layout the loader decodes: WAV PCM 8/16/24/32-bit and
    IEEE float 32/64 (1-6 channels, lengths 1..5000), every AIFF / AIFF-C /
    G.711 case of audio_files, silence and a sub-threshold file."""
    import audio_files
    files = [f for f, _, _ in audio_files.cases(rng).values()]
    gens = [
        lambda n, c: rng.integers(0, 255, (n, c), dtype=np.uint8),
        lambda n, c: rng.integers(-32768, 32767, (n, c), dtype=np.int16),
        lambda n, c: rng.integers(-2**31, 2**31 - 1, (n, c), dtype=np.int32),
        lambda n, c: rng.uniform(-1.3, 1.3, (n, c)).astype(np.float32),
        lambda n, c: rng.uniform(-2, 2, (n, c)),
    ]
    k = 0
    while len(files) < 60:
        n, c = int(rng.integers(1, 5000)), int(rng.integers(1, 7))
        files.append(_wavfile(gens[k % len(gens)](n, c), int(rng.choice([8000, 44100, 48000]))))
        k += 1
    files.append(_wav24(rng.integers(-2**23, 2**23 - 1, (1234, 3)), 3, 96000))
    files.append(_wav24(rng.integers(-2**23, 2**23 - 1, 17), 1, 22050))
    files.append(_wavfile(np.zeros((321, 2), dtype=np.int16), 44100))
    files.append(_wavfile((rng.uniform(-1, 1, 999) * 1e-7).astype(np.float32), 44100))
    return files


def test_loader_batch_64_mixed_files_two_launches(gpu):
    """load_batch of 64 mixed-format files: one host-to-device copy, then
    dsp_pcm_batch_to_mono_f32's two launches (decode + mean + zero padding,
    normalise); every row bitwise the per-file load() (the single-file
    kernels) and the oracle's cargar_senal_audio, zeros past its length."""
    from dspcore import _lib, audio_io
    from oracle import dsp_ref_cpu as orc
    files = _mixed_files(np.random.default_rng(64))
    assert len(files) == 64
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        batch, lengths, rates = audio_io.load_batch(files, gpu)
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    assert names == ["pcm_batch", "pcm_batch_scale"]
    assert batch.shape == (64, max(lengths))
    got = batch.cpu().numpy()
    for i, f in enumerate(files):
        ref, rfs = orc.load_audio(f)
        assert rates[i] == rfs and lengths[i] == ref.size, i
        np.testing.assert_array_equal(got[i, :lengths[i]], ref, err_msg=str(i))
        assert not got[i, lengths[i]:].any(), i
        one, _ = audio_io.load(f, gpu)
        assert torch.equal(batch[i, :lengths[i]], one), i


def test_loader_batch_rejects_bad_descriptors(gpu):
    """dsp_pcm_batch_to_mono_f32 validates the host descriptor table: samples
    outside the buffer, frames past the width, an unknown format."""
    import ctypes
    from dspcore import _lib
    lib = _lib.load()
    pcm = torch.zeros(64, dtype=torch.uint8, device=gpu)
    out = torch.empty((1, 16), dtype=torch.float32, device=gpu)
    peaks = torch.empty(1, dtype=torch.int32, device=gpu)
    ws = torch.empty(4096, dtype=torch.uint8, device=gpu)
    for frames, fmt, bits, off in ((16, 1, 16, 40), (17, 1, 8, 0), (4, 5, 16, 0), (4, 1, 12, 0)):
        d = (_lib.PcmRow * 1)()
        d[0].offset, d[0].frames, d[0].format, d[0].bits, d[0].channels = off, frames, fmt, bits, 1
        rc = lib.dsp_pcm_batch_to_mono_f32(pcm.data_ptr(), 64, ctypes.addressof(d), 1, 16,
                                           out.data_ptr(), 16, 1e-6, peaks.data_ptr(),
                                           ws.data_ptr(), ws.numel(), None)
        assert rc == -1, (frames, fmt, bits, off, rc)


def test_peak_normalize_nan_and_threshold(gpu):
    from dspcore import audio_io
    x = torch.tensor([[0.5, -2.0, 1.0], [float("nan"), 3.0, 1.0], [1e-7, -5e-7, 0.0]],
                     device=gpu)
    peaks = audio_io.peak_normalize(x)
    assert peaks[0].item() == 2.0 and torch.isnan(peaks[1])
    assert x[0].tolist() == [0.25, -1.0, 0.5]
    assert x[1, 1].item() == 3.0 and x[2, 1].item() == np.float32(-5e-7)  # unchanged


def test_playback_quantization_matches_app_bitwise(gpu):
    """app.py:349-355 bitwise, in both dtypes z_final can have: float64 (after
    the SRC or the EQ) and float32 (both bypassed: the loader's array).  The
    data has samples where the two dtypes round to different int16 values, so
    each mode is checked against its own restatement."""
    from dspcore import audio_io
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(8)
    z = rng.uniform(-1, 1, (4, 200000)).astype(np.float32)
    z[1, 10] = np.nan
    z[2, :] = 0.0
    z[3, 7] = np.inf
    z[3, 8] = -np.inf
    zt = torch.from_numpy(z).to(gpu)
    q64 = audio_io.quantize_pcm16(zt).cpu().numpy()
    q32 = audio_io.quantize_pcm16(zt, precision=32).cpu().numpy()
    differ = 0
    for b in range(4):
        r64 = orc.playback_pcm16(z[b].astype(np.float64))
        r32 = orc.playback_pcm16(z[b])
        np.testing.assert_array_equal(q64[b], r64)
        np.testing.assert_array_equal(q32[b], r32)
        differ += int(np.count_nonzero(r64 != r32))
    assert differ > 0          # the two modes are distinguishable on this data
    wav = audio_io.wav_bytes_pcm16(torch.from_numpy(z[0]).to(gpu), 72000)
    buf = io.BytesIO()
    wavfile.write(buf, 72000, orc.playback_pcm16(z[0].astype(np.float64)))
    assert wav == buf.getvalue()
    with pytest.raises(ValueError):
        audio_io.quantize_pcm16(zt, precision=16)


@pytest.mark.gpu
def test_batches_past_the_grid_row_limit(gpu):
    """Batches of more than 65535 rows (the grid's y extent) run as
    consecutive row ranges: quantize and peak-normalise every row of a
    70000-row batch, rows on both sides of the split equal to the oracle."""
    from dspcore import audio_io
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(70)
    B, n = 70000, 16
    z = (rng.uniform(-1, 1, (B, n)) * rng.uniform(0.5, 4.0, (B, 1))).astype(np.float32)
    zt = torch.from_numpy(z).to(gpu)
    q = audio_io.quantize_pcm16(zt).cpu().numpy()
    for b in (0, 65534, 65535, 65536, B - 1):
        np.testing.assert_array_equal(q[b], orc.playback_pcm16(z[b].astype(np.float64)))
    xt = zt.clone()
    peaks = audio_io.peak_normalize(xt).cpu().numpy()
    np.testing.assert_array_equal(peaks, np.max(np.abs(z), axis=1))
    x = xt.cpu().numpy()
    for b in (0, 65535, 65536, B - 1):
        np.testing.assert_array_equal(x[b], z[b] / np.max(np.abs(z[b])))


def test_loader_aiff_and_g711_bitwise(gpu):
    """AIFF / AIFF-C (big- and little-endian PCM 8-32, fl32/fl64, G.711) and
    WAV G.711 decode on the device bitwise equal to the oracle (libsndfile's
    scaling restated; parity unpinned against soundfile itself, which is not
    installed -- the oracle's reader is pinned on stdlib aifc and the Sun
    G.711 end points in test_oracle_golden.py)."""
    import audio_files
    from modules import dsp_core
    from oracle import dsp_ref_cpu as orc
    for name, (f, frames, ch) in audio_files.cases(np.random.default_rng(12)).items():
        x, fs = dsp_core.cargar_senal_audio(io.BytesIO(f))
        ref, rfs = orc.load_audio(f)
        assert fs == rfs and x.dtype == np.float32 and x.shape == (frames,) == ref.shape, name
        np.testing.assert_array_equal(x, ref, err_msg=name)
