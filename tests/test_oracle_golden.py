"""Pins the CPU oracle (oracle/dsp_ref_cpu.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by tests/golden/make_golden.py from
the reference modules/dsp_core.py.  The oracle issues the same numpy/scipy calls,
so agreement is exact (bitwise), except where the fixture itself was composed
from reference primitives -- still exact.
"""
import numpy as np
import pytest

from conftest import golden, golden_gains
from oracle import dsp_ref_cpu as orc


def test_taps_exact():
    g = golden("taps")
    for i, (wc, k) in enumerate(g["cases"]):
        np.testing.assert_array_equal(orc.sinc_taps(wc, int(k)), g[f"h_{i}"])


def test_src_noise_exact():
    g = golden("src")
    for i, (L, M, K, N, fs) in enumerate(g["cases"]):
        x = g[f"x_{i}"]
        for c in range(x.shape[0]):
            y, fs_out = orc.resample(x[c], int(fs), int(M), int(L), None if K < 0 else int(K))
            np.testing.assert_array_equal(y, g[f"y_{i}"][c])
            assert fs_out == int(g[f"fs_{i}"])


def test_src_delta_exact():
    g = golden("src")
    for i, (L, M, K, N) in enumerate(g["delta_cases"]):
        x = g[f"dx_{i}"]
        for r in range(x.shape[0]):
            y, _ = orc.resample(x[r], 48000, int(M), int(L), None if K < 0 else int(K))
            np.testing.assert_array_equal(y, g[f"dy_{i}"][r])


def test_src_identity_returns_same_object():
    x = np.arange(5, dtype=np.float32)
    y, fs = orc.resample(x, 44100, 1, 1)
    assert y is x and fs == 44100


def test_biquad_exact():
    for row in golden("biquad")["rows"]:
        b, a = orc.peaking(row[0], row[1], row[2])
        np.testing.assert_array_equal(b, row[3:6])
        np.testing.assert_array_equal(a, row[6:9])


def test_eq_exact():
    g = golden("eq")
    i = 0
    while f"gains_{i}" in g:
        gains, fs = golden_gains(g[f"gains_{i}"]), int(g[f"fs_{i}"])
        for src, key in (("x64", "z64"), ("x32", "z32")):
            z = orc.equaliser(g[src], fs, gains)
            np.testing.assert_array_equal(np.asarray(z), g[f"{key}_{i}"])
        i += 1
    assert i == 10


def test_fft_exact():
    g = golden("fft")
    for k in range(13):
        for kind in ("r", "c"):
            np.testing.assert_array_equal(orc.fft_dit(g[f"x{kind}_{k}"]), g[f"X{kind}_{k}"])


def test_fft_large_matches_reference():
    """N = 2^13 .. 2^16 (fixtures stored as complex64): the restatement equals
    the reference's outputs to the fixture's rounding."""
    g = golden("fft_large")
    for k in (13, 14, 15, 16):
        kinds = ("r", "c") if k >= 15 else ("r",)
        for kind in kinds:
            x = g[f"x{kind}_{k}"].astype(np.complex128 if kind == "c" else np.float64)
            ref = g[f"X{kind}_{k}"]
            got = orc.fft_dit(x)
            assert np.max(np.abs(got - ref)) <= 1e-6 * np.max(np.abs(ref)), (k, kind)
    f, m = orc.spectrum(g["spec_x"].astype(np.float64), 72000, window=1 << 15)
    np.testing.assert_array_equal(f, g["spec_f"])
    assert np.max(np.abs(m - g["spec_m"])) <= 1e-6 * np.max(g["spec_m"])


def test_spectrum_exact():
    g = golden("spectrum")
    for i, n in enumerate(g["lengths"]):
        with np.errstate(invalid="ignore", divide="ignore"):
            f, m = orc.spectrum(g[f"x_{i}"], 44100)
        np.testing.assert_array_equal(f, g[f"f_{i}"])
        np.testing.assert_array_equal(m, g[f"m_{i}"])


def test_spectrum_raises_where_reference_raises():
    for n, raised in golden("spectrum")["raising"]:
        if raised:
            with pytest.raises(ValueError):
                orc.spectrum(np.ones(int(n)), 44100)


@pytest.mark.parametrize("tag,fs,L,M,K", [("c3", 48000, 3, 2, None),
                                          ("c5", 44100, 160, 147, 1023)])
def test_chain_exact(tag, fs, L, M, K):
    g = golden("chain")
    y, z, f, mag, fs_out = orc.chain(g[f"{tag}_x"], fs, L, M, orc.CONFIG3_GAINS, K, 4096)
    assert fs_out == int(g[f"{tag}_fs_out"])
    np.testing.assert_array_equal(y, g[f"{tag}_y"])
    np.testing.assert_array_equal(z, g[f"{tag}_z"])
    np.testing.assert_array_equal(mag, g[f"{tag}_mag"])
    np.testing.assert_array_equal(orc.spectrum(z, fs_out)[1], g[f"{tag}_mag2048"])


def test_oracle_g711_known_answers():
    """The oracle's G.711 expansion (audioop, the tables libsndfile uses) on the
    Sun g711.c end points: mu-law 0x00/0x80 -> -/+32124, 0x7F/0xFF -> 0; A-law
    0x55/0xD5 -> -/+8, 0x2A/0xAA -> -/+32256."""
    import audio_files
    from oracle import dsp_ref_cpu as orc
    x, fs = orc._g711_or_aiff(audio_files.wav_g711([0x00, 0x80, 0x7F, 0xFF], 1, 8000, 7))
    assert fs == 8000 and (x * 32768).tolist() == [-32124, 32124, 0, 0]
    x, _ = orc._g711_or_aiff(audio_files.wav_g711([0x55, 0xD5, 0x2A, 0xAA], 1, 8000, 6))
    assert (x * 32768).tolist() == [-8, 8, -32256, 32256]


def test_oracle_aiff_reader_matches_stdlib_aifc():
    """Pins the oracle's AIFF/AIFF-C reader on what Python's own aifc module
    decodes (big-endian PCM 8/16/24/32 and the AIFF-C G.711 codecs)."""
    import io
    import warnings

    import audio_files
    from oracle import dsp_ref_cpu as orc
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        import aifc
    rng = np.random.default_rng(9)
    for bits in (8, 16, 24, 32):
        ints = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (300, 2))
        f = audio_files.aiff(audio_files.pcm_be(ints, bits), 2, 44100, bits, extra_chunk=True)
        x, fs = orc._g711_or_aiff(f)
        r = aifc.open(io.BytesIO(f))
        assert (r.getnchannels(), r.getnframes(), r.getframerate()) == (2, 300, fs)
        raw = np.frombuffer(r.readframes(300), dtype=np.uint8).reshape(-1, bits // 8)
        v = np.zeros(raw.shape[0], dtype=np.int64)
        for k in range(bits // 8):
            v = (v << 8) | raw[:, k]
        v = np.where(v >= 1 << (bits - 1), v - (1 << bits), v)
        np.testing.assert_array_equal(v, ints.reshape(-1))
        np.testing.assert_array_equal(x.reshape(-1), v / float(1 << (bits - 1)))
    codes = rng.integers(0, 256, 400, dtype=np.uint8).tobytes()
    for comp in (b"ulaw", b"alaw"):
        f = audio_files.aiff(codes, 2, 8000, 16, comp)
        x, _ = orc._g711_or_aiff(f)
        r = aifc.open(io.BytesIO(f))
        lin = np.frombuffer(r.readframes(200), dtype="<i2")     # aifc expands to native order
        np.testing.assert_array_equal(x.reshape(-1), lin / 32768.0)
