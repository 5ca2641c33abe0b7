"""Parity of the HIP path (through the C-ABI) with the reference.

Expected values come from the reference's own outputs (tests/golden/*.npz) or,
at sizes with no fixture, from the CPU oracle, which tests/test_oracle_golden.py
pins bitwise to those fixtures.  Tolerances (measured in the
survey container):
  * SRC: float32 taps and accumulation -> atol 2e-6; index mapping and output
    length bit-exact (delta inputs reproduce float32(L*h[k]) exactly);
  * EQ: float64 coefficients and state, float32 I/O -> atol 1e-5;
  * FFT: float32 with float64-computed twiddles -> max|dX| <= 1e-5 * max|X|;
  * chain spectrum: the FFT tolerance, max|dmag| <= 1e-5 * max|mag| (observed
    3.5e-7 on the smoke case; round 2 allowed 1e-4).
"""
import contextlib

import numpy as np
import pytest
import torch

from conftest import golden, golden_gains

pytestmark = pytest.mark.gpu

SRC_ATOL = 2e-6
EQ_ATOL = 1e-5
FFT_RTOL = 1e-5
CHAIN_MAG_RTOL = 1e-5


def _dc():
    from modules import dsp_core
    return dsp_core


@contextlib.contextmanager
def _chain_path(path):
    """Path of dsp_chain_f32 on this thread (dsp_chain_path): 0 single-pass
    kernel where it applies, 1 always the two-launch chain."""
    from dspcore import _lib
    prev = _lib.chain_path(path)
    try:
        yield
    finally:
        _lib.chain_path(prev)


def _traced(fn):
    """(results cloned, names of the kernels the library launched)."""
    from dspcore import _lib
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        out = tuple(t.clone() for t in fn())
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    return out, names


def _ops():
    from dspcore import ops
    return ops


# --------------------------------------------------------------------------- SRC
def test_src_noise_matches_reference(gpu):
    from dspcore import design
    g = golden("src")
    for i, (L, M, K, N, fs) in enumerate(g["cases"]):
        plan = design.src_plan(int(N), int(fs), int(M), int(L), None if K < 0 else int(K))
        x = torch.from_numpy(g[f"x_{i}"]).to(gpu)
        y = _ops().src_polyphase(x, plan).cpu().numpy()
        ref = g[f"y_{i}"]
        assert y.shape == ref.shape, (i, y.shape, ref.shape)
        err = np.max(np.abs(y - ref))
        assert err <= SRC_ATOL, f"case {i} (L={L}, M={M}, K={K}): max err {err:.3g}"


def test_src_delta_is_bit_exact(gpu):
    from dspcore import design
    g = golden("src")
    for i, (L, M, K, N) in enumerate(g["delta_cases"]):
        plan = design.src_plan(int(N), 48000, int(M), int(L), None if K < 0 else int(K))
        x = torch.from_numpy(g[f"dx_{i}"]).to(gpu)
        y = _ops().src_polyphase(x, plan).cpu().numpy()
        # bitwise the reference's float32(L*h[k]) at every position but the
        # sinc-zero noise taps the library flushes (include/dspcore.h, ABI 2.1):
        # there y is 0 and the reference's value is float64 rounding noise, <= 2e-16 of the peak
        ref = g[f"dy_{i}"]
        want = ref.astype(np.float32)
        flushed = np.zeros(ref.shape, bool)
        if plan.L > 1:
            flushed = (np.abs(want) <= design.TAP_FLUSH_REL * np.max(np.abs(want))) & (ref != 0)
            assert np.all(y[flushed] == 0.0), i
            assert np.max(np.abs(ref[flushed]), initial=0.0) <= 2e-16 * np.max(np.abs(ref)), i
        np.testing.assert_array_equal(y[~flushed], want[~flushed])


def test_src_drop_in_dtypes_and_identity(gpu):
    dc = _dc()
    g = golden("src")
    x = g["x_0"][0]
    y, fs = dc.conversion_tasa_muestreo(x, 48000, 2, 3)
    assert y.dtype == np.float64 and fs == 72000
    assert np.max(np.abs(y - g["y_0"][0])) <= SRC_ATOL
    same, fs1 = dc.conversion_tasa_muestreo(x, 48000, 1, 1)
    assert same is x and fs1 == 48000
    # keyword-only tap override (configs 2 and 5)
    y255, _ = dc.conversion_tasa_muestreo(g["x_1"][0], 48000, 2, 3, num_taps=255)
    assert np.max(np.abs(y255 - g["y_1"][0])) <= SRC_ATOL
    # batched numpy and device tensors
    yb, _ = dc.conversion_tasa_muestreo(g["x_0"], 48000, 2, 3)
    assert yb.shape == g["y_0"].shape and np.max(np.abs(yb - g["y_0"])) <= SRC_ATOL
    yt, _ = dc.conversion_tasa_muestreo(torch.from_numpy(x).to(gpu), 48000, 2, 3)
    assert yt.is_cuda and yt.dtype == torch.float32


def test_config2_full_length(gpu):
    """BASELINE config 2 at its stated size: 1 channel x 48000 samples, 255-tap
    FIR, L = 3 / M = 2, SRC only, through the drop-in against the oracle."""
    from oracle import dsp_ref_cpu as orc
    dc = _dc()
    rng = np.random.default_rng(22)
    x = rng.uniform(-1, 1, 48000).astype(np.float32)
    y, fs_out = dc.conversion_tasa_muestreo(x, 48000, 2, 3, num_taps=255)
    ry, rfs = orc.resample(x, 48000, 2, 3, 255)
    assert fs_out == rfs == 72000 and y.shape == ry.shape == (72000,)
    assert np.max(np.abs(y - ry)) <= SRC_ATOL


def test_src_misaligned_rows_and_long_taps(gpu):
    from dspcore import design
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(5)
    # odd leading dimension (no float4 path) and the generic kernel (K = 6401)
    for (L, M, K, N) in ((3, 2, None, 1001), (160, 147, None, 300), (7, 5, 289, 777)):
        x = rng.uniform(-1, 1, (3, N)).astype(np.float32)
        buf = torch.zeros((3, N + 1), dtype=torch.float32, device=gpu)
        buf[:, :N] = torch.from_numpy(x).to(gpu)
        plan = design.src_plan(N, 48000, M, L, K)
        y = _ops().src_polyphase(buf[:, :N], plan).cpu().numpy()
        for c in range(3):
            ref, _ = orc.resample(x[c], 48000, M, L, K)
            assert np.max(np.abs(y[c] - ref)) <= SRC_ATOL


# --------------------------------------------------------------------------- EQ
def test_eq_matches_reference(gpu):
    dc = _dc()
    g = golden("eq")
    for i in range(10):
        gains, fs = golden_gains(g[f"gains_{i}"]), int(g[f"fs_{i}"])
        for src, key in (("x64", "z64"), ("x32", "z32")):
            x = g[src]
            z = dc.sistema_ecualizador(x, fs, gains)
            ref = g[f"{key}_{i}"]
            if all(abs(v) < 0.1 for v in gains.values()):
                assert z is x, f"case {i}: bypass must return the input object"
                continue
            assert z.dtype == ref.dtype, (i, src, z.dtype, ref.dtype)
            err = np.max(np.abs(z - ref))
            assert err <= EQ_ATOL, f"case {i} {src}: max err {err:.3g}"


def test_single_biquad_matches_lfilter(gpu):
    import scipy.signal
    dc = _dc()
    x = np.random.default_rng(1).uniform(-1, 1, 5000)
    for fc, g in ((40, 15), (10000, -15), (3000, 6)):
        b, a = dc.disenar_coeficientes_diferencias(fc, 72000, g)
        y = dc.aplicar_ecuacion_diferencias(x, b, a)
        assert y.dtype == np.float64
        assert np.max(np.abs(y - scipy.signal.lfilter(b, a, x))) <= EQ_ATOL


def test_difference_equation_any_order_matches_lfilter(gpu):
    """aplicar_ecuacion_diferencias for any (b, a), as lfilter takes them
    (reference dsp_core.py:214): orders 1-8 (Butterworth, Chebyshev, elliptic,
    random stable), orders 36 and 48 (18 and 24 sections: two cascade
    launches), b longer than a, a[0] != 1, FIRs, a pure gain -- within
    1e-5 of scipy.signal.lfilter (relative to max|y| when that exceeds 1), 1-D
    numpy in -> float64 out, 2-D batches per row."""
    import scipy.signal
    from test_host_logic import _high_order_cases, _lfilter_cases
    dc = _dc()
    x = np.random.default_rng(5).uniform(-1, 1, (2, 20000))
    for name, b, a in _lfilter_cases() + _high_order_cases():
        ref = scipy.signal.lfilter(b, a, x[0])
        y = dc.aplicar_ecuacion_diferencias(x[0], b, a)
        assert y.dtype == np.float64 and y.shape == ref.shape
        err = np.max(np.abs(y - ref))
        assert err <= EQ_ATOL * max(1.0, np.max(np.abs(ref))), (name, err)
        yb = dc.aplicar_ecuacion_diferencias(x, b, a)
        np.testing.assert_array_equal(yb[0], y)
    with pytest.raises(ValueError):
        dc.aplicar_ecuacion_diferencias(x[0], [1.0], [0.0, 1.0])


def test_eq_chunk_carry_is_exact_to_rounding(gpu):
    """Every scan variant vs one chunk per channel (a plain serial recursion),
    at config-3 length: fused kernel with / without the state-response table,
    and the general three-launch path (282 chunks)."""
    from dspcore import design
    ops = _ops()
    rng = np.random.default_rng(2)
    x = torch.from_numpy(rng.uniform(-0.9, 0.9, (6, 72000)).astype(np.float32)).to(gpu)
    sos = design.eq_plan(72000, {"Sub-Bass": 15, "Bass": -15, "Low Mids": 12,
                                 "High Mids": -12, "Presence": 9, "Brilliance": -9}).sos
    z_one = ops.biquad_cascade(x, sos, True, chunk_len=72000 + 32 - 72000 % 32).cpu().numpy()
    variants = {
        "fused+table (4 waves, 250 chunks)": dict(),
        "fused (4 waves, 250 chunks)": dict(use_table=False),
        "fused+table, 1 wave, 63 chunks": dict(chunk_len=1152),
        "fused, 36 chunks": dict(chunk_len=2048),
        "fused 4 waves, 141 chunks": dict(chunk_len=512),
        "fused 2 waves, 125 chunks": dict(chunk_len=576),
        "general, 282 chunks": dict(chunk_len=256),
    }
    for name, kw in variants.items():
        z = ops.biquad_cascade(x, sos, True, **kw).cpu().numpy()
        assert np.max(np.abs(z - z_one)) <= 1e-6, name


def test_eq_many_stages_general_path(gpu):
    """S = 9 (padded to 12: general three-launch path) and S = 7 (padded to 8:
    fused kernel without the state table)."""
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(8)
    y = rng.uniform(-1, 1, (2, 30000))
    for gains in ({f"b{i}": (-1) ** i * (3 + i) for i in range(9)},
                  {**{k: 4 for k in orc.CONFIG3_GAINS}, "extra": -5}):
        z = _dc().sistema_ecualizador(y, 72000, gains)
        for c in range(2):
            assert np.max(np.abs(z[c] - orc.equaliser(y[c], 72000, gains))) <= EQ_ATOL


def test_eq_full_length_matches_oracle(gpu):
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(3)
    y = rng.uniform(-1, 1, (3, 72000))
    z = _dc().sistema_ecualizador(y, 72000, orc.CONFIG3_GAINS)
    for c in range(3):
        ref = orc.equaliser(y[c], 72000, orc.CONFIG3_GAINS)
        assert np.max(np.abs(z[c] - ref)) <= EQ_ATOL


def test_eq_rows_independent_of_batch(gpu):
    """Bitwise: a row's output does not depend on the batch it runs in."""
    from dspcore import design
    ops = _ops()
    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.uniform(-1, 1, (9, 20000)).astype(np.float32)).to(gpu)
    sos = design.eq_plan(72000, {"Sub-Bass": 6, "Bass": -4}).sos
    full = ops.biquad_cascade(x, sos, True).cpu().numpy()
    for lo, hi in ((0, 1), (1, 4), (4, 9)):
        part = ops.biquad_cascade(x[lo:hi].contiguous(), sos, True).cpu().numpy()
        np.testing.assert_array_equal(part, full[lo:hi])


# --------------------------------------------------------------------------- FFT
def test_fft_matches_reference(gpu):
    dc = _dc()
    g = golden("fft")
    for k in range(13):
        for kind in ("r", "c"):
            x, ref = g[f"x{kind}_{k}"], g[f"X{kind}_{k}"]
            X = dc.fft_diezmado_en_tiempo(x)
            if k == 0:
                assert X is x
                continue
            assert X.dtype == np.complex128 and X.shape == ref.shape
            err = np.max(np.abs(X - ref))
            assert err <= FFT_RTOL * np.max(np.abs(ref)), f"N=2^{k} {kind}: {err:.3g}"


def test_fft_large_and_batched(gpu):
    ops = _ops()
    rng = np.random.default_rng(6)
    for lg in (13, 14):
        x = rng.uniform(-1, 1, (3, 1 << lg)) + 1j * rng.uniform(-1, 1, (3, 1 << lg))
        X = ops.fft(torch.from_numpy(x.astype(np.complex64)).to(gpu)).cpu().numpy()
        ref = np.fft.fft(x, axis=1)
        assert np.max(np.abs(X - ref)) <= FFT_RTOL * np.max(np.abs(ref))


def test_any_length_dft_matches_numpy(gpu):
    """The app-side transform (app.py:322-324: np.fft.fft of int(1024*L/M)-sample
    segments) for any length: max|dX| <= 1e-5 * max|X| against np.fft.fft,
    real and complex rows, batched; powers of two go to the radix-2 kernel."""
    rng = np.random.default_rng(21)
    for n in (1, 2, 3, 5, 7, 100, 1000, 1114, 1536, 2047, 4096, 8191):
        for real in (True, False):
            x = rng.uniform(-1, 1, (3, n))
            if not real:
                x = x + 1j * rng.uniform(-1, 1, (3, n))
            xt = torch.from_numpy(x.astype(np.float32 if real else np.complex64)).to(gpu)
            got = _ops().dft(xt).cpu().numpy()
            ref = np.fft.fft(x.astype(np.float32 if real else np.complex64).astype(
                np.complex128), axis=1)
            err = np.max(np.abs(got - ref), axis=1)
            assert np.all(err <= FFT_RTOL * np.max(np.abs(ref), axis=1)), (n, real, err)
    with pytest.raises(ValueError):
        _ops().dft(torch.zeros((1, 9000), device=gpu))


def test_fft_rejects_non_power_of_two(gpu):
    with pytest.raises(ValueError):
        _dc().fft_diezmado_en_tiempo(np.ones(12))
    with pytest.raises(ValueError):
        _dc().fft_diezmado_en_tiempo(np.ones(3))


# --------------------------------------------------------------------------- spectrum
def test_spectrum_matches_reference(gpu):
    dc = _dc()
    g = golden("spectrum")
    for i, n in enumerate(g["lengths"]):
        f, m = dc.calcular_espectro_magnitud(g[f"x_{i}"], 44100)
        np.testing.assert_array_equal(f, g[f"f_{i}"])
        ref = g[f"m_{i}"]
        assert m.dtype == np.float64 and m.shape == ref.shape
        if n == 1:
            assert np.isnan(m).all() and np.isnan(ref).all()
            continue
        err = np.max(np.abs(m - ref))
        assert err <= FFT_RTOL * np.max(ref), f"len {n}: {err:.3g}"
    for n, raised in g["raising"]:
        if raised:
            with pytest.raises(ValueError):
                dc.calcular_espectro_magnitud(np.ones(int(n)), 44100)


def test_spectrum_4096_large_batch_bitwise_small_batch(gpu):
    """The 4096-point spectrum kernel (k_spec_wave12, a persistent grid of
    one transform per wave at a time) over a batch ~10x its resident waves:
    the large batch's rows are bitwise the same rows computed in a small
    batch, and within FFT_RTOL of float64 numpy (Hann of dsp_core.py:87,
    |rfft|) -- on an unaligned segment start."""
    B, n, start = 20000, 4196, 37
    g = torch.Generator(device=gpu).manual_seed(5)
    x = torch.rand((B, n), device=gpu, generator=g) * 2 - 1
    big = _ops().spectrum(x, start, 4096, 4096)
    rows = [0, 1, 4999, 12345, B - 1]
    small = _ops().spectrum(x[rows].contiguous(), start, 4096, 4096)
    assert torch.equal(big[rows], small)
    k = np.arange(4096)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * k / 4095)
    seg = x[rows, start:start + 4096].double().cpu().numpy()
    ref = np.abs(np.fft.rfft(seg * w, axis=1))
    got = small.cpu().numpy()
    assert np.max(np.abs(got - ref), axis=1).max() <= FFT_RTOL * ref.max()


def test_stft_frames_match_reference_recipe(gpu):
    """Every frame of the spectrogram extension equals the reference's spectrum
    recipe (Hann, radix-2 FFT, |X|) on that frame: max|d| <= 1e-5 * max|X|
    per frame; ragged last frame zero-padded; one frame when n < n_fft."""
    from oracle import dsp_ref_cpu as orc
    dc = _dc()
    rng = np.random.default_rng(11)
    for n, n_fft, hop in [(10000, 1024, 256), (4096, 4096, 1000), (3000, 4096, 512),
                          (9999, 256, 100), (72000, 2048, 512), (9001, 4096, 777)]:
        x = rng.uniform(-1, 1, (2, n))
        f, times, mag = dc.calcular_espectrograma_magnitud(x, 72000, n_fft=n_fft, hop=hop)
        frames = 1 + -(-max(0, n - n_fft) // hop)
        assert mag.shape == (2, frames, n_fft // 2 + 1) and mag.dtype == np.float64
        assert f.shape == (n_fft // 2 + 1,) and times.shape == (frames,)
        for b in range(2):
            ref = orc.spectrogram(x[b].astype(np.float32).astype(np.float64), n_fft, hop, frames)
            err = np.max(np.abs(mag[b] - ref), axis=1)
            assert np.all(err <= FFT_RTOL * np.maximum(np.max(ref, axis=1), 1e-30)), (n, n_fft)
    # frames == 1 on the centre segment is the spectrum kernel itself
    x = rng.uniform(-1, 1, (1, 72000)).astype(np.float32)
    xt = torch.from_numpy(x).to(gpu)
    one = _ops().stft_magnitude(xt[:, 36000:36000 + 4096].contiguous(), 4096, 4096, 1)
    spec = _ops().spectrum(xt, 36000, 4096, 4096)
    assert torch.equal(one[:, 0], spec)


# --------------------------------------------------------------------------- chain
@pytest.mark.parametrize("tag,fs,L,M,K", [("c3", 48000, 3, 2, None),
                                          ("c5", 44100, 160, 147, 1023)])
def test_chain_matches_reference(gpu, tag, fs, L, M, K):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    g = golden("chain")
    cfg = ChainConfig(48000, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, 1, gpu)
    x = torch.from_numpy(g[f"{tag}_x"][None, :]).to(gpu)
    y, z, mag = (t.cpu().numpy()[0] for t in ch.run(x))
    assert ch.fs_out == int(g[f"{tag}_fs_out"])
    assert np.max(np.abs(y - g[f"{tag}_y"])) <= SRC_ATOL
    assert np.max(np.abs(z - g[f"{tag}_z"])) <= EQ_ATOL
    ref = g[f"{tag}_mag"]
    assert np.max(np.abs(mag - ref)) <= CHAIN_MAG_RTOL * np.max(ref)
    # the staged path (one ABI call per stage): y bitwise; z within rounding of
    # the chain call, whose chunk states come from other chunkings (the
    # single-pass kernel's 48-sample sub-chunks, or x-domain states)
    y2, z2, m2 = (t.cpu().numpy()[0] for t in ch.run_stages(x))
    np.testing.assert_array_equal(y2, y)
    assert np.max(np.abs(z2 - z)) <= 2e-6
    assert np.max(np.abs(m2 - mag)) <= 1e-5 * np.max(mag)
    if ch.xstate:
        # and the two-launch chain without x-domain states gives the staged bits
        ch2 = Chain(cfg, 1, gpu, use_xstate=False, chunk_len=ch.chunk_len)
        with _chain_path(1):
            y3, z3, m3 = (t.cpu().numpy()[0] for t in ch2.run(x))
        np.testing.assert_array_equal(z3, z2)
        np.testing.assert_array_equal(m3, m2)


def test_chain_config3_full_batch(gpu):
    """Config 3 at full size (4096 x 48000): spot channels vs the oracle, and
    every row bitwise equal to its single-row computation for a few rows."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B = 4096
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, B, gpu)
    gen = torch.Generator(device=gpu).manual_seed(0)
    x = torch.rand((B, 48000), generator=gen, device=gpu) * 2 - 1
    y, z, mag = ch.run(x)
    torch.cuda.synchronize()
    assert torch.isfinite(z).all() and torch.isfinite(mag).all()
    assert float(z.abs().max()) <= 1.0
    # same chunking and single-pass mode (plan_batch: the batch's chained tiles,
    # not one row's three-launch mode): bitwise rows
    one = Chain(cfg, 1, gpu, chunk_len=ch.chunk_len, plan_batch=B)
    for b in (0, 1234, B - 1):
        xb = x[b].cpu().numpy()
        ry, rz, _, rmag, _ = orc.chain(xb.astype(np.float32), 48000, 3, 2, orc.CONFIG3_GAINS,
                                       None, 4096)
        assert np.max(np.abs(y[b].cpu().numpy() - ry)) <= SRC_ATOL
        assert np.max(np.abs(z[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b].cpu().numpy() - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)
        y1, z1, m1 = one.run(x[b:b + 1].contiguous())
        assert torch.equal(y1[0], y[b]) and torch.equal(z1[0], z[b]) and torch.equal(m1[0], mag[b])


def test_app_call_sequence_drop_in(gpu):
    """app.py:164-167 then :203-205 through the drop-in module."""
    dc = _dc()
    g = golden("chain")
    x = g["c3_x"]
    gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3,
             "Presence": 5, "Brilliance": -6}
    y, fs_out = dc.conversion_tasa_muestreo(x, 48000, 2, 3)
    z = dc.sistema_ecualizador(y, fs_out, gains)
    assert fs_out == 72000
    assert np.max(np.abs(z - g["c3_z"])) <= EQ_ATOL
    f, m = dc.calcular_espectro_magnitud(z[:100000], fs_out)
    ref = g["c3_mag2048"]
    assert f.shape == ref.shape
    assert np.max(np.abs(m - ref)) <= CHAIN_MAG_RTOL * np.max(ref)


def test_shard_driver_bitwise_invariant(gpu):
    """Sharding the batch over 1, 2, 4 or 8 'devices' (here repeated cuda:0,
    one host thread each) gives bitwise the same result."""
    from dspcore.chain import Chain, ChainConfig
    from dspcore.shard import run_sharded
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, (16, 48000)).astype(np.float32)
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)

    def fn(xd):
        ch = Chain(cfg, xd.shape[0], xd.device)
        y, z, mag = ch.run(xd)
        return z.clone(), mag.clone()

    base = run_sharded(fn, x, [gpu])
    for parts in (2, 4, 8):
        got = run_sharded(fn, x, [gpu] * parts)
        for a, b in zip(got, base):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n_in,tile", [(48000, True), (4800, True), (96, True), (6144, True),
                                       (47996, True), (100, True), (47999, False)])
def test_chain_single_pass_matches_two_launch(gpu, n_in, tile):
    """The single-pass chain kernel (csrc/chain_tile.hip) against the
    two-launch chain on the same batch: it is the kernel that ran exactly where
    dsp_chain_tile_len says so (n_out a multiple of 4: one tile, whole tiles,
    a ragged last tile; n_out not a multiple of 4: the per-phase kernel of
    csrc/chain_pp.h; n_in not a multiple of 4: the two-launch chain), y is
    bitwise the SRC kernel's, z within float64 rounding of the two-launch z
    (other chunking of the same recursion), |X| likewise; rows against the
    reference recipe; the tile hand-off never gave up."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B = 6
    n_fft = 4096 if n_in >= 10000 else 2048 if n_in >= 2000 else 64
    cfg = ChainConfig(n_in, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu)
    assert (ch.tile_len > 0) == tile
    gen = torch.Generator(device=gpu).manual_seed(3)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[1] *= 40.0                      # drive the clip
    x[2, : n_in // 2] = 0.0           # silence then signal
    (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    with _chain_path(1):
        (y0, z0, m0), names0 = _traced(lambda: ch.run(x))
    assert ("chain_tile" in names1 and "src_poly" not in names1) == tile, names1
    assert "chain_tile" not in names0 and "src_poly" in names0, names0
    assert ch.handoff_ok()
    assert torch.equal(y1, y0)
    assert (z1 - z0).abs().max().item() <= 2e-6
    assert (m1 - m0).abs().max().item() <= 1e-5 * m0.abs().max().item()
    y, z, mag = (t.cpu().numpy() for t in (y1, z1, m1))
    assert np.abs(z[1]).max() == 1.0
    for b in (0, 1, 2, 5):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, 3, 2, orc.CONFIG3_GAINS,
                                       None, cfg.n_fft)
        assert np.max(np.abs(y[b] - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)


@pytest.mark.parametrize("n_in,fs,L,M,K,B", [(48000, 44100, 160, 147, 1023, 6),
                                             (4800, 44100, 160, 147, 1023, 3),
                                             (9000, 48000, 5, 4, 31, 5),
                                             (6600, 48000, 2, 3, 15, 9),
                                             (4000, 48000, 7, 3, 55, 4)])
def test_chain_generic_single_pass(gpu, n_in, fs, L, M, K, B):
    """The generic single-pass kernel (k_chain_gen: run-time L/M, ceil(K/L) <=
    8, e.g. config 5's 160/147 with K = 1023) against the two-launch chain:
    it ran where dsp_chain_tile_len says so, y bitwise the generic SRC kernel's
    (same summation order), z within float64 rounding, odd n_out (ragged float4
    at the row end), batches that leave waves of the last workgroup idle,
    up- and down-sampling; rows against the reference recipe."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    n_fft = 4096 if n_in >= 10000 else 2048
    cfg = ChainConfig(n_in, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 32
    gen = torch.Generator(device=gpu).manual_seed(11)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[1] *= 40.0                      # drive the clip
    x[2, : n_in // 2] = 0.0           # silence then signal
    (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    with _chain_path(1):
        (y0, z0, m0), names0 = _traced(lambda: ch.run(x))
    assert "chain_tile" in names1 and "src_poly" not in names1, names1
    assert "chain_tile" not in names0, names0
    assert ch.handoff_ok()
    assert torch.equal(y1, y0)
    assert (z1 - z0).abs().max().item() <= 2e-6
    assert (m1 - m0).abs().max().item() <= 1e-5 * m0.abs().max().item()
    y, z, mag = (t.cpu().numpy() for t in (y1, z1, m1))
    assert np.abs(z[1]).max() == 1.0
    for b in (0, 1, 2, B - 1):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), fs, L, M, orc.CONFIG3_GAINS, K, n_fft)
        assert np.max(np.abs(y[b] - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)
    # more than 8 taps per branch: the two-launch chain serves the call
    assert Chain(ChainConfig(n_in, fs, L, M, 17 * L, orc.CONFIG3_GAINS, n_fft=n_fft), 1,
                 gpu).tile_len == 0


def test_chain_two_launch_48k_to_44k1(gpu):
    """48 kHz -> 44.1 kHz (L/M = 147/160, K = 1023): 147 phase classes of the
    32-output sub-chunks are more than the single-pass kernels' LDS tables
    hold, so no single-pass SRC kernel serves it: Chain runs the SRC kernel,
    then the single-pass cascade alone on y; its rows against the library's
    two-launch chain and the reference recipe (dsp_core.py:133-173, 216-254,
    68-98), clip driven."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in = 3, 9600
    cfg = ChainConfig(n_in, 48000, 147, 160, 1023, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 0
    gen = torch.Generator(device=gpu).manual_seed(147)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[1] *= 40.0
    # the SRC kernel, then the single-pass cascade alone on y (Chain's route
    # for geometries without a single-pass SRC kernel), against the library's
    # two-launch chain: y bitwise, z within 2e-6
    (y, z, mag), names = _traced(lambda: ch.run(x))
    assert "src_poly" in names and "chain_tile" in names, names
    with _chain_path(1):
        (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    assert "chain_tile" not in names1, names1
    assert torch.equal(y, y1) and (z - z1).abs().max().item() <= 2e-6
    assert (mag - m1).abs().max().item() <= 1e-5 * m1.abs().max().item()
    y, z, mag = (t.cpu().numpy() for t in (y, z, mag))
    for b in range(B):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, 147, 160, orc.CONFIG3_GAINS,
                                       1023, 2048)
        assert y.shape[1] == ry.size and z.shape[1] == rz.size
        assert np.max(np.abs(y[b] - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)


@pytest.mark.parametrize("B,n_in", [(1, 48000), (5, 48000), (9, 12000), (16, 4800)])
def test_chain_config5_persistent_bitwise_chained(gpu, B, n_in):
    """Config 5's ratio (160/147, K = 1023) through the persistent single-pass
    kernel (dsp_chain_path(3): a workgroup walks channel groups, each wave runs
    its channel's tiles in order with the entry state in registers and the next
    window in flight) and through the chained-tile kernel (dsp_chain_path(2)):
    y, z and |X| bitwise equal (same tile code on the same entry states), for
    partial channel groups and ragged last tiles; both match the oracle."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    n_fft = 4096 if n_in >= 10000 else 2048
    cfg = ChainConfig(n_in, 44100, 160, 147, 1023, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 32
    gen = torch.Generator(device=gpu).manual_seed(21)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[B - 1] *= 30.0                   # drive the clip
    with _chain_path(3):
        (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    with _chain_path(2):
        (y0, z0, m0), names0 = _traced(lambda: ch.run(x))
    assert "chain_tile" in names1 and "chain_tile" in names0, (names1, names0)
    assert ch.handoff_ok()
    assert torch.equal(y1, y0) and torch.equal(z1, z0) and torch.equal(m1, m0)
    y, z, mag = (t.cpu().numpy() for t in (y1, z1, m1))
    for b in sorted({0, B - 1}):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 44100, 160, 147, orc.CONFIG3_GAINS,
                                       1023, n_fft)
        assert np.max(np.abs(y[b] - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)


@pytest.mark.parametrize("gains", [{"Sub-Bass": 6, "Bass": 0.0, "Presence": -3, "Otra": 4},
                                   {"Sub-Bass": 0, "Bass": 0.05}])
def test_chain_single_pass_fewer_bands_and_bypass(gpu, gains):
    """Fewer than six bands run through the single-pass kernel padded with
    exact identity stages; an all-bypass EQ (sistema_ecualizador returns its
    input, dsp_core.py:222-223) gives z == y bitwise with no clip -- through
    the two-launch chain (round 6: S = 0 takes no single-pass kernel; its copy
    pass is cheaper, and it keeps the bypass's local inf / NaN)."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(48000, 48000, 3, 2, None, gains, n_fft=4096)
    ch = Chain(cfg, 3, gpu)
    assert (ch.tile_len > 0) == (ch.eq.sos.shape[0] > 0)
    gen = torch.Generator(device=gpu).manual_seed(5)
    x = (torch.rand((3, 48000), generator=gen, device=gpu) * 2 - 1) * 3.0
    (y, z, mag), names = _traced(lambda: ch.run(x))
    assert ("chain_tile" in names) == (ch.eq.sos.shape[0] > 0), names
    if ch.eq.bypass:
        assert torch.equal(y, z) and z.abs().max().item() > 1.0
    for b in range(3):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, 3, 2, gains, None, 4096)
        assert np.max(np.abs(y[b].cpu().numpy() - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b].cpu().numpy() - rz)) <= EQ_ATOL * max(1.0, np.abs(rz).max())
        assert np.max(np.abs(mag[b].cpu().numpy() - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)


def test_chain_unaligned_input_rows_fall_back_to_y_states(gpu):
    """x rows that are not 16-byte aligned (n_in % 4 != 0) cannot feed the
    x-domain chunk states nor the single-pass SRC kernels.  The library's
    two-launch chain (dsp_chain_path(1)) then uses the y-domain table (the
    contract in include/dspcore.h) instead of failing, bitwise equal to the
    staged path; the default (Chain: the SRC kernel, then the single-pass
    cascade alone on y) has the same y and z within 2e-6 of it; both match
    the reference recipe."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    n_in = 47999
    cfg = ChainConfig(n_in, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, 3, gpu)
    gen = torch.Generator(device=gpu).manual_seed(13)
    x = torch.rand((3, n_in), generator=gen, device=gpu) * 2 - 1
    assert ch.tile_len == 0           # n_in % 4 != 0: no single-pass SRC kernel
    with _chain_path(1):
        (y, z, mag), names1 = _traced(lambda: ch.run(x))
    assert "src_poly" in names1 and "chain_tile" not in names1, names1
    y2, z2, m2 = ch.run_stages(x)
    assert torch.equal(y, y2) and torch.equal(z, z2) and torch.equal(mag, m2)
    (y3, z3, m3), names = _traced(lambda: ch.run(x))
    assert "src_poly" in names and "chain_tile" in names, names
    assert ch.handoff_ok()
    assert torch.equal(y3, y) and (z3 - z).abs().max().item() <= 2e-6
    for b in range(3):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, 3, 2, orc.CONFIG3_GAINS,
                                       None, 4096)
        assert np.max(np.abs(z[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b].cpu().numpy() - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)


def _all_rows_match_two_launch(ch, x):
    """Every row of a single-pass run against the two-launch chain (SRC kernel +
    two-pass cascade, dsp_chain_path(1)) on the same input: y bitwise, z within
    2e-6 (include/dspcore.h), |Z| within the spectrum tolerance -- the whole
    batch, not sampled rows."""
    y, z, mag = (t.clone() for t in ch.run(x))
    with _chain_path(1):
        y2, z2, m2 = ch.run(x)
    torch.cuda.synchronize()
    assert torch.equal(y2, y)
    assert float((z2 - z).abs().max()) <= 2e-6
    assert float((m2 - mag).abs().max()) <= CHAIN_MAG_RTOL * float(mag.abs().max())
    del y, z, mag


def test_chain_config4_one_gpu_and_shards(gpu):
    """Config 4 on one GPU (32768 x 48000: 2.36e9 output elements, row offsets
    past 2^31): every row against the two-launch chain, 16 rows (incl. row
    32767) against the oracle, and the last shard of the 2-, 4- and 8-GPU splits (16384 / 8192 / 4096 channels,
    bench.py's per-rank batches) bitwise equal to the full run's rows."""
    from dspcore.chain import Chain, ChainConfig
    from dspcore.shard import shard_ranges
    from oracle import dsp_ref_cpu as orc
    B = 32768
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len > 0
    gen = torch.Generator(device=gpu).manual_seed(4)
    x = torch.rand((B, 48000), generator=gen, device=gpu) * 2 - 1
    y, z, mag = ch.run(x)
    torch.cuda.synchronize()
    assert ch.handoff_ok()
    assert float(z.abs().max()) <= 1.0 and torch.isfinite(mag).all()
    rows = sorted({0, 16383, 16384, 32767} | set(np.random.default_rng(44).integers(0, B, 12)))
    for b in rows:
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, 3, 2, orc.CONFIG3_GAINS,
                                       None, 4096)
        assert np.max(np.abs(y[b].cpu().numpy() - ry)) <= SRC_ATOL
        assert np.max(np.abs(z[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b].cpu().numpy() - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)
    for parts in (2, 4, 8):
        lo, hi = shard_ranges(B, parts)[-1]
        sh = Chain(cfg, hi - lo, gpu, plan_batch=B)
        ys, zs, ms = sh.run(x[lo:hi])
        assert torch.equal(ys, y[lo:hi]) and torch.equal(zs, z[lo:hi]) and torch.equal(ms, mag[lo:hi])
        assert sh.handoff_ok()
        del sh, ys, zs, ms
    del y, z, mag
    _all_rows_match_two_launch(ch, x)


def test_chain_config5_full_batch_and_shards(gpu):
    """Config 5 at full size on one GPU (8192 x 48000 at 44.1 kHz, L/M =
    160/147, K = 1023: the generic single-pass kernel): every row against the
    two-launch chain, 16 rows against the oracle on both sides of the 2-way
    split, and the last shard of the 2-, 4-
    and 8-GPU splits (4096 / 2048 / 1024 channels) bitwise equal to the full
    run's rows (the kernel's arithmetic depends on L, M, K only)."""
    from dspcore.chain import Chain, ChainConfig
    from dspcore.shard import shard_ranges
    from oracle import dsp_ref_cpu as orc
    B = 8192
    cfg = ChainConfig(48000, 44100, 160, 147, 1023, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 32
    gen = torch.Generator(device=gpu).manual_seed(5)
    x = torch.rand((B, 48000), generator=gen, device=gpu) * 2 - 1
    y, z, mag = ch.run(x)
    torch.cuda.synchronize()
    assert ch.handoff_ok()
    assert float(z.abs().max()) <= 1.0 and torch.isfinite(mag).all()
    rows = sorted({0, 4095, 4096, B - 1} | set(np.random.default_rng(55).integers(0, B, 12)))
    for b in rows:
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 44100, 160, 147, orc.CONFIG3_GAINS,
                                       1023, 4096)
        assert np.max(np.abs(y[b].cpu().numpy() - ry)) <= SRC_ATOL
        assert np.max(np.abs(z[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b].cpu().numpy() - rmag)) <= CHAIN_MAG_RTOL * np.max(rmag)
    for parts in (2, 4, 8):
        lo, hi = shard_ranges(B, parts)[-1]
        sh = Chain(cfg, hi - lo, gpu, plan_batch=B)
        ys, zs, ms = sh.run(x[lo:hi])
        assert torch.equal(ys, y[lo:hi]) and torch.equal(zs, z[lo:hi]) and torch.equal(ms, mag[lo:hi])
        assert sh.handoff_ok()
        del sh, ys, zs, ms
    del y, z, mag
    _all_rows_match_two_launch(ch, x)


def test_drop_in_shards_large_batches(gpu, monkeypatch):
    """The drop-in's 2-D numpy calls from SHARD_MIN_ROWS rows run on every
    visible GPU (here four shards on the one card): SRC, EQ (chunk length
    planned for the whole batch), lfilter, FFT and spectrum rows bitwise the
    one-device results; below the threshold nothing is sharded."""
    dc = _dc()
    rng = np.random.default_rng(31)
    B = dc.SHARD_MIN_ROWS + 3
    x = rng.uniform(-0.9, 0.9, (B, 4800)).astype(np.float32)
    gains = {"Sub-Bass": 6, "Bass": -3, "Low Mids": 2, "High Mids": 0, "Presence": 4,
             "Brilliance": -6}

    def calls():
        y, fs = dc.conversion_tasa_muestreo(x, 48000, 2, 3)
        z = dc.sistema_ecualizador(y, fs, gains)
        w = dc.aplicar_ecuacion_diferencias(x, [0.2, 0.3, 0.1], [1.0, -0.5, 0.25])
        X = dc.fft_diezmado_en_tiempo(x[:, :4096])
        _, m = dc.calcular_espectro_magnitud(z, fs)
        return y, z, w, X, m

    monkeypatch.setattr(dc, "_shard_devices", lambda: [gpu])
    one = calls()
    monkeypatch.setattr(dc, "_shard_devices", lambda: [gpu] * 4)
    four = calls()
    for a, b in zip(one, four):
        assert a.dtype == b.dtype and a.shape == b.shape
        np.testing.assert_array_equal(a, b)
    # a sharded call never takes the one-device route (_to_rows); a smaller one does
    got = []
    orig = dc._to_rows
    monkeypatch.setattr(dc, "_to_rows", lambda *a, **k: got.append(1) or orig(*a, **k))
    dc.conversion_tasa_muestreo(x, 48000, 2, 3)
    assert not got
    dc.conversion_tasa_muestreo(x[:dc.SHARD_MIN_ROWS - 1], 48000, 2, 3)
    assert got


def test_drop_in_sharding_stays_on_a_ranks_device(gpu, monkeypatch):
    """_shard_devices: every visible GPU in a single-process program on device
    0; none (the call stays on the current device) once torch.distributed is
    initialised, as in one rank of a multi-process job; DSPCORE_SHARD=0 / 1
    overrides either way."""
    import torch.distributed as tdist
    dc = _dc()
    monkeypatch.delenv("DSPCORE_SHARD", raising=False)
    assert len(dc._shard_devices()) == torch.cuda.device_count()
    monkeypatch.setattr(tdist, "is_initialized", lambda: True)
    assert dc._shard_devices() == []
    monkeypatch.setenv("DSPCORE_SHARD", "1")
    assert len(dc._shard_devices()) == torch.cuda.device_count()
    monkeypatch.setenv("DSPCORE_SHARD", "0")
    monkeypatch.setattr(tdist, "is_initialized", lambda: False)
    assert dc._shard_devices() == []


def test_shards_plan_with_the_job_batch(gpu):
    """Two-launch geometry (config 5's L/M = 160/147), 4096 rows: planned with
    the job's batch (Chain(plan_batch=4096)) every shard of 1, 2 and 4 runs the
    unsharded chunking and the rows are bitwise equal although the per-shard
    batches (2048, 1024) straddle design.WIDE_BATCH; planned per shard they
    agree to float64 rounding."""
    from dspcore.chain import Chain, ChainConfig
    from dspcore.shard import run_sharded
    from oracle import dsp_ref_cpu as orc
    B, n_in = 4096, 4800
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, (B, n_in)).astype(np.float32)
    cfg = ChainConfig(n_in, 44100, 160, 147, 1023, orc.CONFIG3_GAINS, n_fft=2048)

    def fn(plan):
        def run(xd):
            ch = Chain(cfg, xd.shape[0], xd.device, plan_batch=plan)
            with _chain_path(1):          # the two-launch chain (its chunking is planned)
                y, z, mag = ch.run(xd)
            return z.clone(), mag.clone()
        return run

    base = run_sharded(fn(B), x, [gpu])
    for parts in (2, 4):
        got = run_sharded(fn(B), x, [gpu] * parts)
        for a, b in zip(got, base):
            np.testing.assert_array_equal(a, b)
    own = run_sharded(fn(None), x, [gpu] * 4)
    assert np.max(np.abs(own[0] - base[0])) <= 2e-6


def test_shards_of_the_split_route_bitwise(gpu):
    """48 -> 44.1 kHz (147/160, K = 1023: no single-pass SRC kernel; Chain runs
    the SRC kernel, then the single-pass cascade alone on y), 512 rows of
    48000: the job's batch takes the chained tiles, a shard of 128 by itself
    the three-launch mode.  Planned with the job's batch every shard of 1, 2
    and 4 forces the job's mode and the rows are bitwise the unsharded ones;
    planned per shard they agree to float64 rounding."""
    from dspcore import _lib
    from dspcore.chain import Chain, ChainConfig
    from dspcore.shard import run_sharded
    from oracle import dsp_ref_cpu as orc
    B, n_in = 512, 48000
    cfg = ChainConfig(n_in, 48000, 147, 160, 1023, orc.CONFIG3_GAINS, n_fft=4096)
    lib = _lib.load()
    n_out = Chain(cfg, 1, gpu).n_out
    assert lib.dsp_chain_mode(B, n_out, n_out, 1, 1, 1, 0, 6) == 1
    assert lib.dsp_chain_mode(B // 4, n_out, n_out, 1, 1, 1, 0, 6) == 3
    x = np.random.default_rng(147).uniform(-1, 1, (B, n_in)).astype(np.float32)

    def fn(plan):
        def run(xd):
            ch = Chain(cfg, xd.shape[0], xd.device, plan_batch=plan)
            assert ch.tile_len == 0 and ch._split_ws is not None
            y, z, mag = ch.run(xd)
            return y.clone(), z.clone(), mag.clone()
        return run

    base = run_sharded(fn(B), x, [gpu])
    for parts in (2, 4):
        got = run_sharded(fn(B), x, [gpu] * parts)
        for a, b in zip(got, base):
            np.testing.assert_array_equal(a, b)
    own = run_sharded(fn(None), x, [gpu] * 4)
    np.testing.assert_array_equal(own[0], base[0])          # y: one SRC kernel
    assert np.max(np.abs(own[1] - base[1])) <= 2e-6


def test_fft_four_step_matches_reference(gpu):
    """N = 2^13 .. 2^16 through the drop-in against the reference's own outputs
    (tests/golden/fft_large.npz; 2^15 and 2^16 take the four-step path), and
    2^17 .. 2^22 batched and 2^23 / 2^24 / 2^26 against np.fft.fft, 2^27 and
    2^28 against the exact DFT of a sum of tones: max|dX| <= 1e-5 * max|X|
    (2^29 and 2^30: test_fft_nested_four_step)."""
    dc = _dc()
    g = golden("fft_large")
    for k in (13, 14, 15, 16):
        for kind in (("r", "c") if k >= 15 else ("r",)):
            x = g[f"x{kind}_{k}"].astype(np.complex128 if kind == "c" else np.float64)
            ref = g[f"X{kind}_{k}"].astype(np.complex128)
            X = dc.fft_diezmado_en_tiempo(x)
            assert X.dtype == np.complex128 and X.shape == ref.shape
            err = np.max(np.abs(X - ref))
            assert err <= FFT_RTOL * np.max(np.abs(ref)), f"N=2^{k} {kind}: {err:.3g}"
    rng = np.random.default_rng(12)
    for lg, B in ((17, 3), (18, 2), (19, 2), (20, 2), (21, 1), (22, 1)):
        x = (rng.uniform(-1, 1, (B, 1 << lg)) + 1j * rng.uniform(-1, 1, (B, 1 << lg)))
        x = x.astype(np.complex64)
        X = _ops().fft(torch.from_numpy(x).to(gpu)).cpu().numpy()
        ref = np.fft.fft(x.astype(np.complex128), axis=1)
        err = np.max(np.abs(X - ref), axis=1)
        assert np.all(err <= FFT_RTOL * np.max(np.abs(ref), axis=1)), (lg, err)
    xr = rng.uniform(-1, 1, (2, 1 << 20)).astype(np.float32)
    X = _ops().fft(torch.from_numpy(xr).to(gpu)).cpu().numpy()
    ref = np.fft.fft(xr.astype(np.float64), axis=1)
    assert np.max(np.abs(X - ref)) <= FFT_RTOL * np.max(np.abs(ref))
    # 2^23 .. 2^26 (round 3): sub-transforms of 2^12 / 2^13 points with 4 / 2
    # columns per workgroup; one row each, real and complex input
    for lg, real in ((23, True), (24, False), (26, True)):
        n = 1 << lg
        x = rng.uniform(-1, 1, n).astype(np.float32)
        if not real:
            x = (x + 1j * rng.uniform(-1, 1, n).astype(np.float32)).astype(np.complex64)
        X = _ops().fft(torch.from_numpy(x[None, :]).to(gpu)).cpu().numpy()[0]
        ref = np.fft.fft(x.astype(np.complex128))
        err = np.max(np.abs(X - ref))
        assert err <= FFT_RTOL * np.max(np.abs(ref)), (lg, err)
        del X, ref
    # 2^27 and 2^28 (round 4: 2^13 x 2^14 and 2^14 x 2^14): a sum of tones,
    # whose DFT is known exactly (N a_j at bin f_j, zero elsewhere), built and
    # checked on the device
    for lg in (27, 28):
        n = 1 << lg
        f = torch.tensor([1, 12345, n // 3, n - 7], dtype=torch.int64, device=gpu)
        amp = torch.tensor([0.5, -0.25 + 0.5j, 0.75j, 0.3], dtype=torch.complex128, device=gpu)
        idx = torch.arange(n, dtype=torch.int64, device=gpu)
        x = torch.zeros(n, dtype=torch.complex64, device=gpu)
        for fj, aj in zip(f, amp):
            ph = ((fj * idx) % n).double() * (2 * np.pi / n)
            x += (aj * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
            del ph
        del idx
        X = _ops().fft(x[None, :])[0]
        del x
        want = torch.zeros(n, dtype=torch.complex64, device=gpu)
        want[f] = (n * amp).to(torch.complex64)
        err = float(torch.max(torch.abs(X - want)))
        assert err <= FFT_RTOL * n * 0.75, (lg, err)
        del X, want
        torch.cuda.empty_cache()


def _tones(n, f, amp, gpu, real=False):
    """sum_j amp_j exp(2 pi i f_j t / n) (or its real part, cos tones) on the
    device, phases reduced mod n in int64 and formed in float64."""
    idx = torch.arange(n, dtype=torch.int64, device=gpu)
    x = torch.zeros(n, dtype=torch.float32 if real else torch.complex64, device=gpu)
    for fj, aj in zip(f, amp):
        ph = ((fj * idx) % n).double() * (2 * np.pi / n)
        if real:
            x += (aj * torch.cos(ph)).float()
        else:
            x += (aj * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
        del ph
    return x


def test_fft_nested_four_step(gpu):
    """2^29 and 2^30 (round 5, the nested four-step of csrc/fft.hip run_fft6_row;
    the reference's recursion has no size cap, dsp_core.py:41-66): sums of
    tones against their exact DFT (max|dX| <= 1e-5 * max|X|), two complex rows
    at 2^29 and a real row at 2^30; the 2^29 spectrum against |FFT| of the same
    windowed float32 row; an inf at n = 0 (every X[k].real +inf, X.imag the
    DFT of the rest) and in the spectrum's segment (every bin non-finite);
    the three-pass spectrum at 2^25 over three rows against numpy; Parseval
    and linearity on dense random 2^27 input; per-row non-finite flags at
    2^25; 2^33 raises RuntimeError (2^31, 2^32: tests/test_gpu_fft_split.py)."""
    ops = _ops()
    n = 1 << 29
    f = [[3, 777777, n // 3, n - 5], [1, 2, n // 2, n - 1]]
    amp = [[0.5, -0.25 + 0.5j, 0.75j, 0.3], [0.25, 0.5, -0.5, 0.125j]]
    x = torch.stack([_tones(n, f[r], amp[r], gpu) for r in range(2)])
    X = ops.fft(x)
    for r in range(2):
        want = torch.zeros(n, dtype=torch.complex64, device=gpu)
        want[torch.tensor(f[r], device=gpu)] = torch.tensor(
            [n * a for a in amp[r]], dtype=torch.complex64, device=gpu)
        err = float(torch.max(torch.abs(X[r] - want)))
        assert err <= FFT_RTOL * n * 0.75, (r, err)
        del want
    # an inf at n = 0 rides every output's real part unchanged (W^0 = 1)
    xz = x[:1].clone()
    xz[0, 0] = complex(0.0, x[0, 0].imag.item())
    x[0, 0] = complex(np.inf, x[0, 0].imag.item())
    Xi = ops.fft(x[:1])
    Xz = ops.fft(xz)
    assert bool(torch.all(torch.isposinf(Xi.real)))
    assert torch.equal(Xi.imag, Xz.imag)
    del x, X, Xi, Xz, xz
    torch.cuda.empty_cache()
    # the 2^29 spectrum: centre segment shorter than N (zero padded)
    xr = _tones(n, [12345, n // 7], [0.5, 0.25], gpu, real=True)
    mag = ops.spectrum(xr[None, :], 1000, n - 5000, n)[0]
    seg = torch.zeros(n, dtype=torch.float32, device=gpu)
    seg[:n - 5000] = xr[1000:n - 4000]
    seg *= ops._table("hann", n, torch.device(gpu))
    ref = torch.abs(ops.fft(seg[None, :])[0, :n // 2 + 1])
    assert float(torch.max(torch.abs(mag - ref))) <= FFT_RTOL * float(torch.max(ref))
    del seg, ref
    xr[n // 2] = np.inf
    mag = ops.spectrum(xr[None, :], 1000, n - 5000, n)[0]
    assert not bool(torch.any(torch.isfinite(mag)))
    del xr, mag
    torch.cuda.empty_cache()
    # dense random input through the three-pass path: Parseval (sum |X|^2 = N
    # sum |x|^2, in float64 sums) and linearity, size-independent properties
    n = 1 << 27
    gen = torch.Generator(device=gpu).manual_seed(27)
    xa = torch.randn(1, n, dtype=torch.complex64, device=gpu, generator=gen)
    xb = torch.randn(1, n, dtype=torch.complex64, device=gpu, generator=gen)
    Xa, Xb = ops.fft(xa), ops.fft(xb)
    ex = float(torch.sum(torch.abs(xa.to(torch.complex128)) ** 2))
    eX = float(torch.sum(torch.abs(Xa.to(torch.complex128)) ** 2))
    assert abs(eX / (n * ex) - 1) < 1e-5, eX / (n * ex)
    Xs = ops.fft(xa + 2 * xb)
    lin = float(torch.max(torch.abs(Xs - (Xa + 2 * Xb))))
    assert lin <= FFT_RTOL * float(torch.max(torch.abs(Xs))), lin
    del xa, xb, Xa, Xb, Xs
    torch.cuda.empty_cache()
    # the per-row non-finite flags of the three-pass path: an inf only in row 1
    # of a 2^25 batch leaves row 0 bitwise the clean batch's
    n = 1 << 25
    xc = torch.randn(2, n, dtype=torch.complex64, device=gpu)
    Xc = ops.fft(xc)
    xc[1, 0] = complex(np.inf, 0.0)
    Xi = ops.fft(xc)
    assert torch.equal(Xi[0], Xc[0])
    assert bool(torch.all(torch.isposinf(Xi[1].real)))
    assert bool(torch.all(torch.isfinite(Xi[1].imag)))
    del xc, Xc, Xi
    # the three-pass spectrum from 2^25, three rows (row loop, segment offsets,
    # zero padding) against numpy
    n = 1 << 25
    rng = np.random.default_rng(25)
    xs = rng.uniform(-1, 1, (3, n + 3000)).astype(np.float32)
    mag = ops.spectrum(torch.from_numpy(xs).to(gpu), 2000, n - 1000, n).cpu().numpy()
    w = (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))).astype(np.float32)
    seg = np.zeros((3, n), dtype=np.float32)
    seg[:, :n - 1000] = xs[:, 2000:n + 1000]
    ref = np.abs(np.fft.rfft((seg * w).astype(np.float64), axis=1))
    assert np.max(np.abs(mag - ref)) <= FFT_RTOL * np.max(ref)
    del xs, mag, seg, ref
    # 2^30, real input: cos tones, N/2 a_j at bins f_j and N - f_j
    n = 1 << 30
    fr, ar = [5, n // 3, n // 2 - 1], [0.5, -0.75, 0.25]
    X = ops.fft(_tones(n, fr, ar, gpu, real=True)[None, :])[0]
    want = torch.zeros(n, dtype=torch.complex64, device=gpu)
    for fj, aj in zip(fr, ar):
        want[fj] += n / 2 * aj
        want[n - fj] += n / 2 * aj
    err = float(torch.max(torch.abs(X - want)))
    assert err <= FFT_RTOL * n / 2 * 0.75, err
    del X, want
    torch.cuda.empty_cache()
    from dspcore import _lib
    with pytest.raises(RuntimeError):
        ops._log2(1 << 33)          # (2^31 and 2^32: the radix-2 split, test_gpu_fft_split.py)
    with pytest.raises(RuntimeError):
        ops._log2(1 << 31, _lib.DSP_MAX_LOG2N_FOURSTEP)   # the spectrum's limit


def test_spectrum_four_step_matches_reference(gpu):
    """calcular_espectro_magnitud with n_fft = 2^15 (four-step spectrum mode:
    centre segment, Hann window, |X[k]| for k <= N/2) against the reference
    recipe's output in tests/golden/fft_large.npz."""
    dc = _dc()
    g = golden("fft_large")
    f, m = dc.calcular_espectro_magnitud(g["spec_x"].astype(np.float64), 72000, n_fft=1 << 15)
    np.testing.assert_array_equal(f, g["spec_f"])
    ref = g["spec_m"].astype(np.float64)
    assert m.shape == ref.shape
    assert np.max(np.abs(m - ref)) <= FFT_RTOL * np.max(ref)
    # batched device rows against numpy at 2^18 (segment shorter than N: zero padded)
    rng = np.random.default_rng(13)
    x = rng.uniform(-1, 1, (2, 200000)).astype(np.float32)
    mag = _ops().spectrum(torch.from_numpy(x).to(gpu), 1000, 150000, 1 << 18).cpu().numpy()
    n = 1 << 18
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))
    seg = np.zeros((2, n))
    seg[:, :150000] = x[:, 1000:151000]
    ref = np.abs(np.fft.fft(seg * w, axis=1))[:, :n // 2 + 1]
    assert np.max(np.abs(mag - ref)) <= FFT_RTOL * np.max(ref)
