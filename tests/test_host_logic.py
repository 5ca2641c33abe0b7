"""Host-side logic of the product path (no GPU): filter design, band selection,
size rules and the shard partitioning, checked against the reference's outputs."""
import numpy as np
import pytest

from conftest import golden, golden_gains
from dspcore import design
from dspcore.shard import shard_ranges


def test_sinc_taps_match_reference_bitwise():
    g = golden("taps")
    for i, (wc, k) in enumerate(g["cases"]):
        np.testing.assert_array_equal(design.sinc_lowpass(wc, int(k)), g[f"h_{i}"])


def test_biquad_design_matches_reference_bitwise():
    for row in golden("biquad")["rows"]:
        b, a = design.peaking_biquad(row[0], row[1], row[2])
        np.testing.assert_array_equal(b, row[3:6])
        np.testing.assert_array_equal(a, row[6:9])


def test_src_plan_sizes_match_reference_outputs():
    g = golden("src")
    for i, (L, M, K, N, fs) in enumerate(g["cases"]):
        p = design.src_plan(int(N), int(fs), int(M), int(L), None if K < 0 else int(K))
        assert p.n_out == g[f"y_{i}"].shape[1]
        assert p.fs_out == int(g[f"fs_{i}"])
        assert p.K % 2 == 1
        assert p.c_offset == (min(int(N) * int(L), p.K) - 1) // 2


def test_src_plan_default_and_override_taps():
    assert design.src_plan(48000, 48000, 2, 3).K == 121
    assert design.src_plan(48000, 48000, 2, 3, 255).K == 255
    assert design.src_plan(48000, 48000, 1, 2, 126).K == 127      # even -> odd
    p = design.src_plan(48000, 44100, 147, 160, 1023)
    assert (p.n_out, p.fs_out) == (52245, 48000)
    with pytest.raises(ValueError):
        design.src_plan(0, 48000, 2, 3)


def test_eq_plan_rules():
    g = golden("eq")
    # bypass / clip-only / unknown band / clamp / floor, cases 3, 4, 5, 6, 8, 9
    assert design.eq_plan(72000, golden_gains(g["gains_3"])).bypass
    assert design.eq_plan(72000, {}).bypass
    p = design.eq_plan(72000, golden_gains(g["gains_4"]))
    assert not p.bypass and p.sos.shape == (0, 5)       # g == 0.1: no stage, still clips
    p = design.eq_plan(72000, {"Mystery": 9, "Bass": 3})
    assert p.centres == (1000, 150)
    p = design.eq_plan(6000, golden_gains(g["gains_6"]))
    assert max(p.centres) == pytest.approx(0.45 * 6000)
    p = design.eq_plan(20, {"Bass": 6})
    assert not p.bypass and p.sos.shape[0] == 0          # clamped to 9 Hz <= 10: skipped
    p = design.eq_plan(72000, {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3,
                               "High Mids": -3, "Presence": 5, "Brilliance": -6})
    assert p.sos.shape == (6, 5) and p.centres == (40, 150, 1000, 3000, 5000, 10000)


def test_spectrum_plan_matches_reference_segments():
    g = golden("spectrum")
    for i, n in enumerate(g["lengths"]):
        p = design.spectrum_plan(int(n))
        assert p.n_fft // 2 + 1 == g[f"m_{i}"].size
    for n, raised in g["raising"]:
        if raised:
            with pytest.raises(ValueError):
                design.spectrum_plan(int(n))
        else:
            design.spectrum_plan(int(n))
    assert design.spectrum_plan(72000, 4096) == design.SpectrumPlan(36000, 4096, 4096)
    assert design.spectrum_plan(0).n_fft == 2


def test_tf_to_sos_row_normalises_like_lfilter():
    row = design.tf_to_sos_row([2.0, 1.0], [2.0, -1.0, 0.5])
    np.testing.assert_allclose(row, [1.0, 0.5, 0.0, -0.5, 0.25])
    with pytest.raises(ValueError):
        design.tf_to_sos_row([1, 2, 3, 4], [1])


def test_shard_ranges_cover_batch_contiguously():
    for B in (0, 1, 7, 4096, 32768):
        for parts in (1, 2, 4, 8):
            r = shard_ranges(B, parts)
            assert sum(hi - lo for lo, hi in r) == B
            assert all(r[i][1] == r[i + 1][0] for i in range(len(r) - 1))
            assert len(r) <= parts


def _cascade_run(sos, u):
    """The kernels' direct-form-II realisation (design.df2_realization),
    written out independently: returns (outputs, final delay lines)."""
    rows, gain, norm = design.df2_realization(sos)
    S = rows.shape[0]
    st = np.zeros(2 * S)
    out = np.empty(len(u))
    for i, x in enumerate(u):
        v = gain * x if norm else x
        for k in range(S):
            g, c1, c2, a1, a2 = rows[k]
            w = v - a1 * st[2 * k] - a2 * st[2 * k + 1]
            v = g * w + c1 * st[2 * k] + c2 * st[2 * k + 1]
            st[2 * k + 1] = st[2 * k]
            st[2 * k] = w
        out[i] = v
    return out, st


def test_df2_realisation_matches_lfilter():
    """The rearranged recursion computes the reference's lfilter cascade
    (dsp_core.py:205-214, :233-251) to float64 rounding, with and without the
    b0 normalisation (a stage with b0 == 0 keeps its gain)."""
    from scipy.signal import lfilter
    sos = design.eq_plan(72000, {"Sub-Bass": 15, "Bass": -9, "Low Mids": 3, "Presence": 6,
                                 "Brilliance": -6}).sos
    u = np.random.default_rng(3).uniform(-1, 1, 3000)
    ref = u.copy()
    for row in sos:
        ref = lfilter(row[:3], np.r_[1.0, row[3:]], ref)
    got, _ = _cascade_run(sos, u)
    assert design.df2_realization(sos)[2]
    assert np.max(np.abs(got - ref)) <= 1e-11
    odd = np.array([[0.0, 0.5, -0.25, -1.2, 0.5]])
    assert not design.df2_realization(odd)[2]
    got, _ = _cascade_run(odd, u)
    np.testing.assert_allclose(got, lfilter([0.0, 0.5, -0.25], [1.0, -1.2, 0.5], u),
                               rtol=0, atol=1e-12)


def test_state_response_table_gives_chunk_end_states():
    sos = design.eq_plan(72000, {"Sub-Bass": 15, "Bass": -9, "Presence": 6}).sos
    rng = np.random.default_rng(0)
    for T in (32, 96, 1152):
        u = rng.uniform(-1, 1, T)
        G = design.state_response_table(sos, T)
        assert G.shape == (T, 2 * sos.shape[0])
        end = _cascade_run(sos, u)[1]
        np.testing.assert_allclose(u @ G, end, rtol=1e-10, atol=1e-9)


def test_chunk_policy_is_batch_independent_and_fused():
    for n in (1, 31, 32, 100, 4800, 72000, 52245, 10 ** 6):
        T = design.chunk_len_for(n)
        assert T % 32 == 0 and T >= 32
        assert -(-n // T) <= design.MAX_FUSED_CHUNKS
    assert design.chunk_len_for(72000) == 288 and design.chunk_len_for(72000, 64) == 1152


def test_xstate_table_reproduces_output_domain_states():
    """The chain's x-domain state table (design.xstate_table) gives the same
    chunk end states as the output-domain table applied to the float64 SRC
    output of the reference's own algorithm (np.convolve 'same', [::M])."""
    import ctypes

    from dspcore import _lib, design
    lib = _lib.load()
    gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3,
             "Presence": 5, "Brilliance": -6}
    for n_in, fs, L, M, K in [(4800, 48000, 3, 2, None), (4801, 48000, 3, 2, 255),
                              (9600, 44100, 160, 147, 1023), (3000, 48000, 2, 1, None)]:
        plan = design.src_plan(n_in, fs, M, L, K)
        sos = design.eq_plan(plan.fs_out, gains).sos
        T = design.xstate_chunk_len(plan.n_out, L, M)
        assert T % 32 == 0 and (T * M) % (4 * L) == 0 and -(-plan.n_out // T) <= 256
        out = [ctypes.c_int64() for _ in range(3)]
        assert lib.dsp_chain_xstate_geometry(T, plan.K, L, M, plan.c_offset,
                                             *[ctypes.byref(o) for o in out]) == 0
        shift, q0, rows = (o.value for o in out)
        gx = design.xstate_table(sos, plan, T, q0, rows)
        g = design.state_response_table(sos, T)
        x = np.random.default_rng(n_in).uniform(-1, 1, n_in)
        xe = np.zeros(n_in * L)
        xe[::L] = x
        y = np.convolve(xe, plan.taps, "same")[::M]
        for c in range(-(-plan.n_out // T) - 1):
            e_y = g.T @ y[c * T:(c + 1) * T]
            idx = c * shift + q0 + np.arange(rows)
            xv = np.where((idx >= 0) & (idx < n_in), x[np.clip(idx, 0, n_in - 1)], 0.0)
            e_x = gx.T @ xv
            assert np.max(np.abs(e_x - e_y)) <= 1e-12 * max(1.0, np.max(np.abs(e_y)))


def test_stft_plan_framing():
    assert design.stft_plan(10000, 1024, 256) == design.StftPlan(1024, 256, 1 + 36)
    assert design.stft_plan(1024, 1024).frames == 1
    assert design.stft_plan(100, 1024).frames == 1            # zero-padded single frame
    assert design.stft_plan(72000, 2048).hop == 512
    with pytest.raises(ValueError):
        design.stft_plan(1000, 1000)


def test_bluestein_tables_compute_the_dft():
    """The any-length DFT identity with the host tables (float64), as the
    kernel applies it: A = FFT(x w), D = FFT(conj(A Bf)), X = w conj(D)."""
    from dspcore import _lib
    rng = np.random.default_rng(2)
    for n in (1, 3, 1114, 1536, 8192):
        chirp, bf, M = design.bluestein_tables(n)
        assert M == _lib.load().dsp_dft_size(n) and M >= 2 * n - 1 and M & (M - 1) == 0
        x = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
        a = np.zeros(M, complex)
        a[:n] = x * chirp
        d = np.fft.fft(np.conj(np.fft.fft(a) * bf))
        got = chirp * np.conj(d[:n])
        assert np.max(np.abs(got - np.fft.fft(x))) <= 1e-12 * max(1.0, np.max(np.abs(got)))


def _lfilter_cases():
    import scipy.signal as ss
    rng = np.random.default_rng(12)
    poles = 0.9 * np.sqrt(rng.uniform(0, 1, 3)) * np.exp(1j * rng.uniform(0, np.pi, 3))
    a_rand = np.real(np.poly(np.concatenate([poles, np.conj(poles), [0.5]])))
    return [
        ("order 1", [0.5, 0.5], [1.0, -0.3]),
        ("biquad, a0 = 2", [1.0, -1.2, 0.5], [2.0, -1.0, 0.4]),
        ("butter 3 lp", *ss.butter(3, 0.2)),
        ("butter 4 hp", *ss.butter(4, 0.3, "highpass")),
        ("butter 4 bp (order 8)", *ss.butter(4, [0.2, 0.4], "bandpass")),
        ("butter 8 lp", *ss.butter(8, 0.4)),
        ("cheby1 5", *ss.cheby1(5, 1, 0.3)),
        ("ellip 6", *ss.ellip(6, 0.5, 40, 0.35)),
        ("random stable order 7", rng.uniform(-1, 1, 8), a_rand),
        ("b longer than a", [0.2, 0.3, -0.1, 0.05, 0.4, 0.1], [1.0, -0.5, 0.2]),
        ("fir 31", ss.firwin(31, 0.2), [1.0]),
        ("fir 5, a = [2]", [1.0, 2.0, 3.0, 2.0, 1.0], [2.0]),
        ("gain", [3.0], [4.0]),
        ("fir 3 with a zero tap", [1.0, 0.0, 2.0], [1.0]),
        ("fir 2, a = [2]", [0.5, -0.5], [2.0]),
        ("fir 5 through the recursion (a = [1, 0])", [1.0, 2.0, 3.0, 4.0, 5.0], [1.0, 0.0]),
        ("gain through the recursion (a = [2, 0])", [3.0], [2.0, 0.0]),
        # long FIRs through the recursion: convolved, not factored (tf2sos of a
        # degree-300 polynomial is off by 5e30)
        ("fir 101 through the recursion (a = [1, 0])", ss.firwin(101, 0.2), [1.0, 0.0]),
        ("fir 301 through the recursion (a = [2, 0, 0])", ss.firwin(301, 0.1), [2.0, 0.0, 0.0]),
    ]


def test_lfilter_plan_any_order_matches_lfilter():
    """design.lfilter_plan (aplicar_ecuacion_diferencias, any order): the
    second-order sections it hands the cascade kernel filter exactly like
    scipy.signal.lfilter (checked in float64 with sosfilt), the FIR and gain
    plans are lfilter's normalised b; a[0] == 0 raises lfilter's ValueError."""
    import scipy.signal as ss
    from dspcore import design
    x = np.random.default_rng(3).uniform(-1, 1, 4000)
    for name, b, a in _lfilter_cases():
        ref = ss.lfilter(b, a, x)
        plan = design.lfilter_plan(b, a)
        if plan.kind == "sos":
            sos6 = np.column_stack([plan.sos[:, :3], np.ones(plan.sos.shape[0]), plan.sos[:, 3:]])
            got = ss.sosfilt(sos6, x)
            assert plan.sos.shape[0] <= design.MAX_LFILTER_SECTIONS
        else:
            assert (plan.kind == "fir" and np.size(a) == 1) or (
                plan.kind == "fir_rec" and not np.any(np.asarray(a)[1:]))
            got = np.convolve(x, plan.taps)[:x.size]
        assert np.max(np.abs(got - ref)) <= 1e-9 * max(1.0, np.max(np.abs(ref))), name
    with pytest.raises(ValueError, match="a\\[0\\] == 0"):
        design.lfilter_plan([1.0], [0.0, 1.0])
    # any order (round 4): more than DSP_MAX_STAGES sections run in groups
    for name, b, a in _high_order_cases():
        plan = design.lfilter_plan(b, a)
        groups = design.lfilter_groups(plan.sos)
        assert plan.kind == "sos" and plan.sos.shape[0] > design.MAX_LFILTER_SECTIONS
        assert all(g.shape[0] <= design.MAX_LFILTER_SECTIONS for g in groups)
        assert np.array_equal(np.concatenate(groups), plan.sos)
        got = x
        for g in groups:
            got = ss.sosfilt(np.column_stack([g[:, :3], np.ones(g.shape[0]), g[:, 3:]]), got)
        ref = ss.lfilter(b, a, x)
        assert np.max(np.abs(got - ref)) <= 1e-9 * max(1.0, np.max(np.abs(ref))), name


def _high_order_cases():
    """IIR orders 36 and 48 from random stable sections (pole radius <= 0.85:
    lfilter's direct form stays accurate there, unlike a Butterworth of that
    order)."""
    import scipy.signal as ss
    rng = np.random.default_rng(21)
    out = []
    for order in (36, 48):
        secs = []
        for _ in range(order // 2):
            r, th = rng.uniform(0.3, 0.85), rng.uniform(0.1, 3.0)
            secs.append([1.0, rng.uniform(-1, 1), rng.uniform(-0.5, 0.5), 1.0,
                         -2 * r * np.cos(th), r * r])
        out.append((f"random stable order {order}", *ss.sos2tf(np.array(secs))))
    return out


def test_kernel_taps_flush_only_sinc_zero_noise():
    """design.kernel_taps: for upsampling plans (wc = 1/L) exactly the taps at
    the sinc's zeros (every L-th from the centre, float64 noise of sin(k pi))
    become 0 -- the centre branch is then a pure delay (the single-pass kernel's
    DLY path) -- every other tap is float32(L h) bitwise; L = 1 plans keep all
    taps; the flushed taps change y by less than 1e-14 per unit input."""
    for L, M, K in ((3, 2, None), (2, 1, 127), (3, 2, 255), (160, 147, 1023)):
        p = design.src_plan(48000, 48000, M, L, K)
        kt = design.kernel_taps(p)
        flushed = kt == 0
        c = (p.K - 1) // 2
        idx = np.arange(p.K)
        # the sinc zeros of wc = 1/max(L, M) sit every max(L, M) taps from the
        # centre; the Blackman window's end taps (~1e-34) are its zeros
        sinc_zero = (idx - c) % max(L, M) == 0
        win_end = (idx == 0) | (idx == p.K - 1)
        assert np.all((sinc_zero | win_end)[flushed])
        assert flushed.sum() >= (p.K - 1) // max(L, M) - 2
        np.testing.assert_array_equal(kt[~flushed], p.taps[~flushed].astype(np.float32))
        assert np.sum(np.abs(p.taps[flushed])) < 1e-14
        assert kt[c] != 0
    p = design.src_plan(48000, 48000, 2, 3)          # the benchmark's K = 121
    kt = design.kernel_taps(p)
    branch0 = kt[0::3]                               # taps ph = 0: indices 0, 3, .., 120
    assert np.count_nonzero(branch0) == 1 and branch0[20] == kt[60]
    fir = design.src_plan(100, 48000, 1, 1, 31)      # L = 1: nothing flushed
    np.testing.assert_array_equal(design.kernel_taps(fir), fir.taps.astype(np.float32))


def test_chain_tile_tables_flush_and_mark_the_delay_branch():
    """dsp_chain_tile_tables flushes the caller's taps itself (csrc/common.h,
    kTapFlushRel): the reference's float32 taps and design.kernel_taps give
    byte-identical tables, with branch 0 a pure delay and the DLY key; a
    branch-0 tap above the flush threshold takes the plain key; a tap at
    1e-20 is flushed like the sinc-zero noise (host only)."""
    import ctypes
    from dspcore import _lib
    lib = _lib.load()
    p = design.src_plan(48000, 48000, 2, 3)
    sos = np.ascontiguousarray(design.eq_plan(72000, {"Bass": 6.0}).sos)
    nbytes = lib.dsp_chain_tile_tables_bytes()

    def tables(t32):
        buf = np.zeros(nbytes, np.uint8)
        k = ctypes.c_uint64(0)
        rc = lib.dsp_chain_tile_tables(buf.ctypes.data, nbytes, 48000, p.n_out, t32.ctypes.data,
                                       p.K, 3, 2, p.c_offset, _lib.sos_pointer(sos),
                                       sos.shape[0], ctypes.byref(k))
        assert rc == 0
        return buf, k.value

    kt = np.ascontiguousarray(design.kernel_taps(p))
    raw = design.caller_taps(p)
    assert np.any(raw[0::3] != 0) and np.count_nonzero(kt[0::3]) == 1
    (bk, kk), (br, kr) = tables(kt), tables(raw)
    np.testing.assert_array_equal(bk, br)
    noisy = raw.copy()
    noisy[3] = 1e-20
    assert tables(noisy)[1] == kr
    loud = raw.copy()
    loud[3] = 1e-3
    assert tables(loud)[1] != kr
