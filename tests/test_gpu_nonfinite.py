"""Non-finite input through the SRC -> EQ -> spectrum chain, against the
reference's semantics.

The reference convolves the zero-stuffed x with its float64 taps, every one of
them non-zero -- the sinc's zeros are rounding noise, |L h| ~ 1e-17 .. 1e-34
(/root/reference/modules/dsp_core.py:120-129, :162, :166) -- so an inf or NaN
reaches every output whose window covers it: NaN stays NaN, inf * tap keeps
the tap's sign, infs of both signs make NaN.  lfilter (:205-214) then turns
every output after the first non-finite sample into NaN (the peaking sections
have b1 == a1, so b1 x - a1 y = inf - inf), the clip (:254) maps +-inf to +-1,
and a NaN anywhere in the spectrum's segment makes every bin NaN (:92-93).

Rows of each config carry NaN, +inf and -inf at a delay output's window edge
(L3/M2: the branch whose only flushed-free tap is the centre), off its centre,
at tile and sub-chunk boundaries of the single-pass kernels and of the SRC
kernel's blocks, and at a channel's first and last samples.  Every path --
the drop-in module, Chain.run's single-pass kernel and its two-launch chain
(dsp_chain_path(1)), and the host-resident HostChain -- must give the oracle's
(oracle/dsp_ref_cpu.py) non-finite masks exactly: y's NaN / +inf / -inf, z's
NaN (and +-inf where the EQ is bypassed), |X|'s NaN and +inf; finite values
within the parity tolerances.  With the EQ bypassed (config 1) z carries y's
infs into the spectrum, where numpy's |.| is hypot -- +inf for a bin with an
infinite component even when the other is NaN -- and the labels of the
reference's radix-2 recursion decide which bins are which: the non-finite
repair (csrc/fft_nf.hip) restores them, and the masks are compared exactly.

The FFT and spectrum entry points are also called directly
(fft_diezmado_en_tiempo, calcular_espectro_magnitud, the spectrogram) on rows
with +-inf / NaN at the segment's edges (the Hann window's zeros), its centre
and outside it: every output component's class is the oracle's (NaN / +inf /
-inf of Re X and Im X, of |X|), and the finite components of X within the FFT
tolerance.
"""
import contextlib
import time
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SRC_ATOL = 2e-6
EQ_ATOL = 1e-5
MAG_RTOL = 1e-5
NAN, INF = float("nan"), float("inf")

CONFIGS = {
    # name: (fs, L, M, K, n_in, gains, n_fft, limit_pts, single-pass tile / sub-chunk outputs)
    "c1": (44100, 2, 1, 127, 441000, "flat", 1024, 100000, (3840, 3840)),
    "c3": (48000, 3, 2, None, 48000, "c3", 4096, None, (3072, 48)),
    "c5": (44100, 160, 147, 1023, 12000, "c3", 4096, None, (2048, 32)),
    # the generic single-pass kernel (k_chain_gen), up- and down-sampling
    "g54": (48000, 5, 4, 31, 9000, "c3", 2048, None, (2048, 32)),
    "g23": (48000, 2, 3, 15, 6600, "c3", 2048, None, (2048, 32)),
}
FLAT = {"Sub-Bass": 0, "Bass": 0, "Low Mids": 0, "High Mids": 0, "Presence": 0, "Brilliance": 0}


def _gains(which):
    from oracle import dsp_ref_cpu as orc
    return FLAT if which == "flat" else orc.CONFIG3_GAINS


def _rows(name):
    """x [B, n_in] float32 and the (position, value) list of every row."""
    from dspcore import design
    fs, L, M, K, n, _, _, _, (tile, sub) = CONFIGS[name]
    plan = design.src_plan(n, fs, M, L, K)
    T = -(-plan.K // L)

    def q(m):                                  # last input sample output m reads
        return (m * M + plan.c_offset) // L

    # a delay output (polyphase branch 0) in the middle of the row
    m_d = next(m for m in range(plan.n_out // 3, plan.n_out) if (m * M + plan.c_offset) % L == 0)
    qd = q(m_d)
    m_t = 2 * tile if 2 * tile < plan.n_out - tile else tile   # a tile boundary
    m_s = m_t + 5 * sub                                        # a sub-chunk boundary
    specs = [
        [],
        [(qd - (T - 1), NAN)],                  # the delay output's window edge
        [(qd, INF)],                            # its other edge
        [(qd - (T - 1) // 2 - 1, -INF)],        # off its centre
        [(q(m_t), INF), (q(m_t) + 3, -INF)],    # both signs, one window: NaN
        [(q(m_t - 1), NAN)],                    # last sample of the tile before
        [(q(m_t) - (T - 1), -INF)],             # first sample of the tile's first window
        [(q(m_s), INF), (q(m_s) - 1, INF)],     # sub-chunk boundary, one sign
        [(0, NAN)],
        [(n - 1, -INF)],
        [(n - 1, NAN)],
        [(n - 5, INF), (n - 3, INF)],
    ]
    rng = np.random.default_rng(404)
    x = rng.uniform(-0.9, 0.9, (len(specs), n)).astype(np.float32)
    for r, sp in enumerate(specs):
        for pos, val in sp:
            assert 0 <= pos < n
            x[r, pos] = val
    return x, specs


def _oracle(name, x):
    from oracle import dsp_ref_cpu as orc
    fs, L, M, K, n, g, n_fft, limit, _ = CONFIGS[name]
    out = []
    with warnings.catch_warnings(), np.errstate(invalid="ignore", over="ignore"):
        warnings.simplefilter("ignore")
        for row in x:
            y, z, _, mag, _ = orc.chain(row, fs, L, M, _gains(g), K, n_fft, limit_pts=limit)
            out.append((y, z, mag))
    return out


_CACHE = {}


def _case(name):
    if name not in _CACHE:
        x, specs = _rows(name)
        _CACHE[name] = (x, specs, _oracle(name, x))
    return _CACHE[name]


def _same(got, want, tol, what, masks=("nan", "+inf", "-inf"), rel=False):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    tests = {"nan": np.isnan, "+inf": np.isposinf, "-inf": np.isneginf,
             "nonfinite": lambda a: ~np.isfinite(a)}
    for m in masks:
        gm, wm = tests[m](got), tests[m](want)
        if not np.array_equal(gm, wm):
            bad = np.nonzero(gm != wm)[0]
            raise AssertionError(f"{what}: {m} mask differs at {bad[:8]} of {bad.size} "
                                 f"(got {got[bad[:4]]}, want {want[bad[:4]]})")
    fin = np.isfinite(want) & np.isfinite(got)
    if fin.any():
        scale = float(np.max(np.abs(want[fin]))) if rel else 1.0
        err = float(np.max(np.abs(got[fin] - want[fin])))
        assert err <= tol * max(scale, 1e-30), f"{what}: max finite error {err:.3g}"


def _check(name, y, z, mag, label):
    x, specs, ref = _case(name)
    bypass = CONFIGS[name][5] == "flat"
    for r, (ry, rz, rm) in enumerate(ref):
        tag = f"{name} {label} row {r} {specs[r]}"
        if y is not None:
            _same(y[r], ry, SRC_ATOL, tag + " y")
        _same(z[r], rz, SRC_ATOL if bypass else EQ_ATOL, tag + " z",
              masks=("nan", "+inf", "-inf") if bypass else ("nan",))
        _same(mag[r], rm, MAG_RTOL, tag + " |X|", masks=("nan", "+inf", "-inf"), rel=True)


@contextlib.contextmanager
def _chain_path(path):
    from dspcore import _lib
    prev = _lib.chain_path(path)
    try:
        yield
    finally:
        _lib.chain_path(prev)


def _cfg(name):
    from dspcore.chain import ChainConfig
    fs, L, M, K, n, g, n_fft, limit, _ = CONFIGS[name]
    return ChainConfig(n, fs, L, M, K, _gains(g), n_fft=n_fft, limit_pts=limit)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_nonfinite_chain_paths_match_reference(gpu, name):
    """Chain.run (single-pass where it applies) and the two-launch chain."""
    from dspcore.chain import Chain
    x, _, _ = _case(name)
    ch = Chain(_cfg(name), x.shape[0], gpu)
    if name != "c1":
        assert ch.tile_len in (32, 48)
    xd = torch.from_numpy(x).to(gpu)
    y, z, mag = (t.cpu().numpy() for t in ch.run(xd))
    _check(name, y, z, mag, "single-pass" if ch.tile_len else "two-launch")
    with _chain_path(1):
        y2, z2, m2 = (t.cpu().numpy() for t in ch.run(xd))
    _check(name, y2, z2, m2, "two-launch")
    # finite outputs are the same numbers on both paths; y bitwise
    fin = np.isfinite(y)
    np.testing.assert_array_equal(y[fin], y2[fin])


def test_nonfinite_persistent_kernel_matches_reference(gpu):
    """Config 5's persistent single-pass kernel (dsp_chain_path(3): each wave
    runs its channels' tiles in order, the entry state in registers), then the
    repair kernel: the oracle's masks, and y and z bitwise the chained-tile
    kernel's (dsp_chain_path(2))."""
    from dspcore.chain import Chain
    x, _, _ = _case("c5")
    ch = Chain(_cfg("c5"), x.shape[0], gpu)
    xd = torch.from_numpy(x).to(gpu)
    with _chain_path(3):
        y, z, mag = (t.cpu().numpy() for t in ch.run(xd))
    _check("c5", y, z, mag, "persistent")
    with _chain_path(2):
        y2, z2, m2 = (t.cpu().numpy() for t in ch.run(xd))
    np.testing.assert_array_equal(y, y2)
    np.testing.assert_array_equal(z, z2)
    np.testing.assert_array_equal(mag, m2)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_nonfinite_drop_in_matches_reference(gpu, name):
    """The drop-in module's calls, as app.py makes them, on the [B, n] batch."""
    from modules import dsp_core as dc
    fs, L, M, K, n, g, n_fft, limit, _ = CONFIGS[name]
    x, _, _ = _case(name)
    with np.errstate(invalid="ignore"):
        y, fs_out = dc.conversion_tasa_muestreo(x, fs, M, L, num_taps=K)
        z = dc.sistema_ecualizador(y, fs_out, _gains(g))
        zs = z if limit is None else z[:, :limit]
        _, mag = dc.calcular_espectro_magnitud(zs, fs_out, n_fft=n_fft)
    _check(name, y, z, mag, "drop-in")


@pytest.mark.parametrize("name", ["c3", "c5", "g54"])
def test_nonfinite_host_chain_matches_reference(gpu, name):
    """HostChain (numpy in and out, pipelined blocks of 5 rows, 2 slots)."""
    from dspcore.host import HostChain
    x, _, _ = _case(name)
    with HostChain(_cfg(name), gpu, block=5, slots=2) as hc:
        y, z, mag = hc.run(x, copy=True)
    _check(name, y, z, mag, "HostChain")


def test_finite_input_keeps_the_canonical_sums(gpu):
    """The non-finite path is taken only by tiles whose window holds an inf
    or NaN: a row with one NaN gives, in every tile before it, y and z bitwise
    equal to the same row without it, and the call after it is unaffected."""
    from dspcore.chain import Chain
    x, _ = _rows("c3")
    clean = x[0:1].copy()
    dirty = clean.copy()
    dirty[0, 40000] = NAN
    ch = Chain(_cfg("c3"), 1, gpu)
    y0, z0, _ = (t.cpu().numpy() for t in ch.run(torch.from_numpy(clean).to(gpu)))
    y1, z1, _ = (t.cpu().numpy() for t in ch.run(torch.from_numpy(dirty).to(gpu)))
    first = int(np.argmax(~np.isfinite(y1[0])))
    assert 0 < first < y1.shape[1]
    np.testing.assert_array_equal(y1[0, :first], y0[0, :first])
    np.testing.assert_array_equal(z1[0, :first], z0[0, :first])
    assert np.isnan(z1[0, first + 1:]).all()
    # the repair leaves no hand-off flag or state behind: a clean call after it
    # is bitwise the first one
    y2, z2, _ = (t.cpu().numpy() for t in ch.run(torch.from_numpy(clean).to(gpu)))
    np.testing.assert_array_equal(y2, y0)
    np.testing.assert_array_equal(z2, z0)
    assert ch.handoff_ok()


# ---------------------------------------------------------------------------
# Direct calls of the FFT and spectrum entry points (dsp_core.py:41-98)
# ---------------------------------------------------------------------------
@contextlib.contextmanager
def _quiet():
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        yield


def _fft_rows(N, cplx, seed):
    """Rows of length N with +-inf / NaN at the ends, the centre, both
    components, several at once, and one finite row."""
    rng = np.random.default_rng(seed)
    c = N // 2
    specs = [
        [(0, INF, 0)], [(N - 1, NAN, 0)], [(c, -INF, 0)], [(c - 1, INF, 0), (c + 1, INF, 0)],
        [(1, INF, 0), (N - 2, -INF, 0)], [(c, NAN, 0), (0, INF, 0)], [],
    ]
    if cplx:
        specs += [[(c, INF, 1)], [(0, NAN, 1), (c, -INF, 0)], [(N - 1, INF, 0), (N - 1, -INF, 1)]]
    x = rng.uniform(-1, 1, (len(specs), N))
    if cplx:
        x = x + 1j * rng.uniform(-1, 1, (len(specs), N))
    for r, sp in enumerate(specs):
        for pos, val, part in sp:
            pos = min(max(pos, 0), N - 1)
            if part:
                x[r, pos] = complex(x[r, pos].real, val)
            elif cplx:
                x[r, pos] = complex(val, x[r, pos].imag)
            else:
                x[r, pos] = val
    return x.astype(np.complex64 if cplx else np.float32)


def _same_complex(got, want, what):
    got = np.asarray(got, dtype=np.complex128)
    want = np.asarray(want, dtype=np.complex128)
    scale = max(float(np.max(np.abs(np.where(np.isfinite(want.real), want.real, 0)))),
                float(np.max(np.abs(np.where(np.isfinite(want.imag), want.imag, 0)))), 1e-30)
    for part, g, w in (("re", got.real, want.real), ("im", got.imag, want.imag)):
        _same(g, w, MAG_RTOL * scale, f"{what} {part}")


@pytest.mark.parametrize("N", [2, 16, 1024, 4096, 16384, 32768])
@pytest.mark.parametrize("cplx", [False, True])
def test_nonfinite_fft_direct_matches_reference(gpu, N, cplx):
    """fft_diezmado_en_tiempo on a [B, N] batch and on one 1-D row: Re X and
    Im X carry the oracle's NaN / +inf / -inf exactly, finite components
    within 1e-5 of the largest (2^15: the four-step transform and its
    workspace-header repair)."""
    from modules import dsp_core as dc
    x = _fft_rows(N, cplx, N + cplx)
    with _quiet():
        want = [np.asarray(orc_fft(r), dtype=np.complex128) for r in x]
        X = dc.fft_diezmado_en_tiempo(x)
        X1 = dc.fft_diezmado_en_tiempo(x[0])
    assert X.dtype == np.complex128 and X.shape == x.shape
    for r in range(x.shape[0]):
        _same_complex(X[r], want[r], f"N={N} complex={cplx} row {r}")
    _same_complex(X1, want[0], f"N={N} 1-D")


def orc_fft(row):
    from oracle import dsp_ref_cpu as orc
    return orc.fft_dit(row.astype(np.complex128) if np.iscomplexobj(row) else row.astype(np.float64))


@pytest.mark.parametrize("n,n_fft", [(100000, 2048), (100000, 4096), (1000, 2048), (6, 2048),
                                     (100000, 32768)])
def test_nonfinite_spectrum_direct_matches_reference(gpu, n, n_fft):
    """calcular_espectro_magnitud with +-inf / NaN at the segment's first and
    last samples (the Hann window's zeros: inf * 0 = NaN), its centre, next to
    it, and outside it (no effect): |X| has the oracle's NaN / +inf masks
    exactly (hypot: +inf wherever a component is infinite); finite rows within
    the spectrum tolerance.  (1000 and 6 samples take the zero-padded path,
    32768 points the four-step spectrum.)"""
    from dspcore import design
    from modules import dsp_core as dc
    from oracle import dsp_ref_cpu as orc
    plan = design.spectrum_plan(n, n_fft)
    s0, sl = plan.seg_start, plan.seg_len
    rng = np.random.default_rng(n + n_fft)
    spots = [[(s0, INF)], [(s0 + sl - 1, -INF)], [(s0 + sl // 2, NAN)], [(s0 + sl // 2, INF)],
             [(s0 + sl // 2 - 1, -INF)], [(s0 + 1, INF), (s0 + sl - 2, INF)],
             [(s0 + sl // 3, INF), (s0 + sl // 3 + 1, -INF)], []]
    if s0 > 0:
        spots.append([(s0 - 1, INF)])                      # outside the segment
    if s0 + sl < n:
        spots.append([(s0 + sl, NAN)])
    x = rng.uniform(-1, 1, (len(spots), n)).astype(np.float32)
    for r, sp in enumerate(spots):
        for pos, val in sp:
            x[r, pos] = val
    with _quiet():
        want = [orc.spectrum(r.astype(np.float64), 48000, n_fft)[1] for r in x]
        _, mag = dc.calcular_espectro_magnitud(x, 48000, n_fft=n_fft)
        _, mag1 = dc.calcular_espectro_magnitud(x[2], 48000, n_fft=n_fft)
    for r in range(x.shape[0]):
        _same(mag[r], want[r], MAG_RTOL, f"n={n} n_fft={n_fft} row {r} {spots[r]}",
              masks=("nan", "+inf", "-inf"), rel=True)
        if spots[r] and s0 <= spots[r][0][0] < s0 + sl:
            assert not np.isfinite(mag[r]).any()
    _same(mag1, want[2], MAG_RTOL, "1-D", masks=("nan", "+inf", "-inf"), rel=True)


def test_nonfinite_spectrogram_matches_reference(gpu):
    """Every frame of calcular_espectrograma_magnitud (the spectrum recipe per
    frame): frames that hold an inf or NaN get the oracle's masks, the others
    stay finite and within tolerance."""
    from dspcore import design
    from modules import dsp_core as dc
    from oracle import dsp_ref_cpu as orc
    n, n_fft = 9000, 1024
    plan = design.stft_plan(n, n_fft, None)
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, (3, n)).astype(np.float32)
    x[0, 0] = INF                    # first frame's first sample (a window zero)
    x[0, 4000] = -INF
    x[1, n - 1] = NAN                # the last, zero-padded frame
    x[1, 2 * plan.hop + 17] = INF
    x[1, 2 * plan.hop + 18] = INF
    with _quiet():
        want = [orc.spectrogram(r.astype(np.float64), plan.n_fft, plan.hop, plan.frames)
                for r in x]
        _, _, mag = dc.calcular_espectrograma_magnitud(x, 48000, n_fft=n_fft)
    for r in range(x.shape[0]):
        for f in range(plan.frames):
            _same(mag[r, f], want[r][f], MAG_RTOL, f"row {r} frame {f}",
                  masks=("nan", "+inf", "-inf"), rel=True)


def test_nonfinite_repair_leaves_finite_batches_alone(gpu):
    """The repair launch after a finite batch changes nothing: the spectrum of
    finite rows is bitwise the same with and without a non-finite row beside
    them, and the non-finite row's neighbours are untouched."""
    from dspcore import ops
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.uniform(-1, 1, (300, 4096)).astype(np.float32)).to(gpu)
    a = ops.spectrum(x, 1024, 2048, 2048).cpu().numpy()
    x[137, 2000] = INF
    b = ops.spectrum(x, 1024, 2048, 2048).cpu().numpy()
    keep = np.arange(300) != 137
    np.testing.assert_array_equal(a[keep], b[keep])
    assert not np.isfinite(b[137]).any()


# ---------------------------------------------------------------------------
# aplicar_ecuacion_diferencias (dsp_core.py:205-214: scipy.signal.lfilter)
# ---------------------------------------------------------------------------
LFILTER_CASES = [
    # len(a) == 1: lfilter's convolution (SRC kernel, L = M = 1)
    ("gain", [3.0], [4.0]),
    ("fir 2", [0.5, -0.5], [1.0]),
    ("fir 3 with a zero tap", [1.0, 0.0, 2.0], [1.0]),
    ("fir 31", list(np.hanning(31)), [2.0]),
    # len(a) >= 2: the recursion (cascade kernel + dsp_lfilter_nonfinite_f32)
    ("one-pole low-pass (inf persists)", [0.5, 0.5], [1.0, -0.3]),
    ("one-pole, negative pole (inf alternates)", [1.0], [1.0, 0.6]),
    ("peaking biquad (b1 == a1: NaN)", None, None),
    ("fir through the recursion (a = [1, 0])", [1.0, 2.0, 3.0], [1.0, 0.0]),
    ("trailing zeros of a count", [1.0], [1.0, -0.5, 0.0, 0.0]),
    ("b longer than a", [0.2, 0.3, -0.1, 0.05, 0.4, 0.1], [1.0, -0.5, 0.2]),
    ("butter 4 (four sections' worth of order)", "butter", None),
    # a = [1, 0, ...] with a long b: convolved, then the recursion's labels
    # (dsp_lfilter_nonfinite_f32 scans x: y[n-1] is finite again after len(b))
    ("fir 101 through the recursion (a = [1, 0])", "firwin101", None),
    ("fir 301 through the recursion (a = [2, 0, 0])", "firwin301", None),
]


def _lfilter_coeffs(b, a):
    import scipy.signal as ss
    if b is None:
        from dspcore import design
        return design.peaking_biquad(1000.0, 48000.0, 6.0)
    if b == "butter":
        return ss.butter(4, 0.2)
    if b == "firwin101":
        return ss.firwin(101, 0.2), np.array([1.0, 0.0])
    if b == "firwin301":
        return ss.firwin(301, 0.1), np.array([2.0, 0.0, 0.0])
    return np.asarray(b, dtype=np.float64), np.asarray(a, dtype=np.float64)


@pytest.mark.parametrize("name,b,a", LFILTER_CASES, ids=[c[0] for c in LFILTER_CASES])
def test_nonfinite_lfilter_matches_scipy(gpu, name, b, a):
    """aplicar_ecuacion_diferencias on rows with NaN / +inf / -inf at the
    first and last samples, in the middle, two of opposite sign, one of each:
    y's NaN / +inf / -inf masks are lfilter's exactly (a gain or FIR keeps an
    inf within len(b) samples; a recursion labels everything after it, a
    one-pole low-pass +inf forever, a peaking section NaN), finite samples
    within 1e-5 (relative to max|y| above 1), 2-D batch and 1-D row."""
    import scipy.signal as ss
    from modules import dsp_core as dc
    b, a = _lfilter_coeffs(b, a)
    n = 3000
    specs = [[(0, INF)], [(n - 1, NAN)], [(1500, -INF)], [(700, INF), (701, -INF)],
             [(900, NAN), (2000, INF)], [(1200, INF), (1260, INF)], []]
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, (len(specs), n)).astype(np.float32)
    for r, sp in enumerate(specs):
        for pos, val in sp:
            x[r, pos] = val
    with _quiet():
        want = [ss.lfilter(b, a, row.astype(np.float64)) for row in x]
        y = dc.aplicar_ecuacion_diferencias(x, b, a)
        y1 = dc.aplicar_ecuacion_diferencias(x[3], b, a)
    assert y.dtype == np.float64 and y.shape == x.shape
    for r in range(x.shape[0]):
        fin = np.isfinite(want[r])
        scale = max(1.0, float(np.max(np.abs(want[r][fin]))) if fin.any() else 1.0)
        _same(y[r], want[r], EQ_ATOL * scale, f"{name} row {r} {specs[r]}")
    _same(y1, want[3], EQ_ATOL * 10, f"{name} 1-D")


@pytest.mark.parametrize("name,b,a", [("one-pole low-pass", [0.5, 0.5], [1.0, -0.3]),
                                      ("negative pole", [1.0], [1.0, 0.6]),
                                      ("fir 101, a = [1, 0]", "firwin101", None)],
                         ids=["lowpass", "negpole", "fir101"])
def test_nonfinite_lfilter_long_rows(gpu, name, b, a):
    """Rows of 2^21 samples whose labels never turn all-NaN (+inf kept by a
    one-pole low-pass, a sign alternating with a negative pole) and a second
    inf of the other sign 1.5 M samples later (NaN from there): the relabel
    kernel fills the periodic stretches without running the class recursion
    sample by sample (seconds per row before), and y's masks
    are scipy.signal.lfilter's exactly."""
    import scipy.signal as ss
    from modules import dsp_core as dc
    b, a = _lfilter_coeffs(b, a)
    n = 1 << 21
    x = np.random.default_rng(9).uniform(-1, 1, (3, n)).astype(np.float32)
    x[0, 5] = INF
    x[1, 70] = -INF
    x[2, 64] = INF
    x[2, 1_500_000] = -INF
    with _quiet():
        want = [ss.lfilter(b, a, row.astype(np.float64)) for row in x]
        t0 = time.perf_counter()
        y = dc.aplicar_ecuacion_diferencias(x, b, a)
        wall = time.perf_counter() - t0
    for r in range(x.shape[0]):
        fin = np.isfinite(want[r])
        scale = max(1.0, float(np.max(np.abs(want[r][fin]))) if fin.any() else 1.0)
        _same(y[r], want[r], EQ_ATOL * scale, f"{name} row {r}")
    assert wall < 5.0, wall


def test_fft_all_inf_2_23_row_repair_is_bounded(gpu):
    """A 2^23-point row that is +inf everywhere: every input
    is on the four-step repair's list, and k_nf_fix walks the list per output
    until both components are NaN.  The class algebra saturates within 8
    entries for every k here (a host simulation of the walk: mean 4.25, worst
    8, for 2^10..2^16), so the repair is bounded; the reference's recursion
    gives NaN in both components of every X[k] for N >= 4 (E[0] + W O[0] with W
    = 1 + 0j: 0 * inf = NaN), and so must this."""
    from modules import dsp_core as dc
    x = np.full(1 << 23, np.inf, dtype=np.float32)
    with _quiet():
        dc.fft_diezmado_en_tiempo(x[: 1 << 15])      # warm the tables
        t0 = time.perf_counter()
        X = dc.fft_diezmado_en_tiempo(x)
        wall = time.perf_counter() - t0
    assert X.shape == x.shape
    assert np.isnan(X.real).all() and np.isnan(X.imag).all()
    assert wall < 10.0, wall
