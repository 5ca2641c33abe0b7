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
NaN (and +-inf where the EQ is bypassed), |X|'s NaN; finite values within the
parity tolerances.  With the EQ bypassed (config 1) z carries y's infs into the
spectrum, where numpy's |.| gives inf for a (NaN, inf) bin and the kernels NaN:
there only |X|'s finite mask is compared.
"""
import contextlib
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
        _same(mag[r], rm, MAG_RTOL, tag + " |X|", masks=("nonfinite",) if bypass else ("nan",),
              rel=True)


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
