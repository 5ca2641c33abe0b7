"""The chain's contract beyond plain parity (ABI 2.0, round 3), on the GPU
through the C-ABI:

  * config 1 (BASELINE.json configs[0]) end to end: app.py:164-167 then
    :203-205 through the drop-in module, and the same job through Chain.run,
    whose geometry (L2/M1, K = 127: 64 taps per branch) takes the two-launch
    path with the EQ bypassed (S = 0: the cascade launch is a copy);
  * the single-pass kernel's float32 pass 1 (input-normal coordinates) at the
    reference's gain extremes (+-15 dB on every band, eq.npz's sets), at both
    single-pass geometries, within the EQ tolerance of the oracle;
  * a tile hand-off wait that gives up surfaces as HandoffError and the reset
    workspace serves the next call correctly;
  * y = NULL (keep_y=False) skips the y store and leaves z and |Z| bitwise;
  * the two paths never share workspace bytes (a general-path cascade between
    single-pass calls on one workspace changes nothing);
  * tables whose key does not match the call are not used.
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
CHAIN_MAG_RTOL = 1e-5     # max|dX| <= 1e-5 max|X|


@contextlib.contextmanager
def _chain_path(path):
    from dspcore import _lib
    prev = _lib.chain_path(path)
    try:
        yield
    finally:
        _lib.chain_path(prev)


def _traced(fn):
    from dspcore import _lib
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        out = tuple(None if t is None else t.clone() for t in fn())
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    return out, names


def _fastcar_stand_in():
    """Config 1's input: 10 s at 44.1 kHz, a synthetic stand-in for the missing
    examples/FastCar.wav (.MISSING_LARGE_BLOBS): noise plus two tones,
    peak-normalised as cargar_senal_audio does (dsp_core.py:26-31)."""
    fs, n = 44100, 441000
    t = np.arange(n) / fs
    rng = np.random.default_rng(2024)
    x = 0.3 * rng.standard_normal(n) + 0.5 * np.sin(2 * np.pi * 440 * t) \
        + 0.2 * np.sin(2 * np.pi * 3100 * t)
    x = x.astype(np.float32)
    return x / np.max(np.abs(x)), fs


FLAT = {"Sub-Bass": 0, "Bass": 0, "Low Mids": 0, "High Mids": 0, "Presence": 0, "Brilliance": 0}


def test_config1_drop_in_end_to_end(gpu):
    """BASELINE configs[0] through the drop-in, as app.py calls it: SRC L2/M1
    with 127 taps (keyword extension), flat EQ (the bypass returns its input
    object), 1024-point spectrum of z[:100000] (app.py:202)."""
    from modules import dsp_core as dc
    from oracle import dsp_ref_cpu as orc
    x, fs = _fastcar_stand_in()
    y, fs_out = dc.conversion_tasa_muestreo(x, fs, 1, 2, num_taps=127)
    z = dc.sistema_ecualizador(y, fs_out, FLAT)
    f, m = dc.calcular_espectro_magnitud(z[:100000], fs_out, n_fft=1024)
    ry, rz, rf, rm, rfs = orc.chain(x, fs, 2, 1, FLAT, 127, 1024, limit_pts=100000)
    assert fs_out == rfs == 88200 and y.dtype == np.float64 and y.shape == ry.shape
    assert z is y                                   # dsp_core.py:222-223
    assert np.max(np.abs(y - ry)) <= SRC_ATOL
    np.testing.assert_array_equal(f, rf)
    assert np.max(np.abs(m - rm)) <= CHAIN_MAG_RTOL * np.max(rm)


def test_config1_chain_two_launch_bypass(gpu):
    """Config 1 through Chain.run: the EQ is bypassed (S = 0), which takes no
    single-pass kernel (round 6: the two-launch chain's copy pass is cheaper
    than an identity cascade and keeps the bypass's local inf / NaN), so SRC
    then the S = 0 cascade launch (the bypass copy, no clip: z == y bitwise)
    then the spectrum; with the config-3 gains the same geometry (2/1, K =
    127: 64 taps per branch) takes the per-phase single-pass kernel (csrc/
    chain_pp.h; for two channels this long, its three-launch mode), whose y
    is bitwise the two-launch chain's; against the oracle."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    x, fs = _fastcar_stand_in()
    cfg = ChainConfig(x.size, fs, 2, 1, 127, FLAT, n_fft=1024, limit_pts=100000)
    ch = Chain(cfg, 2, gpu)
    assert ch.tile_len == 0 and ch.eq.bypass and ch.sos.shape[0] == 0
    xs = torch.from_numpy(np.stack([x, -x])).to(gpu)
    (y, z, mag), names = _traced(lambda: ch.run(xs))
    # S = 0: one copy pass; no clip, so z may carry infs and the spectrum's
    # non-finite repair follows it (csrc/fft_nf.hip)
    assert names == ["src_poly", "iir_apply", "spectrum", "spectrum_nf"], names
    assert torch.equal(y, z)
    cfg3 = ChainConfig(x.size, fs, 2, 1, 127, orc.CONFIG3_GAINS, n_fft=1024, limit_pts=100000)
    ch3 = Chain(cfg3, 2, gpu)
    assert ch3.tile_len == 48
    (y3, _, _), names3 = _traced(lambda: ch3.run(xs))
    # (two 441000-sample channels: the single-pass kernel's three-launch mode)
    assert names3[:4] == ["chain_tile_agg", "chain_tile_carry", "chain_tile", "chain_repair"], \
        names3
    assert torch.equal(y3, y)
    ry, rz, _, rm, _ = orc.chain(x, fs, 2, 1, FLAT, 127, 1024, limit_pts=100000)
    y, mag = y.cpu().numpy(), mag.cpu().numpy()
    assert np.max(np.abs(y[0] - ry)) <= SRC_ATOL
    np.testing.assert_array_equal(y[1], -y[0])      # odd symmetry of the linear SRC
    assert np.max(np.abs(mag[0] - rm)) <= CHAIN_MAG_RTOL * np.max(rm)
    np.testing.assert_array_equal(mag[1], mag[0])
    # a clip-only EQ (S = 0 with clip, gains of exactly 0.1 dB: dsp_core.py:234
    # applies no band but still clips) through the same copy launch
    cfg2 = ChainConfig(x.size, fs, 2, 1, 127, {"Bass": 0.1}, n_fft=1024, limit_pts=100000)
    ch2 = Chain(cfg2, 2, gpu)
    assert not ch2.eq.bypass and ch2.sos.shape[0] == 0
    y2, z2, m2 = ch2.run(xs * 3)
    rz2 = orc.equaliser(orc.resample(3 * x, fs, 1, 2, 127)[0], 88200, {"Bass": 0.1})
    assert np.max(np.abs(z2[0].cpu().numpy() - rz2)) <= SRC_ATOL * 3
    assert float(z2.abs().max()) == 1.0


EXTREME_CASES = [1, 2, 0, 5, 7]     # eq.npz: all +15, all -15, config 3, unknown band, 2 bands


@pytest.mark.parametrize("fs,L,M,K", [(48000, 3, 2, None), (44100, 160, 147, 1023)])
def test_single_pass_extreme_gains_within_eq_tolerance(gpu, fs, L, M, K):
    """The single-pass kernel's carry (float32 pass-1 sums in input-normal
    coordinates, float64 scan and pass 2) against the oracle at the gain sets
    of tests/golden/eq.npz, including +-15 dB on all six bands: z within the
    EQ tolerance of the reference recipe and of the two-launch chain (float64
    throughout), |Z| within 1e-5 max|Z|.  Rows 0-1 noise, row 2 driven into
    the clip."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    g = golden("eq")
    rng = np.random.default_rng(31)
    x = rng.uniform(-1, 1, (3, 48000)).astype(np.float32)
    x[2] *= 4.0
    xd = torch.from_numpy(x).to(gpu)
    worst = {}
    for case in EXTREME_CASES:
        gains = golden_gains(g[f"gains_{case}"])
        cfg = ChainConfig(48000, fs, L, M, K, gains, n_fft=4096)
        ch = Chain(cfg, 3, gpu)
        assert ch.tile_len in (32, 48), (case, ch.tile_len)
        (y1, z1, m1), names = _traced(lambda: ch.run(xd))
        assert "chain_tile" in names
        with _chain_path(1):
            y0, z0, m0 = (t.clone() for t in ch.run(xd))
        assert torch.equal(y1, y0)
        assert (z1 - z0).abs().max().item() <= EQ_ATOL
        err = err0 = 0.0
        for b in range(3):
            ry, rz, _, rm, _ = orc.chain(x[b], fs, L, M, gains, K, 4096)
            e = float(np.max(np.abs(z1[b].cpu().numpy() - rz)))
            err = max(err, e)
            err0 = max(err0, float(np.max(np.abs(z0[b].cpu().numpy() - rz))))
            assert e <= EQ_ATOL, (case, b, e)
            assert np.max(np.abs(m1[b].cpu().numpy() - rm)) <= CHAIN_MAG_RTOL * np.max(rm)
        worst[case] = (f"{err:.3g}", f"two-launch {err0:.3g}")
    print(f"max|z - oracle| per eq.npz case at L/M={L}/{M}: {worst}")


def test_handoff_give_up_surfaces_and_reset_recovers(gpu):
    """With a spin limit of 0 (dsp_chain_spin_limit: every wait gives up at its
    first unanswered poll) one channel's tiles, all in flight at once, cannot
    hand off: run() raises HandoffError, and after its reset the workspace
    serves a normal call bitwise like a fresh chain.  (The chained tiles
    forced: one channel alone would take the three-launch mode, which waits
    for nothing.)"""
    with _chain_path(2):
        _handoff_give_up(gpu)


def _handoff_give_up(gpu):
    from dspcore import _lib
    from dspcore.chain import Chain, ChainConfig, HandoffError
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, 1, gpu)
    assert ch.tile_len == 48
    gen = torch.Generator(device=gpu).manual_seed(17)
    x = torch.rand((1, 48000), generator=gen, device=gpu) * 2 - 1
    prev = _lib.spin_limit(0)
    try:
        with pytest.raises(HandoffError):
            ch.run(x)
    finally:
        _lib.spin_limit(prev)
    assert ch.handoff_ok()                          # reset by the raise
    y, z, mag = (t.clone() for t in ch.run(x))
    fresh = Chain(cfg, 1, gpu)
    y2, z2, m2 = fresh.run(x)
    assert torch.equal(y, y2) and torch.equal(z, z2) and torch.equal(mag, m2)
    # graph-capture-free callers can defer the check
    prev = _lib.spin_limit(0)
    try:
        ch.run(x, check=False)
    finally:
        _lib.spin_limit(prev)
    assert not ch.handoff_ok()
    with pytest.raises(HandoffError):
        ch.check()
    assert ch.handoff_ok()


@pytest.mark.parametrize("fs,L,M,K,n_in", [(48000, 3, 2, None, 48000), (44100, 160, 147, 1023, 48000),
                                           (48000, 3, 2, None, 47996)])
def test_chain_without_y(gpu, fs, L, M, K, n_in):
    """keep_y=False: the single-pass kernel gets y = NULL (no y store, no y
    buffer) and z and |Z| are bitwise those of the run that writes y; where
    the two-launch chain serves the geometry (n_out % 4 != 0) y lives in an
    internal buffer.  Either way run() returns (None, z, mag)."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(n_in, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=4096)
    gen = torch.Generator(device=gpu).manual_seed(23)
    x = torch.rand((5, n_in), generator=gen, device=gpu) * 2 - 1
    full = Chain(cfg, 5, gpu)
    bare = Chain(cfg, 5, gpu, keep_y=False)
    assert (bare.y is None) == (bare.tile_len > 0)
    y1, z1, m1 = (t.clone() for t in full.run(x))
    (y0, z0, m0), names = _traced(lambda: bare.run(x))
    assert y0 is None
    assert torch.equal(z0, z1) and torch.equal(m0, m1)
    assert ("chain_tile" in names) == (full.tile_len > 0)


def test_two_paths_never_share_workspace(gpu):
    """a two-launch call whose cascade runs the general path (282
    chunks: scratch in the workspace) between single-pass calls on the SAME
    workspace leaves the hand-off region intact: the next single-pass call is
    bitwise a fresh chain's and its hand-off never gave up."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, 4, gpu, chunk_len=256)          # 282 chunks: the general cascade path
    assert ch.tile_len == 48 and not ch.xstate
    gen = torch.Generator(device=gpu).manual_seed(29)
    x = torch.rand((4, 48000), generator=gen, device=gpu) * 2 - 1
    ref = [t.clone() for t in Chain(cfg, 4, gpu).run(x)]
    ch.run(x)
    with _chain_path(1):
        (_, zg, _), names = _traced(lambda: ch.run(x))
    assert "iir_carry" in names, names              # the general path ran, using scratch
    assert (zg - ref[1]).abs().max().item() <= 2e-6
    out = ch.run(x)
    assert ch.handoff_ok()
    for a, b in zip(out, ref):
        assert torch.equal(a, b)


def test_tables_with_another_key_are_not_used(gpu):
    """Tables built for another cascade (other gains) handed to a call: the
    key differs, the library takes the two-launch path (correct z), not the
    single-pass kernel with the wrong coefficients."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg_a = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=4096)
    gains_b = {"Sub-Bass": -6, "Presence": 9}
    cfg_b = ChainConfig(48000, 48000, 3, 2, None, gains_b, n_fft=4096)
    a, b = Chain(cfg_a, 2, gpu), Chain(cfg_b, 2, gpu)
    assert a.tile_key != b.tile_key
    gen = torch.Generator(device=gpu).manual_seed(37)
    x = torch.rand((2, 48000), generator=gen, device=gpu) * 2 - 1
    with _chain_path(1):
        want = [t.clone() for t in b.run(x)]
    b.tile_tables, b.tile_key = a.tile_tables, a.tile_key
    (y, z, mag), names = _traced(lambda: b.run(x))
    assert "chain_tile" not in names and "src_poly" in names, names
    for got, w in zip((y, z, mag), want):
        assert torch.equal(got, w)
    rz = orc.chain(x[0].cpu().numpy(), 48000, 3, 2, gains_b, None, 4096)[1]
    assert np.max(np.abs(z[0].cpu().numpy() - rz)) <= EQ_ATOL


def test_chain_app_rerun_spectra_x_y_z(gpu):
    """Chain(spectra=("x", "y", "z")) is app.py:203-205's rerun: the spectra of
    the input (at fs), the SRC output and the EQ output (at fs') over the first
    limit_pts samples, each within 1e-5 max|X| of the oracle's
    calcular_espectro_magnitud and on its frequency axis; z's spectrum is the
    chain's own, bitwise the same as without the extras."""
    import numpy as np
    import torch

    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(31)
    x = rng.uniform(-1, 1, (2, 48000)).astype(np.float32)
    cfg = ChainConfig(48000, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=2048, limit_pts=100000)
    ch = Chain(cfg, 2, gpu, spectra=("x", "y", "z"))
    xt = torch.from_numpy(x).to(gpu)
    y, z, mag = ch.run(xt)
    plain = Chain(cfg, 2, gpu)
    _, _, mag0 = plain.run(xt)
    assert torch.equal(mag, mag0) and ch.mags["z"] is mag
    for b in range(2):
        ry, _ = orc.resample(x[b], 48000, 2, 3)
        rz = orc.equaliser(ry, 72000, orc.CONFIG3_GAINS)
        for which, sig, fs in (("x", x[b], 48000), ("y", ry, 72000), ("z", rz, 72000)):
            f_ref, m_ref = orc.spectrum(np.asarray(sig)[:100000], fs)
            got = ch.mags[which][b].cpu().numpy()
            assert got.shape == m_ref.shape, which
            assert np.max(np.abs(got - m_ref)) <= 1e-5 * np.max(m_ref), which
            np.testing.assert_allclose(ch.frequencies(which), f_ref, rtol=1e-12, atol=0)
    with pytest.raises(ValueError):
        Chain(cfg, 2, gpu, spectra=("x",))
    with pytest.raises(ValueError):
        Chain(cfg, 2, gpu, keep_y=False, spectra=("y", "z"))


def test_host_chain_pipelined_numpy_matches_chain_run(gpu):
    """dspcore.host.HostChain (numpy in/out, channel blocks through a ring of
    slots with pinned staging and overlapped copies): 300 channels in blocks of
    64 (a short, zero-padded last block) are bitwise Chain.run's rows on the
    whole batch -- the single-pass kernel's rows do not depend on the batch --
    and spot rows match the oracle; keep_y=False returns y = None with z and
    |Z| unchanged; a second call reuses the pinned outputs."""
    from dspcore.chain import Chain, ChainConfig
    from dspcore.host import HostChain
    from oracle import dsp_ref_cpu as orc
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, (300, 4800)).astype(np.float32)
    cfg = ChainConfig(4800, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=2048)
    hc = HostChain(cfg, gpu, block=64, slots=3)
    y, z, mag = hc.run(x, copy=True)
    ch = Chain(cfg, 300, gpu)
    ry, rz, rmag = (t.cpu().numpy() for t in ch.run(torch.from_numpy(x).to(gpu)))
    assert ch.tile_len > 0
    np.testing.assert_array_equal(y, ry)
    np.testing.assert_array_equal(z, rz)
    np.testing.assert_array_equal(mag, rmag)
    for b in (0, 299):
        oy, oz, _, om, _ = orc.chain(x[b], 48000, 3, 2, orc.CONFIG3_GAINS, None, 2048)
        assert np.max(np.abs(y[b] - oy)) <= SRC_ATOL
        assert np.max(np.abs(z[b] - oz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - om)) <= CHAIN_MAG_RTOL * np.max(om)
    y2, z2, mag2 = hc.run(x[::-1])
    np.testing.assert_array_equal(z2, rz[::-1])
    np.testing.assert_array_equal(mag2, rmag[::-1])
    hn = HostChain(cfg, gpu, block=128, slots=2, keep_y=False)
    yn, zn, mn = hn.run(x)
    assert yn is None
    np.testing.assert_array_equal(zn, rz)
    np.testing.assert_array_equal(mn, rmag)
    with pytest.raises(ValueError):
        hc.run(x[:, :100])


def test_run_sharded_host_bitwise(gpu):
    """shard.run_sharded_host: a numpy batch over 1, 2 and 3 "devices" (all
    cuda:0 here: the 1-GPU rehearsal of one HostChain and host thread per GPU)
    gives the same bits for every shard count."""
    from dspcore.chain import ChainConfig
    from dspcore.shard import run_sharded_host
    from oracle import dsp_ref_cpu as orc
    x = np.random.default_rng(12).uniform(-1, 1, (150, 4800)).astype(np.float32)
    cfg = ChainConfig(4800, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=2048)
    base = run_sharded_host(cfg, x, [gpu], block=32, slots=2)
    for parts in (2, 3):
        got = run_sharded_host(cfg, x, [gpu] * parts, block=32, slots=2)
        for a, b in zip(base, got):
            np.testing.assert_array_equal(a, b)
    oy, oz, _, om, _ = orc.chain(x[77], 48000, 3, 2, orc.CONFIG3_GAINS, None, 2048)
    assert np.max(np.abs(base[1][77] - oz)) <= EQ_ATOL


def test_single_pass_delay_branch_index_map_bit_exact(gpu):
    """The single-pass kernel's delay-branch path (k_chain_tile<Geo3241, DLY>):
    unit impulses through Chain.run give y[m] = kernel_taps[2 m + c - 3 p]
    bitwise (0 outside the taps) -- every third output from the one-multiply
    path, the others from the FMA chains -- at tile and sub-chunk edges."""
    from dspcore import design
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    n = 4800
    pos = [0, 1, 2, 31, 32, 2047, 2048, 2049, 4799]
    x = np.zeros((len(pos), n), np.float32)
    for r, p in enumerate(pos):
        x[r, p] = 1.0
    cfg = ChainConfig(n, 48000, 3, 2, None, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, len(pos), gpu)
    assert ch.tile_len > 0
    kt = design.kernel_taps(ch.src)
    y = ch.run(torch.from_numpy(x).to(gpu))[0].cpu().numpy()
    m = np.arange(ch.n_out)
    for r, p in enumerate(pos):
        k = 2 * m + ch.src.c_offset - 3 * p
        want = np.where((k >= 0) & (k < ch.src.K), kt[np.clip(k, 0, ch.src.K - 1)], 0.0)
        np.testing.assert_array_equal(y[r], want.astype(np.float32))
