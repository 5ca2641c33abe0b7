"""The cascade alone through the single-pass kernels (ABI 2.7): the SRC bypass
L = M = 1 (/root/reference/modules/dsp_core.py:144-145, the app's default
ratio, app.py:149-150) followed by sistema_ecualizador (:216-254) runs as the
one-tap SRC y = 1.0 x on the per-phase kernel k_chain_pp<PpGeo<1, 1, 48, 1, 0,
...>> (csrc/chain_pp.h): x read once, z written once, y never stored (it is x).

Against the two-launch path (Chain.run_stages: the two-pass cascade k_iir_wave
over y = x) on the same batch: z within 2e-6, |X| within 1e-5 of the largest,
the same inf / NaN masks; rows against the oracle (dsp_core.py:216-254 and
:68-98 restated in oracle/dsp_ref_cpu.py) within the parity tolerances; one
tile, ragged last tiles, a row driven into the clip, a row silent for its
first half, +-15 dB gain sets (tests/golden/eq.npz), rows of x that are not
16-byte aligned (the two-pass cascade serves them).
"""
import contextlib
import os
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

EQ_ATOL = 1e-5
MAG_RTOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))


def _traced(fn):
    from dspcore import _lib
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        out = tuple(t.clone() if t is not None else None for t in fn())
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    return out, names


@contextlib.contextmanager
def _chain_path(path):
    from dspcore import _lib
    prev = _lib.chain_path(path)
    try:
        yield
    finally:
        _lib.chain_path(prev)


@pytest.mark.parametrize("n_in,B", [(48000, 6), (3072, 3), (96, 4), (100, 5), (47996, 4),
                                    (441000, 3)])
def test_cascade_alone_single_pass(gpu, n_in, B):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    fs = 48000
    n_fft = 4096 if n_in >= 3000 else 128   # (the reference's segment rule: 2^k points)
    cfg = ChainConfig(n_in, fs, 1, 1, None, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 48 and ch.identity_src
    gen = torch.Generator(device=gpu).manual_seed(n_in % 1000 + B)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[1] *= 40.0                      # drive the clip
    x[2, : n_in // 2] = 0.0           # silence then signal
    (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    (y0, z0, m0), names0 = _traced(lambda: ch.run_stages(x))
    assert "chain_tile" in names1 and not any(n.startswith("iir") for n in names1), names1
    assert "chain_tile" not in names0, names0
    assert ch.handoff_ok()
    assert torch.equal(y1, x) and torch.equal(y0, x)     # y is x (the bypass)
    assert (z1 - z0).abs().max().item() <= 2e-6
    assert (m1 - m0).abs().max().item() <= MAG_RTOL * m0.abs().max().item()
    z, mag = z1.cpu().numpy(), m1.cpu().numpy()
    assert np.abs(z[1]).max() == 1.0
    for b in (0, 1, 2, B - 1):
        xb = x[b].cpu().numpy()
        ry, rz, _, rmag, _ = orc.chain(xb, fs, 1, 1, orc.CONFIG3_GAINS, None, n_fft)
        np.testing.assert_array_equal(ry, xb)
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= MAG_RTOL * np.max(rmag)
    # without y: the same z, and run() hands back None for y
    ch2 = Chain(cfg, B, gpu, keep_y=False)
    y2, z2, m2 = ch2.run(x)
    assert y2 is None and torch.equal(z2, z1) and torch.equal(m2, m1)
    # the forced two-launch path is the staged one
    with _chain_path(1):
        (y3, z3, m3), _ = _traced(lambda: ch.run(x))
    assert torch.equal(z3, z0) and torch.equal(m3, m0)


def test_cascade_alone_golden_eq_cases(gpu):
    """Every gain set of tests/golden/eq.npz (the reference's own
    sistema_ecualizador outputs: config 3's gains, +-15 dB on every band,
    single bands, the unknown band, g = 0.1 edges, the Nyquist clamp) on its
    7200-sample x32 through the single-pass cascade where it takes it: within
    1e-5 of the reference's z32, within 2e-6 of the two-pass cascade, the
    bypass sets returning x itself."""
    from conftest import golden, golden_gains
    from dspcore.chain import Chain, ChainConfig
    g = golden("eq")
    x32 = g["x32"]
    n = x32.size - x32.size % 4
    x = torch.from_numpy(np.ascontiguousarray(x32[:n])[None, :]).to(gpu)
    cases = sorted(int(k[6:]) for k in g.keys() if k.startswith("gains_"))
    served = 0
    for k in cases:
        gains, fs = golden_gains(g[f"gains_{k}"]), int(g[f"fs_{k}"])
        cfg = ChainConfig(n, fs, 1, 1, None, gains, n_fft=8192)
        ch = Chain(cfg, 1, gpu)
        (y1, z1, _), names = _traced(lambda: ch.run(x))
        assert torch.equal(y1, x)
        ref = g[f"z32_{k}"][:n]
        if ch.tile_len:
            served += 1
            assert "chain_tile" in names, (k, names)
            _, z0, _ = ch.run_stages(x)
            assert (z1 - z0).abs().max().item() <= 2e-6, k
        err = float(np.max(np.abs(z1[0].cpu().numpy() - ref)))
        assert err <= EQ_ATOL, (k, gains, err)
    assert served >= 5, served


def test_cascade_alone_nonfinite_matches_two_pass(gpu):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in = 4, 12000
    cfg = ChainConfig(n_in, 48000, 1, 1, None, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    gen = torch.Generator(device=gpu).manual_seed(11)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0, 3072] = float("nan")         # a tile's first sample
    x[1, n_in // 2] = float("inf")
    x[1, n_in // 2 + 3] = float("-inf")
    x[2, n_in - 1] = float("-inf")    # the last sample
    x[3, 0] = float("inf")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        (_, z1, m1), names1 = _traced(lambda: ch.run(x))
        (_, z0, m0), _ = _traced(lambda: ch.run_stages(x))
    assert "chain_tile" in names1 and "chain_repair" in names1, names1
    a, b = z1.cpu().numpy(), z0.cpu().numpy()
    for f in (np.isnan, np.isposinf, np.isneginf):
        np.testing.assert_array_equal(f(a), f(b))
    fin = np.isfinite(b)
    assert np.max(np.abs(a[fin] - b[fin])) <= 2e-6
    np.testing.assert_array_equal(np.isnan(m1.cpu().numpy()), np.isnan(m0.cpu().numpy()))
    # and the oracle's masks (lfilter + np.clip on the row)
    for r in range(B):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            _, rz, _, _, _ = orc.chain(x[r].cpu().numpy(), 48000, 1, 1, orc.CONFIG3_GAINS, None, 2048)
        np.testing.assert_array_equal(np.isnan(a[r]), np.isnan(rz))


def test_cascade_alone_unaligned_rows_take_two_pass(gpu):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in = 3, 9600
    cfg = ChainConfig(n_in, 48000, 1, 1, None, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    buf = torch.rand((B, n_in + 1), device=gpu) * 2 - 1
    x = buf[:, 1:]                    # rows 4 bytes past a 16-byte boundary
    (_, z1, _), names = _traced(lambda: ch.run(x))
    assert "chain_tile" not in names, names
    (_, z0, _), _ = _traced(lambda: ch.run(x.contiguous()))
    assert (z1 - z0).abs().max().item() <= 2e-6


@pytest.mark.parametrize("B,n_in", [(1, 441000), (3, 441000), (5, 48000), (2, 3072), (4, 96),
                                    (2, 882000)])
def test_three_launch_mode_matches_chained(gpu, B, n_in):
    """The three-launch mode of the cascade alone (dsp_chain_path 4, chain_tile.h
    AggEntry / GivenEntry, k_tile_carry): every tile from a zero state, the
    channel's tile states scanned, every tile again from its entry state.
    Against the chained tiles (path 2) on the same batch: z within 2e-6 (the
    carries sum in another order), |X| within 1e-5; rows against the oracle;
    the default takes it for small batches of long rows (one 441000-sample
    channel: 144 tiles) and leaves the hand-off flags clear."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    n_fft = 4096 if n_in >= 3000 else 128
    cfg = ChainConfig(n_in, 44100, 1, 1, None, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu, keep_y=False)
    gen = torch.Generator(device=gpu).manual_seed(B * 7 + n_in % 97)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0] *= 8.0
    with _chain_path(4):
        (_, z4, m4), names4 = _traced(lambda: ch.run(x))
    with _chain_path(2):
        (_, z2, m2), names2 = _traced(lambda: ch.run(x))
    (_, z0, m0), names0 = _traced(lambda: ch.run(x))
    assert "chain_tile_agg" in names4 and "chain_tile_carry" in names4, names4
    assert "chain_tile_agg" not in names2, names2
    ntiles = -(-n_in // (64 * 48))
    if B <= 3 and ntiles >= 16:
        assert "chain_tile_agg" in names0, names0        # the default's pick
    assert ch.handoff_ok()
    assert (z4 - z2).abs().max().item() <= 2e-6
    assert (m4 - m2).abs().max().item() <= MAG_RTOL * m2.abs().max().item()
    z = z4.cpu().numpy()
    for b in (0, B - 1):
        _, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 44100, 1, 1, orc.CONFIG3_GAINS, None,
                                      n_fft)
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(m4[b].cpu().numpy() - rmag)) <= MAG_RTOL * np.max(rmag)


def test_three_launch_mode_nonfinite(gpu):
    """Non-finite input through the three-launch mode: the repair kernel reruns
    the channels from their first non-finite tile state (launch 3 published
    the end states), masks equal to the two-pass cascade's."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in = 3, 96000
    cfg = ChainConfig(n_in, 48000, 1, 1, None, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, B, gpu)
    gen = torch.Generator(device=gpu).manual_seed(5)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0, 40000] = float("nan")
    x[1, 3072 * 7] = float("inf")
    x[2, n_in - 2] = float("-inf")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with _chain_path(4):
            (_, z4, _), names = _traced(lambda: ch.run(x))
        (_, z0, _), _ = _traced(lambda: ch.run_stages(x))
    assert "chain_tile_agg" in names and "chain_repair" in names, names
    a, b = z4.cpu().numpy(), z0.cpu().numpy()
    for f in (np.isnan, np.isposinf, np.isneginf):
        np.testing.assert_array_equal(f(a), f(b))
    fin = np.isfinite(b)
    assert np.max(np.abs(a[fin] - b[fin])) <= 2e-6
    assert ch.handoff_ok()


def test_drop_in_equaliser_one_long_channel(gpu):
    """sistema_ecualizador on one 441000-sample channel, as app.py:167 calls it
    after the 2/1 SRC (882000 samples) and at L = M = 1: the single-pass cascade
    alone in its three-launch mode (traced), float64 out, within 1e-5 of the
    oracle (dsp_core.py:216-254) and of the two-pass cascade."""
    from dspcore import _lib
    from oracle import dsp_ref_cpu as orc
    import modules.dsp_core as dc
    rng = np.random.default_rng(12)
    for n in (441000, 882000):
        x = rng.uniform(-1, 1, n).astype(np.float64) * 0.8
        _lib.trace_enable(True)
        _lib.trace_read()
        try:
            z = dc.sistema_ecualizador(x, 44100 if n == 441000 else 88200, orc.CONFIG3_GAINS)
            names = [nm for nm, _ in _lib.trace_read()]
        finally:
            _lib.trace_enable(False)
        assert "chain_tile_agg" in names and "chain_tile_carry" in names, names
        assert not any(nm.startswith("iir") for nm in names), names
        assert z.dtype == np.float64 and z.shape == (n,)
        rz = orc.equaliser(x, 44100 if n == 441000 else 88200, orc.CONFIG3_GAINS)
        assert np.max(np.abs(z - rz)) <= EQ_ATOL


def test_drop_in_equaliser_shards_take_the_jobs_mode(gpu, monkeypatch):
    """A sharded drop-in batch runs, on every shard, the single-pass mode the
    whole batch takes (dsp_chain_mode, ops.forced_chain_path): 400 rows of
    48000 samples take chained tiles whole, while a 100-row shard alone would
    take the three-launch mode; the four-shard rows are bitwise the one-device
    rows."""
    from dspcore import _lib
    from oracle import dsp_ref_cpu as orc
    import modules.dsp_core as dc
    lib = _lib.load()
    assert lib.dsp_chain_mode(400, 48000, 48000, 1, 1, 1, 0, 6) == 1
    assert lib.dsp_chain_mode(100, 48000, 48000, 1, 1, 1, 0, 6) == 3
    assert lib.dsp_chain_mode(1, 48000, 48000, 41, 1, 1, 20, 6) == 0
    rng = np.random.default_rng(3)
    x = rng.uniform(-0.9, 0.9, (400, 48000)).astype(np.float32)
    monkeypatch.setattr(dc, "_shard_devices", lambda: [gpu])
    one = dc.sistema_ecualizador(x, 48000, orc.CONFIG3_GAINS)
    monkeypatch.setattr(dc, "_shard_devices", lambda: [gpu] * 4)
    four = dc.sistema_ecualizador(x, 48000, orc.CONFIG3_GAINS)
    np.testing.assert_array_equal(one, four)
    assert _lib.chain_path() == 0            # restored


@pytest.mark.parametrize("L,M,B,n_in", [(2, 1, 1, 441000), (3, 2, 2, 96000), (1, 2, 2, 441000),
                                        (3, 4, 3, 96000), (5, 4, 1, 48000), (8, 8, 2, 96000)])
def test_three_launch_mode_src_ratios(gpu, L, M, B, n_in):
    """The three-launch mode on the SRC kernels (k_chain_tile3 for 3/2,
    k_chain_pp3 for the per-phase ratios): against the chained tiles (path 2)
    y bitwise (one SRC), z within 2e-6, |X| within 1e-5; rows against the
    oracle; the default takes it for one or two long channels."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(n_in, 48000, L, M, None, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len > 0
    gen = torch.Generator(device=gpu).manual_seed(L * 9 + M + B)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0] *= 8.0
    with _chain_path(4):
        (y4, z4, m4), names4 = _traced(lambda: ch.run(x))
    with _chain_path(2):
        (y2, z2, m2), names2 = _traced(lambda: ch.run(x))
    (_, _, _), names0 = _traced(lambda: ch.run(x))
    assert "chain_tile_agg" in names4 and "chain_tile_carry" in names4, names4
    assert "chain_tile_agg" not in names2, names2
    if n_in * L // M >= 96000 * 2:
        assert "chain_tile_agg" in names0, names0
    assert ch.handoff_ok()
    assert torch.equal(y4, y2)
    assert (z4 - z2).abs().max().item() <= 2e-6
    assert (m4 - m2).abs().max().item() <= MAG_RTOL * m2.abs().max().item()
    for b in range(B):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), 48000, L, M, orc.CONFIG3_GAINS, None,
                                       2048)
        assert np.max(np.abs(y4[b].cpu().numpy() - ry)) <= 2e-6 * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z4[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(m4[b].cpu().numpy() - rmag)) <= MAG_RTOL * np.max(rmag)


@pytest.mark.parametrize("L,M", [(3, 2), (2, 1)])
def test_three_launch_mode_src_nonfinite(gpu, L, M):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in = 3, 48000
    cfg = ChainConfig(n_in, 48000, L, M, None, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    gen = torch.Generator(device=gpu).manual_seed(8)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0, 20000] = float("nan")
    x[1, 4096] = float("inf")
    x[2, n_in - 1] = float("-inf")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with _chain_path(4):
            (y4, z4, _), names = _traced(lambda: ch.run(x))
        with _chain_path(1):
            (y0, z0, _), _ = _traced(lambda: ch.run(x))
    assert "chain_tile_agg" in names and "chain_repair" in names, names
    for a, b, tol in ((y4, y0, 0.0), (z4, z0, 2e-6)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        for f in (np.isnan, np.isposinf, np.isneginf):
            np.testing.assert_array_equal(f(a), f(b))
        fin = np.isfinite(b)
        assert np.max(np.abs(a[fin] - b[fin])) <= tol
    assert ch.handoff_ok()


def test_drop_in_host_conversions_match_numpy(gpu):
    """The drop-in's numpy edges (modules/dsp_core.py _to_rows / _from_rows):
    float64 and complex128 rows narrowed on the device give numpy astype's
    float32 / complex64 bits (denormals, halfway cases, inf, NaN included);
    results come back widened exactly, as float64 / complex128 arrays backed
    by page-locked memory that stays valid after later calls."""
    import modules.dsp_core as dc
    rng = np.random.default_rng(4)
    a = rng.standard_normal(4099) * np.logspace(-46, 38, 4099)
    a[:6] = [1e-40, -3e-39, 5e-45, np.inf, -np.inf, np.nan]
    a[6] = 1.0 + 2.0 ** -24            # halfway: ties to even
    a[7] = 1.0 + 3 * 2.0 ** -24
    t, how = dc._to_rows(a)
    got = t.cpu().numpy()[0]
    want = a.astype(np.float32)
    np.testing.assert_array_equal(got.view(np.uint32)[6:], want.view(np.uint32)[6:])
    np.testing.assert_array_equal(got[:6], want[:6])
    c = a[:2048] + 1j * a[2048:4096]
    tc, _ = dc._to_rows(c, complex_ok=True)
    np.testing.assert_array_equal(tc.cpu().numpy()[0].view(np.uint32)[16:],
                                  c.astype(np.complex64).view(np.uint32)[16:])
    back = dc._from_rows(t, how, np.float64)
    assert back.dtype == np.float64 and back.shape == a.shape
    np.testing.assert_array_equal(back[6:], want.astype(np.float64)[6:])
    keep = back.copy()
    for _ in range(3):                   # later calls do not touch a returned array
        dc._from_rows(torch.zeros_like(t), how, np.float64)
    np.testing.assert_array_equal(back, keep)


@pytest.mark.parametrize("fs,L,M,K,B,n_in", [(44100, 160, 147, 1023, 1, 441000),
                                             (48000, 5, 4, 31, 2, 96000)])
def test_three_launch_mode_generic_kernels(gpu, fs, L, M, K, B, n_in):
    """The three-launch mode on the generic single-pass kernels (160/147:
    k_chain_gct3; others: k_chain_gen3): against the chained tiles (path 2) y
    bitwise, z within 2e-6; the default takes it for a long channel or two;
    rows against the oracle."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    cfg = ChainConfig(n_in, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=4096)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 32
    gen = torch.Generator(device=gpu).manual_seed(L + M + B)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0] *= 4.0
    (y0, z0, m0), names0 = _traced(lambda: ch.run(x))
    with _chain_path(2):
        (y2, z2, m2), names2 = _traced(lambda: ch.run(x))
    assert "chain_tile_agg" in names0 and "chain_tile_carry" in names0, names0
    assert "chain_tile_agg" not in names2, names2
    assert ch.handoff_ok()
    assert torch.equal(y0, y2)
    assert (z0 - z2).abs().max().item() <= 2e-6
    assert (m0 - m2).abs().max().item() <= MAG_RTOL * m2.abs().max().item()
    for b in range(B):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), fs, L, M, orc.CONFIG3_GAINS, K, 4096)
        assert np.max(np.abs(y0[b].cpu().numpy() - ry)) <= 2e-6 * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z0[b].cpu().numpy() - rz)) <= EQ_ATOL
        assert np.max(np.abs(m0[b].cpu().numpy() - rmag)) <= MAG_RTOL * np.max(rmag)


def test_drop_in_equaliser_handoff_give_up_falls_back(gpu):
    """The drop-in's single-pass cascade reads the hand-off status for numpy
    calls: with every wait giving up at once (spin limit 0, chained tiles
    forced) it resets the workspace and reruns the rows on the two-pass
    cascade, so the result is still the reference's; the next call is clean."""
    from dspcore import _lib
    from oracle import dsp_ref_cpu as orc
    import modules.dsp_core as dc
    x = np.random.default_rng(9).uniform(-1, 1, (4, 48000)) * 0.8
    ref = np.stack([orc.equaliser(r, 48000, orc.CONFIG3_GAINS) for r in x])
    prev = _lib.spin_limit(0)
    try:
        with _chain_path(2):
            z = dc.sistema_ecualizador(x, 48000, orc.CONFIG3_GAINS)
    finally:
        _lib.spin_limit(prev)
    assert np.max(np.abs(z - ref)) <= EQ_ATOL
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        with _chain_path(2):
            z2 = dc.sistema_ecualizador(x, 48000, orc.CONFIG3_GAINS)
        names = [nm for nm, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    assert "chain_tile" in names and not any(nm.startswith("iir") for nm in names), names
    assert np.max(np.abs(z2 - ref)) <= EQ_ATOL


def test_library_dtype_conversions(gpu):
    """ops.convert (dsp_convert_f64_f32 / dsp_convert_f32_f64): numpy's astype
    bits both ways, real and complex, odd lengths; no torch kernel."""
    from dspcore import _lib, ops
    rng = np.random.default_rng(2)
    a = rng.standard_normal(10007) * np.logspace(-45, 38, 10007)
    t = torch.from_numpy(a).to(gpu)
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        f = ops.convert(t, torch.float32)
        d = ops.convert(f, torch.float64)
        names = [nm for nm, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    assert names == ["convert", "convert"], names
    np.testing.assert_array_equal(f.cpu().numpy().view(np.uint32), a.astype(np.float32).view(np.uint32))
    np.testing.assert_array_equal(d.cpu().numpy(), a.astype(np.float32).astype(np.float64))
    c = (a[:5000] + 1j * a[5000:10000]).reshape(50, 100)
    tc = ops.convert(torch.from_numpy(c).to(gpu), torch.complex64)
    assert tc.shape == (50, 100)
    np.testing.assert_array_equal(tc.cpu().numpy().view(np.uint32),
                                  c.astype(np.complex64).view(np.uint32))


@pytest.mark.parametrize("B,n_in", [(1, 441001), (1, 3073), (1, 97), (1, 48002), (3, 48001)])
def test_cascade_alone_any_length(gpu, B, n_in):
    """The one-tap single-pass cascade for rows whose length is not a multiple
    of 4 (an arbitrary clip): one row runs it (its x loads stop at the row's
    end by the buffer range check), a batch of such rows (pitch not a
    multiple of 4) the two-pass cascade; both within 1e-5 of the oracle, a
    NaN at the last sample relabelled as the two-pass cascade does."""
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    import modules.dsp_core as dc
    n_fft = 4096 if n_in >= 3000 else 128
    cfg = ChainConfig(n_in, 48000, 1, 1, None, orc.CONFIG3_GAINS, n_fft=n_fft)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len == 48
    gen = torch.Generator(device=gpu).manual_seed(n_in)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0, -1] = float("nan")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        (_, z1, _), names = _traced(lambda: ch.run(x))
        (_, z0, _), _ = _traced(lambda: ch.run_stages(x))
    assert ("chain_tile" in names) == (B == 1), names
    a, b = z1.cpu().numpy(), z0.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    fin = np.isfinite(b)
    assert np.max(np.abs(a[fin] - b[fin])) <= 2e-6
    xh = x.cpu().numpy()
    for r in range(B):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            rz = orc.equaliser(xh[r].astype(np.float64), 48000, orc.CONFIG3_GAINS)
        np.testing.assert_array_equal(np.isnan(a[r]), np.isnan(rz))
        f = np.isfinite(rz)
        assert np.max(np.abs(a[r][f] - rz[f])) <= EQ_ATOL
    # the drop-in on the numpy row (one channel: the single-pass kernel)
    xs = xh[0].astype(np.float64)
    xs[-1] = 0.25
    z = dc.sistema_ecualizador(xs, 48000, orc.CONFIG3_GAINS)
    assert np.max(np.abs(z - orc.equaliser(xs, 48000, orc.CONFIG3_GAINS))) <= EQ_ATOL
