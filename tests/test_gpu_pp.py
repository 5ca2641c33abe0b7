"""The per-phase single-pass chain kernels (csrc/chain_pp.h, round 6) on the
GPU: every SRC ratio of the reference app's sliders (L, M in 1..8,
/root/reference/app.py:149-150) at the default tap rule K = 40 max(L, M) + 1
(/root/reference/modules/dsp_core.py:158), and config 1's 2/1 at K = 127.

For each: the single-pass kernel is what ran (dsp_chain_tile_len > 0, the
traced launch is chain_tile, no src_poly); against the two-launch chain
(dsp_chain_path(1): SRC kernel + two-pass cascade) on the same batch y is
bitwise equal (one summation order, csrc/src_poly.hip), z within 2e-6 and |X|
within 1e-5 of the largest; rows against the oracle (dsp_core.py:133-254 and
:68-98 restated in oracle/dsp_ref_cpu.py) within the parity tolerances; a row
driven into the clip, a row silent for its first half, ragged last tiles.
Non-finite input (NaN, +inf, -inf at a tile's first sample, mid-row and the
last sample) through the repair kernel: y's NaN / +inf / -inf masks and z's NaN
mask equal to the two-launch chain's (itself pinned to the reference's
semantics, tests/test_gpu_nonfinite.py), finite values as above.
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

CASES = [(L, M, None) for L in range(1, 9) for M in range(1, 9) if (L, M) != (1, 1)]
CASES += [(2, 1, 127)]


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
        out = tuple(t.clone() for t in fn())
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    return out, names


@pytest.mark.parametrize("L,M,K", CASES, ids=[f"{L}/{M}" + (f"K{K}" if K else "") for L, M, K in CASES])
def test_app_ratio_single_pass(gpu, L, M, K):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, fs = 5, 48000
    n_in = 9600 if L >= M else 40000   # n_out > 4096: the spectrum's centre segment (2048)
    cfg = ChainConfig(n_in, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len > 0
    gen = torch.Generator(device=gpu).manual_seed(L * 16 + M)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    # drive the clip (x 8: at x 40, as config 3's tests drive it, the float32
    # rounding of y -- both paths' EQ input, while the oracle filters float64
    # y and the two-launch chain's carries come from float64 taps -- is worth
    # 2-3e-6 of z at the app's low output rates 6..35 kHz, the whole budget)
    x[1] *= 8.0
    x[2, : n_in // 2] = 0.0           # silence then signal
    (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
    with _chain_path(1):
        (y0, z0, m0), names0 = _traced(lambda: ch.run(x))
    assert "chain_tile" in names1 and "src_poly" not in names1, names1
    assert "chain_tile" not in names0, names0
    assert ch.handoff_ok()
    assert torch.equal(y1, y0), float((y1 - y0).abs().max())
    assert (z1 - z0).abs().max().item() <= 2e-6
    assert (m1 - m0).abs().max().item() <= MAG_RTOL * m0.abs().max().item()
    y, z, mag = (t.cpu().numpy() for t in (y1, z1, m1))
    if not ch.eq.bypass and ch.eq.sos.shape[0]:
        assert np.abs(z[1]).max() == 1.0
    for b in (0, 1, 2):
        ry, rz, _, rmag, _ = orc.chain(x[b].cpu().numpy(), fs, L, M, orc.CONFIG3_GAINS, K, 2048)
        assert y.shape[1] == ry.size
        assert np.max(np.abs(y[b] - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
        assert np.max(np.abs(z[b] - rz)) <= EQ_ATOL
        assert np.max(np.abs(mag[b] - rmag)) <= MAG_RTOL * np.max(rmag)


NF_CASES = [(2, 1, None), (4, 3, None), (1, 2, None), (3, 4, None), (8, 7, None), (2, 1, 127),
            (5, 5, None)]


@pytest.mark.parametrize("L,M,K", NF_CASES, ids=[f"{L}/{M}" + (f"K{K}" if K else "")
                                                 for L, M, K in NF_CASES])
def test_app_ratio_nonfinite_matches_two_launch(gpu, L, M, K):
    from dspcore.chain import Chain, ChainConfig
    from oracle import dsp_ref_cpu as orc
    B, n_in, fs = 4, 12000, 48000
    cfg = ChainConfig(n_in, fs, L, M, K, orc.CONFIG3_GAINS, n_fft=2048)
    ch = Chain(cfg, B, gpu)
    assert ch.tile_len > 0
    tile_in = 64 * ch.tile_len * M // L          # inputs per tile (approx.)
    gen = torch.Generator(device=gpu).manual_seed(99)
    x = torch.rand((B, n_in), generator=gen, device=gpu) * 2 - 1
    x[0, min(tile_in, n_in - 1)] = float("nan")
    x[1, n_in // 2] = float("inf")
    x[1, n_in // 2 + 3] = float("-inf")
    x[2, n_in - 1] = float("-inf")
    x[3, 0] = float("inf")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        (y1, z1, m1), names1 = _traced(lambda: ch.run(x))
        with _chain_path(1):
            (y0, z0, m0), _ = _traced(lambda: ch.run(x))
    assert "chain_tile" in names1 and "chain_repair" in names1, names1
    for a, b, what in ((y1, y0, "y"), (z1, z0, "z")):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        for f in (np.isnan, np.isposinf, np.isneginf):
            np.testing.assert_array_equal(f(a), f(b), err_msg=what)
        fin = np.isfinite(b)
        tol = 0.0 if what == "y" else 2e-6
        assert np.max(np.abs(a[fin] - b[fin])) <= tol, what
    mg1, mg0 = m1.cpu().numpy(), m0.cpu().numpy()
    np.testing.assert_array_equal(np.isnan(mg1), np.isnan(mg0))
