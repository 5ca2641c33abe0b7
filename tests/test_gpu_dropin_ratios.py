"""Every slider position of the app's SRC (L, M in 1..8, /root/reference/app.py:
149-150) through the drop-in exactly as app.py calls it -- conversion_tasa_muestreo
(:164), sistema_ecualizador (:167), the three calcular_espectro_magnitud calls on
the first 100000 samples of x, y and z (:203-205) -- against the oracle's
restatement of dsp_core.py:133-173, 216-254 and 68-98 on the same numpy input:
y within the SRC tolerance, z within the EQ tolerance, |X| within 1e-5 of its
peak, the same frequency axes and fs', and the reference's ValueError wherever
its segment rule meets a length that is not a power of two."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SRC_ATOL = 2e-6
EQ_ATOL = 1e-5
MAG_RTOL = 1e-5
GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5,
         "Brilliance": -6}


def _spectrum_or_error(fn, x, fs):
    try:
        return fn(x, fs)
    except ValueError:
        return None


@pytest.mark.parametrize("M", range(1, 9))
@pytest.mark.parametrize("L", range(1, 9))
def test_app_rerun_every_ratio(gpu, L, M):
    from modules import dsp_core as dc
    from oracle import dsp_ref_cpu as orc
    fs, n = 44100, 8192
    rng = np.random.default_rng(10 * L + M)
    x = (0.6 * np.sin(2 * np.pi * 440.0 * np.arange(n) / fs)
         + 0.4 * rng.uniform(-1, 1, n)).astype(np.float32)
    x /= np.max(np.abs(x))
    y, fs2 = dc.conversion_tasa_muestreo(x, fs, M, L)
    ry, rfs2 = orc.resample(x, fs, M, L)
    assert fs2 == rfs2 and y.shape == ry.shape
    if L == M == 1:
        assert y is x                      # dsp_core.py:144-145 returns its input
    else:
        assert y.dtype == np.float64
        assert np.max(np.abs(y - ry)) <= SRC_ATOL * max(1.0, np.abs(ry).max())
    z = dc.sistema_ecualizador(y, fs2, GAINS)
    rz = orc.equaliser(ry, rfs2, GAINS)
    assert z.shape == rz.shape and z.dtype == np.float64
    assert np.max(np.abs(z - rz)) <= EQ_ATOL
    lim = 100000
    for v, rv, f in ((x, x, fs), (y, ry, fs2), (z, rz, fs2)):
        n_v = min(len(v), lim)
        seg = min(2048, n_v - n_v // 2) if n_v > 2048 else 1 << (n_v - 1).bit_length()
        got = _spectrum_or_error(dc.calcular_espectro_magnitud, v[:lim], f)
        if seg & (seg - 1):
            # a segment that is not a power of two: the reference's recursion
            # raises there (dsp_core.py:55-64 adds halves of unequal length),
            # and so does the drop-in (design.spectrum_plan)
            assert got is None, (n_v, seg)
            assert _spectrum_or_error(orc.spectrum, rv[:lim], f) is None, (n_v, seg)
            continue
        (fg, mg), (fr, mr) = got, orc.spectrum(rv[:lim], f)
        np.testing.assert_array_equal(fg, fr)
        assert mg.shape == mr.shape and mg.dtype == np.float64
        assert np.max(np.abs(mg - mr)) <= MAG_RTOL * np.max(mr)
