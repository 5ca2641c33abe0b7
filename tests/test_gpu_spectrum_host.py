"""The drop-in spectrum's and FFT's zero-copy routes (ops.spectrum_host,
ops.fft_host; the FFT's rows are dsp_core.py:41-66's input): the centre
segments of calcular_espectro_magnitud (/root/reference/modules/dsp_core.py:
74-98) are cast by numpy into page-locked host memory, which the spectrum
kernel reads directly, and |X| comes back the same way.  Same kernel, same
float32 rows: every result is bitwise the device route's (ops.spectrum on a
device copy of the rows), including across calls that reuse the staging
buffers with new data and for inf / NaN rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _device_route(ops, seg, n_fft, dev):
    t = torch.from_numpy(np.ascontiguousarray(seg, dtype=np.float32)).to(dev)
    return ops.spectrum(t, 0, seg.shape[1], n_fft).cpu().numpy()


@pytest.mark.parametrize("B,seg_len,n_fft", [(1, 2048, 2048), (1, 1000, 1024), (3, 4096, 4096),
                                             (5, 128, 128), (1, 16384, 16384), (2, 3, 4)])
def test_host_route_bitwise_device_route(gpu, B, seg_len, n_fft):
    from dspcore import ops
    rng = np.random.default_rng(seg_len + B)
    for rep in range(3):            # the staging buffers reused with new data
        seg = rng.uniform(-1, 1, (B, seg_len))
        got = ops.spectrum_host(seg, n_fft, gpu)
        assert got is not None and got.dtype == np.float32 and got.shape == (B, n_fft // 2 + 1)
        np.testing.assert_array_equal(got, _device_route(ops, seg, n_fft, gpu))


def test_host_route_nonfinite(gpu):
    from dspcore import ops
    seg = np.random.default_rng(9).uniform(-1, 1, (4, 2048))
    seg[0, 0] = np.inf
    seg[1, 1000] = np.nan
    seg[2, 5] = -np.inf
    seg[2, 6] = np.inf
    got = ops.spectrum_host(seg, 2048, gpu)
    np.testing.assert_array_equal(got, _device_route(ops, seg, 2048, gpu))   # (NaN == NaN here)
    # and a finite call right after one that took the repair path
    fin = np.random.default_rng(10).uniform(-1, 1, (4, 2048))
    np.testing.assert_array_equal(ops.spectrum_host(fin, 2048, gpu),
                                  _device_route(ops, fin, 2048, gpu))


def test_host_route_declines(gpu):
    from dspcore import ops
    assert ops.spectrum_host(np.zeros((1, 1 << 15)), 1 << 15, gpu) is None   # four-step length
    big = (ops.SPECTRUM_HOST_MAX_BYTES // (4 * 2048)) + 1
    assert ops.spectrum_host(np.zeros((big, 2048)), 2048, gpu) is None


@pytest.mark.parametrize("n", [441000, 100000, 2049 + 2047, 2048, 1500, 1])
def test_dropin_matches_tensor_call(gpu, n):
    """The drop-in on numpy (host route) against the same call on a device
    tensor (device route): bitwise, float64 out for numpy."""
    from modules import dsp_core as dc
    x = np.random.default_rng(n).uniform(-1, 1, n)
    f, m = dc.calcular_espectro_magnitud(x, 44100)
    ft, mt = dc.calcular_espectro_magnitud(torch.from_numpy(x.astype(np.float32)).to(gpu), 44100)
    assert m.dtype == np.float64 and isinstance(m, np.ndarray)
    np.testing.assert_array_equal(f, ft)
    np.testing.assert_array_equal(m, mt.cpu().numpy().astype(np.float64))
    # 2-D numpy batch: per row the same
    xb = np.stack([x, -x, 0.5 * x])
    _, mb = dc.calcular_espectro_magnitud(xb, 44100)
    assert mb.shape == (3, m.shape[0])
    np.testing.assert_array_equal(mb[0], m)


# --------------------------------------------------------------------------- FFT
def _fft_device_route(ops, x, dev):
    ft = np.complex64 if np.iscomplexobj(x) else np.float32
    return ops.fft(torch.from_numpy(np.ascontiguousarray(x, dtype=ft)).to(dev)).cpu().numpy()


@pytest.mark.parametrize("B,n,cplx", [(1, 2, False), (1, 1024, False), (3, 2048, True),
                                      (2, 16384, False), (1, 16384, True), (4, 8, True)])
def test_fft_host_route_bitwise_device_route(gpu, B, n, cplx):
    """fft_diezmado_en_tiempo's host route (dsp_core.py:41-66 on a few short
    rows): X bitwise the device route's, with the staging buffers reused."""
    from dspcore import ops
    rng = np.random.default_rng(n + B)
    for rep in range(3):
        x = rng.uniform(-1, 1, (B, n))
        if cplx:
            x = x + 1j * rng.uniform(-1, 1, (B, n))
        got = ops.fft_host(x, gpu, np.complex128)
        assert got is not None and got.dtype == np.complex128 and got.shape == (B, n)
        np.testing.assert_array_equal(got, _fft_device_route(ops, x, gpu).astype(np.complex128))


def test_fft_host_route_nonfinite_and_declines(gpu):
    from dspcore import ops
    x = np.random.default_rng(4).uniform(-1, 1, (3, 4096))
    x[0, 3] = np.inf
    x[1, 100] = np.nan
    x[2, 0] = -np.inf
    np.testing.assert_array_equal(ops.fft_host(x, gpu), _fft_device_route(ops, x, gpu))
    assert ops.fft_host(np.zeros((1, 1 << 15)), gpu) is None          # four-step length
    big = ops.SPECTRUM_HOST_MAX_BYTES // (8 * 4096) + 1
    assert ops.fft_host(np.zeros((big, 4096)), gpu) is None


@pytest.mark.parametrize("n", [2, 64, 4096])
def test_fft_dropin_matches_tensor_call(gpu, n):
    from modules import dsp_core as dc
    x = np.random.default_rng(n).uniform(-1, 1, n)
    X = dc.fft_diezmado_en_tiempo(x)
    Xt = dc.fft_diezmado_en_tiempo(torch.from_numpy(x.astype(np.float32)).to(gpu))
    assert X.dtype == np.complex128 and X.shape == (n,)
    np.testing.assert_array_equal(X, Xt.cpu().numpy().astype(np.complex128))
    xb = np.stack([x, 2 * x])
    Xb = dc.fft_diezmado_en_tiempo(xb)
    assert Xb.shape == (2, n) and Xb.dtype == np.complex128
    np.testing.assert_array_equal(Xb[0], X)
