"""FFTs above one four-step transform (ABI 2.7, csrc/fft_split.hip): the
reference's top radix-2 level (/root/reference/modules/dsp_core.py:41-66:
pares / impares, t = W_N^k impares, X = [pares + t, pares - t]) around two
transforms of half the length, for 2^31 and 2^32 points.

At small sizes the test hook dsp_fft_split_log2n sends four-step lengths
through the same code (nested twice at 2^18), against one four-step transform
of the row: within 1e-5 of max|X|, the same inf / NaN classes; with the odd
samples zero both output halves are the even samples' transform bit for bit.
At 2^31 (real input, 8 GB): against the top level restated in float64 torch
arithmetic over two 2^30 transforms of the same halves, and the zero-odd
identity."""
import contextlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FFT_RTOL = 1e-5


@contextlib.contextmanager
def _split_from(log2n):
    from dspcore import _lib
    lib = _lib.load()
    prev = lib.dsp_fft_split_log2n(log2n)
    assert prev >= 0, _lib.last_error()
    try:
        yield
    finally:
        lib.dsp_fft_split_log2n(prev)


def _traced(fn):
    from dspcore import _lib
    _lib.trace_enable(True)
    _lib.trace_read()
    try:
        out = fn().clone()
        names = [n for n, _ in _lib.trace_read()]
    finally:
        _lib.trace_enable(False)
    return out, names


@pytest.mark.parametrize("log2n,real,B", [(16, True, 2), (17, False, 3), (18, True, 1),
                                          (20, False, 2), (23, True, 1)])
def test_split_matches_one_transform(gpu, log2n, real, B):
    from dspcore import ops
    N = 1 << log2n
    gen = torch.Generator(device=gpu).manual_seed(log2n)
    x = torch.rand((B, N), generator=gen, device=gpu) * 2 - 1
    if not real:
        x = torch.complex(x, torch.rand((B, N), generator=gen, device=gpu) * 2 - 1)
    ref, names0 = _traced(lambda: ops.fft(x))
    with _split_from(16):
        got, names = _traced(lambda: ops.fft(x))
    assert "fft_split" not in names0 and "fft_split" in names, names
    # nested: 2^18 splits into 2^17, which splits into 2^16, which splits again
    assert names.count("fft_split") >= 2 ** (min(log2n, 18) - 15), names
    err = (got - ref).abs().max().item()
    assert err <= FFT_RTOL * ref.abs().max().item(), err
    # odd samples zero: both halves are the even samples' transform, bitwise
    xe = x.clone()
    xe[:, 1::2] = 0
    with _split_from(16):
        ge = ops.fft(xe)
        half = ops.fft(xe[:, 0::2].contiguous())   # (the same code for 2^(n-1))
    assert torch.equal(ge[:, : N // 2], half) and torch.equal(ge[:, N // 2:], half)


def test_split_nonfinite_classes(gpu):
    """inf / NaN through the split: every output component's class equals the
    one-transform path's (both the reference's, tests/test_gpu_nonfinite.py)."""
    from dspcore import ops
    N = 1 << 17
    gen = torch.Generator(device=gpu).manual_seed(5)
    x = torch.rand((3, N), generator=gen, device=gpu) * 2 - 1
    x[0, 7] = float("inf")
    x[1, 1000] = float("nan")
    x[2, 2] = float("inf")
    x[2, 3] = float("-inf")
    xc = torch.complex(x, torch.zeros_like(x))
    xc[1, 5] = complex(0.0, float("inf"))
    for inp in (x, xc):
        ref = ops.fft(inp).cpu().numpy()
        with _split_from(16):
            got = ops.fft(inp).cpu().numpy()
        for part in (np.real, np.imag):
            a, b = part(got), part(ref)
            for f in (np.isnan, np.isposinf, np.isneginf):
                np.testing.assert_array_equal(f(a), f(b))
            fin = np.isfinite(b)
            if fin.any():       # (a row with an inf and a NaN is NaN everywhere)
                assert np.max(np.abs(a[fin] - b[fin])) <= FFT_RTOL * np.max(np.abs(b[fin]))


@pytest.mark.timeout(400)
def test_fft_2_31_real(gpu):
    """One 2^31-point real row: X against the top level restated in float64
    over the halves' two 2^30 transforms (the split's own inputs), and the
    zero-odd identity at full size."""
    from dspcore import ops
    N = 1 << 31
    h = N // 2
    gen = torch.Generator(device=gpu).manual_seed(31)
    x = torch.rand((1, N), generator=gen, device=gpu) * 2 - 1
    X = ops.fft(x)
    assert X.shape == (1, N) and X.dtype == torch.complex64
    E = ops.fft(x[:, 0::2].contiguous())[0]
    O = ops.fft(x[:, 1::2].contiguous())[0]
    del x
    torch.cuda.empty_cache()
    scale = 0.0
    worst = 0.0
    step = 1 << 26
    for k0 in range(0, h, step):
        k = torch.arange(k0, k0 + step, device=gpu, dtype=torch.float64)
        w = torch.polar(torch.ones_like(k), -2 * np.pi * k / N)
        t = w * O[k0:k0 + step].to(torch.complex128)
        e = E[k0:k0 + step].to(torch.complex128)
        lo, hi = e + t, e - t
        scale = max(scale, lo.abs().max().item(), hi.abs().max().item())
        worst = max(worst, (X[0, k0:k0 + step].to(torch.complex128) - lo).abs().max().item(),
                    (X[0, h + k0:h + k0 + step].to(torch.complex128) - hi).abs().max().item())
    assert worst <= FFT_RTOL * scale, (worst, scale)
    del X, E, O
    torch.cuda.empty_cache()
    # odd samples zero: both halves are the 2^30 transform of the even ones
    xe = torch.zeros((1, N), device=gpu)
    xe[0, 0::2] = torch.rand(h, generator=gen, device=gpu) * 2 - 1
    Xe = ops.fft(xe)
    half = ops.fft(xe[:, 0::2].contiguous())
    assert torch.equal(Xe[:, :h], half) and torch.equal(Xe[:, h:], half)
