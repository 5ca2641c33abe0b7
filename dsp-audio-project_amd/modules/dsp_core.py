"""Drop-in replacement for reference modules/dsp_core.py, backed by gfx950 HIP.

`from modules.dsp_core import cargar_senal_audio, conversion_tasa_muestreo,
sistema_ecualizador, calcular_espectro_magnitud` (reference app.py:13-18) works
unchanged with this directory on sys.path.  All eight public functions keep the
reference names, argument order and meaning (dsp_core.py:10,41,68,104,133,179,
205,216), return types and error behaviour:

* 1-D numpy in -> numpy out with the reference dtypes (float64 / complex128);
  identity paths return the very same object (SRC with L == M == 1, the EQ
  bypass, an FFT of length <= 1);
* 2-D numpy [B, n] in -> the same, per row (batched; the reference cannot take
  2-D signals, so this extends rather than changes its contract); from
  SHARD_MIN_ROWS rows on a node with several GPUs the rows are sharded over
  all of them (bitwise the one-GPU result) -- only in a single-process
  program on device 0: with torch.distributed initialised, or another current
  device (a rank that picked its GPU with set_device), every call stays on the
  current device; DSPCORE_SHARD=0 / 1 in the environment turns sharding off /
  on regardless;
* a ROCm torch tensor ([n] or [B, n]) in -> a device tensor out, float32 /
  complex64, left on the GPU with no synchronisation.

The numeric work (SRC convolution, biquad recursion, FFT, window, magnitude)
runs only in libdspcore.so.  Host numpy is used for what the reference itself
does once per call in float64: filter design, band selection, size rules and
the frequency axis.  Without a GPU these functions raise RuntimeError.

Deliberate differences, documented in DESIGN.md:
* the SRC/EQ/FFT data path computes in float32 with float64 IIR state, within
  the tolerances of tests/ (SRC atol 2e-6, EQ atol 1e-5, FFT 1e-5 * max|X|);
* fft_diezmado_en_tiempo raises ValueError for every length that is not a
  power of two (the reference raises for most and returns a wrong-length
  array for N = 3), and RuntimeError above 2^32 points (the reference's
  pure-Python recursion has no limit but takes hours there);
* keyword-only extensions: conversion_tasa_muestreo(..., num_taps=None) and
  calcular_espectro_magnitud(..., n_fft=2048); one added function,
  calcular_espectrograma_magnitud (every frame).
"""
from __future__ import annotations

import numpy as np

from dspcore import design as _design

__all__ = [
    "cargar_senal_audio", "fft_diezmado_en_tiempo", "calcular_espectro_magnitud",
    "generar_respuesta_impulso_sinc", "conversion_tasa_muestreo",
    "disenar_coeficientes_diferencias", "aplicar_ecuacion_diferencias",
    "sistema_ecualizador", "calcular_espectrograma_magnitud",
]


def _ops():
    from dspcore import ops
    ops.require_gpu()
    return ops


def _is_tensor(x) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


def _to_rows(x, complex_ok=False):
    """-> (device tensor [B, n], how) where how in {'np1', 'np2', 't1', 't2'}."""
    import torch
    ops = _ops()
    dev = torch.device("cuda", torch.cuda.current_device())
    if _is_tensor(x):
        t = x if x.is_cuda else x.to(dev)
        how = "t1" if t.dim() == 1 else "t2"
        if t.dim() == 1:
            t = t.unsqueeze(0)
        if not (complex_ok and t.is_complex()):
            t = t.to(torch.float32)
        else:
            t = t.to(torch.complex64)
        return t.contiguous(), how
    a = np.asarray(x)
    if a.ndim not in (1, 2):
        raise ValueError(f"expected a 1-D signal or a [B, n] batch, got shape {a.shape}")
    how = "np1" if a.ndim == 1 else "np2"
    a2 = a.reshape(1, -1) if a.ndim == 1 else a
    cplx = complex_ok and np.iscomplexobj(a2)
    if a2.flags.c_contiguous and a2.dtype == (np.complex128 if cplx else np.float64):
        # float64 / complex128 rows (what the reference's functions return and
        # app.py passes on): copied as stored and narrowed on the device by the
        # library (ops.convert: numpy's astype rounding), without a fresh host
        # array to fault in
        return ops.convert(torch.from_numpy(a2).to(dev),
                           torch.complex64 if cplx else torch.float32), how
    host = np.ascontiguousarray(a2, dtype=np.complex64 if cplx else np.float32)
    return torch.from_numpy(host).to(dev), how


# Results up to this size come back through page-locked host memory (torch's
# caching host allocator: reused across calls, one DMA, no page faults on a
# fresh array); larger ones through a pageable copy.
PINNED_MAX_BYTES = 256 << 20


def _from_rows(t, how, np_dtype):
    if how in ("t1", "t2"):
        return t[0] if how == "t1" else t
    import torch
    tdt = {np.dtype(np.float64): torch.float64, np.dtype(np.complex128): torch.complex128,
           np.dtype(np.float32): torch.float32,
           np.dtype(np.complex64): torch.complex64}.get(np.dtype(np_dtype))
    if tdt is None or t.numel() * tdt.itemsize > PINNED_MAX_BYTES:
        host = t.cpu().numpy().astype(np_dtype)
    else:
        # into a pinned buffer that the returned array keeps alive: as stored
        # by one copy, or widened by the library's cast kernel (float32 ->
        # float64 is exact) writing straight into the pinned buffer (no copy
        # launch: 0.094 -> 0.079 ms for 441000 samples, tools/host_io_probe.py)
        pinned = torch.empty(tuple(t.shape), dtype=tdt, pin_memory=True)
        if t.dtype == tdt:
            pinned.copy_(t)
        else:
            _ops().convert(t.contiguous(), tdt, out=pinned)
            torch.cuda.current_stream(t.device).synchronize()
        host = pinned.numpy()
    return host[0] if how == "np1" else host


# 2-D numpy batches of at least this many rows use every visible GPU.
SHARD_MIN_ROWS = 256


def _run(x, fn, np_dtype, complex_ok=False):
    """fn(device rows [b, n], B) -> device rows, applied to x as _to_rows takes
    it, the result as _from_rows gives it.  A 2-D numpy batch of at least
    SHARD_MIN_ROWS rows on a node with several GPUs is cut into contiguous row
    shards, one per visible device (dspcore.shard.shard_ranges), each run from
    its own host thread; B is the whole batch's row count, so a shard plans as
    the whole batch does and its rows are bitwise the unsharded ones."""
    import torch
    devices = _shard_devices() if not _is_tensor(x) else []
    if len(devices) > 1 and np.ndim(x) == 2 and np.shape(x)[0] >= SHARD_MIN_ROWS:
        import threading
        from dspcore.shard import shard_ranges
        a = np.asarray(x)
        B = a.shape[0]
        host = np.complex64 if complex_ok and np.iscomplexobj(a) else np.float32
        ranges = shard_ranges(B, len(devices))
        results: list = [None] * len(ranges)
        errors: list = []

        def worker(i, lo, hi):
            try:
                dev = devices[i]
                with torch.cuda.device(dev):
                    t = torch.from_numpy(np.ascontiguousarray(a[lo:hi], dtype=host)).to(dev)
                    results[i] = fn(t, B).cpu().numpy()
            except BaseException as e:  # re-raised on the caller's thread
                errors.append(e)

        threads = [threading.Thread(target=worker, args=(i, lo, hi))
                   for i, (lo, hi) in enumerate(ranges)]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        if errors:
            raise errors[0]
        return np.concatenate(results, axis=0).astype(np_dtype)
    t, how = _to_rows(x, complex_ok)
    return _from_rows(fn(t, t.shape[0]), how, np_dtype)


def _shard_devices():
    """The devices a large 2-D numpy batch is sharded over: every visible GPU,
    unless this looks like one rank of a multi-process job (torch.distributed
    initialised, or a current device other than 0), which must keep to its own
    GPU; DSPCORE_SHARD=0 / 1 overrides."""
    import os

    import torch
    env = os.environ.get("DSPCORE_SHARD", "")
    if env == "0":
        return []
    if env != "1":
        import torch.distributed as tdist
        if (tdist.is_available() and tdist.is_initialized()) or torch.cuda.current_device() != 0:
            return []
    return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]


def _cascade(ops, t, sos, clip, B):
    """The biquad cascade with the chunk length planned for B rows."""
    chunk = _design.chunk_len_for(int(t.shape[1]), _design.max_chunks_for(B))
    return ops.biquad_cascade(t, sos, clip=clip, chunk_len=chunk)


def _length(x) -> int:
    return int(x.shape[-1]) if (_is_tensor(x) or np.ndim(x) == 2) else len(x)


# ---------------------------------------------------------------------------
# I/O (app.py:14)
# ---------------------------------------------------------------------------
def cargar_senal_audio(buffer_archivo):
    """Load x[n]: read, average to mono, float32, peak-normalise (dsp_core.py:10-35).

    The WAV header is parsed on the host; decoding, the channel mean and the
    peak normalisation run on the GPU with the reference's arithmetic
    (dspcore/audio_io.py).  Any failure to read or decode returns
    (zeros(100, float32), 44100), as the reference's bare `except` does
    (:34-35); a missing GPU or library still raises RuntimeError.
    """
    from dspcore import audio_io
    try:
        x, fs = audio_io.load(buffer_archivo)
    except RuntimeError:
        raise
    except Exception:
        return np.zeros(100, dtype=np.float32), 44100
    return x.cpu().numpy(), fs


# ---------------------------------------------------------------------------
# Frequency analysis (dsp_core.py:41-98)
# ---------------------------------------------------------------------------
def fft_diezmado_en_tiempo(x):
    """Radix-2 decimation-in-time FFT (dsp_core.py:41-66), batched HIP kernel.

    Length <= 1 returns x unchanged (:52).  Power-of-two lengths up to 2^32
    give the natural-order DFT (complex128 for numpy input): one LDS-resident
    launch up to 2^14, a four-step transform (two launches, three from 2^23)
    up to 2^30, and above it the reference's own top radix-2 level around two
    transforms of half the length (csrc/fft_split.hip).  Other lengths raise
    ValueError; powers of two above 2^32 raise RuntimeError.
    """
    n = _length(x)
    if n <= 1:
        return x
    if n & (n - 1):
        raise ValueError(f"fft_diezmado_en_tiempo: length {n} is not a power of two")
    ops = _ops()
    if not _is_tensor(x):
        # a few short rows: read and answered in page-locked host memory
        # (ops.fft_host, as the spectrum's segments), no copy launches
        a = np.asarray(x)
        if a.ndim in (1, 2) and (a.ndim == 1 or a.shape[0] < SHARD_MIN_ROWS
                                 or len(_shard_devices()) <= 1):
            import torch
            X = ops.fft_host(a[None, :] if a.ndim == 1 else a,
                             torch.device("cuda", torch.cuda.current_device()), np.complex128)
            if X is not None:
                return X[0] if a.ndim == 1 else X
    return _run(x, lambda t, B: ops.fft(t), np.complex128, complex_ok=True)


def calcular_espectro_magnitud(x_n, fs, *, n_fft: int = _design.SPECTRUM_WINDOW):
    """|X[k]| of the Hann-windowed centre segment (dsp_core.py:68-98).

    Returns (frequencies, magnitudes), both of length N/2 + 1 where N is the
    transform length chosen by the reference's rule (see design.spectrum_plan).
    """
    plan = _design.spectrum_plan(_length(x_n), n_fft)
    ops = _ops()
    half = plan.n_fft // 2 + 1
    freqs = np.fft.rfftfreq(plan.n_fft, d=1 / fs)[:half]
    seg_start = plan.seg_start
    if not _is_tensor(x_n):
        # only the centre segment leaves the host (dsp_core.py:76-78 reads
        # nothing else); a few short segments (the app's call) are read and
        # answered by the kernel in page-locked host memory, no copy launches
        a = np.asarray(x_n)
        if a.ndim in (1, 2):
            seg = a[..., seg_start:seg_start + plan.seg_len]
            seg_start = 0
            if plan.seg_len and (a.ndim == 1 or a.shape[0] < SHARD_MIN_ROWS
                                 or len(_shard_devices()) <= 1):
                import torch
                mag = ops.spectrum_host(seg[None, :] if a.ndim == 1 else seg, plan.n_fft,
                                        torch.device("cuda", torch.cuda.current_device()),
                                        np.float64)
                if mag is not None:
                    return freqs, (mag[0] if a.ndim == 1 else mag)
            x_n = np.ascontiguousarray(seg)
    mag = _run(x_n, lambda t, B: ops.spectrum(t, seg_start, plan.seg_len, plan.n_fft),
               np.float64)
    return freqs, mag


def calcular_espectrograma_magnitud(x_n, fs, *, n_fft: int = _design.SPECTRUM_WINDOW,
                                    hop: int | None = None):
    """Extension (not in the reference): the recipe of calcular_espectro_magnitud
    (Hann window of dsp_core.py:87, FFT, |X[k]| for k <= N/2) applied to every
    frame of the signal instead of its centre segment.  Frames of n_fft samples
    every `hop` (default n_fft // 4) from the start, the last zero-padded
    (design.stft_plan).  Returns (frequencies [N/2+1], frame start times in
    seconds [frames], magnitudes [frames, N/2+1] -- or [B, frames, N/2+1])."""
    plan = _design.stft_plan(_length(x_n), n_fft, hop)
    ops = _ops()
    mag = _run(x_n, lambda t, B: ops.stft_magnitude(t, plan.n_fft, plan.hop, plan.frames),
               np.float64)
    freqs = np.fft.rfftfreq(plan.n_fft, d=1 / fs)[:plan.n_fft // 2 + 1]
    times = np.arange(plan.frames) * plan.hop / fs
    return freqs, times, mag


# ---------------------------------------------------------------------------
# Sampling and convolution (dsp_core.py:104-173)
# ---------------------------------------------------------------------------
def generar_respuesta_impulso_sinc(w_c_norm, L_taps):
    """Blackman-windowed sinc low-pass with unit DC gain (dsp_core.py:104-131)."""
    return _design.sinc_lowpass(w_c_norm, L_taps)


def conversion_tasa_muestreo(x_n, fs_original, M, L, *, num_taps=None):
    """Rational L/M sample-rate converter (dsp_core.py:133-173).

    Note the reference's argument order (x, fs, M, L).  L == M == 1 returns
    (x_n, fs_original) unchanged.  `num_taps` (keyword-only extension) overrides
    the default 40*max(L, M)+1 tap count.
    """
    if M == 1 and L == 1:
        return x_n, fs_original
    plan = _design.src_plan(_length(x_n), fs_original, M, L, num_taps)
    ops = _ops()
    return _run(x_n, lambda t, B: ops.src_polyphase(t, plan), np.float64), plan.fs_out


# ---------------------------------------------------------------------------
# IIR filtering (dsp_core.py:179-254)
# ---------------------------------------------------------------------------
def disenar_coeficientes_diferencias(fc, fs, ganancia_db):
    """Peaking-EQ biquad (b, a) with Q = 1, a[0] = 1 (dsp_core.py:179-203)."""
    return _design.peaking_biquad(fc, fs, ganancia_db)


def aplicar_ecuacion_diferencias(x_n, b, a):
    """y = lfilter(b, a, x), zero initial state (dsp_core.py:205-214), any order.

    Biquads and second-order sections of higher IIR orders (design.lfilter_plan,
    float64 on the host) run on the float64 biquad-cascade kernel, 16 sections
    a launch (float32 between launches, above order 32); with a of length 1,
    where lfilter convolves, b runs as a causal convolution on the SRC kernel
    (L = M = 1, float32 taps and sums; a gain is one tap), so an inf or NaN
    stays within len(b) samples as in lfilter; otherwise, after the cascade,
    one launch gives every output from the first inf or NaN on the +inf / -inf
    / NaN that lfilter's recursion gives it (dsp_lfilter_nonfinite_f32; orders
    up to 4096; above that the relabelling is skipped and a row keeps the
    cascade's all-NaN after its first non-finite sample).  a = [1, 0, ...] with
    a long b (an FIR through lfilter's recursion) convolves like the len(a) == 1
    case and then takes the recursion's labels.  a[0] == 0 raises ValueError as
    lfilter does.
    """
    plan = _design.lfilter_plan(b, a)
    ops = _ops()
    from dspcore import _lib
    # lfilter's recursion order (D = max(len(a), len(b)) - 1); above
    # DSP_LFILTER_NF_MAX the inf / NaN relabelling is not run: such rows keep
    # the cascade's all-NaN after the first non-finite sample (finite input is
    # unaffected).
    relabel = plan.kind != "fir" and max(plan.a.size, plan.b.size) - 1 <= _lib.DSP_LFILTER_NF_MAX

    def run(t, B):
        x0 = t
        if plan.kind in ("fir", "fir_rec"):
            n = int(t.shape[1])
            src = _design.SrcPlan(1, 1, int(plan.taps.size), plan.taps, 0, n, n, 0)
            t = ops.src_polyphase(t, src)
        else:
            for group in _design.lfilter_groups(plan.sos):   # any order: <= 16 sections a launch
                t = _cascade(ops, t, group, False, B)
        # inf / NaN from x's first non-finite sample on as lfilter labels them
        return ops.lfilter_nonfinite(x0, t, plan.b, plan.a) if relabel else t
    return _run(x_n, run, np.float64)


def sistema_ecualizador(x_n, fs, ganancias_bandas):
    """6-band peaking-EQ cascade + clip to [-1, 1] (dsp_core.py:216-254).

    One channel of any length, or rows of a multiple of 4 samples, run the
    single-pass kernel of the cascade alone (ops.eq_single_pass: x read once,
    z written once; a single long channel, as app.py:167 passes, takes its
    three-launch mode instead of chained tiles); other batches the two-pass
    cascade (ops.biquad_cascade)."""
    plan = _design.eq_plan(fs, ganancias_bandas)
    if plan.bypass:
        return x_n
    ops = _ops()
    if plan.sos.shape[0] > 0:
        out_dtype = np.float64
    else:  # no stage applied: np.clip of x_n.copy() keeps a floating dtype
        dt = np.asarray(x_n).dtype if not _is_tensor(x_n) else np.float32
        out_dtype = dt if np.issubdtype(dt, np.floating) else np.float64

    def run(t, B):
        # the single-pass cascade alone where it serves the rows (x read once,
        # z written once; one long channel takes its three-launch mode), else
        # the two-pass cascade
        # (numpy in: the hand-off status is read, as the result is synchronised
        # anyway; a tensor call stays asynchronous)
        z = (ops.eq_single_pass(t, plan.sos, plan_batch=B, check=not _is_tensor(x_n))
             if plan.sos.shape[0] else None)
        return z if z is not None else _cascade(ops, t, plan.sos, True, B)
    return _run(x_n, run, out_dtype)
