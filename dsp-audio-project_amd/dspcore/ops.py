"""Device-level operators: torch CUDA tensors in, torch CUDA tensors out.

Each function launches the matching libdspcore entry point on the current
torch stream of the tensor's device and returns without synchronising.  The
tensors are only device buffers (PyTorch-ROCm plumbing); all arithmetic is in
the hand-written HIP kernels.  Layout: row-major [B, n] float32 (complex64 for
FFT data), one row per audio channel.
"""
from __future__ import annotations

import threading
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .design import SrcPlan, chunk_len_for, hann, max_chunks_for, state_response_table, twiddles
from .design import xstate_table as xstate_table_host

_tables_lock = threading.Lock()
_tables: OrderedDict = OrderedDict()   # every device LUT kind, one LRU
TABLE_CACHE_MAX = 256                  # entries (slider sweeps make new keys)


def _cached(key, build):
    """The device LUT for `key`, built by `build()` on a miss; one LRU of at
    most TABLE_CACHE_MAX entries for every kind (hann, twiddles, Bluestein,
    G, GX).  Callers that hold a table keep it alive past its eviction."""
    with _tables_lock:
        t = _tables.get(key)
        if t is not None:
            _tables.move_to_end(key)
            return t
    t = build()
    with _tables_lock:
        t = _tables.setdefault(key, t)
        _tables.move_to_end(key)
        while len(_tables) > TABLE_CACHE_MAX:
            _tables.popitem(last=False)
    return t


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "dspcore needs a ROCm GPU (MI355X/gfx950): torch.cuda.is_available() is False; "
            "there is no CPU fallback")
    _lib.load()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _table(kind: str, n: int, device: torch.device) -> torch.Tensor:
    """Cached per-device LUTs: Hann window (fp32[n]) and twiddles (fp32[2*(n/2)])."""
    def build():
        if kind == "hann":
            host = hann(n).astype(np.float32)
        else:  # in slices: 2^29 float64 twiddles at once would hold ~24 GB of host temporaries
            half = max(n // 2, 1)
            host = np.empty(half, dtype=np.complex64)
            for k0 in range(0, half, 1 << 22):
                k1 = min(half, k0 + (1 << 22))
                host[k0:k1] = twiddles(n, k0, k1)
            host = host.view(np.float32)
        return torch.from_numpy(np.ascontiguousarray(host)).to(device)
    return _cached((kind, n, device.index), build)


def _rows(x: torch.Tensor, name: str) -> torch.Tensor:
    if not x.is_cuda:
        raise ValueError(f"{name} must be a CUDA (ROCm) tensor")
    if x.dim() != 2:
        raise ValueError(f"{name} must be [B, n], got shape {tuple(x.shape)}")
    if x.stride(1) != 1 or (x.shape[0] > 1 and x.stride(0) < x.shape[1]):
        x = x.contiguous()
    return x


def ld(x: torch.Tensor) -> int:
    """Row pitch in elements.  A single row's stride(0) is only a pitch when it
    covers the row (a [1, n] view of a padded buffer keeps its padded pitch,
    which the aligned kernels need); otherwise the row length stands in."""
    if x.shape[0] > 1:
        return x.stride(0)
    return x.stride(0) if x.stride(0) >= x.shape[1] else x.shape[1]


def taps_tensor(plan: SrcPlan, device: torch.device) -> torch.Tensor:
    """The library's float32 taps (design.caller_taps; it flushes the sinc-zero
    noise itself, design.kernel_taps)."""
    from .design import caller_taps
    host = caller_taps(plan)
    # cached: the app's reruns take the same few designs (one fewer copy a call)
    return _cached(("taps", host.tobytes(), device.index),
                   lambda: torch.from_numpy(host).to(device))


def src_polyphase(x: torch.Tensor, plan: SrcPlan, taps: torch.Tensor | None = None,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """y = SRC(x) for every row (dsp_core.py:148-170), fp32."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    B, n_in = x.shape
    if n_in != plan.n_in:
        raise ValueError(f"plan is for n_in={plan.n_in}, got {n_in}")
    if taps is None:
        taps = taps_tensor(plan, x.device)
    if out is None:
        out = torch.empty((B, plan.n_out), dtype=torch.float32, device=x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_src_polyphase_f32(
            _ptr(x), _ptr(out), B, n_in, ld(x), plan.n_out, ld(out),
            _ptr(taps), plan.K, plan.L, plan.M, plan.c_offset, _stream(x.device))
    _lib.check(rc, "dsp_src_polyphase_f32")
    return out


_NARROW = {torch.float64: torch.float32, torch.complex128: torch.complex64}
_WIDEN = {torch.float32: torch.float64, torch.complex64: torch.complex128}


def convert(x: torch.Tensor, dtype: torch.dtype, out: torch.Tensor | None = None) -> torch.Tensor:
    """x cast to `dtype` on the device by the library (dsp_convert_f64_f32 /
    dsp_convert_f32_f64: numpy's astype rounding), for the float64 <-> float32
    and complex128 <-> complex64 pairs; a contiguous copy of x keeps its
    shape."""
    if x.dtype == dtype:
        return x
    if _NARROW.get(x.dtype) == dtype:
        fn = "dsp_convert_f64_f32"
    elif _WIDEN.get(x.dtype) == dtype:
        fn = "dsp_convert_f32_f64"
    else:
        raise ValueError(f"no library conversion {x.dtype} -> {dtype}")
    if not x.is_cuda:
        raise ValueError("x must be a CUDA (ROCm) tensor")
    x = x.contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=dtype, device=x.device)
    n = x.numel() * (2 if x.is_complex() else 1)
    with torch.cuda.device(x.device):
        rc = getattr(_lib.load(), fn)(_ptr(x), _ptr(out), n, _stream(x.device))
    _lib.check(rc, fn)
    return out


def biquad_workspace(B: int, n: int, S: int, device: torch.device,
                     chunk_len: int | None = None) -> torch.Tensor:
    chunk_len = chunk_len_for(n, max_chunks_for(B)) if chunk_len is None else chunk_len
    nbytes = _lib.load().dsp_biquad_workspace_bytes(B, n, S, chunk_len)
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def state_table(sos: np.ndarray, chunk_len: int, device: torch.device) -> torch.Tensor | None:
    """Cached device copy of design.state_response_table (None when the fused
    kernel cannot use it: S == 0, S == 7 or S > 8)."""
    S = sos.shape[0]
    if S == 0 or S == 7 or S > 8:
        return None
    return _cached(("G", sos.tobytes(), chunk_len, device.index),
                   lambda: torch.from_numpy(state_response_table(sos, chunk_len)).to(device))


def xstate_geometry(chunk_len: int, plan: SrcPlan) -> tuple[int, int, int]:
    """(shift, q0, rows) of the chain's x-domain chunk states, from the library
    (dsp_chain_xstate_geometry) so host table and kernel agree by construction."""
    import ctypes
    sh, q0, rows = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = _lib.load().dsp_chain_xstate_geometry(int(chunk_len), plan.K, plan.L, plan.M,
                                               plan.c_offset, ctypes.byref(sh),
                                               ctypes.byref(q0), ctypes.byref(rows))
    _lib.check(rc, "dsp_chain_xstate_geometry")
    return sh.value, q0.value, rows.value


def xstate_table(sos: np.ndarray, plan: SrcPlan, chunk_len: int,
                 device: torch.device) -> tuple[torch.Tensor, int]:
    """Cached device copy of design.xstate_table and its row count."""
    _, q0, rows = xstate_geometry(chunk_len, plan)
    key = ("GX", sos.tobytes(), plan.L, plan.M, plan.K, plan.c_offset, chunk_len, device.index)
    t = _cached(key, lambda: torch.from_numpy(
        xstate_table_host(sos, plan, chunk_len, q0, rows)).to(device))
    return t, rows


def biquad_cascade(x: torch.Tensor, sos: np.ndarray, clip: bool,
                   out: torch.Tensor | None = None, workspace: torch.Tensor | None = None,
                   chunk_len: int | None = None, use_table: bool = True) -> torch.Tensor:
    """z = clip(cascade(x)) per row (dsp_core.py:233-254), fp64 inside, fp32 I/O."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    sos = np.ascontiguousarray(sos, dtype=np.float64).reshape(-1, 5)
    B, n = x.shape
    S = sos.shape[0]
    chunk_len = chunk_len_for(n, max_chunks_for(B)) if chunk_len is None else int(chunk_len)
    if out is None:
        out = torch.empty_like(x)
    if workspace is None:
        workspace = biquad_workspace(B, n, S, x.device, chunk_len)
    table = state_table(sos, chunk_len, x.device) if use_table else None
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_biquad_cascade_f32(
            _ptr(x), _ptr(out), B, n, ld(x), ld(out), _lib.sos_pointer(sos),
            S, int(bool(clip)), chunk_len, _ptr(table), _ptr(workspace), workspace.numel(),
            _stream(x.device))
    _lib.check(rc, "dsp_biquad_cascade_f32")
    return out


_ONE_TAP = SrcPlan(1, 1, 1, np.ones(1), 0, 0, 0, 0)


def _eq_tile_plan(n: int, sos: np.ndarray, device: torch.device):
    """(device tables, key, one-tap taps) of the single-pass cascade alone for
    rows of n samples (dsp_chain_tile_tables for the SRC bypass as the one-tap
    SRC, include/dspcore.h), cached; None where no single-pass kernel serves
    it (S outside 1..6, a b0 == 0 band, shared poles)."""
    import ctypes
    S = sos.shape[0]
    lib = _lib.load()
    if not 1 <= S <= 6 or lib.dsp_chain_tile_len(n, n, 1, 1, 1, 0, S) <= 0:
        return None

    def build():
        nbytes = int(lib.dsp_chain_tile_tables_bytes())
        host = np.zeros(nbytes, dtype=np.uint8)
        one = np.ones(1, dtype=np.float32)
        key = ctypes.c_uint64(0)
        rc = lib.dsp_chain_tile_tables(host.ctypes.data, nbytes, n, n, one.ctypes.data, 1, 1, 1,
                                       0, _lib.sos_pointer(sos), S, ctypes.byref(key))
        if rc < 0:
            _lib.check(rc, "dsp_chain_tile_tables")
        if rc != 0:
            return ()
        return (torch.from_numpy(host).to(device), int(key.value),
                torch.ones(1, dtype=torch.float32, device=device))
    plan = _cached(("EQT", sos.tobytes(), n, device.index), build)
    return plan or None


class forced_chain_path:
    """Sets dsp_chain_path on the calling thread to the single-pass mode the
    default takes for a batch of plan_batch rows (dsp_chain_mode: 2 chained
    tiles, 4 the three-launch mode) where the call's own batch of B rows would
    take the other one, unless a path is already forced; restores it after.
    Shards of one job use it so that every shard's rows are bitwise the
    unsharded call's (the two modes agree to float64 rounding only; chained
    and persistent tiles are bitwise one, so a batch both would run chained
    or persistent is left to the default)."""

    def __init__(self, plan_batch: int | None, n_in: int, n_out: int, K: int, L: int, M: int,
                 c: int, S: int, B: int | None = None):
        self.path = None
        if plan_batch is not None:
            lib = _lib.load()
            mode = lib.dsp_chain_mode(int(plan_batch), n_in, n_out, K, L, M, c, S)
            own = None if B is None else lib.dsp_chain_mode(int(B), n_in, n_out, K, L, M, c, S)
            if mode != own:
                self.path = 4 if mode == 3 else 2 if mode == 1 else None

    def __enter__(self):
        self.prev = None
        if self.path is not None and _lib.chain_path() == 0:
            self.prev = _lib.chain_path(self.path)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            _lib.chain_path(self.prev)


_eq_ws_lock = threading.Lock()
_eq_ws: OrderedDict = OrderedDict()   # (device, stream, thread, bytes) -> zero-filled workspace
EQ_WS_CACHE_MAX = 16


def _eq_workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """A chain workspace of at least nbytes for the calling thread's current
    stream, zero-filled once and reused: every call that completes leaves its
    hand-off flags clear (include/dspcore.h), and calls of one thread on one
    stream run in order."""
    key = (device.index, _stream(device), threading.get_ident(), int(nbytes))
    with _eq_ws_lock:
        ws = _eq_ws.get(key)
        if ws is not None:
            _eq_ws.move_to_end(key)
            return ws
    ws = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
    with _eq_ws_lock:
        ws = _eq_ws.setdefault(key, ws)
        _eq_ws.move_to_end(key)
        while len(_eq_ws) > EQ_WS_CACHE_MAX:
            _eq_ws.popitem(last=False)
    return ws


def eq_single_pass(x: torch.Tensor, sos: np.ndarray, out: torch.Tensor | None = None,
                   plan_batch: int | None = None, check: bool = False,
                   workspace: torch.Tensor | None = None) -> torch.Tensor | None:
    """z = clip(cascade(x)) per row (dsp_core.py:233-254) through the
    single-pass kernel of the cascade alone: dsp_chain_f32 with the SRC bypass
    as the one-tap SRC (L = M = 1, K = 1, tap 1.0), y = NULL, mag = NULL -- x
    read once, z written once; small batches of long rows take its
    three-launch mode (the library picks it, for plan_batch rows when given:
    forced_chain_path).  Returns None where that kernel does not serve the
    call (biquad_cascade does) -- and, with check (it synchronises the
    stream), where a chained tile's hand-off wait gave up (dsp_chain_status;
    the workspace is reset): the caller reruns the rows on biquad_cascade.
    workspace: the caller's zero-filled chain workspace of at least
    dsp_chain_workspace_bytes for this call, used on one stream (every call
    that completes leaves it clear); by default one is made or reused here."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    sos = np.ascontiguousarray(sos, dtype=np.float64).reshape(-1, 5)
    B, n = x.shape
    if B == 0 or (B > 1 and ld(x) % 4) or x.data_ptr() % 16:
        return None
    plan = _eq_tile_plan(n, sos, x.device)
    if plan is None:
        return None
    tables, key, taps = plan
    if out is None:
        out = torch.empty((B, n), dtype=torch.float32, device=x.device)
    if (B > 1 and ld(out) % 4) or out.data_ptr() % 16 or out.stride(1) != 1:
        return None
    lib = _lib.load()
    S = sos.shape[0]
    chunk = chunk_len_for(n, max_chunks_for(B))
    ws_bytes = int(lib.dsp_chain_workspace_bytes(B, n, n, 1, 1, 1, 0, S, chunk))
    # (reused only where a give-up is detected and the workspace reset: a flag
    # a give-up left raised would mislead the next call's tiles)
    if workspace is not None:
        if workspace.numel() < ws_bytes or not workspace.is_cuda:
            raise ValueError(f"workspace of {workspace.numel()} bytes < {ws_bytes}")
        ws = workspace
    else:
        ws = (_eq_workspace(x.device, ws_bytes) if check else
              torch.zeros(max(ws_bytes, 256), dtype=torch.uint8, device=x.device))
    force = forced_chain_path(plan_batch if plan_batch != B else None, n, n, 1, 1, 1, 0, S, B)
    with torch.cuda.device(x.device), force:
        rc = lib.dsp_chain_f32(
            _ptr(x), None, _ptr(out), None, B, n, ld(x), n, ld(out), _ptr(taps), 1, 1, 1, 0,
            _lib.sos_pointer(sos), S, 1, chunk, None, None, 0, _ptr(tables), key, 0, 0, 0, 0,
            None, None, _ptr(ws), ws.numel(), _stream(x.device))
        _lib.check(rc, "dsp_chain_f32")
        # the three-launch mode has no hand-off wait that could give up: no
        # status read (and no stream synchronisation) for it
        path = _lib.chain_path()
        if check and not (path == 4 or (path == 0 and lib.dsp_chain_mode(
                B, n, n, 1, 1, 1, 0, S) == 3)):
            st = lib.dsp_chain_status(_ptr(ws), ws.numel(), 0, _stream(x.device))
            if st < 0:
                _lib.check(st, "dsp_chain_status")
            if st:
                lib.dsp_chain_status(_ptr(ws), ws.numel(), 1, _stream(x.device))
                return None
    return out


def lfilter_nonfinite(x: torch.Tensor, y: torch.Tensor, b: np.ndarray, a: np.ndarray) -> torch.Tensor:
    """Gives y = lfilter(b, a, x) (len(a) >= 2), computed by the cascade kernel,
    scipy's inf / NaN labels from x's first non-finite sample on
    (dsp_lfilter_nonfinite_f32); rows without one are left as they are."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    b = np.ascontiguousarray(b, dtype=np.float64)
    a = np.ascontiguousarray(a, dtype=np.float64)
    B, n = x.shape
    if tuple(y.shape) != (B, n) or y.dtype != torch.float32 or y.stride(1) != 1:
        raise ValueError("y must be float32 [B, n] with unit column stride")
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_lfilter_nonfinite_f32(_ptr(x), _ptr(y), B, n, ld(x), ld(y),
                                           b.ctypes.data_as(_lib._dp), b.size,
                                           a.ctypes.data_as(_lib._dp), a.size, _stream(x.device))
    _lib.check(rc, "dsp_lfilter_nonfinite_f32")
    return y


def _dft_tables(n: int, device: torch.device) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    def build():
        from .design import bluestein_tables
        chirp, bf, M = bluestein_tables(n)
        if M != _lib.load().dsp_dft_size(n):
            raise RuntimeError("Bluestein size mismatch between host and library")
        return tuple(torch.from_numpy(a.astype(np.complex64).view(np.float32)).to(device)
                     for a in (chirp, bf)) + (_table("tw", M, device),)
    return _cached(("BLU", n, device.index), build)


def dft(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Natural-order DFT of every row for ANY length n <= 8192 (np.fft.fft's
    contract, app.py:322-324), complex64: the radix-2 kernel for powers of two,
    Bluestein (dsp_dft_f32) otherwise."""
    x = _rows(x, "x")
    B, n = x.shape
    if n >= 1 and n & (n - 1) == 0 and n.bit_length() - 1 <= _lib.DSP_MAX_LOG2N:
        return fft(x, out)
    if n < 1 or n > _lib.DSP_MAX_DFT:
        raise ValueError(f"DFT length {n} outside [1, {_lib.DSP_MAX_DFT}]")
    real = not x.is_complex()
    x = x.float() if real else x.to(torch.complex64)
    if out is None:
        out = torch.empty((B, n), dtype=torch.complex64, device=x.device)
    chirp, bf, tw = _dft_tables(n, x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_dft_f32(_ptr(x), _ptr(out), B, n, int(real), ld(x), ld(out), _ptr(chirp),
                             _ptr(bf), _ptr(tw), _stream(x.device))
    _lib.check(rc, "dsp_dft_f32")
    return out


def _log2(n: int, limit: int | None = None) -> int:
    """log2 of a power-of-two length; `limit` defaults to the largest FFT
    (DSP_MAX_LOG2N_FFT; the STFT stays within one LDS-resident launch)."""
    if n < 1 or n & (n - 1):
        raise ValueError(f"length {n} is not a power of two; the radix-2 FFT needs 2^k points")
    lg = n.bit_length() - 1
    limit = _lib.DSP_MAX_LOG2N_FFT if limit is None else limit
    if lg > limit:
        raise RuntimeError(f"FFT length 2^{lg} exceeds the supported 2^{limit}")
    return lg


def _fft_workspace(B: int, lg: int, device: torch.device) -> torch.Tensor | None:
    """Scratch of the four-step transform above DSP_MAX_LOG2N (else None)."""
    nbytes = int(_lib.load().dsp_fft_workspace_bytes(B, lg))
    return torch.empty(nbytes, dtype=torch.uint8, device=device) if nbytes else None


def fft(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Natural-order radix-2 DIT FFT of every row (dsp_core.py:41-66), complex64."""
    x = _rows(x, "x")
    B, n = x.shape
    lg = _log2(n)
    real = not x.is_complex()
    if real:
        x = x.float()
    elif x.dtype != torch.complex64:
        x = x.to(torch.complex64)
    if out is None:
        out = torch.empty((B, n), dtype=torch.complex64, device=x.device)
    tw = _table("tw", n, x.device)
    ws = _fft_workspace(B, lg, x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_fft_c2c_f32(_ptr(x), _ptr(out), B, lg, int(real), ld(x),
                                    ld(out), _ptr(tw), _ptr(ws), 0 if ws is None else ws.numel(),
                                    _stream(x.device))
    _lib.check(rc, "dsp_fft_c2c_f32")
    return out


def spectrum(x: torch.Tensor, seg_start: int, seg_len: int, n_fft: int,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """|FFT(hann * x[seg])|[:n_fft/2+1] per row (dsp_core.py:74-98), fp32."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    B = x.shape[0]
    lg = _log2(n_fft, _lib.DSP_MAX_LOG2N_FOURSTEP)
    if out is None:
        out = torch.empty((B, n_fft // 2 + 1), dtype=torch.float32, device=x.device)
    win = _table("hann", n_fft, x.device)
    tw = _table("tw", n_fft, x.device)
    ws = _fft_workspace(B, lg, x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_spectrum_f32(_ptr(x), _ptr(out), B, ld(x), seg_start, seg_len,
                                  lg, ld(out), _ptr(win), _ptr(tw), _ptr(ws),
                                  0 if ws is None else ws.numel(), _stream(x.device))
    _lib.check(rc, "dsp_spectrum_f32")
    return out


# Page-locked staging buffers of spectrum_host / fft_host, per thread and
# device (grown, never shrunk; calls are synchronous, so a thread's next call
# may reuse them).
_host_stage = threading.local()
# spectrum_host / fft_host take up to this many bytes (float32 / complex64) per call.
SPECTRUM_HOST_MAX_BYTES = 4 << 20


def _pinned(slot: str, device: torch.device, nbytes: int) -> torch.Tensor:
    bufs = getattr(_host_stage, "bufs", None)
    if bufs is None:
        bufs = _host_stage.bufs = {}
    key = (slot, device.index)
    t = bufs.get(key)
    if t is None or t.numel() < nbytes:
        t = bufs[key] = torch.empty(max(nbytes, 4096), dtype=torch.uint8, pin_memory=True)
    return t


def spectrum_host(seg: np.ndarray, n_fft: int, device: torch.device,
                  out_dtype=np.float32) -> np.ndarray | None:
    """|FFT(hann * row)|[:n_fft/2+1] of every row of a host array [B, seg_len]
    (the already-cut segments of dsp_core.py:76-82), float32, for a few small
    segments: the rows go, cast to float32 by numpy (astype's rounding, as
    `convert`), into page-locked host memory that the spectrum kernel reads
    directly over the bus, and the kernel writes |X| into page-locked memory
    too -- no copy launches, one stream synchronisation; returned as a fresh
    array of out_dtype.  None when the call is not of that kind (the caller
    takes the device path)."""
    B, seg_len = seg.shape
    half = n_fft // 2 + 1
    lg = _log2(n_fft, _lib.DSP_MAX_LOG2N_FOURSTEP)
    if B < 1 or lg > _lib.DSP_MAX_LOG2N or B * max(seg_len, half) * 4 > SPECTRUM_HOST_MAX_BYTES:
        return None
    xin = _pinned("spec_in", device, max(B * seg_len * 4, 16))
    xout = _pinned("spec_out", device, B * half * 4)
    xv = xin.numpy()[:B * seg_len * 4].view(np.float32).reshape(B, seg_len)
    np.copyto(xv, seg, casting="unsafe")
    win = _table("hann", n_fft, device)
    tw = _table("tw", n_fft, device)
    lib = _lib.load()
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device)
        rc = lib.dsp_spectrum_f32(xin.data_ptr(), xout.data_ptr(), B, seg_len, 0, seg_len, lg,
                                  half, _ptr(win), _ptr(tw), None, 0, stream.cuda_stream)
        _lib.check(rc, "dsp_spectrum_f32")
        stream.synchronize()
    return xout.numpy()[:B * half * 4].view(np.float32).reshape(B, half).astype(out_dtype)


def fft_host(x: np.ndarray, device: torch.device, out_dtype=np.complex64) -> np.ndarray | None:
    """The DFT of every row of a host array [B, n] (real or complex, n a power
    of two up to one LDS-resident launch), as spectrum_host does it: numpy
    casts the rows (float32 / complex64, astype's rounding) into page-locked
    memory, dsp_fft_c2c_f32 reads them and writes X there, no copy launches;
    returned as a fresh array of out_dtype.  None when the call is not of that
    kind (the caller takes the device path)."""
    B, n = x.shape
    lg = _log2(n)
    if B < 1 or lg > _lib.DSP_MAX_LOG2N or B * n * 8 > SPECTRUM_HOST_MAX_BYTES:
        return None
    real = not np.iscomplexobj(x)
    ft = np.float32 if real else np.complex64
    nin = B * n * np.dtype(ft).itemsize
    xin = _pinned("fft_in", device, nin)
    xout = _pinned("fft_out", device, B * n * 8)
    np.copyto(xin.numpy()[:nin].view(ft).reshape(B, n), x, casting="unsafe")
    tw = _table("tw", n, device)
    lib = _lib.load()
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device)
        rc = lib.dsp_fft_c2c_f32(xin.data_ptr(), xout.data_ptr(), B, lg, int(real), n, n,
                                 _ptr(tw), None, 0, stream.cuda_stream)
        _lib.check(rc, "dsp_fft_c2c_f32")
        stream.synchronize()
    return xout.numpy()[:B * n * 8].view(np.complex64).reshape(B, n).astype(out_dtype)


def stft_magnitude(x: torch.Tensor, n_fft: int, hop: int, frames: int,
                   out: torch.Tensor | None = None) -> torch.Tensor:
    """|FFT(hann * frame)|[:n_fft/2+1] of every frame x[b, f*hop : f*hop + n_fft]
    (zero-padded past the row's end) -> [B, frames, n_fft/2+1] float32."""
    x = _rows(x, "x")
    if x.dtype != torch.float32:
        x = x.float()
    B, n = x.shape
    lg = _log2(n_fft, _lib.DSP_MAX_LOG2N)
    half = n_fft // 2 + 1
    if out is None:
        out = torch.empty((B, frames, half), dtype=torch.float32, device=x.device)
    if B == 0:
        return out
    win = _table("hann", n_fft, x.device)
    tw = _table("tw", n_fft, x.device)
    lib = _lib.load()
    with torch.cuda.device(x.device):
        rc = lib.dsp_stft_mag_f32(_ptr(x), _ptr(out), B, ld(x), 0, n, hop, frames, lg,
                                  out.stride(1), _ptr(win), _ptr(tw), _stream(x.device))
    _lib.check(rc, "dsp_stft_mag_f32")
    return out
