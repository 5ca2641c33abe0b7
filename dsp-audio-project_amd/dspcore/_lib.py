"""ctypes binding of libdspcore.so (the C-ABI declared in include/dspcore.h).

The library is the product: there is no CPU fallback.  If it is missing, or no
GPU is visible, every compute entry point raises RuntimeError.

torch is imported before the library is loaded so that both share the one HIP
runtime already mapped into the process (soname libamdhip64.so.7).  ctypes
releases the GIL for the duration of each call, which lets the shard driver run
one host thread per GPU.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_ROOT)
# DSPCORE_LIB: alternate build of the same ABI (tuning experiments only).
LIB_PATH = os.environ.get("DSPCORE_LIB") or os.path.join(PKG_ROOT, "lib", "libdspcore.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "dspcore.h")

DSP_OK = 0
DSP_EINVAL = -1
DSP_EHIP = -2
DSP_ENOTSUP = -3
DSP_MAX_STAGES = 16
DSP_MAX_LOG2N = 14
DSP_MAX_LOG2N_FOURSTEP = 30
DSP_MAX_LOG2N_FFT = 32
DSP_MAX_DFT = 8192
DSP_LFILTER_NF_MAX = 4096

_c_i32, _c_i64, _c_u64, _c_sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t
_vp, _dp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); mirrors include/dspcore.h one to one.
_SIGNATURES = {
    "dsp_version": (ctypes.c_int, []),
    "dsp_last_error": (ctypes.c_char_p, []),
    "dsp_src_polyphase_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _c_i32, _c_i32,
        _c_i32, _c_i64, _vp]),
    "dsp_biquad_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i32, _c_i64]),
    "dsp_biquad_cascade_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _dp, _c_i32, _c_i32, _c_i64,
        _vp, _vp, _c_sz, _vp]),
    "dsp_lfilter_nonfinite_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _dp, _c_i32, _dp, _c_i32, _vp]),
    "dsp_fft_workspace_bytes": (_c_sz, [_c_i64, _c_i32]),
    "dsp_fft_c2c_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i32, _c_i32, _c_i64, _c_i64, _vp, _vp, _c_sz, _vp]),
    "dsp_spectrum_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i32, _c_i64, _vp, _vp,
        _vp, _c_sz, _vp]),
    "dsp_dft_size": (ctypes.c_int, [_c_i64]),
    "dsp_dft_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i32, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "dsp_stft_mag_f32": (ctypes.c_int, [
        _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i32, _c_i64, _vp, _vp,
        _vp]),
    "dsp_chain_f32": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _vp,
        _c_i32, _c_i32, _c_i32, _c_i64, _dp, _c_i32, _c_i32, _c_i64, _vp, _vp, _c_i64,
        _vp, _c_u64, _c_i64, _c_i64, _c_i32, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "dsp_chain_tile_tables_bytes": (_c_sz, []),
    "dsp_chain_tile_tables": (ctypes.c_int, [_vp, _c_sz, _c_i64, _c_i64, _vp, _c_i32, _c_i32,
                                             _c_i32, _c_i64, _dp, _c_i32,
                                             ctypes.POINTER(_c_u64)]),
    "dsp_chain_status": (ctypes.c_int, [_vp, _c_sz, _c_i32, _vp]),
    "dsp_chain_spin_limit": (_c_i64, [_c_i64]),
    "dsp_chain_path": (ctypes.c_int, [_c_i32]),
    "dsp_chain_tile_len": (_c_i64, [_c_i64, _c_i64, _c_i32, _c_i32, _c_i32, _c_i64, _c_i32]),
    "dsp_chain_mode": (_c_i32, [_c_i64, _c_i64, _c_i64, _c_i32, _c_i32, _c_i32, _c_i64, _c_i32]),
    "dsp_convert_f64_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _vp]),
    "dsp_fft_split_log2n": (ctypes.c_int, [_c_i32]),
    "dsp_convert_f32_f64": (ctypes.c_int, [_vp, _vp, _c_i64, _vp]),
    "dsp_chain_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i64, _c_i32, _c_i32, _c_i32,
                                          _c_i64, _c_i32, _c_i64]),
    "dsp_chain_xstate_geometry": (ctypes.c_int, [
        _c_i64, _c_i32, _c_i32, _c_i32, _c_i64, ctypes.POINTER(_c_i64),
        ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)]),
    "dsp_wav_parse": (ctypes.c_int, [ctypes.c_char_p, _c_sz, _vp]),
    "dsp_audio_parse": (ctypes.c_int, [ctypes.c_char_p, _c_sz, _vp]),
    "dsp_pcm_to_mono_f32": (ctypes.c_int, [
        _vp, _c_i32, _c_i32, _c_i32, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp]),
    "dsp_peak_normalize_f32": (ctypes.c_int, [
        _vp, _c_i64, _c_i64, _c_i64, ctypes.c_double, _vp, _vp]),
    "dsp_pcm_batch_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "dsp_pcm_batch_to_mono_f32": (ctypes.c_int, [
        _vp, _c_sz, _vp, _c_i64, _c_i64, _vp, _c_i64, ctypes.c_double, _vp, _vp, _c_sz, _vp]),
    "dsp_quantize_pcm16": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _vp, _c_i32,
                                          _vp]),
    "dsp_wav_header_pcm16": (ctypes.c_int, [ctypes.c_char_p, _c_i32, _c_i32, _c_i64]),
    "dsp_trace_enable": (ctypes.c_int, [_c_i32]),
    "dsp_trace_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_float), _c_i32]),
}
DSP_TRACE_NAME = 32
DSP_WAV_PCM = 1
DSP_WAV_FLOAT = 3
DSP_WAV_ALAW = 6
DSP_WAV_ULAW = 7
DSP_AUDIO_BE = 0x100
DSP_AUDIO_S8 = 0x200


class WavInfo(ctypes.Structure):
    """dsp_wav_info of include/dspcore.h."""
    _fields_ = [("format", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("sample_rate", ctypes.c_int32), ("bits", ctypes.c_int32),
                ("frames", ctypes.c_int64), ("data_offset", ctypes.c_int64),
                ("data_bytes", ctypes.c_int64)]


class PcmRow(ctypes.Structure):
    """dsp_pcm_row of include/dspcore.h."""
    _fields_ = [("offset", ctypes.c_int64), ("frames", ctypes.c_int64),
                ("format", ctypes.c_int32), ("bits", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_lock = threading.Lock()
_lib = None


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Function names declared in include/dspcore.h."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(dsp_[a-z0-9_]+)\s*\(", text)))


def load() -> ctypes.CDLL:
    """Loads libdspcore.so once (thread-safe) and attaches the signatures."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libdspcore.so not found at {LIB_PATH}; build it with "
                    "`make -C dsp-audio-project_amd/csrc` (or __graft_entry__.build())")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def last_error() -> str:
    return load().dsp_last_error().decode(errors="replace")


def check(rc: int, what: str) -> None:
    """Maps an ABI status code to the reference's exception types."""
    if rc == DSP_OK:
        return
    msg = f"{what}: {last_error()} (status {rc})"
    if rc == DSP_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(msg)


def chain_path(path: int = -1) -> int:
    """Path of dsp_chain_f32 on the calling thread (dsp_chain_path): 0 the
    single-pass kernel where it applies (default), 1 always the two-launch
    chain, 2 / 3 the single-pass path with its chained-tile / persistent
    kernel, 4 the three-launch mode of the cascade alone (include/dspcore.h);
    -1 only queries.  Returns the previous setting."""
    rc = load().dsp_chain_path(int(path))
    if rc < 0:
        check(rc, "dsp_chain_path")
    return rc


def spin_limit(spins: int = -1) -> int:
    """Polls before a single-pass hand-off wait gives up, on the calling
    thread (dsp_chain_spin_limit); -1 only queries.  Returns the previous one."""
    rc = load().dsp_chain_spin_limit(int(spins))
    if rc < 0:
        check(int(rc), "dsp_chain_spin_limit")
    return int(rc)


def trace_enable(on: bool) -> None:
    """Per-launch HIP-event tracing on the calling thread (dsp_trace_enable)."""
    check(load().dsp_trace_enable(int(bool(on))), "dsp_trace_enable")


def trace_read(max_records: int = 4096) -> list[tuple[str, float]]:
    """[(kernel name, milliseconds)] recorded since the last read (waits for them)."""
    names = ctypes.create_string_buffer(max_records * DSP_TRACE_NAME)
    ms = (ctypes.c_float * max_records)()
    n = load().dsp_trace_read(names, ms, max_records)
    if n < 0:
        check(n, "dsp_trace_read")
    raw = names.raw
    out = []
    for i in range(n):
        name = raw[i * DSP_TRACE_NAME:(i + 1) * DSP_TRACE_NAME].split(b"\0", 1)[0].decode()
        out.append((name, float(ms[i])))
    return out


def sos_pointer(sos):
    """float64 [S][5] host array -> ctypes double* (keeps `sos` alive in caller)."""
    if sos is None or sos.size == 0:
        return None
    return sos.ctypes.data_as(_dp)
