"""The C-ABI library loads and exports exactly what include/dspcore.h declares;
argument validation answers without touching a GPU."""
import ctypes

import pytest

from dspcore import _lib


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = _lib.header_symbols()
    assert len(names) == 35
    for name in names:
        assert hasattr(lib, name), name
        assert name in _lib._SIGNATURES, f"{name} has no ctypes signature"


def test_version_and_error_string():
    lib = _lib.load()
    assert lib.dsp_version() == 20700     # 2.7.0: the SRC bypass single-pass, mag may be NULL (2.6.0: single-pass ratios)
    assert isinstance(_lib.last_error(), str)


def test_invalid_arguments_are_rejected_before_any_launch():
    lib = _lib.load()
    rc = lib.dsp_src_polyphase_f32(None, None, 1, 10, 10, 10, 10, None, 121, 0, 2, 0, None)
    assert rc == _lib.DSP_EINVAL and "L=0" in _lib.last_error()
    rc = lib.dsp_fft_c2c_f32(None, None, 1, 31, 1, 1 << 31, 1 << 31, None, None, 0, None)
    assert rc == _lib.DSP_EINVAL
    # four-step sizes: the two-pass split (2^15..2^22) needs B * N complex, the
    # three-pass one (2^23..2^30, row by row) 2 N complex; above 2^20 the
    # coarse twiddle table, 2^floor(log2n / 2) complex; then the non-finite
    # header, 8 bytes per row (of a launch part of <= 65535 rows: two-pass)
    assert lib.dsp_fft_workspace_bytes(3, 14) == 0
    assert lib.dsp_fft_workspace_bytes(3, 15) == 3 * (1 << 15) * 8 + 3 * 8
    assert lib.dsp_fft_workspace_bytes(2, 22) == 2 * (1 << 22) * 8 + (1 << 11) * 8 + 2 * 8
    assert lib.dsp_fft_workspace_bytes(3, 23) == 2 * (1 << 23) * 8 + (1 << 11) * 8 + 3 * 8
    assert lib.dsp_fft_workspace_bytes(3, 24) == 2 * (1 << 24) * 8 + (1 << 12) * 8 + 3 * 8
    assert lib.dsp_fft_workspace_bytes(3, 25) == 2 * (1 << 25) * 8 + (1 << 12) * 8 + 3 * 8
    assert lib.dsp_fft_workspace_bytes(3, 26) == 2 * (1 << 26) * 8 + (1 << 13) * 8 + 3 * 8
    assert lib.dsp_fft_workspace_bytes(1, 28) == 2 * (1 << 28) * 8 + (1 << 14) * 8 + 8
    assert lib.dsp_fft_workspace_bytes(1, 29) == 2 * (1 << 29) * 8 + (1 << 14) * 8 + 8
    assert lib.dsp_fft_workspace_bytes(5, 30) == 2 * (1 << 30) * 8 + (1 << 15) * 8 + 5 * 8
    # 2^31, 2^32 (ABI 2.7): the radix-2 split -- even / odd halves, an N/2-point
    # twiddle table, the halves' own workspace (2^32 splits once more)
    G = 1 << 30
    w31 = 2 * (G * 8) + (G // 2) * 8 + lib.dsp_fft_workspace_bytes(1, 30) + 255
    assert lib.dsp_fft_workspace_bytes(1, 31) == w31
    assert lib.dsp_fft_workspace_bytes(7, 31) == w31                 # rows one at a time
    assert lib.dsp_fft_workspace_bytes(1, 32) == 2 * (2 * G * 8) + G * 8 + w31 + 255
    assert lib.dsp_fft_workspace_bytes(1, 33) == 0
    # the test hook sends four-step sizes through the split (the larger
    # workspace of the two), and answers the range
    prev = lib.dsp_fft_split_log2n(-1)
    assert prev == 31
    assert lib.dsp_fft_split_log2n(15) == _lib.DSP_EINVAL
    assert lib.dsp_fft_split_log2n(20) == 31
    try:
        h = 1 << 19
        w20 = 2 * (h * 8) + (h // 2) * 8 + lib.dsp_fft_workspace_bytes(1, 19) + 255
        assert lib.dsp_fft_workspace_bytes(1, 20) == max(w20, (1 << 20) * 8 + (1 << 10) * 8 + 8)
    finally:
        assert lib.dsp_fft_split_log2n(prev) == 20
    assert lib.dsp_fft_workspace_bytes(70000, 15) == 70000 * (1 << 15) * 8 + 65535 * 8
    rc = lib.dsp_fft_c2c_f32(1024, 1024, 1, 15, 1, 1 << 15, 1 << 15, 1024, None, 0, None)
    assert rc == _lib.DSP_EINVAL and "workspace" in _lib.last_error()
    sos = (ctypes.c_double * 5)(1, 0, 0, 0, 0)
    rc = lib.dsp_biquad_cascade_f32(None, None, 1, 100, 100, 100, sos, 17, 1, 2048, None, None, 0, None)
    assert rc == _lib.DSP_EINVAL
    rc = lib.dsp_biquad_cascade_f32(None, None, 1, 100, 100, 100, sos, 1, 1, 100, None, None, 0, None)
    assert rc == _lib.DSP_EINVAL and "chunk_len" in _lib.last_error()
    with pytest.raises(ValueError):
        _lib.check(_lib.DSP_EINVAL, "x")
    with pytest.raises(RuntimeError):
        _lib.check(_lib.DSP_EHIP, "x")


def test_zero_batch_is_a_no_op():
    lib = _lib.load()
    assert lib.dsp_src_polyphase_f32(None, None, 0, 10, 10, 15, 15, None, 121, 3, 2, 5, None) == 0
    assert lib.dsp_spectrum_f32(None, None, 0, 10, 0, 10, 4, 9, None, None, None, 0, None) == 0


def test_workspace_query():
    lib = _lib.load()
    D = 12
    B, n, T = 4096, 72000, 2048
    C = -(-n // T)
    assert lib.dsp_biquad_workspace_bytes(B, n, 6, 1152) == 0       # fused: none
    need = lib.dsp_biquad_workspace_bytes(B, n, 6, 256)             # 282 chunks
    C = -(-n // 256)
    assert need >= 8 * (D * D + B * (C - 1) * D + B * C * D)
    need9 = lib.dsp_biquad_workspace_bytes(B, n, 9, T)              # S > 8: general
    assert need9 > 0
    assert lib.dsp_biquad_workspace_bytes(B, 2000, 6, T) == 0   # single chunk: none
    assert lib.dsp_biquad_workspace_bytes(B, n, 0, T) == 0      # clip-only: none


def test_trace_toggle_without_gpu():
    assert _lib.load().dsp_trace_enable(1) == 0
    assert _lib.trace_read() == []          # nothing launched
    assert _lib.load().dsp_trace_enable(0) == 0


def test_xstate_geometry_query():
    """dsp_chain_xstate_geometry is host-only: shift = T*M/L, q0 a multiple of 4
    at or below the lowest input index a chunk's outputs touch, rows a multiple
    of 32 covering the highest."""
    lib = _lib.load()
    out = [ctypes.c_int64() for _ in range(3)]
    refs = [ctypes.byref(o) for o in out]
    assert lib.dsp_chain_xstate_geometry(1152, 121, 3, 2, 60, *refs) == 0
    shift, q0, rows = (o.value for o in out)
    assert shift == 768 and q0 % 32 == 0 and rows % 32 == 0
    assert q0 <= -((121 - 1 - 60) // 3) and q0 + rows > (1151 * 2 + 60) // 3
    # chunk_len*M not a multiple of L, or a shift that is not a multiple of 4
    assert lib.dsp_chain_xstate_geometry(1000, 121, 3, 2, 60, *refs) == _lib.DSP_EINVAL
    assert lib.dsp_chain_xstate_geometry(1149, 121, 3, 2, 60, *refs) == _lib.DSP_EINVAL


def _wav(fmt_tag, channels, rate, bits, payload, extensible=False, extra_chunk=False):
    import struct
    block = channels * bits // 8
    if extensible:
        fmt = struct.pack("<HHIIHH", 0xFFFE, channels, rate, rate * block, block, bits)
        fmt += struct.pack("<HHI", 22, bits, 0) + struct.pack("<H", fmt_tag) + bytes(14)
    else:
        fmt = struct.pack("<HHIIHH", fmt_tag, channels, rate, rate * block, block, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra_chunk:   # odd-sized chunk: padded to a word boundary
        body += b"LIST" + struct.pack("<I", 3) + b"abc" + b"\0"
    body += b"data" + struct.pack("<I", len(payload)) + payload
    return b"RIFF" + struct.pack("<I", len(body)) + body


def test_wav_parse_host_only():
    """dsp_wav_parse reads headers without a GPU: PCM, float, extensible,
    chunks before data; rejects what soundfile would not give as PCM/float."""
    lib = _lib.load()
    info = _lib.WavInfo()
    f = _wav(1, 2, 44100, 16, bytes(400), extra_chunk=True)
    assert lib.dsp_wav_parse(f, len(f), ctypes.byref(info)) == 0
    assert (info.format, info.channels, info.sample_rate, info.bits, info.frames) == \
        (_lib.DSP_WAV_PCM, 2, 44100, 16, 100)
    assert f[info.data_offset - 8:info.data_offset - 4] == b"data"
    f = _wav(3, 1, 48000, 32, bytes(64), extensible=True)
    assert lib.dsp_wav_parse(f, len(f), ctypes.byref(info)) == 0
    assert (info.format, info.bits, info.frames) == (_lib.DSP_WAV_FLOAT, 32, 16)
    f = _wav(1, 1, 8000, 24, bytes(30))
    assert lib.dsp_wav_parse(f, len(f), ctypes.byref(info)) == 0 and info.frames == 10
    for bad in (b"RIFX" + bytes(40), _wav(2, 1, 8000, 4, bytes(8)), _wav(1, 1, 8000, 12, bytes(8)),
                b"RIFF\x04\0\0\0WAVE"):
        assert lib.dsp_wav_parse(bad, len(bad), ctypes.byref(info)) == _lib.DSP_EINVAL


def test_wav_header_matches_scipy_writer():
    """The playback header is byte-identical to scipy.io.wavfile.write's for
    int16 (what app.py:352 calls)."""
    import io

    import numpy as np
    from scipy.io import wavfile
    pcm = (np.arange(-500, 500) * 31).astype(np.int16)
    buf = io.BytesIO()
    wavfile.write(buf, 72000, pcm)
    hdr = ctypes.create_string_buffer(44)
    assert _lib.load().dsp_wav_header_pcm16(hdr, 72000, 1, pcm.size) == 0
    assert hdr.raw + pcm.tobytes() == buf.getvalue()


def test_chain_path_tile_len_and_workspace_query():
    """dsp_chain_path takes 0..4 (-1 queries); dsp_chain_tile_len names the
    single-pass geometries (config 3's L3/M2, K = 121: 48-sample sub-chunks;
    any L/M with ceil(K/L) <= 8, e.g. config 5's 160/147, K = 1023: 32) and
    declines others; the chain workspace holds a 256-byte status header, the
    tile hand-off (a 12-double state and a flag per tile, 3072- or 2048-output
    tiles) and, after it, the two-launch cascade's scratch (never shared)."""
    lib = _lib.load()
    prev = lib.dsp_chain_path(-1)
    assert prev in (0, 1, 2, 3, 4)
    assert lib.dsp_chain_path(5) == _lib.DSP_EINVAL
    assert lib.dsp_chain_path(-2) == _lib.DSP_EINVAL
    assert lib.dsp_chain_path(-1) == prev
    assert lib.dsp_chain_tile_len(48000, 72000, 121, 3, 2, 60, 6) == 48
    assert lib.dsp_chain_tile_len(48000, 72000, 121, 3, 2, 60, 3) == 48   # padded stages
    # n_out % 4 != 0: not k_chain_tile, but the per-phase kernel (chain_pp.h, 6/4's geometry)
    assert lib.dsp_chain_tile_len(47996, 71994, 121, 3, 2, 60, 6) == 48
    assert lib.dsp_chain_tile_len(48000, 96000, 81, 2, 1, 40, 6) == 48     # app ratio 2/1
    assert lib.dsp_chain_tile_len(48000, 24000, 81, 1, 2, 40, 6) == 24     # app ratio 1/2
    assert lib.dsp_chain_tile_len(48000, 52245, 1023, 160, 147, 511, 6) == 32   # generic
    assert lib.dsp_chain_tile_len(48000, 52245, 6401, 160, 147, 3200, 6) == 0   # 41 taps/branch
    assert lib.dsp_chain_tile_len(47999, 52244, 1023, 160, 147, 511, 6) == 0    # n_in % 4
    assert lib.dsp_chain_tile_len(48000, 72000, 121, 3, 2, 60, 7) == 0    # > 6 stages
    # the SRC bypass as the one-tap SRC (ABI 2.7): the cascade alone; any
    # other L = M = 1 call, or no EQ stage, takes the two-launch chain
    assert lib.dsp_chain_tile_len(48000, 48000, 1, 1, 1, 0, 6) == 48
    assert lib.dsp_chain_tile_len(48000, 48000, 41, 1, 1, 20, 6) == 0
    assert lib.dsp_chain_tile_len(48000, 48000, 1, 1, 1, 0, 0) == 0
    assert lib.dsp_chain_tile_len(454231, 454231, 1, 1, 1, 0, 6) == 48   # any length (one tap)
    assert lib.dsp_chain_tile_len(47999, 71998, 121, 3, 2, 60, 6) == 0   # n_in % 4 with an SRC
    # dsp_chain_mode (host): the default's single-pass mode for a batch -- the
    # three-launch mode for a few long rows, chained tiles for full batches
    # (DESIGN.md §3.0.9), 0 where the two-launch chain serves the geometry
    assert lib.dsp_chain_mode(1, 441000, 441000, 1, 1, 1, 0, 6) == 3          # the EQ alone
    assert lib.dsp_chain_mode(32768, 48000, 48000, 1, 1, 1, 0, 6) == 1
    assert lib.dsp_chain_mode(16, 441000, 661500, 121, 3, 2, 60, 6) == 3      # L3/M2 kernel
    assert lib.dsp_chain_mode(32768, 48000, 72000, 121, 3, 2, 60, 6) == 1     # config 4
    assert lib.dsp_chain_mode(2, 441000, 882000, 81, 2, 1, 40, 6) == 3        # per-phase 2/1
    assert lib.dsp_chain_mode(1, 441000, 480000, 1023, 160, 147, 511, 6) == 3  # generic
    assert lib.dsp_chain_mode(8192, 48000, 52245, 1023, 160, 147, 511, 6) == 1  # config 5
    assert lib.dsp_chain_mode(1, 48000, 44100, 1023, 147, 160, 511, 6) == 0   # two-launch
    assert lib.dsp_chain_mode(0, 48000, 72000, 121, 3, 2, 60, 6) == 0
    B, n_in, n_out = 4096, 48000, 72000
    tiles = -(-n_out // 3072)
    ws = lib.dsp_chain_workspace_bytes(B, n_in, n_out, 121, 3, 2, 60, 6, 1152)
    assert ws >= B * tiles * (12 * 8 + 4)
    assert lib.dsp_chain_workspace_bytes(B, n_in, 52245, 1023, 160, 147, 511, 6, 1152) >= \
        B * -(-52245 // 2048) * (12 * 8 + 4)
    # no single-pass kernel and a fused cascade: the status header alone
    assert lib.dsp_chain_workspace_bytes(B, n_in, 52245, 6401, 160, 147, 3200, 6, 1152) == 256
    # the two-launch cascade's scratch (282 chunks: general path) follows the hand-off region
    head = lib.dsp_chain_workspace_bytes(B, n_in, n_out, 121, 3, 2, 60, 6, 1152)
    assert lib.dsp_chain_workspace_bytes(B, n_in, n_out, 121, 3, 2, 60, 6, 256) == \
        head + lib.dsp_biquad_workspace_bytes(B, n_out, 6, 256)


def test_chain_status_spin_limit_and_null_y_validation():
    """dsp_chain_spin_limit is per thread (default 2^23 polls, -1 queries);
    dsp_chain_status rejects a null workspace; y == NULL is refused where the
    single-pass kernel does not serve the call (no tables), before any launch."""
    import threading
    lib = _lib.load()
    assert _lib.spin_limit() == 1 << 23
    assert _lib.spin_limit(0) == 1 << 23 and _lib.spin_limit() == 0
    seen = []
    t = threading.Thread(target=lambda: seen.append(_lib.spin_limit()))
    t.start()
    t.join()
    assert seen == [1 << 23]                       # another thread keeps the default
    assert _lib.spin_limit(1 << 23) == 0
    assert lib.dsp_chain_spin_limit(-2) == _lib.DSP_EINVAL
    assert lib.dsp_chain_status(None, 0, 0, None) == _lib.DSP_EINVAL
    ws = lib.dsp_chain_workspace_bytes(1, 48000, 72000, 121, 3, 2, 60, 6, 1152)
    rc = lib.dsp_chain_f32(16, None, 32, 48, 1, 48000, 48000, 72000, 72000, 64, 121, 3, 2, 60,
                           None, 0, 0, 1152, None, None, 0, None, 0, 0, 2048, 11, 1025, 80, 96,
                           112, ws, None)
    assert rc == _lib.DSP_EINVAL and "NULL" in _lib.last_error()
    rc = lib.dsp_chain_f32(16, None, 32, 48, 1, 48000, 48000, 72000, 72000, 64, 121, 3, 2, 60,
                           None, 0, 0, 1152, None, None, 0, None, 0, 0, 2048, 11, 1025, 80, 96,
                           112, 16, None)
    assert rc == _lib.DSP_EINVAL and "workspace" in _lib.last_error()


def _tables_dtype():
    """numpy mirror of csrc/chain_tile.hip's TileTables (C layout)."""
    import numpy as np
    return np.dtype([("key", "<u8"), ("G", "<f8", (64, 12)), ("Gc", "<f4", (32, 12, 2)),
                     ("Q", "<f8", (12, 12)), ("Dp", "<f8", (6, 6, 2, 2)), ("T", "<f8", (12, 12)),
                     ("TP", "<f4", (32, 4, 2)), ("geo", "<i4", (6,)), ("cf", "<f8", (6, 4)),
                     ("gain", "<f8"), ("seq", "<f4", (8, 32, 8)), ("adv", "<u4", (8,)),
                     ("classes", "<i4"), ("pad", "<i4"), ("seqs", "<f4", (8, 32, 12)),
                     ("flush_thr", "<f4"), ("pad3", "<i4", (3,)), ("tpw", "<f4", (1024,)),
                     ("pp_td", "<f4"), ("pp_np", "<i4"), ("pp_geo", "<i4"), ("pad4", "<i4")],
                    align=True)


def _table_step(tb, X, u):
    """One sample of the tables' NORM DF2 realisation (cascade.h): u *= gain;
    per stage w = u - a1 w1 - a2 w2, v = w + c1 w1 + c2 w2.  State X (12,) in
    place; returns the output."""
    cf = tb["cf"]
    u = u * float(tb["gain"])
    for k in range(6):
        c1, c2, a1, a2 = cf[k]
        w1, w2 = X[2 * k], X[2 * k + 1]
        w = u - a1 * w1 - a2 * w2
        v = w + c1 * w1 + c2 * w2
        X[2 * k + 1], X[2 * k] = w1, w
        u = v
    return u


def _table_cascade(tb, y):
    import numpy as np
    X = np.zeros(12)
    return np.array([_table_step(tb, X, float(v)) for v in y])


def _table_state_space(tb):
    """(A, B) of the tables' realisation: X' = A X + B u."""
    import numpy as np
    A = np.zeros((12, 12))
    for c in range(12):
        X = np.zeros(12)
        X[c] = 1.0
        _table_step(tb, X, 0.0)
        A[:, c] = X
    X = np.zeros(12)
    _table_step(tb, X, 1.0)
    return A, X.copy()


def _tables(lib, nbytes, *args):
    import numpy as np
    buf = np.zeros(nbytes, np.uint8)
    key = ctypes.c_uint64(0)
    rc = lib.dsp_chain_tile_tables(buf.ctypes.data, nbytes, *args, ctypes.byref(key))
    return rc, buf.view(_tables_dtype())[0], key.value


def test_chain_tile_tables_host_only():
    """dsp_chain_tile_tables (host, no GPU) for config 3's geometry: the
    block-diagonal carry tables reproduce the cascade's dense state algebra
    (T D^(48 2^d) T^-1 = A^(48 2^d); T sum_i G'[i] y[i] = the zero-state end
    state of a 48-sample sub-chunk); the float32 pass-1 rows in input-normal
    coordinates give the same end state through Q (gain T Q sum_i Gc[i] y[i]:
    pass 2 applies the realisation's gain at the output, so its states and Q
    carry 1 / gain), Q is lower triangular and the coordinates have unit
    variance under white noise;
    the tap pairs are the reversed polyphase branches shifted by their window
    parity; the key fingerprints geometry and cascade; config 5's geometry
    builds 32-sample tables for the generic kernel; others decline with 1."""
    import numpy as np

    from dspcore import design
    lib = _lib.load()
    gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3,
             "Presence": 5, "Brilliance": -6}
    plan = design.src_plan(48000, 48000, 2, 3)
    sos = np.ascontiguousarray(design.eq_plan(72000, gains).sos)
    nbytes = lib.dsp_chain_tile_tables_bytes()
    assert nbytes == _tables_dtype().itemsize
    taps32 = np.ascontiguousarray(plan.taps, dtype=np.float32)
    rc, tb, key = _tables(lib, nbytes, 48000, 72000, taps32.ctypes.data, plan.K, 3, 2,
                          plan.c_offset, _lib.sos_pointer(sos), 6)
    assert rc == 0 and key != 0 and int(tb["key"]) == key
    G, Dp, T, TP = tb["G"], tb["Dp"], tb["T"], tb["TP"]
    assert tuple(tb["geo"]) == (48, 21, 3, 2, 121, 6)
    # the DF2 realisation pass 2 reads: per stage {b1/b0, b2/b0, a1, a2}, gain
    # prod(b0); it filters as the reference's cascade does
    rows, gain, norm = design.df2_realization(sos)
    assert norm
    np.testing.assert_array_equal(tb["cf"], rows[:, 1:])
    assert tb["gain"] == gain
    from scipy.signal import sosfilt
    yy = np.random.default_rng(4).uniform(-1, 1, 400)
    np.testing.assert_allclose(_table_cascade(tb, yy),
                               sosfilt(np.c_[sos[:, :3], np.ones(6), sos[:, 3:]], yy),
                               rtol=1e-9, atol=1e-12)
    A, B = _table_state_space(tb)
    Ti = np.linalg.inv(T)
    for d in range(6):
        D = np.zeros((12, 12))
        for k in range(6):
            D[2 * k:2 * k + 2, 2 * k:2 * k + 2] = Dp[d, k]
        An = np.linalg.matrix_power(A, 48 << d)
        np.testing.assert_allclose(T @ D @ Ti, An, atol=1e-9 * max(1.0, np.abs(An).max()))
    y = np.random.default_rng(0).uniform(-1, 1, 48).astype(np.float32)
    X = np.zeros(12)
    for v in y:
        X = A @ X + B * float(v)
    # (G carries 1 / gain like Q: pass 2 applies the gain at the output)
    np.testing.assert_allclose(float(tb["gain"]) * (T @ (G[:48].T @ y)), X, rtol=1e-10, atol=1e-12)
    # input-normal pass 1: float32 rows, Q = T^-1 P lower triangular
    Q = tb["Q"]
    Gc = tb["Gc"].astype(np.float64).transpose(0, 2, 1).reshape(64, 12)   # rows 2j, 2j+1
    assert np.array_equal(Q, np.tril(Q)) and not Gc[48:].any()
    g0 = float(tb["gain"])
    np.testing.assert_allclose(g0 * (T @ (Q @ (Gc[:48].T @ y))), X, rtol=1e-5,
                               atol=1e-6 * np.abs(X).max())
    P = g0 * (T @ Q)                            # DF2 coordinates = P * input-normal ones
    W = np.zeros((12, 12))                      # state covariance, unit white noise
    g = B.copy()
    for _ in range(60000):
        W += np.outer(g, g)
        g = A @ g
    np.testing.assert_allclose(np.linalg.solve(P, np.linalg.solve(P, W).T), np.eye(12), atol=1e-5)
    # the key follows the cascade and the geometry
    sos2 = sos.copy()
    sos2[0, 0] *= 1 + 1e-15
    assert _tables(lib, nbytes, 48000, 72000, taps32.ctypes.data, plan.K, 3, 2, plan.c_offset,
                   _lib.sos_pointer(np.ascontiguousarray(sos2)), 6)[2] not in (0, key)
    assert _tables(lib, nbytes, 48008, 72012, taps32.ctypes.data, plan.K, 3, 2, plan.c_offset,
                   _lib.sos_pointer(sos), 6)[2] not in (0, key)
    # tap pairs: branch ph, pair p = (h[2p - a], h[2p + 1 - a]), h[u] = taps[ph + 3 (40 - u)]
    # of the taps the library flushed itself (design.kernel_taps models it)
    kt = design.kernel_taps(plan)
    assert tb["flush_thr"] == np.float32(1e-12) * np.max(np.abs(taps32))
    for ph in range(3):
        a = [((2 * i) // 3) & 1 for i in range(48) if (2 * i) % 3 == ph][0]
        h = np.array([kt[ph + 3 * (40 - u)] if 0 <= u < 41 and ph + 3 * (40 - u) < 121
                      else 0.0 for u in range(-1, 43)], dtype=np.float32)
        want = np.array([[h[2 * p - a + 1], h[2 * p + 2 - a]] for p in range(21)])
        np.testing.assert_array_equal(TP[:21, ph], want)
    assert not TP[21:].any() and not TP[:, 3].any()
    c5 = design.src_plan(48000, 44100, 147, 160, 1023)
    t5c = np.ascontiguousarray(c5.taps, dtype=np.float32)   # what the caller passes
    t5 = design.kernel_taps(c5)                               # what the tables hold
    # config 5 (generic kernel): 32-sample sub-chunks, no tap pairs (the kernel
    # reads the device taps); 41 taps per branch declines with 1.
    sos5 = np.ascontiguousarray(design.eq_plan(c5.fs_out, gains).sos)
    rc, tb, key5 = _tables(lib, nbytes, 48000, c5.n_out, t5c.ctypes.data, c5.K, 160, 147,
                           c5.c_offset, _lib.sos_pointer(sos5), 6)
    assert rc == 0 and key5 not in (0, key)
    assert tuple(tb["geo"]) == (32, 0, 160, 147, 1023, 6)
    A5, B5 = _table_state_space(tb)
    y = np.random.default_rng(1).uniform(-1, 1, 32).astype(np.float32)
    X = np.zeros(12)
    for v in y:
        X = A5 @ X + B5 * float(v)
    np.testing.assert_allclose(float(tb["gain"]) * (tb["T"] @ (tb["G"][:32].T @ y)), X,
                               rtol=1e-10, atol=1e-12)
    Gc5 = tb["Gc"].astype(np.float64).transpose(0, 2, 1).reshape(64, 12)
    np.testing.assert_allclose(float(tb["gain"]) * (tb["T"] @ (tb["Q"] @ (Gc5[:32].T @ y))), X,
                               rtol=1e-5, atol=1e-6 * np.abs(X).max())
    assert not tb["TP"].any()
    # class tables: sub-chunks start at outputs 32 j; class j mod 5 (32*147 mod 160 = 64)
    seq, adv = tb["seq"], tb["adv"]
    assert tb["classes"] == 5
    L, M, K, c = 160, 147, 1023, c5.c_offset
    for k in range(5):
        phi = (c + k * 64) % L
        for i in range(32):
            want = [t5[phi + L * (6 - u)] if u < 7 and phi + L * (6 - u) < K else 0.0
                    for u in range(8)]
            np.testing.assert_array_equal(seq[k, i], np.array(want, dtype=np.float32))
            assert ((int(adv[k]) >> i) & 1) == int(phi + M >= L)
            phi = (phi + M) % L
    # k_chain_gct's rows: output i reads window pairs from (i M div L) rounded
    # down to even; its T = 7 taps sit shifted by (i M div L) mod 2 + the
    # class's carry d_i in 10 of 12 slots
    seqs = tb["seqs"]
    for k in range(5):
        phi0 = (c + k * 64) % L
        for i in range(32):
            g = i * M // L
            d = (phi0 + i * M) // L - g
            phi = (phi0 + i * M) % L
            sh = (g & 1) + d
            want = [t5[phi + L * (6 - (v - sh))] if 0 <= v - sh < 7 and v < 10
                    and phi + L * (6 - (v - sh)) < K else 0.0 for v in range(12)]
            np.testing.assert_array_equal(seqs[k, i], np.array(want, dtype=np.float32))
    assert not seqs[5:].any()
    c6 = design.src_plan(48000, 44100, 147, 160)
    t6 = np.ascontiguousarray(c6.taps, dtype=np.float32)
    rc, _, key6 = _tables(lib, nbytes, 48000, c6.n_out, t6.ctypes.data, c6.K, 160, 147,
                          c6.c_offset, _lib.sos_pointer(sos5), 6)
    assert rc == 1 and key6 == 0


def test_audio_parse_aiff_and_g711_host_only():
    """dsp_audio_parse: FORM/AIFF and AIFF-C layouts (PCM 8-32 big- and
    little-endian, fl32/fl64, G.711) and WAV G.711 give the right format word,
    width, frame count and sample offset without a GPU; WAV still parses."""
    import numpy as np
    import audio_files
    lib = _lib.load()
    info = _lib.WavInfo()
    BE, S8 = _lib.DSP_AUDIO_BE, _lib.DSP_AUDIO_S8
    for name, (f, frames, ch) in audio_files.cases(np.random.default_rng(3)).items():
        assert lib.dsp_audio_parse(f, len(f), ctypes.byref(info)) == 0, (name, _lib.last_error())
        assert (info.frames, info.channels) == (frames, ch), name
        fmt = info.format
        if name.startswith("aiff s") or "twos" in name or "NONE" in name or "short" in name:
            assert fmt & 0xFF == _lib.DSP_WAV_PCM and fmt & BE, name
            assert bool(fmt & S8) == (info.bits == 8), name
        elif "sowt" in name:
            assert fmt & 0xFF == _lib.DSP_WAV_PCM and not fmt & BE, name
        elif "fl32" in name or "FL64" in name:
            assert fmt == (_lib.DSP_WAV_FLOAT | BE) and info.bits in (32, 64), name
        else:
            mu = "ulaw" in name.lower()
            assert fmt & 0xFF == (_lib.DSP_WAV_ULAW if mu else _lib.DSP_WAV_ALAW), name
            assert info.bits == 8 and bool(fmt & BE) == name.startswith("aifc"), name
    f = audio_files.aiff(bytes(16), 1, 44100, 16, b"twos", ssnd_offset=6)
    assert lib.dsp_audio_parse(f, len(f), ctypes.byref(info)) == 0
    assert f[info.data_offset - 6 - 16:info.data_offset - 6 - 12] == b"SSND"
    assert info.sample_rate == 44100 and info.frames == 8
    f = _wav(1, 2, 44100, 16, bytes(400))
    assert lib.dsp_audio_parse(f, len(f), ctypes.byref(info)) == 0 and info.frames == 100
    for bad in (audio_files.aiff(bytes(8), 1, 44100, 16, b"ima4"),    # unsupported codec
                audio_files.aiff(bytes(8), 1, 44100, 12),             # 12-bit PCM
                audio_files.aiff(bytes(8), 0, 44100, 16, comm_frames=4),  # no channels
                b"FORM\0\0\0\x04AIFF",                                # no chunks
                audio_files.aiff(bytes(8), 1, 44100, 16)[:40]):       # cut inside COMM
        assert lib.dsp_audio_parse(bad, len(bad), ctypes.byref(info)) == _lib.DSP_EINVAL
    # a zero rate (80-bit zero) is refused like WAV's
    z = bytearray(audio_files.aiff(bytes(8), 1, 44100, 16))
    at = z.index(b"COMM") + 16
    z[at:at + 10] = bytes(10)
    assert lib.dsp_audio_parse(bytes(z), len(z), ctypes.byref(info)) == _lib.DSP_EINVAL
