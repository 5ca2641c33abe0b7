"""Host-side filter design and call planning (float64, numpy).

These are the parts of reference modules/dsp_core.py that run once per call
and are O(taps) or O(bands): the FIR designer, the peaking-biquad designer,
the EQ band selection and the SRC / spectrum size rules.  They stay on the host
in float64 exactly as the reference computes them; only their results (fp32
taps, fp64 second-order sections, sizes) cross into the HIP kernels.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# Band centres of the 6-band EQ, in the reference's order
# (reference modules/dsp_core.py:225-228).
BAND_CENTRES_HZ = {
    "Sub-Bass": 40, "Bass": 150, "Low Mids": 1000,
    "High Mids": 3000, "Presence": 5000, "Brilliance": 10000,
}
DEFAULT_CENTRE_HZ = 1000      # unknown band name (dsp_core.py:235)
BYPASS_DB = 0.1               # |g| threshold (dsp_core.py:222, :234)
NYQUIST_FRACTION = 0.90       # fc ceiling = 0.9 * fs/2 (dsp_core.py:240)
MIN_CENTRE_HZ = 10            # fc floor (dsp_core.py:249)
SPECTRUM_WINDOW = 2048        # N_ventana (dsp_core.py:74)


def sinc_lowpass(w_c_norm: float, num_taps: int) -> np.ndarray:
    """Windowed-sinc low-pass, unit DC gain (reference dsp_core.py:104-131).

    An even tap count is bumped to odd (:114); taps are sinc(wc*n), n centred on
    0 (:116-120), times a Blackman window (:123-124), normalised to sum 1 when
    the sum is non-zero (:127-129).
    """
    k = int(num_taps) + (1 - int(num_taps) % 2)
    half = k // 2
    n = np.arange(-half, half + 1)
    h = np.sinc(w_c_norm * n) * np.blackman(n.size)
    total = np.sum(h)
    if total != 0:
        h /= total
    return h


def default_num_taps(L: int, M: int) -> int:
    """Tap rule of dsp_core.py:158: 40 * max(L, M) + 1."""
    return 40 * max(L, M) + 1


@dataclass(frozen=True)
class SrcPlan:
    """Sizes and taps of one polyphase SRC call (dsp_core.py:133-173)."""
    L: int
    M: int
    K: int                 # odd tap count actually used
    taps: np.ndarray       # float64 L*h, length K
    c_offset: int          # 'same' centring offset into the full convolution
    n_in: int
    n_out: int
    fs_out: int


def src_plan(n_in: int, fs: int, M: int, L: int, num_taps: int | None = None) -> SrcPlan:
    """Plans conversion_tasa_muestreo(x, fs, M, L) for a signal of n_in samples.

    wc = 1/max(L, M) (:155); K from `num_taps` or the default rule (:158);
    h *= L (:162).  np.convolve(x_e, h, 'same') keeps max(NL, K) samples of the
    full convolution starting at c = (min(NL, K) - 1) // 2 (:166); [::M] keeps
    ceil(max(NL, K) / M) of them (:170); fs' = int(fs * L / M) (:172).
    """
    L, M = int(L), int(M)
    if L < 1 or M < 1:
        raise ValueError(f"L and M must be >= 1 (got L={L}, M={M})")
    if n_in < 1:
        raise ValueError("conversion_tasa_muestreo needs at least one sample")
    taps_req = default_num_taps(L, M) if num_taps is None else int(num_taps)
    h = sinc_lowpass(1.0 / max(L, M), taps_req)
    h *= L
    K = h.size
    nl = n_in * L
    c = (min(nl, K) - 1) // 2
    n_out = -(-max(nl, K) // M)
    return SrcPlan(L, M, K, h, c, n_in, n_out, int(fs * L / M))


# The library's flush rule (csrc/common.h, kTapFlushRel): taps at or below
# this fraction of the largest (float32 arithmetic) are zero in its finite sums.
TAP_FLUSH_REL = np.float32(1e-12)


def caller_taps(plan: SrcPlan) -> np.ndarray:
    """float32 L*h, the taps every SRC entry point of the library takes
    (include/dspcore.h): the reference's float64 design (dsp_core.py:159-162)
    rounded once."""
    return np.ascontiguousarray(np.asarray(plan.taps, dtype=np.float64).astype(np.float32))


def kernel_taps(plan: SrcPlan) -> np.ndarray:
    """What the library's finite arithmetic makes of caller_taps (a model, for
    tests: the flush happens inside the library, csrc/common.h): for L > 1 the
    taps with |t| <= 1e-12 max|t| (float32) are zero -- the taps at the sinc's
    zeros, every L-th tap from the centre when wc = 1/L (upsampling,
    dsp_core.py:155), whose float64 values are the rounding noise of sin(k pi)
    (|L h| ~ 1e-17 .. 1e-34 at K = 121), and the Blackman window's end taps.
    Their contribution to y is below 1e-14 of the signal, far inside the SRC
    tolerance (2e-6), and the polyphase branch that holds the centre tap
    becomes a pure scaled delay: the single-pass kernel computes its outputs
    (1/L of them) with one multiply instead of ceil(K/L) FMAs
    (csrc/chain_tile.hip, DLY).  Windows that hold an inf or NaN take the
    caller's unflushed taps, so non-finite input propagates as through the
    reference's convolution.  Plans with L = 1 keep every tap."""
    out = caller_taps(plan).copy()
    if plan.L > 1 and out.size:
        thr = TAP_FLUSH_REL * np.max(np.abs(out))
        out[np.abs(out) <= thr] = 0.0
    return out


def peaking_biquad(fc: float, fs: float, gain_db: float) -> tuple[np.ndarray, np.ndarray]:
    """RBJ-style peaking EQ with Q = 1 (reference dsp_core.py:179-203).

    Returns (b, a), both float64[3] normalised so a[0] == 1.
    """
    w0 = 2 * np.pi * fc / fs
    alpha = np.sin(w0) / 2.0
    amp = 10 ** (gain_db / 40.0)
    cosw = np.cos(w0)
    a0 = 1 + alpha / amp
    b = np.array([1 + alpha * amp, -2 * cosw, 1 - alpha * amp]) / a0
    a = np.array([a0, -2 * cosw, 1 - alpha / amp]) / a0
    return b, a


@dataclass(frozen=True)
class EqPlan:
    """What sistema_ecualizador does for given (fs, gains) (dsp_core.py:216-254)."""
    bypass: bool           # all |g| < 0.1: the input object is returned as is
    sos: np.ndarray        # float64 [S][5] = b0 b1 b2 a1 a2, in dict order
    centres: tuple         # effective fc of each stage (after the clamp)


def eq_plan(fs: float, gains: dict) -> EqPlan:
    """Band selection of dsp_core.py:222-251.

    Bypass when every |g| < 0.1 (an empty dict bypasses too).  Otherwise, in
    dict order, every band with |g| > 0.1 gets fc from the centre table (1000 Hz
    for an unknown name), clamped to 0.9*fs/2 when fc >= that ceiling, and is
    applied only if fc > 10 Hz.  The clip to [-1, 1] always follows.
    """
    values = list(gains.values())
    if all(abs(g) < BYPASS_DB for g in values):
        return EqPlan(True, np.zeros((0, 5)), ())
    ceiling = (fs / 2.0) * NYQUIST_FRACTION
    rows, centres = [], []
    for name, g in gains.items():
        if not abs(g) > BYPASS_DB:
            continue
        fc = BAND_CENTRES_HZ.get(name, DEFAULT_CENTRE_HZ)
        if fc >= ceiling:
            fc = ceiling
        if fc > MIN_CENTRE_HZ:
            b, a = peaking_biquad(fc, fs, g)
            rows.append([b[0], b[1], b[2], a[1], a[2]])
            centres.append(fc)
    sos = np.asarray(rows, dtype=np.float64).reshape(-1, 5)
    return EqPlan(False, sos, tuple(centres))


def tf_to_sos_row(b, a) -> np.ndarray:
    """(b, a) of order <= 2 -> one normalised DF2T row {b0 b1 b2 a1 a2}.

    lfilter divides every coefficient by a[0]; shorter vectors are zero-padded.
    """
    b = np.atleast_1d(np.asarray(b, dtype=np.float64))
    a = np.atleast_1d(np.asarray(a, dtype=np.float64))
    if b.ndim != 1 or a.ndim != 1 or b.size == 0 or a.size == 0:
        raise ValueError("b and a must be non-empty 1-D coefficient vectors")
    if b.size > 3 or a.size > 3:
        raise ValueError("the GPU cascade takes biquads: len(b), len(a) <= 3")
    if a[0] == 0:
        raise ValueError("BUG: filter coefficient a[0] == 0 not supported yet")
    bb = np.zeros(3)
    aa = np.zeros(3)
    bb[: b.size] = b
    aa[: a.size] = a
    bb /= aa[0]
    aa /= aa[0]
    return np.array([bb[0], bb[1], bb[2], aa[1], aa[2]])


@dataclass(frozen=True)
class LfilterPlan:
    """How aplicar_ecuacion_diferencias runs lfilter(b, a, x) of any order
    (reference dsp_core.py:205-214): 'sos' -- the transfer function as
    second-order sections (float64, host) for the biquad-cascade kernel;
    'fir' -- a of length 1, where lfilter is the convolution np.convolve(b / a0,
    x)[:n] (a gain when b has length 1), as a causal convolution on the SRC
    kernel with L = M = 1.  That keeps lfilter's non-finite semantics of the
    case: an inf or NaN meets every tap of b, a zero tap included (0 * inf =
    NaN), and stays within len(b) samples; 'fir_rec' -- a = [1, 0, ...] with
    more than 3 coefficients: the same convolution for the finite values, then
    lfilter's recursion labels (b, a kept for dsp_lfilter_nonfinite_f32)."""
    kind: str
    sos: np.ndarray | None = None
    taps: np.ndarray | None = None
    b: np.ndarray | None = None     # 'sos': lfilter's b / a0 and a / a0 (the
    a: np.ndarray | None = None     # non-finite relabelling, dsp_lfilter_nonfinite_f32)


MAX_LFILTER_SECTIONS = 16     # include/dspcore.h DSP_MAX_STAGES: sections per cascade launch


def lfilter_plan(b, a) -> LfilterPlan:
    """Plan of scipy.signal.lfilter(b, a, x) for 1-D b, a of any length.

    Like lfilter, every coefficient is divided by a[0] (a[0] == 0 raises the
    ValueError lfilter raises).  Orders <= 2 keep the direct biquad row; higher
    IIR orders are factored into second-order sections with
    scipy.signal.tf2sos (poles and zeros in float64; the cascade is the same
    transfer function as lfilter's direct form II transposed, and better
    conditioned).  Any order: a cascade of more than DSP_MAX_STAGES sections
    runs as consecutive launches of up to that many (lfilter_groups).
    """
    b = np.atleast_1d(np.asarray(b, dtype=np.float64))
    a = np.atleast_1d(np.asarray(a, dtype=np.float64))
    if b.ndim != 1 or a.ndim != 1 or b.size == 0 or a.size == 0:
        raise ValueError("b and a must be non-empty 1-D coefficient vectors")
    if a[0] == 0:
        raise ValueError("BUG: filter coefficient a[0] == 0 not supported yet")
    b = b / a[0]
    a = a / a[0]
    if a.size == 1:      # scipy's lfilter convolves here (the DF2T recursion below)
        return LfilterPlan("fir", taps=b.copy())
    a_tail = np.trim_zeros(a[1:], "b")
    if max(a.size, b.size) <= 3:
        return LfilterPlan("sos", sos=tf_to_sos_row(b, a).reshape(1, 5), b=b, a=a)
    if a_tail.size == 0:
        # a = [1, 0, ...]: the transfer function is the FIR b, but lfilter runs
        # its recursion (0 * inf = NaN labels everything after an inf).  The
        # finite values are the convolution (tf2sos of a long b would factor a
        # degree len(b) - 1 polynomial: 0.33 error at 101 taps, 5e30 at 301);
        # the labels come from dsp_lfilter_nonfinite_f32, which scans x for
        # this a (include/dspcore.h).
        return LfilterPlan("fir_rec", taps=b.copy(), b=b, a=a)
    import scipy.signal
    sos6 = scipy.signal.tf2sos(b, np.concatenate([[1.0], a_tail]))  # rows b0 b1 b2 1 a1 a2
    sos = np.ascontiguousarray(np.column_stack([sos6[:, 0:3] / sos6[:, 3:4],
                                                sos6[:, 4:6] / sos6[:, 3:4]]))
    # (b and the untrimmed a: lfilter's recursion order counts a's trailing zeros)
    return LfilterPlan("sos", sos=sos, b=b, a=a)


def lfilter_groups(sos: np.ndarray) -> list[np.ndarray]:
    """The sections of an 'sos' plan in launch-sized groups (<= DSP_MAX_STAGES
    rows each), applied in order; between groups the signal is float32 (the
    cascade kernel's I/O), within a group the state is float64."""
    sos = np.asarray(sos, dtype=np.float64).reshape(-1, 5)
    return [sos[g:g + MAX_LFILTER_SECTIONS] for g in range(0, max(1, sos.shape[0]),
                                                               MAX_LFILTER_SECTIONS)]


MAX_FUSED_CHUNKS = 256   # csrc/iir.hip kCBMax: four waves of 64 chunk lanes per channel
WIDE_BATCH = 2048        # from this many channels one wave (<= 64 chunks) per channel fills the chip


def max_chunks_for(batch: int) -> int:
    """Chunks per channel the cascade plans for a batch of `batch` channels:
    <= 64 (one wavefront per channel, no barriers) once the batch alone fills
    the chip with waves, else <= 256 (four wavefronts per channel) so that small
    batches still do.  Rows are bitwise independent of the batch size for a
    given chunk length; across this threshold they agree to rounding."""
    return 64 if int(batch) >= WIDE_BATCH else MAX_FUSED_CHUNKS


def chunk_len_for(n: int, max_chunks: int = MAX_FUSED_CHUNKS) -> int:
    """Chunk length of the biquad carry scan for a row of n samples: the
    smallest multiple of 32 that splits the row into <= max_chunks chunks, so the
    cascade runs as one fused launch (include/dspcore.h) with enough chunk lanes
    to fill the chip at small batches.  A function of n only: every row's
    result is independent of the batch size."""
    per = -(-int(n) // max_chunks)
    return max(32, -(-per // 32) * 32)


def df2_realization(sos: np.ndarray) -> tuple[np.ndarray, float, bool]:
    """The kernels' realisation of a [S][5] {b0 b1 b2 a1 a2} cascade
    (csrc/iir.hip:realize): direct form II per stage, rows {g, c1, c2, a1, a2}
    and an input gain G.  With every b0 != 0 (NORM): g = 1, c = b/b0,
    G = prod(b0); otherwise g = b0, c = (b1, b2), G = 1."""
    sos = np.asarray(sos, dtype=np.float64).reshape(-1, 5)
    norm = bool(np.all(sos[:, 0] != 0))
    rows = np.empty_like(sos)
    if norm:
        rows[:, 0] = 1.0
        rows[:, 1] = sos[:, 1] / sos[:, 0]
        rows[:, 2] = sos[:, 2] / sos[:, 0]
        gain = float(np.prod(sos[:, 0])) if sos.shape[0] else 1.0
    else:
        rows[:, :3] = sos[:, :3]
        gain = 1.0
    rows[:, 3:] = sos[:, 3:]
    return rows, gain, norm


def state_space(sos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """(A, B) of the S-stage cascade as one D = 2S state system X' = A X + B u
    in the kernels' realisation (df2_realization), state order
    (w1_0, w2_0, w1_1, w2_1, ...): the delay lines of each stage."""
    rows, gain, norm = df2_realization(sos)
    S = rows.shape[0]
    D = 2 * S

    def step(X, u):
        X = X.copy()
        if norm:
            u = gain * u
        for k in range(S):
            g, c1, c2, a1, a2 = rows[k]
            w = u - a1 * X[2 * k] - a2 * X[2 * k + 1]
            v = g * w + c1 * X[2 * k] + c2 * X[2 * k + 1]
            X[2 * k + 1] = X[2 * k]
            X[2 * k] = w
            u = v
        return X

    A = np.column_stack([step(np.eye(D)[i], 0.0) for i in range(D)]) if D else np.zeros((0, 0))
    B = step(np.zeros(D), 1.0)
    return A, B


def state_response_table(sos: np.ndarray, chunk_len: int) -> np.ndarray:
    """float64 [chunk_len][2S]: row t = A^(chunk_len-1-t) B, the cascade state at
    the end of a chunk caused by a unit sample t samples into it.  The GPU
    cascade turns its chunk end states into one dot product per state with it."""
    A, B = state_space(sos)
    D = B.size
    G = np.empty((chunk_len, D))
    G[0] = B
    m, Am = 1, A.copy()
    while m < chunk_len:
        k = min(m, chunk_len - m)
        G[m:m + k] = G[:k] @ Am.T          # A^m applied to rows 0..k-1
        m += k
        Am = Am @ Am
    return np.ascontiguousarray(G[::-1])


def xstate_chunk_len(n_out: int, L: int, M: int, max_chunks: int = MAX_FUSED_CHUNKS) -> int:
    """Chunk length for the chain's x-domain chunk states (include/dspcore.h,
    dsp_chain_f32): the smallest multiple of 32 with chunk_len*M/L an integer
    multiple of 32 (128-byte aligned x rows) that splits n_out into between
    max_chunks/2 and max_chunks chunks, else the smallest with chunk_len*M/L a
    multiple of 4.  A function of (n_out, L, M) only, so rows stay independent
    of the batch size."""
    per = -(-int(n_out) // max_chunks)
    best = None
    for q in (32, 4):   # prefer 128-byte aligned chunk rows of x (csrc/iir.hip)
        unit = q * L // math.gcd(M, q * L)      # chunk_len*M % (qL) == 0
        step = 32 * unit // math.gcd(32, unit)  # lcm(32, unit)
        T = max(step, -(-per // step) * step)
        if best is None or T < best:
            best = T
        if -(-int(n_out) // T) >= max_chunks // 2:  # keeps >= half the chunk lanes
            return T
    return best


def xstate_table(sos: np.ndarray, plan: "SrcPlan", chunk_len: int, q0: int,
                 rows: int) -> np.ndarray:
    """float64 [rows][2S]: the state-response table of `chunk_len` composed with
    the SRC taps, so that a chunk's zero-state end state is a dot product over
    the SRC input instead of its output (include/dspcore.h, dsp_chain_f32):

        E_c = sum_t G[t] y[cT + t],  y[m] = sum_k (L h)[k] x[(m M + c - k) / L]
            = sum_j Gx[j] x[c T M / L + q0 + j],
        Gx[q' - q0] = sum_t G[t] (L h)[t M + c - q' L]   (0 <= t M + c - q' L < K).

    Everything in float64 from the reference's own taps (dsp_core.py:159-162)."""
    G = state_response_table(sos, chunk_len)
    T, D = G.shape
    L, M, K, c = plan.L, plan.M, plan.K, plan.c_offset
    taps = np.asarray(plan.taps, dtype=np.float64)
    base = np.arange(T, dtype=np.int64) * M + c
    ph, qb = base % L, base // L
    out = np.zeros((rows, D))
    for j in range(-(-K // L) + 1):
        k = ph + j * L
        ok = k < K
        q = qb[ok] - j - q0
        if q.size and (q.min() < 0 or q.max() >= rows):
            raise ValueError("x-state geometry does not cover the taps")
        np.add.at(out, q, G[ok] * taps[k[ok], None])
    return np.ascontiguousarray(out)


@dataclass(frozen=True)
class SpectrumPlan:
    seg_start: int
    seg_len: int
    n_fft: int             # transform length actually used (power of two)


def spectrum_plan(length: int, window: int = SPECTRUM_WINDOW) -> SpectrumPlan:
    """Segment rule of calcular_espectro_magnitud (dsp_core.py:74-82).

    len > window: x[len//2 : len//2 + window] (numpy slicing may truncate it);
    otherwise zero-pad to the next power of two of len.  The reference's FFT
    only works on power-of-two lengths, so a truncated segment whose length is
    not a power of two raises ValueError exactly where the reference does
    (e.g. 2048 < len < 4095 with the default window).
    """
    length = int(length)
    if length > window:
        start = length // 2
        seg = min(window, length - start)
        n = seg
    else:
        start = 0
        seg = length
        n = 1 << (length - 1).bit_length()
    if n & (n - 1):
        raise ValueError(
            f"segment of {n} samples is not a power of two "
            f"(signal length {length}, window {window}); the radix-2 FFT needs 2^k points")
    return SpectrumPlan(start, seg, n)


@dataclass(frozen=True)
class StftPlan:
    n_fft: int
    hop: int
    frames: int


def stft_plan(length: int, n_fft: int = SPECTRUM_WINDOW, hop: int | None = None) -> StftPlan:
    """Framing of the spectrogram extension: frames of
    n_fft samples (a power of two, as the reference's FFT requires) every `hop`
    samples (default n_fft // 4) from the start of the signal; every frame that
    starts inside the signal while the previous one did not reach its end, i.e.
    1 + ceil(max(0, length - n_fft) / hop) frames, the last zero-padded."""
    n_fft = int(n_fft)
    if n_fft < 1 or n_fft & (n_fft - 1):
        raise ValueError(f"n_fft={n_fft} is not a power of two; the radix-2 FFT needs 2^k points")
    hop = max(1, n_fft // 4) if hop is None else int(hop)
    if hop < 1:
        raise ValueError("hop must be >= 1")
    frames = 1 + -(-max(0, int(length) - n_fft) // hop)
    return StftPlan(n_fft, hop, frames)


def hann(n: int) -> np.ndarray:
    """Window of dsp_core.py:85-87: 0.5 - 0.5 cos(2 pi n / (N - 1)), float64."""
    k = np.arange(n)
    with np.errstate(divide="ignore", invalid="ignore"):
        return 0.5 - 0.5 * np.cos(2 * np.pi * k / (n - 1))


def twiddles(n: int, start: int = 0, stop: int | None = None) -> np.ndarray:
    """exp(-2j pi k / N), start <= k < stop (default N/2), computed in float64
    (dsp_core.py:59-60)."""
    k = np.arange(start, max(n // 2, 1) if stop is None else stop)
    return np.exp(-2j * np.pi * k / n)


def bluestein_tables(n: int) -> tuple[np.ndarray, np.ndarray, int]:
    """(chirp[n], FFT_M(b)/M [M], M) of the any-length DFT (include/dspcore.h,
    dsp_dft_f32), float64: chirp[k] = exp(-i pi (k^2 mod 2n) / n) (the modulus
    keeps the phase argument small and exact), b[j] = b[M-j] = conj(chirp[j])."""
    n = int(n)
    m = 1
    while (1 << m) < 2 * n - 1:
        m += 1
    M = 1 << m
    k = np.arange(n, dtype=np.int64)
    chirp = np.exp(-1j * np.pi * ((k * k) % (2 * n)) / n)
    b = np.zeros(M, dtype=np.complex128)
    b[:n] = np.conj(chirp)
    if n > 1:
        b[M - np.arange(1, n)] = np.conj(chirp[1:])
    return chirp, np.fft.fft(b) / M, M
