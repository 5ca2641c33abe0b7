/*
 * dspcore.h — C-ABI of libdspcore.so, the MI355X (gfx950) hot path of
 * Renatovela-ctrl/dsp-audio-project's modules/dsp_core.py.
 *
 * The reference has no native code and no FFI: its "operator API" is the set of
 * module-level Python functions in modules/dsp_core.py.  Each entry point below
 * replaces the numeric inner loop of one of them; the Python drop-in
 * (dsp-audio-project_amd/modules/dsp_core.py) keeps the reference signatures and
 * binds these symbols with ctypes.
 *
 * Conventions (all entry points):
 *   - every data pointer is a DEVICE pointer owned by the caller; the library
 *     never allocates device memory.  Scratch space comes from the caller via
 *     `workspace` (size from the matching *_workspace_bytes query);
 *   - `stream` is a hipStream_t (NULL = legacy default stream); every launch is
 *     asynchronous on it, nothing synchronises, so calls are graph-capturable;
 *   - kernels run on the calling thread's current HIP device;
 *   - batches are row-major [B][ld] float32 (complex data interleaved re,im);
 *   - return 0 (DSP_OK) on success, a negative DSP_E* code otherwise; the
 *     thread-local dsp_last_error() string says why.  Nothing throws across
 *     the ABI and no global mutable state is shared between threads.
 */
#ifndef DSPCORE_H
#define DSPCORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSP_OK 0
#define DSP_EINVAL (-1)   /* invalid argument: maps to Python ValueError      */
#define DSP_EHIP (-2)     /* HIP runtime error: maps to Python RuntimeError   */
#define DSP_ENOTSUP (-3)  /* valid but unsupported size: RuntimeError         */

#define DSP_MAX_STAGES 16 /* biquad stages per cascade call                   */
#define DSP_MAX_LOG2N 14  /* largest FFT handled in one LDS-resident launch   */
#define DSP_MAX_LOG2N_FOURSTEP 30 /* largest spectrum, and largest FFT in one
                                     four-step transform (above 2^14)            */
#define DSP_MAX_LOG2N_FFT 32 /* largest FFT (ABI 2.7: the reference's radix-2
                                split into two transforms above 2^30)            */
#define DSP_MAX_DFT 8192  /* largest any-length DFT (Bluestein, M <= 2^14)     */
#define DSP_LFILTER_NF_MAX 4096 /* largest order dsp_lfilter_nonfinite_f32 takes */

/* ABI version (major*10000 + minor*100 + patch). */
int dsp_version(void);

/* Last error message of the calling thread ("" if none). */
const char* dsp_last_error(void);

/* ---------------------------------------------------------------------------
 * Sample-rate conversion, polyphase L/M.
 * Replaces dsp_core.py:148-170 (conversion_tasa_muestreo): zero-stuff by L
 * (:149-150), np.convolve(x_e, h*L, mode='same') (:162,:166), keep every M-th
 * sample (:170).  For every output m < n_out:
 *     j = m*M + c_offset,  phi = j mod L,  q = j div L
 *     y[m] = sum_{t >= 0, phi + L t < K} taps[phi + L t] * x[q - t]
 * with x == 0 outside [0, n_in).  `taps` are the K gain-compensated filter
 * coefficients L*h (dsp_core.py:159-162) rounded to float32,
 * c_offset = (min(n_in*L, K) - 1) / 2 ('same' centring),
 * n_out = ceil(max(n_in*L, K) / M).  Accumulation is float32.
 * Tap flush (ABI 2.1): for L > 1 the sums use every tap with |t| <= 1e-12 *
 * max|t| (float32) as zero -- the float64 rounding noise of the reference's
 * sinc at its zeros and the Blackman window's end taps (|L h| ~ 1e-17 ..
 * 1e-34), which move y by less than 1e-14 per unit input.  Windows that hold
 * an inf or NaN give the reference's result: +-inf or NaN exactly as
 * np.convolve with the float64 taps (every one of them non-zero) gives it,
 * from the caller's unflushed taps; finite outputs beside them keep their
 * finite sums.
 * ------------------------------------------------------------------------- */
int dsp_src_polyphase_f32(const float* x, float* y, int64_t B, int64_t n_in,
                          int64_t ld_x, int64_t n_out, int64_t ld_y,
                          const float* taps, int32_t K, int32_t L, int32_t M,
                          int64_t c_offset, void* stream);

/* ---------------------------------------------------------------------------
 * Biquad cascade (direct form II transposed), zero initial state.
 * Replaces dsp_core.py:233-254 (sistema_ecualizador's serial loop of
 * aplicar_ecuacion_diferencias = scipy.signal.lfilter, dsp_core.py:205-214,
 * then np.clip(y, -1, 1) when clip != 0).
 * `sos_host` is a HOST array [S][5] = {b0, b1, b2, a1, a2} per stage, a0 == 1,
 * float64; coefficients and state are float64 inside the kernel, I/O float32.
 * The time axis is cut into chunks of `chunk_len` samples (multiple of 32)
 * whose initial states are recovered by a linear-recurrence carry scan, so
 * results do not depend on B or on how a batch is sharded.  x may equal y.
 * With S <= 8 (S != 7) and ceil(n / chunk_len) <= 64 the whole cascade is one
 * launch and needs no workspace.  `state_table` (optional, device, may be
 * NULL) is float64 [chunk_len][2S]: row t = A^(chunk_len-1-t) B, the state
 * response of the S-stage cascade (state order s1_0, s2_0, s1_1, ...) to a
 * unit sample t samples into a chunk; with it the chunk end states cost 2S
 * FMAs per sample instead of a cascade run.
 * ------------------------------------------------------------------------- */
size_t dsp_biquad_workspace_bytes(int64_t B, int64_t n, int32_t S,
                                  int64_t chunk_len);
int dsp_biquad_cascade_f32(const float* x, float* y, int64_t B, int64_t n,
                           int64_t ld_x, int64_t ld_y, const double* sos_host,
                           int32_t S, int32_t clip, int64_t chunk_len,
                           const double* state_table, void* workspace,
                           size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * lfilter's inf / NaN labels after a cascade (ABI 2.4).
 * Replaces nothing numeric: it relabels, after dsp_biquad_cascade_f32 (or
 * consecutive calls of it) has filtered x into y with the second-order
 * sections of lfilter(b, a) (dsp_core.py:214, len(a) >= 2), the outputs that
 * a non-finite input reaches: scipy's recursion (direct form II transposed
 * over b / a0 and a / a0 zero-padded to one length D + 1) gives every y from
 * the first inf or NaN of x on the class -- +inf, -inf or NaN -- that its
 * float64 arithmetic gives (a one-pole low-pass keeps +inf, a section with b1
 * == a1 makes NaN), while the cascade makes them all NaN.  Rows whose y[n-1]
 * is finite (no non-finite input) are left as they are, after one read --
 * except when a / a0 = [1, 0, ...] (an FIR through lfilter's recursion, whose
 * finite values the caller computes as a convolution on dsp_src_polyphase_f32:
 * y[n-1] is finite again len(b) samples after an inf), where every row's x is
 * scanned.  Long stretches of finite x after the first inf or NaN whose class
 * state repeats (a pole that keeps +inf, or alternates its sign) are filled
 * without running the recursion sample by sample.
 * b (nb >= 1) and a (na >= 2, a[0] != 0) are HOST float64 arrays; D =
 * max(na, nb) - 1 <= DSP_LFILTER_NF_MAX.  x and y are [B][ld] float32 device
 * rows and must not alias.  (len(a) == 1 is lfilter's convolution: run it on
 * dsp_src_polyphase_f32 with L = M = 1, c_offset = 0, which keeps its labels.)
 * ------------------------------------------------------------------------- */
int dsp_lfilter_nonfinite_f32(const float* x, float* y, int64_t B, int64_t n, int64_t ld_x,
                              int64_t ld_y, const double* b, int32_t nb, const double* a,
                              int32_t na, void* stream);

/* ---------------------------------------------------------------------------
 * Batched complex FFT of power-of-two length, natural-order output: the DFT
 * that dsp_core.py:41-66 (fft_diezmado_en_tiempo, a recursive radix-2 DIT)
 * computes, here as radix-16 Stockham passes in LDS (round 1 named the entry
 * dsp_fft_r2_c2c_f32 after the reference's radix-2).  N = 2^log2n,
 * 0 <= log2n <= DSP_MAX_LOG2N_FFT.  real_input != 0: `in` is float32
 * [B][ld_in] real samples; otherwise interleaved complex [B][ld_in] (ld in
 * complex elements).  `out` is interleaved complex [B][ld_out].  `twiddles` is
 * the interleaved complex table exp(-2*pi*i*k/N), k < N/2, in float32.
 * Up to DSP_MAX_LOG2N one launch keeps each transform in LDS and needs no
 * workspace; above it a four-step transform keeps its intermediate in
 * `workspace` (device, 8-byte aligned, >= dsp_fft_workspace_bytes(B, log2n);
 * 0 below): up to 2^22 two launches over all rows, B * N * 8 bytes; from 2^23
 * (ABI 2.5, up to 2^30) three launches (a four-step nested in step B) row by
 * row, 2 * N * 8 bytes whatever B; plus, above 2^20, a coarse twiddle table of
 * 2^floor(log2n / 2) * 8 bytes, and a header of 8 bytes per row (per launch
 * part of at most 65535 rows for two launches).  Above DSP_MAX_LOG2N_FOURSTEP
 * (ABI 2.7, 2^31 and 2^32) the reference's own top level: each row's even and
 * odd samples gathered into the workspace, transformed (as above; 2^32 splits
 * once more), and combined in place, X[k] = E[k] + W^k O[k], X[k + N/2] =
 * E[k] - W^k O[k] with W from the caller's table; the workspace (256-byte
 * aligned) then holds the halves, an N/2-point twiddle table and the halves'
 * own workspace, ~9 N complex-float bytes whatever B.  Size the workspace with
 * dsp_fft_workspace_bytes, never with a formula of your own: the size grew in
 * ABI 2.4 (per-row header), 2.5 (coarse table, three-pass rows) and 2.7 (the
 * split), and a smaller buffer is refused with DSP_EINVAL.
 * dsp_fft_split_log2n(log2n) (a test hook) sets the calling thread's smallest
 * log2n (>= 16) that takes the split, default DSP_MAX_LOG2N_FOURSTEP + 1, so
 * the split can be checked against one four-step transform; -1 queries;
 * returns the previous value.
 * Non-finite input (ABI 2.4): every output component gets the class --
 * finite, +inf, -inf or NaN -- that the reference's recursive radix-2 DIT in
 * complex128 numpy arithmetic gives it (inf * 0 = NaN at the k = 0 twiddles,
 * inf - inf = NaN), and a finite component the DFT of the input with its
 * non-finite components zeroed (the reference's value there).  A repair
 * launch after the transform does it; on finite data it exits at once (up to
 * 2^14: one launch reading X[0] of every transform; above: the header flags).
 * The same holds for dsp_spectrum_f32 and dsp_stft_mag_f32, whose |X| is +inf
 * wherever a component is infinite and NaN where one is NaN, as np.abs
 * (hypot) gives it (dsp_core.py:91).
 * ------------------------------------------------------------------------- */
size_t dsp_fft_workspace_bytes(int64_t B, int32_t log2n);
int dsp_fft_split_log2n(int32_t log2n);
int dsp_fft_c2c_f32(const float* in, float* out, int64_t B, int32_t log2n,
                       int32_t real_input, int64_t ld_in, int64_t ld_out,
                       const float* twiddles, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ---------------------------------------------------------------------------
 * Any-length DFT, batched (app.py:322-324 calls
 * np.fft.fft on segments of int(1024*L/M) samples, not powers of two).
 * Bluestein: 1 <= n <= DSP_MAX_DFT, M = 2^m the smallest power of two
 * >= 2n - 1 (dsp_dft_size).  Tables from the caller, float64-computed and
 * rounded to float32, interleaved complex:
 *   chirp[k]     = exp(-i pi (k^2 mod 2n) / n),            k < n
 *   chirp_fft[k] = FFT_M(b)[k] / M, b[j] = b[M-j] = conj(chirp[j]) (j < n),
 *                  0 elsewhere,                            k < M
 *   twiddles_m   = exp(-2 pi i k / M),                     k < M/2
 * in: real float32 [B][ld_in] (real_input != 0) or complex; out complex [B][ld_out].
 * ------------------------------------------------------------------------- */
int dsp_dft_size(int64_t n);
int dsp_dft_f32(const float* in, float* out, int64_t B, int64_t n, int32_t real_input,
                int64_t ld_in, int64_t ld_out, const float* chirp, const float* chirp_fft,
                const float* twiddles_m, void* stream);

/* ---------------------------------------------------------------------------
 * Windowed magnitude spectrum of one segment per row.
 * Replaces dsp_core.py:74-98 (calcular_espectro_magnitud): segment
 * x[seg_start : seg_start + seg_len] zero-padded to N = 2^log2n (:76-82),
 * times window[N] (Hann, :85-87), FFT (:90), |X[k]| for k <= N/2 (:91,:97-98).
 * mag is float32 [B][ld_mag], ld_mag >= N/2 + 1.  log2n <= DSP_MAX_LOG2N_FOURSTEP;
 * above DSP_MAX_LOG2N the workspace rules of dsp_fft_c2c_f32 apply.
 * ------------------------------------------------------------------------- */
int dsp_spectrum_f32(const float* x, float* mag, int64_t B, int64_t ld_x,
                     int64_t seg_start, int64_t seg_len, int32_t log2n,
                     int64_t ld_mag, const float* window,
                     const float* twiddles, void* workspace, size_t workspace_bytes,
                     void* stream);

/* ---------------------------------------------------------------------------
 * Framed magnitude spectrogram (every frame instead of
 * calcular_espectro_magnitud's centre segment, dsp_core.py:74-98).
 * Frame f < `frames` of row b is x[b][seg_start + f*hop + j], j < N = 2^log2n,
 * zero past seg_start + seg_len; mag[(b*frames + f)*ld_mag + k] =
 * |FFT(window * frame)[k]| for k <= N/2.  frames == 1 is dsp_spectrum_f32.
 * ------------------------------------------------------------------------- */
int dsp_stft_mag_f32(const float* x, float* mag, int64_t B, int64_t ld_x,
                     int64_t seg_start, int64_t seg_len, int64_t hop, int64_t frames,
                     int32_t log2n, int64_t ld_mag, const float* window,
                     const float* twiddles, void* stream);

/* ---------------------------------------------------------------------------
 * Whole hot path of app.py:164-167 + :203-205 for a batch of channels:
 *   y   = SRC(x)                     (dsp_src_polyphase_f32)
 *   z   = clip(cascade(y))           (dsp_biquad_cascade_f32; S == 0 and
 *                                     clip == 0 is the EQ bypass: z := y)
 *   mag = |FFT(window * z[seg])|     (dsp_spectrum_f32; ABI 2.7: mag == NULL
 *                                     skips it)
 * y and z must not alias.  workspace_bytes >= dsp_chain_workspace_bytes();
 * the workspace must be zero-filled before its first use, and every call that
 * completes with status 0 (dsp_chain_status) leaves it ready for the next one,
 * whichever path served it: its first 256 bytes are a status header (word 0),
 * followed by the single-pass kernel's hand-off region, followed by the
 * two-launch cascade's scratch; the two paths never share bytes.  Each row's
 * result is bitwise independent of B for a given path and mode: y always;
 * z and mag across the default's choice of the single-pass mode (chained
 * tiles, or from ABI 2.7 the three-launch mode for small batches of long
 * rows) to float64 rounding only -- dsp_chain_mode(B, ...) names the mode, and
 * dsp_chain_path 2 / 4 fix it, for callers that split one batch over calls.
 *
 * Single-pass path (default).  When dsp_chain_tile_len() is nonzero, i.e.
 * 1 <= S <= 6 with every b0 != 0 (ABI 2.6: S = 0, the EQ bypassed, takes the
 * two-launch chain's copy pass), n_in a multiple of 4 (any n_in for the
 * one-tap SRC bypass below), and
 *   48: (L, M, ceil(K/L)) = (3, 2, 41), c_offset mod 3 == 0,
 *       (c_offset/3 - 40) mod 4 == 0 and n_out a multiple of 4 (the kernel
 *       with wave-uniform taps: configs 3 and 4), or
 *   4..48 (ABI 2.6, the per-phase kernels): every reduced ratio L'/M' with
 *       L', M' <= 8 at the default tap rule K = 40 max(L, M) + 1, i.e. every
 *       L, M in 1..8 of the reference app's sliders (and 2/1 at K = 127):
 *       the sub-chunk length depends on L'/M' (DESIGN.md §3.0.8), and
 *       (ABI 2.7) the SRC bypass as the one-tap SRC -- L = M = 1, K = 1,
 *       c_offset = 0, taps {1.0f}: y = x, so the kernel is the cascade alone,
 *       x read once and z written once (pass y = NULL: y is x) -- or
 *   32: any other L/M with ceil(K/L) <= 8, at most 8 branch classes of the
 *       32-output sub-chunk starts (L / gcd(32 M mod L, L)) and four x windows
 *       that fit 64 KB of LDS with the class tables (config 5's 160/147,
 *       K = 1023: 5 classes; 160/147 itself runs a compile-time-ratio
 *       instantiation whose class rows carry the window shift),
 * `tile_tables` is a device copy (256-byte aligned) of the tables
 * dsp_chain_tile_tables built for this call's geometry, taps and sos,
 * `tile_key` is the key it returned with them (a call whose n_in, n_out, K,
 * L, M, c_offset, S or sos differ from the tables' has another key and takes
 * the two-launch path; the taps must be the ones the tables were built from),
 * and the rows of x, y and z are 16-byte aligned with pitches that are
 * multiples of 4 (n_out itself need not be; with B == 1 the pitch is not
 * used), ONE kernel computes y and z from
 * x: x is read once, y and z are written once, y is never read back.  Its y
 * is bitwise that of dsp_src_polyphase_f32; z agrees with the two-launch
 * chain's within 2e-6 (its carry sums run in float32 in input-normal
 * coordinates).  y may be NULL on this path only: the y store
 * is skipped (a caller that needs z and |Z| alone); anywhere else y == NULL is
 * DSP_EINVAL.  chunk_len, state_table and xstate_table are not used by it; the
 * sos host array only keys the tables (the kernel reads its coefficients from
 * them).  Non-finite input: y, z and mag follow the reference (inf and NaN
 * as dsp_src_polyphase_f32 gives them; every z after the first non-finite y
 * of a channel NaN, as lfilter gives it): the single-pass kernel is followed
 * on `stream` by a repair launch that reruns, with the non-finite semantics,
 * the tiles of every channel whose carried state became non-finite, and
 * exits at once when none did.
 *
 * The single-pass kernel hands each tile's end state to the next tile of the
 * channel through the workspace; a wait that polls more than the calling
 * thread's spin limit gives up, sets workspace word 0 and leaves that call's z
 * wrong (nothing hangs).  dsp_chain_status(workspace, bytes, reset, stream)
 * synchronises `stream`, returns 0 when word 0 is clear and 1 when a wait gave
 * up since the last reset (negative DSP_E* on error) and, with reset != 0,
 * zero-fills the whole workspace (required after a give-up: flags of the
 * failed call may be left set).  Not graph-capturable.
 * dsp_chain_spin_limit(spins) sets the calling thread's limit (0 gives up at
 * the first unanswered poll: a test hook; -1 queries) and returns the previous
 * one (default 2^23 polls, ~0.4 s).
 *
 * dsp_chain_tile_tables (HOST, no device work) fills `tables_host`
 * (>= dsp_chain_tile_tables_bytes()) with the single-pass kernel's float64
 * carry tables (the cascade in block-diagonal coordinates: the sub-chunk
 * state-response rows, the powers of the diagonal blocks, the change of basis)
 * and, for the 48-sample kernel, its packed tap pairs (for the 32-sample
 * kernel, its per-class tap rows), from the HOST float32 taps and sos, and
 * stores their key in *key (may be NULL).  Returns 0 when the single-pass
 * kernel serves the geometry (copy the buffer to the device once and pass it
 * and the key to every call), 1 when it does not (the two-launch path serves
 * it; nothing to copy; *key = 0), DSP_EINVAL on bad arguments.  With
 * tile_tables == NULL dsp_chain_f32 takes the two-launch path.
 * Delay branch (L3/M2 kernel): when the flushed taps (dsp_src_polyphase_f32)
 * of polyphase branch 0 are all zero but its centre tap -- as the reference's
 * wc = 1/L design makes them -- the key says so and dsp_chain_f32 computes
 * that branch's outputs (every third) with one multiply each, bitwise what the
 * FMAs give on those taps.  Pass the same taps to dsp_chain_f32 and to the
 * SRC entry points so y stays bitwise equal across paths.
 *
 * Two-launch path (any other geometry, or dsp_chain_path(1)): SRC, then the
 * cascade.  With `xstate_table` (device, float64 [xstate_rows][2S], may be
 * NULL) the cascade's first pass reads x instead of y: chunk c's zero-state
 * end state is
 *     E_c = sum_j xstate_table[j] * x[c*shift + q0 + j],   j < xstate_rows
 * (x == 0 outside [0, n_in)), where (shift, q0, xstate_rows) come from
 * dsp_chain_xstate_geometry and row j = sum_t G[t] (L h)[t*M + c_offset -
 * (q0 + j)*L] composes the state-response table G of chunk_len (see
 * dsp_biquad_cascade_f32) with the float64 taps.  It needs 1 <= S <= 8,
 * S != 7, ceil(n_out / chunk_len) <= 64, chunk_len a multiple of 32,
 * chunk_len*M/L an integer multiple of 4 and 16-byte aligned rows of x.
 * Otherwise `state_table` (G, may be NULL) is used as in
 * dsp_biquad_cascade_f32.
 *
 * dsp_chain_path sets the path for the calling thread: 0 (default) the
 * single-pass kernel where it applies, 1 always the two-launch chain, 2 the
 * single-pass path with chained tiles only (one workgroup per tile, the
 * hand-off above), 3 the single-pass path with its persistent kernel where
 * one is built (L/M = 160/147: each wave runs its channels' tiles in order,
 * the entry state in registers; the default picks it for batches that fill
 * the chip), 4 (ABI 2.7) the three-launch mode of every single-pass kernel:
 * every tile from a zero entry state, a scan of the tiles' end states per
 * channel, every tile again from its entry state -- no tile waits for
 * another; the default picks it for small batches of long rows, where the
 * chained hand-off (~2 us a tile) would bound the launch; -1 only queries; returns the previous setting
 * (DSP_EINVAL for anything else).  Every variant gives bitwise the same y;
 * z agrees across variants to float64 rounding (bitwise for 2 and 3).
 * ------------------------------------------------------------------------- */
int dsp_chain_path(int32_t path);
int64_t dsp_chain_tile_len(int64_t n_in, int64_t n_out, int32_t K, int32_t L, int32_t M,
                           int64_t c_offset, int32_t S);
/* (ABI 2.7, HOST) The path dsp_chain_f32 with dsp_chain_path 0 takes for a
 * batch of B rows of this geometry: 0 the two-launch chain, 1 a single-pass
 * kernel (chained tiles or persistent), 3 its three-launch mode.  A caller that shards one job's rows over several calls passes the
 * job's B and forces the answer (dsp_chain_path 2 for 1, 4 for 3) on every
 * shard, so that every shard's rows are bitwise the unsharded call's. */
int32_t dsp_chain_mode(int64_t B, int64_t n_in, int64_t n_out, int32_t K, int32_t L, int32_t M,
                       int64_t c_offset, int32_t S);
size_t dsp_chain_workspace_bytes(int64_t B, int64_t n_in, int64_t n_out, int32_t K,
                                 int32_t L, int32_t M, int64_t c_offset, int32_t S,
                                 int64_t chunk_len);
size_t dsp_chain_tile_tables_bytes(void);
int dsp_chain_tile_tables(void* tables_host, size_t tables_bytes, int64_t n_in, int64_t n_out,
                          const float* taps_host, int32_t K, int32_t L, int32_t M,
                          int64_t c_offset, const double* sos_host, int32_t S, uint64_t* key);
int dsp_chain_status(void* workspace, size_t workspace_bytes, int32_t reset, void* stream);
int64_t dsp_chain_spin_limit(int64_t spins);
int dsp_chain_xstate_geometry(int64_t chunk_len, int32_t K, int32_t L, int32_t M,
                              int64_t c_offset, int64_t* shift, int64_t* q0,
                              int64_t* rows);
int dsp_chain_f32(const float* x, float* y, float* z, float* mag, int64_t B,
                  int64_t n_in, int64_t ld_x, int64_t n_out, int64_t ld_y,
                  const float* taps, int32_t K, int32_t L, int32_t M,
                  int64_t c_offset, const double* sos_host, int32_t S,
                  int32_t clip, int64_t chunk_len, const double* state_table,
                  const double* xstate_table, int64_t xstate_rows,
                  const void* tile_tables, uint64_t tile_key, int64_t seg_start,
                  int64_t seg_len, int32_t log2n, int64_t ld_mag,
                  const float* window, const float* twiddles, void* workspace,
                  size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Audio I/O edges.
 *
 * Loader, replacing dsp_core.py:10-35 (cargar_senal_audio: soundfile read,
 * channel mean, float32, divide by max|x| when > 1e-6):
 *   dsp_wav_parse        HOST: RIFF/WAVE header of an in-memory file (PCM 8/16/
 *                        24/32-bit, IEEE float 32/64, G.711 A-law/mu-law,
 *                        WAVE_FORMAT_EXTENSIBLE); no sample is touched;
 *   dsp_audio_parse      HOST: the same for RIFF/WAVE and FORM/AIFF or AIFF-C
 *                        ('NONE'/'twos'/'sowt' PCM, 'fl32'/'fl64', 'ulaw'/
 *                        'alaw'); `format` then carries DSP_AUDIO_BE for
 *                        big-endian samples and DSP_AUDIO_S8 for AIFF's
 *                        signed 8-bit PCM, and `bits` is the stored width
 *                        (8 for G.711);
 *   dsp_pcm_to_mono_f32  DEVICE: raw interleaved sample bytes [B][ld_bytes] ->
 *                        float32 [B][ld_out]: each sample scaled as soundfile
 *                        returns it (float64: ints / 2^(bits-1), u8 - 128,
 *                        G.711 expanded to 16-bit linear / 2^15), the
 *                        channel mean in float64 in numpy's summation order,
 *                        rounded to float32 (bit-identical to the reference);
 *   dsp_peak_normalize_f32  DEVICE: per row, peak = max|x| (float32; a NaN
 *                        propagates like np.max) and x /= peak where
 *                        (double)peak > threshold (the reference uses 1e-6).
 *                        peak_out: caller's device uint32[B], receives the
 *                        peaks as float32 bit patterns.
 *   dsp_pcm_batch_to_mono_f32  DEVICE: a batch of files in two launches
 *                        (load_batch): `pcm` (device)
 *                        holds every row's raw sample bytes, `rows` (HOST,
 *                        B descriptors: byte offset into pcm, frames, format,
 *                        bits, channels as dsp_audio_parse gives them; the
 *                        library validates them against pcm_bytes and copies
 *                        the table to its workspace) says where; out [B][ld_out]
 *                        receives row b's dsp_pcm_to_mono_f32 result in
 *                        [0, frames_b), zeros in [frames_b, width), each row
 *                        divided by its peak as dsp_peak_normalize_f32 does
 *                        (threshold, peak_out likewise); workspace (device,
 *                        256-byte aligned) >= dsp_pcm_batch_workspace_bytes(B,
 *                        width).  Bitwise the per-file calls.
 * Playback, replacing app.py:349-355 (nan_to_num, divide by max|z| when > 0,
 * * 32767, astype(int16), all in z_final's dtype):
 *   dsp_quantize_pcm16   DEVICE: float32 z [B][ld_z] -> int16 [B][ld_out],
 *                        peak_out as above (after nan_to_num); `precision`
 *                        64: the arithmetic in float64 (z_final came out of
 *                        the SRC or the EQ, both return float64), 32: in
 *                        float32 (SRC and EQ both bypassed: z_final is the
 *                        loader's float32 array);
 *   dsp_wav_header_pcm16 HOST: the 44-byte header scipy.io.wavfile.write puts
 *                        in front of 16-bit PCM (app.py:352).
 * ------------------------------------------------------------------------- */
#define DSP_WAV_PCM 1    /* integer PCM (8-bit unsigned, 16/24/32-bit signed) */
#define DSP_WAV_FLOAT 3  /* IEEE float, 32 or 64 bits                           */
#define DSP_WAV_ALAW 6   /* G.711 A-law, one byte per sample (-> 16-bit linear) */
#define DSP_WAV_ULAW 7   /* G.711 mu-law, one byte per sample                   */
#define DSP_AUDIO_BE 0x100 /* format flag: big-endian samples (AIFF)           */
#define DSP_AUDIO_S8 0x200 /* format flag: 8-bit PCM is signed (AIFF)          */
typedef struct dsp_wav_info {
  int32_t format;       /* DSP_WAV_PCM/FLOAT/ALAW/ULAW, | DSP_AUDIO_*    */
  int32_t channels;     /* interleaved channels, 1..128                  */
  int32_t sample_rate;  /* Hz                                            */
  int32_t bits;         /* bits per sample                               */
  int64_t frames;       /* samples per channel in the data chunk         */
  int64_t data_offset;  /* byte offset of the first sample in the file   */
  int64_t data_bytes;   /* bytes of sample data present                  */
} dsp_wav_info;

int dsp_wav_parse(const uint8_t* file, size_t len, dsp_wav_info* info);
int dsp_audio_parse(const uint8_t* file, size_t len, dsp_wav_info* info);
int dsp_pcm_to_mono_f32(const void* pcm, int32_t format, int32_t bits, int32_t channels,
                        int64_t B, int64_t frames, int64_t ld_bytes, float* out,
                        int64_t ld_out, void* stream);
int dsp_peak_normalize_f32(float* x, int64_t B, int64_t n, int64_t ld, double threshold,
                           uint32_t* peak_out, void* stream);
typedef struct dsp_pcm_row {
  int64_t offset;       /* byte offset of the row's first sample in pcm  */
  int64_t frames;       /* samples per channel (<= width)                */
  int32_t format;       /* as dsp_wav_info.format                        */
  int32_t bits;         /* as dsp_wav_info.bits                          */
  int32_t channels;     /* 1..128                                        */
  int32_t reserved;     /* 0                                             */
} dsp_pcm_row;
size_t dsp_pcm_batch_workspace_bytes(int64_t B, int64_t width);
int dsp_pcm_batch_to_mono_f32(const void* pcm, size_t pcm_bytes, const dsp_pcm_row* rows,
                              int64_t B, int64_t width, float* out, int64_t ld_out,
                              double threshold, uint32_t* peak_out, void* workspace,
                              size_t workspace_bytes, void* stream);
/* (ABI 2.7) DEVICE dtype edges of the drop-in: out[i] = in[i] for i < n over
 * flat arrays, float64 -> float32 rounded to nearest even (numpy's astype) or
 * float32 -> float64 (exact); complex arrays pass as 2n reals. */
int dsp_convert_f64_f32(const double* in, float* out, int64_t n, void* stream);
int dsp_convert_f32_f64(const float* in, double* out, int64_t n, void* stream);
int dsp_quantize_pcm16(const float* z, int16_t* out, int64_t B, int64_t n, int64_t ld_z,
                       int64_t ld_out, uint32_t* peak_out, int32_t precision, void* stream);
int dsp_wav_header_pcm16(uint8_t* header44, int32_t sample_rate, int32_t channels,
                         int64_t frames);

/* ---------------------------------------------------------------------------
 * Per-launch tracing (the reference has no tracing; this is the build's).
 * While enabled on the calling thread, every kernel this thread launches
 * through the library is bracketed by two hipEventRecord calls on its stream
 * (events are created once and reused).  dsp_trace_read waits for the
 * recorded events, copies up to `max` records (name: NUL-terminated, stride
 * DSP_TRACE_NAME bytes; duration in milliseconds) and clears the list; it
 * returns the number of records copied or a negative DSP_E* code.
 * ------------------------------------------------------------------------- */
#define DSP_TRACE_NAME 32
int dsp_trace_enable(int32_t enable);
int dsp_trace_read(char* names, float* ms, int32_t max);

#ifdef __cplusplus
}
#endif

#endif /* DSPCORE_H */
