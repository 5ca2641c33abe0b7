"""Generates the golden fixtures in tests/golden/ from the reference itself.

Run in the build container only (the reference is not on the GPU box):
    python tests/golden/make_golden.py [/root/reference]

It imports the reference's modules/dsp_core.py (soundfile, absent from this
image and used only by the WAV loader at dsp_core.py:2,20, is stubbed for the
import), calls its functions on seeded inputs and stores inputs and outputs as
.npz data.  Where a configuration needs a tap count the reference's signature
cannot express (num_taps 127 / 255 / 1023, SURVEY.md §7 hard part 4), the
expected output is composed from the reference's own primitives in the order
conversion_tasa_muestreo uses them (dsp_core.py:148-172) with its
generar_respuesta_impulso_sinc, and the spectrum with n_fft != 2048 uses the
reference's fft_diezmado_en_tiempo on the segment/window rule of :74-98.
No reference source is copied into the repository; only these vectors are.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import scipy

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference(root):
    sys.modules.setdefault("soundfile", types.ModuleType("soundfile"))
    sys.path.insert(0, root)
    import modules.dsp_core as ref  # noqa: E402
    return ref


def noise(rng, shape):
    """uniform(-1, 1) float32, peak-normalised per row like dsp_core.py:29-31."""
    x = rng.uniform(-1.0, 1.0, size=shape).astype(np.float32)
    peak = np.max(np.abs(x), axis=-1, keepdims=True)
    return (x / peak).astype(np.float32)


def src_via_primitives(ref, x, fs, M, L, K):
    """conversion_tasa_muestreo's steps (dsp_core.py:148-172) with an explicit K."""
    if K is None:
        return ref.conversion_tasa_muestreo(x, fs, M, L)
    xe = np.zeros(len(x) * L, dtype=x.dtype)
    xe[::L] = x
    h = ref.generar_respuesta_impulso_sinc(1.0 / max(L, M), K)
    h *= L
    return np.convolve(xe, h, mode="same")[::M], int(fs * L / M)


def spectrum_via_primitives(ref, z, fs, n_fft):
    """calcular_espectro_magnitud's steps (dsp_core.py:74-98) with N_ventana = n_fft."""
    if n_fft == 2048:
        return ref.calcular_espectro_magnitud(z, fs)
    if len(z) > n_fft:
        mid = len(z) // 2
        seg = z[mid:mid + n_fft]
    else:
        seg = np.pad(z, (0, (1 << (len(z) - 1).bit_length()) - len(z)))
    n = len(seg)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))
    mag = np.abs(ref.fft_diezmado_en_tiempo(seg * w))
    return np.fft.rfftfreq(n, d=1 / fs)[: n // 2 + 1], mag[: n // 2 + 1]


CONFIG3_GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3,
                 "High Mids": -3, "Presence": 5, "Brilliance": -6}


def main(root="/root/reference"):
    ref = load_reference(root)
    rng = np.random.default_rng(20261015)
    out = {}

    # (1) FIR taps.
    taps_cases = [(1 / 2, 81), (1 / 3, 121), (1 / 2, 127), (1 / 3, 255), (1 / 8, 321),
                  (1 / 160, 1023), (1 / 160, 6401), (1 / 2, 8)]
    np.savez_compressed(os.path.join(HERE, "taps.npz"), **{
        f"h_{i}": ref.generar_respuesta_impulso_sinc(wc, k) for i, (wc, k) in enumerate(taps_cases)},
        cases=np.array(taps_cases))

    # (2)+(3) SRC: noise (4 channels) and delta inputs.
    src_cases = [  # L, M, K (None = default rule), N, fs
        (3, 2, None, 4800, 48000), (3, 2, 255, 4800, 48000), (2, 1, 127, 4800, 44100),
        (2, 1, None, 4800, 44100), (160, 147, 1023, 480, 44100), (8, 8, None, 4800, 48000),
        (1, 3, None, 7, 48000), (3, 2, None, 7, 48000), (5, 7, None, 500, 48000),
        (4, 3, None, 1000, 32000), (1, 2, None, 999, 48000)]
    src = {"cases": np.array([[L, M, -1 if K is None else K, N, fs]
                              for L, M, K, N, fs in src_cases])}
    for i, (L, M, K, N, fs) in enumerate(src_cases):
        x = noise(rng, (4, N))
        ys = [src_via_primitives(ref, x[c], fs, M, L, K) for c in range(4)]
        src[f"x_{i}"] = x
        src[f"y_{i}"] = np.stack([y for y, _ in ys])
        src[f"fs_{i}"] = np.array(ys[0][1])
    delta_cases = [(3, 2, None, 300, [0, 1, 150, 299]), (160, 147, 1023, 50, [0, 7, 49]),
                   (2, 1, 127, 200, [0, 100, 199]), (3, 2, 255, 120, [3, 60])]
    src["delta_cases"] = np.array([[L, M, -1 if K is None else K, N]
                                   for L, M, K, N, _ in delta_cases])
    for i, (L, M, K, N, pos) in enumerate(delta_cases):
        x = np.zeros((len(pos), N), np.float32)
        for r, p in enumerate(pos):
            x[r, p] = 1.0
        src[f"dx_{i}"] = x
        src[f"dy_{i}"] = np.stack([src_via_primitives(ref, x[r], 48000, M, L, K)[0]
                                   for r in range(len(pos))])
    np.savez_compressed(os.path.join(HERE, "src.npz"), **src)

    # (4) biquad coefficients.
    rows = []
    for fs in (48000, 72000, 96000, 6000):
        for fc in (40, 150, 1000, 3000, 5000, 10000):
            for g in (-15, -6, 0.1, 6, 15):
                b, a = ref.disenar_coeficientes_diferencias(fc, fs, g)
                rows.append([fc, fs, g, *b, *a])
    np.savez_compressed(os.path.join(HERE, "biquad.npz"), rows=np.array(rows))

    # (5) EQ outputs on an SRC output (float64) and on raw float32 input.
    x = noise(rng, (7200,))
    y72, _ = ref.conversion_tasa_muestreo(x[:4800], 48000, 2, 3)
    eq_cases = [
        (72000, CONFIG3_GAINS),
        (72000, {k: 15 for k in CONFIG3_GAINS}),
        (72000, {k: -15 for k in CONFIG3_GAINS}),
        (72000, {k: 0 for k in CONFIG3_GAINS}),                      # bypass
        (72000, {"Sub-Bass": 0.1, "Bass": 0, "Low Mids": 0.05}),     # g == 0.1: clip only
        (72000, {"Mystery": 9, "Bass": 3}),                          # unknown -> 1000 Hz
        (6000, CONFIG3_GAINS),                                        # Nyquist clamp
        (48000, {"Brilliance": 12, "Presence": -9}),
        (20, {"Bass": 6}),                                            # fc <= 10 after clamp
        (72000, {}),                                                  # empty dict bypasses
    ]
    eq = {"x64": y72, "x32": x}
    for i, (fs, g) in enumerate(eq_cases):
        eq[f"gains_{i}"] = np.array(json.dumps(g))
        eq[f"fs_{i}"] = np.array(fs)
        eq[f"z64_{i}"] = np.asarray(ref.sistema_ecualizador(y72, fs, g))
        eq[f"z32_{i}"] = np.asarray(ref.sistema_ecualizador(x, fs, g))
    np.savez_compressed(os.path.join(HERE, "eq.npz"), **eq)

    # (6) FFT, N = 2^0 .. 2^12, real and complex.
    fft = {}
    for k in range(13):
        n = 1 << k
        xr = rng.uniform(-1, 1, n)
        xc = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
        fft[f"xr_{k}"], fft[f"Xr_{k}"] = xr, np.asarray(ref.fft_diezmado_en_tiempo(xr))
        fft[f"xc_{k}"], fft[f"Xc_{k}"] = xc, np.asarray(ref.fft_diezmado_en_tiempo(xc))
    np.savez_compressed(os.path.join(HERE, "fft.npz"), **fft)

    # (7) spectrum for several lengths, and the lengths where the reference raises.
    spec = {}
    lengths = [1, 2, 6, 1000, 2048, 4095, 4096, 5000, 100000]
    for i, n in enumerate(lengths):
        xs = noise(rng, (n,)).astype(np.float64)
        f, m = ref.calcular_espectro_magnitud(xs, 44100)
        spec[f"x_{i}"], spec[f"f_{i}"], spec[f"m_{i}"] = xs, f, m
    spec["lengths"] = np.array(lengths)
    raising = []
    for n in (2049, 2050, 3000, 4000, 4094):
        try:
            ref.calcular_espectro_magnitud(np.ones(n), 44100)
            raising.append([n, 0])
        except ValueError:
            raising.append([n, 1])
    spec["raising"] = np.array(raising)
    np.savez_compressed(os.path.join(HERE, "spectrum.npz"), **spec)

    # (8) chain: config 3 (1 ch x 48000) and config 5 (1 ch x 48000).
    chain = {}
    for tag, fs, L, M, K, nfft in (("c3", 48000, 3, 2, None, 4096),
                                   ("c5", 44100, 160, 147, 1023, 4096)):
        x = noise(rng, (48000,))
        y, fs_out = src_via_primitives(ref, x, fs, M, L, K)
        z = ref.sistema_ecualizador(y, fs_out, CONFIG3_GAINS)
        f, m = spectrum_via_primitives(ref, z, fs_out, nfft)
        f2, m2 = ref.calcular_espectro_magnitud(z, fs_out)
        chain.update({f"{tag}_x": x, f"{tag}_y": y, f"{tag}_z": z, f"{tag}_mag": m,
                      f"{tag}_f": f, f"{tag}_mag2048": m2, f"{tag}_fs_out": np.array(fs_out)})
    np.savez_compressed(os.path.join(HERE, "chain.npz"), **chain)

    # (9) FFT above the one-launch size, N = 2^13 .. 2^16: real rows for every
    # size, complex rows for 2^15 and 2^16, plus the spectrum recipe at
    # n_fft = 2^15 on a 100000-sample signal.  Own seed (the fixtures above
    # stay as they were); inputs stored as float32 / complex64 (exactly what
    # the reference was given), outputs rounded to complex64 / float32
    # (6e-8 relative, far inside the 1e-5 tolerance) to keep the file small.
    rng9 = np.random.default_rng(20261016)
    big = {}
    for k in (13, 14, 15, 16):
        n = 1 << k
        xr = rng9.uniform(-1, 1, n).astype(np.float32)
        big[f"xr_{k}"] = xr
        big[f"Xr_{k}"] = np.asarray(ref.fft_diezmado_en_tiempo(xr.astype(np.float64)),
                                    dtype=np.complex128).astype(np.complex64)
        if k >= 15:
            xc = (rng9.uniform(-1, 1, n) + 1j * rng9.uniform(-1, 1, n)).astype(np.complex64)
            big[f"xc_{k}"] = xc
            big[f"Xc_{k}"] = np.asarray(ref.fft_diezmado_en_tiempo(xc.astype(np.complex128)),
                                        dtype=np.complex128).astype(np.complex64)
    zs = noise(rng9, (100000,))
    fs15, ms15 = spectrum_via_primitives(ref, zs.astype(np.float64), 72000, 1 << 15)
    big["spec_x"], big["spec_f"], big["spec_m"] = zs, fs15, ms15.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "fft_large.npz"), **big)

    manifest = {"numpy": np.__version__, "scipy": scipy.__version__,
                "reference": "Renatovela-ctrl/dsp-audio-project modules/dsp_core.py",
                "generator": "tests/golden/make_golden.py", "seed": 20261015}
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
