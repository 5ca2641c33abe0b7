"""The drop-in under concurrent callers: Streamlit runs each session's script
in its own thread (SURVEY.md §8(b) Threading; /root/reference/app.py:162-167,
203-205), so the app's rerun -- conversion_tasa_muestreo, sistema_ecualizador,
three calcular_espectro_magnitud calls -- and fft_diezmado_en_tiempo may run
from several threads at once.  Every thread's results must be bitwise the
ones the same calls give when run one after another (the per-thread EQ
workspace and page-locked staging buffers, the shared LUT caches)."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GAINS = [{"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5,
          "Brilliance": -6},
         {"Sub-Bass": -15, "Bass": 15, "Presence": 2},
         {"Brilliance": 9, "Low Mids": -7}]
RATIOS = [(1, 1), (2, 1), (3, 2), (1, 2)]


def _rerun(dc, x, fs, L, M, gains):
    y, fs2 = dc.conversion_tasa_muestreo(x, fs, M, L)
    z = dc.sistema_ecualizador(y, fs2, gains)
    lim = 100000
    spectra = [dc.calcular_espectro_magnitud(v[:lim], f)[1]
               for v, f in ((x, fs), (y, fs2), (z, fs2))]
    X = dc.fft_diezmado_en_tiempo(z[:2048])
    return [np.asarray(y), np.asarray(z)] + spectra + [X]


def test_concurrent_reruns_bitwise_sequential(gpu):
    from modules import dsp_core as dc
    fs, n = 44100, 120000
    jobs = []
    for i in range(6):
        rng = np.random.default_rng(100 + i)
        x = (0.5 * np.sin(2 * np.pi * (220 + 70 * i) * np.arange(n) / fs)
             + 0.3 * rng.uniform(-1, 1, n)).astype(np.float32)
        L, M = RATIOS[i % len(RATIOS)]
        jobs.append((x, fs, L, M, GAINS[i % len(GAINS)]))
    expected = [_rerun(dc, *j) for j in jobs]

    got = [None] * len(jobs)
    errors = []
    start = threading.Barrier(len(jobs))

    def worker(i):
        try:
            start.wait()
            out = None
            for _ in range(3):          # the staging buffers and workspaces reused
                out = _rerun(dc, *jobs[i])
                for a, b in zip(out, expected[i]):
                    np.testing.assert_array_equal(a, b)
            got[i] = out
        except BaseException as e:  # noqa: BLE001  (re-raised on the test's thread)
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "a drop-in thread did not finish"
    if errors:
        raise errors[0]
    assert all(g is not None for g in got)
