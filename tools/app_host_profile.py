"""cProfile of the app's rerun through the drop-in (bench.py app_rerun's calls,
one 441000-sample channel, L/M from argv, default 2/1): where the host time
of a rerun goes besides the kernels.  Prints the top functions by cumulative
and by own time over 20 reruns."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dsp-audio-project_amd"))

from modules import dsp_core as dc  # noqa: E402

GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5,
         "Brilliance": -6}


def main():
    L, M = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2/1").split("/"))
    fs, n, lim = 44100, 441000, 100000
    t = np.arange(n) / fs
    x = (0.6 * np.sin(2 * np.pi * 440.0 * t)
         + 0.3 * np.random.default_rng(7).uniform(-1, 1, n)).astype(np.float32)
    x /= np.max(np.abs(x))

    def rerun():
        y, fs2 = dc.conversion_tasa_muestreo(x, fs, M, L)
        z = dc.sistema_ecualizador(y, fs2, GAINS)
        r = (dc.calcular_espectro_magnitud(x[:lim], fs), dc.calcular_espectro_magnitud(y[:lim], fs2),
             dc.calcular_espectro_magnitud(z[:lim], fs2))
        torch.cuda.synchronize()
        return r

    for _ in range(3):
        rerun()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        rerun()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(35)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
