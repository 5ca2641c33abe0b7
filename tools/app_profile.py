"""Where one app rerun's time goes: the drop-in calls of app.py:162-167 and
:203-205 on one 441000-sample channel (bench.py app_rerun's input) at the given
L/M ratios, each call timed on the host (synchronised), so that a
`rocprofv3 --kernel-trace --stats` run of this script splits kernels from host
work.  Usage: python tools/app_profile.py [L/M ...] (default 1/1 2/1 3/2)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dsp-audio-project_amd"))

from modules import dsp_core as dc  # noqa: E402

GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5,
         "Brilliance": -6}


def main():
    ratios = [tuple(int(v) for v in a.split("/")) for a in sys.argv[1:]] or [(1, 1), (2, 1), (3, 2)]
    fs, n, lim = 44100, 441000, 100000
    t = np.arange(n) / fs
    x = (0.6 * np.sin(2 * np.pi * 440.0 * t)
         + 0.3 * np.random.default_rng(7).uniform(-1, 1, n)).astype(np.float32)
    x /= np.max(np.abs(x))
    dev = torch.device("cuda", 0)

    def timed(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        return out, (time.perf_counter() - t0) * 1e3

    for L, M in ratios:
        rows = []
        for rep in range(6):
            (y, fs2), a = timed(lambda: dc.conversion_tasa_muestreo(x, fs, M, L))
            z, b = timed(lambda: dc.sistema_ecualizador(y, fs2, GAINS))
            _, c = timed(lambda: dc.calcular_espectro_magnitud(x[:lim], fs))
            _, d = timed(lambda: dc.calcular_espectro_magnitud(y[:lim], fs2))
            _, e = timed(lambda: dc.calcular_espectro_magnitud(z[:lim], fs2))
            if rep:
                rows.append((a, b, c, d, e))
        med = np.median(np.array(rows), axis=0)
        print(f"L/M {L}/{M}: src {med[0]:.3f} ms, eq {med[1]:.3f} ms, spectra "
              f"{med[2]:.3f} + {med[3]:.3f} + {med[4]:.3f} ms, total {med.sum():.3f} ms", flush=True)


if __name__ == "__main__":
    main()
