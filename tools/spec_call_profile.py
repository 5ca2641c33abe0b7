"""Host-side cost of one drop-in call of the app's rerun (app.py:162-167,
203-205) on a 441000-sample numpy channel: `spec` (calcular_espectro_magnitud
on the app's 100000-sample slice), `eq` (sistema_ecualizador) or `src`
(conversion_tasa_muestreo 3/2).  Per call: the synchronised mean over N calls,
then cProfile over N calls sorted by own time; for `spec` also the median of
each step timed alone (host -> device, the kernel call, device -> host).
Usage: python tools/spec_call_profile.py [spec|eq|src] [N]."""
import cProfile
import os
import pstats
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
    what = sys.argv[1] if len(sys.argv) > 1 else "spec"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    x = np.random.default_rng(3).uniform(-1, 1, 441000).astype(np.float32)
    call = {"spec": lambda: dc.calcular_espectro_magnitud(x[:100000], 44100),
            "eq": lambda: dc.sistema_ecualizador(x, 44100, GAINS),
            "src": lambda: dc.conversion_tasa_muestreo(x, 44100, 2, 3)}[what]
    dev = torch.device("cuda", 0)
    for _ in range(20):
        call()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(n):
        call()
    torch.cuda.synchronize(dev)
    print(f"{what} call: {(time.perf_counter() - t0) / n * 1e3:.4f} ms", flush=True)

    if what == "spec":
        from dspcore import design, ops
        xs = x[:100000].astype(np.float64)
        plan = design.spectrum_plan(len(xs), 2048)
        seg = np.ascontiguousarray(xs[plan.seg_start:plan.seg_start + plan.seg_len])

        def med(fn, k=200):
            ts = []
            for _ in range(k):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t)
            return np.median(ts) * 1e3

        t_rows = med(lambda: dc._to_rows(seg))
        rows, _ = dc._to_rows(seg)
        t_spec = med(lambda: ops.spectrum(rows, 0, plan.seg_len, plan.n_fft))
        mag = ops.spectrum(rows, 0, plan.seg_len, plan.n_fft)
        t_back = med(lambda: dc._from_rows(mag, "np1", np.float64))
        t_host = med(lambda: ops.spectrum_host(seg[None, :], plan.n_fft, dev))
        print(f"steps (median, synchronised): to_rows {t_rows:.4f}, spectrum {t_spec:.4f}, "
              f"from_rows {t_back:.4f} ms; the zero-copy spectrum_host {t_host:.4f} ms",
              flush=True)

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        call()
    torch.cuda.synchronize(dev)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
