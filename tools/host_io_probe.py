"""Host <-> device conversion costs of the drop-in's numpy calls (one app rerun
moves a 441000..882000-sample channel in and out several times): the current
route (host dtype conversion + pageable copies) against device-side casts and
pinned (page-locked) host buffers.  ms per variant, median of 20."""
import time

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dsp-audio-project_amd"))


def med(fn, k=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return sorted(ts)[k // 2]


def main():
    from dspcore import ops
    dev = torch.device("cuda", 0)
    for n in (441000, 882000):
        t = torch.rand(n, device=dev)
        a64 = np.random.default_rng(0).uniform(-1, 1, n)
        a32 = a64.astype(np.float32)
        pin64 = torch.empty(n, dtype=torch.float64, pin_memory=True)
        pin32 = torch.empty(n, dtype=torch.float32, pin_memory=True)
        rows = {
            "D2H f32 pageable + host astype f64 (current)":
                lambda: t.cpu().numpy().astype(np.float64),
            "device cast f64 + D2H pageable":
                lambda: t.to(torch.float64).cpu().numpy(),
            "device cast f64 + D2H into fresh pinned":
                lambda: torch.empty(n, dtype=torch.float64, pin_memory=True).copy_(
                    t.to(torch.float64)).numpy(),
            "device cast f64 + D2H into held pinned":
                lambda: pin64.copy_(t.to(torch.float64)).numpy(),
            "library cast kernel writing f64 into held pinned (zero-copy)":
                lambda: ops.convert(t, torch.float64, out=pin64).numpy(),
            "library cast kernel writing f64 into fresh pinned (zero-copy)":
                lambda: ops.convert(t, torch.float64, out=torch.empty(
                    n, dtype=torch.float64, pin_memory=True)).numpy(),
            "D2H f32 into held pinned + host astype":
                lambda: pin32.copy_(t).numpy().astype(np.float64),
            "H2D: host astype f32 + pageable (current, f64 in)":
                lambda: torch.from_numpy(np.ascontiguousarray(a64, dtype=np.float32)).to(dev),
            "H2D: f64 pageable + device cast":
                lambda: torch.from_numpy(a64).to(dev).float(),
            "H2D: f64 via held pinned + device cast":
                lambda: (pin64.numpy().__setitem__(slice(None), a64),
                         pin64.to(dev, non_blocking=True).float())[1],
            "H2D: f64 from a numpy view of pinned memory + device cast":
                lambda: torch.from_numpy(pin64.numpy()).to(dev).float(),
            "H2D: f64 pinned tensor non_blocking + device cast":
                lambda: pin64.to(dev, non_blocking=True).float(),
            "H2D: f32 pageable (f32 in)":
                lambda: torch.from_numpy(a32).to(dev),
            "H2D: f32 via held pinned":
                lambda: (pin32.numpy().__setitem__(slice(None), a32),
                         pin32.to(dev, non_blocking=True))[1],
        }
        for name, fn in rows.items():
            print(f"n={n} {name}: {med(fn):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
