"""Per-kernel times of the config-3 chain (HIP-event traced) for the library
named by DSPCORE_LIB -- A/B experiments between builds of the same ABI."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dspcore import _lib  # noqa: E402
from dspcore.chain import Chain, ChainConfig  # noqa: E402

gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5, "Brilliance": -6}
B = int(os.environ.get("CHAIN_B", 4096))
cfg = ChainConfig(48000, 48000, 3, 2, None, gains, n_fft=4096)
dev = torch.device("cuda", 0)
x = torch.rand((B, 48000), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
x = x * 2 - 1
variants = {"xstate": dict(), "ytable": dict(use_xstate=False),
            "xstate1152": dict(chunk_len=1152), "ytable1152": dict(use_xstate=False, chunk_len=1152)}
if os.environ.get("CHAIN_C5"):
    B = int(os.environ.get("CHAIN_B", 1024))
    cfg = ChainConfig(48000, 44100, 160, 147, 1023, gains, n_fft=4096)
    x = torch.rand((B, 48000), device=dev) * 2 - 1
    variants = {"c5": dict(), "c5_T1280": dict(chunk_len=1280)}
res = {}
for name, kw in variants.items():
    ch = Chain(cfg, B, dev, **kw)
    for _ in range(3):
        ch.run(x, check=False)
    torch.cuda.synchronize()
    _lib.trace_enable(True)
    _lib.trace_read()
    for _ in range(10):
        ch.run(x, check=False)
    recs = _lib.trace_read()
    _lib.trace_enable(False)
    per = {}
    for k, ms in recs:
        per.setdefault(k, []).append(ms)
    res[name] = {k: round(float(np.median(v)), 4) for k, v in per.items()}
    res[name]["z00"] = float(ch.z[0, 1000])
print(os.path.basename(_lib.LIB_PATH), res)

# Copy ceiling on this box: torch device copy of a y-sized buffer (read + write).
a = torch.empty((B, 72000), device=dev)
b2 = torch.empty_like(a)
for _ in range(3):
    b2.copy_(a)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(10):
    b2.copy_(a)
ev[1].record()
torch.cuda.synchronize()
ms = ev[0].elapsed_time(ev[1]) / 10
print(f"copy {a.numel() * 4 / 1e9:.2f} GB: {ms:.4f} ms = {2 * a.numel() * 4 / ms / 1e9:.0f} GB/s (read+write)")
