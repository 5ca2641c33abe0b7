"""Times the fused IIR cascade (config-3 size, chunk 1152) for the library
named by DSPCORE_LIB (tile-width experiments)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dspcore import _lib, design, ops  # noqa: E402

B, n = 4096, 72000
dev = torch.device("cuda", 0)
gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5, "Brilliance": -6}
sos = design.eq_plan(72000, gains).sos
x = torch.rand((B, n), device=dev) * 2 - 1
out = torch.empty_like(x)
ref = None
res = []
for rnd in range(6):
    ws = ops.biquad_workspace(B, n, 6, dev, 1152)
    ops.biquad_cascade(x, sos, True, out=out, workspace=ws, chunk_len=1152)
    torch.cuda.synchronize()
    if ref is None:
        ref = out[:8].clone()
    _lib.trace_enable(True)
    _lib.trace_read()
    for _ in range(3):
        ops.biquad_cascade(x, sos, True, out=out, workspace=ws, chunk_len=1152)
    recs = _lib.trace_read()
    _lib.trace_enable(False)
    if rnd > 0:
        res.append(sum(ms for _, ms in recs) / 3)
print(f"{os.path.basename(_lib.LIB_PATH):24s} {recs[0][0]} median {np.median(res):.4f} ms "
      f"min {np.min(res):.4f} ms  row0[:4]={out[0, :4].tolist()}")
