"""Config-3 chain kernel times (HIP-event traced) with the fused SRC + cascade
launch on and off, for the library named by DSPCORE_LIB (A/B of builds)."""
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
L, M = (int(v) for v in os.environ.get("CHAIN_LM", "3,2").split(","))
cfg = ChainConfig(48000, 48000, L, M, None, gains, n_fft=4096)
dev = torch.device("cuda", 0)
x = torch.rand((B, 48000), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
x = x * 2 - 1
T = int(os.environ.get("CHAIN_T", 0)) or None
ch = Chain(cfg, B, dev, chunk_len=T)
res = {}
modes = [int(m) for m in os.environ.get("FUSION_MODES", "1,0").split(",")]
for rnd in range(3):
    for mode in modes:
        _lib.chain_fusion(mode)
        for _ in range(3):
            ch.run(x)
        torch.cuda.synchronize()
        _lib.trace_enable(True)
        _lib.trace_read()
        for _ in range(10):
            ch.run(x)
        recs = _lib.trace_read()
        _lib.trace_enable(False)
        for k, ms in recs:
            res.setdefault((mode, k), []).append(ms)
print(os.path.basename(_lib.LIB_PATH), f"L/M={L}/{M} T={ch.chunk_len}",
      {f"m{m}:{k}": round(float(np.median(v)), 4) for (m, k), v in res.items()},
      "z00", float(ch.z[0, 1000]))
