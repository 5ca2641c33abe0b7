"""Runs the config-3 chain a few times (for rocprofv3 --pmc passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import torch  # noqa: E402

from dspcore.chain import Chain, ChainConfig  # noqa: E402

gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5, "Brilliance": -6}
cfg = ChainConfig(48000, 48000, 3, 2, None, gains, n_fft=4096)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
ch = Chain(cfg, 4096, dev)
x = torch.rand((4096, 48000), device=dev) * 2 - 1
for _ in range(reps):
    ch.run(x)
torch.cuda.synchronize()
print("done")
