"""Runs a bench workload's chain a few times on cuda:0 (the program the
rocprofv3 --pmc passes of tools/pmc_chain.sh profile).

    python tools/kernels_once.py [reps] [config] [channels]
    config: c3 (default) | c4 | c5 | eq (the EQ alone, L = M = 1, at config 4's
    batch), channels default the config's one-GPU batch.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from dspcore.chain import Chain, ChainConfig  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
key = sys.argv[2] if len(sys.argv) > 2 else "c3"
if key == "eq":   # the EQ alone (L = M = 1) at config 4's batch
    wl = dict(bench.WORKLOADS["c4"], L=1, M=1, num_taps=None, name="eq alone")
else:
    wl = bench.WORKLOADS[key]
B = int(sys.argv[3]) if len(sys.argv) > 3 else wl["channels"]
cfg = ChainConfig(wl["n_in"], wl["fs"], wl["L"], wl["M"], wl["num_taps"], bench.CONFIG3_GAINS,
                  n_fft=wl["n_fft"])
dev = torch.device("cuda", 0)
ch = Chain(cfg, B, dev, plan_batch=wl["channels"])
x = torch.rand((B, wl["n_in"]), device=dev) * 2 - 1
for _ in range(reps):
    ch.run(x)
torch.cuda.synchronize()
assert ch.handoff_ok()
print("done", wl["name"], B)
