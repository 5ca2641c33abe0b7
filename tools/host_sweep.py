"""Host-inclusive HostChain timing over block / slot counts (config-4
geometry, 1024 channels): python tools/host_sweep.py [block:slots ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dspcore.chain import ChainConfig  # noqa: E402
from dspcore.host import HostChain  # noqa: E402

dev = torch.device("cuda", 0)
wl = bench.WORKLOADS["c4"]
cfg = ChainConfig(wl["n_in"], wl["fs"], wl["L"], wl["M"], wl["num_taps"], bench.CONFIG3_GAINS,
                  n_fft=wl["n_fft"])
x = np.random.default_rng(5).uniform(-1, 1, (1024, wl["n_in"])).astype(np.float32)
for spec in sys.argv[1:] or ["64:3", "64:4", "32:4", "128:3"]:
    parts = [int(v) for v in spec.split(":")]
    blk, sl = parts[0], parts[1]
    th = parts[2] if len(parts) > 2 else 4
    hc = HostChain(cfg, dev, block=blk, slots=sl, copy_threads=th)
    hc.run(x)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        hc.run(x)
        ts.append(time.perf_counter() - t0)
    w = float(np.median(ts))
    print(f"block {blk} slots {sl} threads {th}: median {w * 1e3:.2f} ms, {1024 * 48000 / w / 1e6:.1f} "
          f"Msamples/s (min {min(ts) * 1e3:.2f} max {max(ts) * 1e3:.2f})", flush=True)
    del hc
    torch.cuda.empty_cache()
