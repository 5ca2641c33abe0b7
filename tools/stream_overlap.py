"""Throughput of the config-3 chain with consecutive batches on one stream vs
alternating over two streams (double-buffered y/z): does SRC of batch i+1
overlap the EQ of batch i?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import torch  # noqa: E402

from dspcore.chain import Chain, ChainConfig  # noqa: E402

gains = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5, "Brilliance": -6}
B = 4096
cfg = ChainConfig(48000, 48000, 3, 2, None, gains, n_fft=4096)
dev = torch.device("cuda", 0)
x = torch.rand((B, 48000), device=dev) * 2 - 1
chains = [Chain(cfg, B, dev) for _ in range(2)]
streams = [torch.cuda.Stream(dev) for _ in range(2)]
K = 20


def run(nstreams):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        s = streams[i % nstreams] if nstreams > 1 else torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            chains[i % 2].run(x, check=False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for n in (1, 2, 1, 2):
    run(n)
    print(f"{n} stream(s): {run(n):.4f} ms/step")
