"""The cascade alone (L = M = 1, config-3 gains; --ratio L/M for another
ratio, y not kept): the single-pass one-tap
kernel (Chain.run) against the two-pass cascade (Chain.run_stages) on the same
box, HIP-graph replay like bench.py, for the batch shapes given as BxN
(default 4096x48000 32768x48000 1x441000 1x48000 16x441000).  Prints ms per
call of each path, the single-pass kernel's algorithmic GB/s (x read + z
written), the speedup, and the default's two modes forced (dsp_chain_path 2:
chained tiles, 4: three launches).  The graph capture runs on the calling
thread, so the forced path holds during capture."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dsp-audio-project_amd"))

from dspcore import _lib  # noqa: E402
from dspcore.chain import Chain, ChainConfig  # noqa: E402

GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3, "High Mids": -3, "Presence": 5,
         "Brilliance": -6}


def graph_ms(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    args = sys.argv[1:]
    L = M = 1
    K = None
    if "--ratio" in args:   # another SRC ratio (L/M or L/M/K) through the same paths
        i = args.index("--ratio")
        v = [int(t) for t in args[i + 1].split("/")]
        L, M = v[0], v[1]
        K = v[2] if len(v) > 2 else None
        del args[i:i + 2]
    shapes = [tuple(int(v) for v in a.split("x")) for a in args] or \
        [(4096, 48000), (32768, 48000), (1, 441000), (1, 48000), (16, 441000)]
    dev = torch.device("cuda", 0)
    print(f"L/M {L}/{M}" + (f" K {K}" if K else ""), flush=True)
    for B, n in shapes:
        cfg = ChainConfig(n, 48000, L, M, K, GAINS, n_fft=4096)
        ch = Chain(cfg, B, dev, keep_y=False)
        x = torch.rand((B, n), device=dev) * 2 - 1
        reps = max(5, min(200, int(2e9 // (B * n * 8))))
        t1 = graph_ms(lambda: ch.run(x, check=False), reps)
        t0 = graph_ms(lambda: ch.run_stages(x), reps)
        paths = {}
        for p in (2, 4):   # the chained tiles, the three-launch mode
            prev = _lib.chain_path(p)
            try:
                paths[p] = graph_ms(lambda: ch.run(x, check=False), reps)
            finally:
                _lib.chain_path(prev)
        ch.check()
        gbs = B * (n * 4 + ch.n_out * 4) / (t1 * 1e-3) / 1e9
        print(f"B={B} n={n}: single-pass {t1:.4f} ms ({gbs:.0f} GB/s x+z, "
              f"{B * n / t1 / 1e6:.1f} G samples/s), two-pass {t0:.4f} ms, x{t0 / t1:.2f} "
              f"(tile_len {ch.tile_len}); chained {paths[2]:.4f} ms, three-launch "
              f"{paths[4]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
