"""Same-box A/B of dsp_chain_f32's paths: the single-pass kernel (path 0) and
the two-launch chain (path 1), per-kernel HIP-event means over K traced steps.

    python tools/chain_ab.py [--config c3|c5] [--channels B] [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dsp-audio-project_amd"), ROOT]

import torch  # noqa: E402

from bench import CONFIG3_GAINS, WORKLOADS  # noqa: E402
from dspcore import _lib  # noqa: E402
from dspcore.chain import Chain, ChainConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--channels", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    wl = dict(WORKLOADS[args.config])
    B = args.channels or wl["channels"]
    dev = torch.device("cuda", 0)
    cfg = ChainConfig(wl["n_in"], wl["fs"], wl["L"], wl["M"], wl["num_taps"], CONFIG3_GAINS,
                      n_fft=wl["n_fft"])
    ch = Chain(cfg, B, dev)
    x = torch.rand((B, wl["n_in"]), device=dev) * 2 - 1
    out = {"config": args.config, "channels": B, "tile_len": ch.tile_len}
    for path in (0, 1):
        prev = _lib.chain_path(path)
        for _ in range(3):
            ch.run(x, check=False)
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(args.steps):
            ch.run(x, check=False)
        end.record()
        torch.cuda.synchronize()
        _lib.trace_enable(True)
        _lib.trace_read()
        for _ in range(args.steps):
            ch.run(x, check=False)
        recs = _lib.trace_read()
        _lib.trace_enable(False)
        _lib.chain_path(prev)
        per = {}
        for n, ms in recs:
            per.setdefault(n, []).append(ms)
        out[f"path{path}"] = {"ms_per_step": round(start.elapsed_time(end) / args.steps, 4),
                              "kernels_ms": {k: round(sum(v) / len(v), 4) for k, v in per.items()}}
    out["handoff_ok"] = ch.handoff_ok()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
