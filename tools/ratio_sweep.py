#!/usr/bin/env python3
"""bench.py's ratio_sweep alone (every app L/M at 4096 channels, single-pass
vs two-launch): one JSON object on stdout.
    python tools/ratio_sweep.py [channels] [L/M[:K] ...]   (DSPCORE_LIB picks a build;
    naming ratios times those only, without the two-launch chain)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cases = None
    if len(sys.argv) > 2:
        cases = []
        for a in sys.argv[2:]:
            lm, _, k = a.partition(":")
            L, M = (int(v) for v in lm.split("/"))
            cases.append((L, M, int(k) if k else None))
    print(json.dumps(bench.ratio_sweep(dev, channels=ch, cases=cases,
                                       two_launch=cases is None)), flush=True)
