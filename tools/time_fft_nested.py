"""Times the four-step FFT paths on the device with HIP events; prints one
line per size: ms per transform and the rate of its algorithmic traffic
(read + write of N complex64 per pass: 2 passes for the two-step split, 3 for
the three-pass one from 2^NEST, default 23; DSPCORE_LIB picks a build).
    python tools/time_fft_nested.py [reps] [nest_from] [log2 sizes ...]
FFT_ROWS_LOG2=k: 2^k / N rows per call (batched transforms) instead of one."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dsp-audio-project_amd"))
from dspcore import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    nest = int(sys.argv[2]) if len(sys.argv) > 2 else 23
    sizes = [int(v) for v in sys.argv[3:]] or [22, 24, 26, 28, 29, 30]
    dev = torch.device("cuda:0")
    for lg in sizes:
        n = 1 << lg
        rows = max(1, (1 << int(os.environ.get("FFT_ROWS_LOG2", "0"))) // n)
        x = torch.randn(rows, n, dtype=torch.complex64, device=dev)
        out = torch.empty_like(x)
        ops.fft(x, out)  # tables, workspace
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.fft(x, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        passes = 1 if lg <= 14 else (3 if lg >= nest else 2)  # one LDS-resident launch to 2^14
        gbs = passes * 2 * n * rows * 8 / (ms * 1e-3) / 1e9
        print(f"2^{lg} x {rows}: {ms:.3f} ms per call, {passes} passes, {gbs:.0f} GB/s of "
              f"read+write traffic", flush=True)
        del x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
