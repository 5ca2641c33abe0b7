"""Multi-GPU shard driver for the channel batch.

Channels never interact, so a batch is cut into contiguous channel ranges of
ceil(B/g) rows, one per device; each device gets its own copy of the LUTs and
runs the same kernels on its own stream from its own host thread (ctypes drops
the GIL while the ABI runs).  No collective, no device-to-device traffic: the
per-device results are gathered on the host.

Bitwise invariance: no kernel's arithmetic depends on the batch size, only on
the plan.  The single-pass chain kernel's geometry depends on (L, M, K) only;
the two-launch cascade's chunk length depends on the batch the chain is
planned for (design.max_chunks_for: <= 64 chunks from 2048 channels, <= 256
below), so shards must plan with the job's total batch
(`Chain(..., plan_batch=B_total)`, as bench.py does) to be bitwise equal to the
unsharded run; planned per shard they agree to float64 rounding only.
"""
from __future__ import annotations

import threading

import numpy as np
import torch


def shard_ranges(B: int, parts: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) ranges of ceil(B/parts) rows (the last may be short;
    trailing empty ranges are dropped)."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    step = -(-B // parts) if B else 0
    out = []
    for p in range(parts):
        lo, hi = p * step, min(B, (p + 1) * step)
        if lo < hi:
            out.append((lo, hi))
    return out


def run_sharded(fn, x: np.ndarray, devices: list | None = None) -> list:
    """Applies fn(x_dev) -> tuple of CUDA tensors to each shard of x's rows on its
    own device and returns the tuple of host arrays concatenated along rows.

    fn runs inside `torch.cuda.device(dev)` on that device's current stream."""
    if devices is None:
        devices = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    ranges = shard_ranges(x.shape[0], len(devices))
    results: list = [None] * len(ranges)
    errors: list = []

    def worker(i, dev, lo, hi):
        try:
            with torch.cuda.device(dev):
                xd = torch.from_numpy(np.ascontiguousarray(x[lo:hi], dtype=np.float32)).to(dev)
                outs = fn(xd)
                results[i] = tuple(o.cpu().numpy() for o in outs)
        except BaseException as e:  # re-raised on the caller's thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i, devices[i], lo, hi))
               for i, (lo, hi) in enumerate(ranges)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return [np.concatenate([r[k] for r in results], axis=0) for k in range(len(results[0]))]


def run_sharded_host(cfg, x: np.ndarray, devices: list | None = None, block: int = 64,
                     slots: int = 4) -> tuple:
    """y, z, |Z| of a host-resident [B, n_in] batch over several devices: one
    dspcore.host.HostChain per device on its contiguous channel range, each
    driven from its own host thread (pinned staging, overlapped copies), the
    rows gathered into fresh numpy arrays.  Rows are bitwise those of one
    HostChain on the whole batch (the chain is planned per block, the same
    on every device)."""
    from .host import HostChain
    if devices is None:
        devices = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    x = np.asarray(x, dtype=np.float32)
    ranges = shard_ranges(x.shape[0], len(devices))
    runners = [HostChain(cfg, devices[i], block=block, slots=slots) for i in range(len(ranges))]
    n_out, n_mag = runners[0].n_out, runners[0].n_mag
    B = x.shape[0]
    y = np.empty((B, n_out), np.float32)
    z = np.empty((B, n_out), np.float32)
    mag = np.empty((B, n_mag), np.float32)
    errors: list = []

    def worker(i, lo, hi):
        try:
            with torch.cuda.device(runners[i].device):
                oy, oz, om = runners[i].run(x[lo:hi])
            y[lo:hi], z[lo:hi], mag[lo:hi] = oy, oz, om
        except BaseException as e:  # re-raised on the caller's thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i, lo, hi))
               for i, (lo, hi) in enumerate(ranges)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for r in runners:
        r.close()
    if errors:
        raise errors[0]
    return y, z, mag
