"""Host-resident batches through the chain: numpy in, numpy out, PCIe overlapped.

The drop-in's callers hold their audio in host memory (app.py:164-167 and
203-205 hand numpy arrays to dsp_core).  A single `Chain.run` on a pageable
numpy batch moves it in three serial steps -- a staged H2D copy, the chain, a
staged D2H copy of y, z and |Z| -- and the PCIe transfers dominate: 768 KB of
traffic per config-4 channel against ~6 us of GPU work per 32 channels.

`HostChain` cuts the batch into channel blocks and runs them through a small
ring of slots, each with its own `Chain` (device buffers, hand-off workspace),
pinned input staging buffer and HIP stream:

    host copy of block i+1 into pinned staging       (CPU)
    H2D of block i+1                                  (copy engine, stream s+1)
    chain of block i                                  (CUs, stream s)
    D2H of y, z, |Z| of block i-1 into pinned output  (other copy engine)

so the host copy, both PCIe directions and the kernels overlap.  The outputs
are numpy views of pinned host buffers the object owns and reuses: the next
`run` overwrites them (pass `copy=True` to keep a call's results).

Each block is a full `Chain` call of `block` channels (a short last block is
zero-padded); the rows equal `Chain(cfg, block).run` bitwise, and on the
single-pass geometries (configs 3, 4, 5) those equal any batch's rows
(dspcore/shard.py: the kernel's arithmetic depends on (L, M, K) only).  The
hand-off status of every slot is checked once at the end of `run` (HandoffError
as in Chain.run).
"""
from __future__ import annotations

import numpy as np
import torch

from concurrent.futures import ThreadPoolExecutor

from .chain import Chain, ChainConfig


class HostChain:
    """Pipelined numpy -> device -> numpy runner of one ChainConfig."""

    def __init__(self, cfg: ChainConfig, device: torch.device | str = "cuda", block: int = 64,
                 slots: int = 4, keep_y: bool = True, copy_threads: int = 4):
        if block < 1 or slots < 1:
            raise ValueError("block and slots must be >= 1")
        self.cfg = cfg
        self.block = int(block)
        self.keep_y = bool(keep_y)
        self.chains = [Chain(cfg, self.block, device, keep_y=keep_y) for _ in range(slots)]
        self.device = self.chains[0].device
        self.n_out = self.chains[0].n_out
        self.n_mag = self.chains[0].mag.shape[1]
        n_in = cfg.n_in
        self.streams = [torch.cuda.Stream(self.device) for _ in range(slots)]
        # The chains' workspace zero-fill and table uploads were queued on the
        # current stream; the slot streams (non-blocking) wait for them.
        setup = torch.cuda.current_stream(self.device)
        for st in self.streams:
            st.wait_stream(setup)
        self.xpin = [torch.zeros((self.block, n_in), dtype=torch.float32, pin_memory=True)
                     for _ in range(slots)]
        self.xdev = [torch.empty((self.block, n_in), dtype=torch.float32, device=self.device)
                     for _ in range(slots)]
        self.done: list = [None] * slots
        # numpy releases the GIL in its copy loops: the copy into pinned staging
        # runs on a few threads, row slices each
        self._pool = ThreadPoolExecutor(copy_threads) if copy_threads > 1 else None
        self._nthreads = max(1, int(copy_threads))
        self._out_B = -1
        self._out: tuple = ()

    def _outputs(self, B: int):
        if B != self._out_B:
            pin = dict(dtype=torch.float32, pin_memory=True)
            y = torch.empty((B, self.n_out), **pin) if self.keep_y else None
            self._out = (y, torch.empty((B, self.n_out), **pin), torch.empty((B, self.n_mag), **pin))
            self._out_B = B
        return self._out

    def close(self) -> None:
        """Stops the staging-copy threads (the device buffers go with the object)."""
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        pool = getattr(self, "_pool", None)
        if pool is not None:
            pool.shutdown(wait=False)

    def _fill(self, xp: np.ndarray, x: np.ndarray, lo: int, nb: int) -> None:
        if self._pool is None or nb < 2 * self._nthreads:
            np.copyto(xp[:nb], x[lo:lo + nb])
            return
        step = -(-nb // self._nthreads)
        futs = [self._pool.submit(np.copyto, xp[r:min(nb, r + step)], x[lo + r:lo + min(nb, r + step)])
                for r in range(0, nb, step)]
        for f in futs:
            f.result()

    def run(self, x: np.ndarray, copy: bool = False):
        """y, z, |Z| (numpy float32, [B, n_out], [B, n_out], [B, n_fft/2+1]) of a
        [B, n_in] float32 batch; y is None with keep_y=False."""
        x = np.asarray(x)
        if x.ndim != 2 or x.shape[1] != self.cfg.n_in:
            raise ValueError(f"expected [B, {self.cfg.n_in}] samples, got {x.shape}")
        if x.dtype != np.float32:
            x = x.astype(np.float32)
        B = x.shape[0]
        oy, oz, om = self._outputs(B)
        ns = len(self.chains)
        for i, lo in enumerate(range(0, B, self.block)):
            hi = min(B, lo + self.block)
            nb = hi - lo
            s = i % ns
            if self.done[s] is not None:
                self.done[s].synchronize()  # the slot's previous block has left the device
            xp = self.xpin[s].numpy()
            self._fill(xp, x, lo, nb)
            if nb < self.block:
                xp[nb:] = 0.0
            st = self.streams[s]
            with torch.cuda.stream(st):
                self.xdev[s].copy_(self.xpin[s], non_blocking=True)
                y, z, mag = self.chains[s].run(self.xdev[s], check=False)
                if oy is not None:
                    oy[lo:hi].copy_(y[:nb], non_blocking=True)
                oz[lo:hi].copy_(z[:nb], non_blocking=True)
                om[lo:hi].copy_(mag[:nb], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                self.done[s] = ev
        for st in self.streams:
            st.synchronize()
        for c in self.chains:
            c.check()
        outs = tuple(None if t is None else t.numpy() for t in (oy, oz, om))
        if copy:
            outs = tuple(None if a is None else a.copy() for a in outs)
        return outs
