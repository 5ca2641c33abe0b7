"""Batched SRC -> EQ -> spectrum chain: the hot path of app.py:164-167 and
app.py:203-205 for B channels at once, planned once and replayed.

A Chain owns every device buffer (taps, LUTs, y, z, mag, workspace) so that
`run()` is only kernel launches: graph-capturable, no allocation, no sync.

Where the library has a single-pass kernel for the geometry
(dsp_chain_tile_len > 0, include/dspcore.h) one launch computes y and z from x
and a second the spectrum; otherwise the SRC kernel writes y, the single-pass
cascade alone (the one-tap kernel) reads it once and writes z, and the
spectrum follows -- or, with dsp_chain_path(1), an explicit two-launch
variant, or more than six bands, the library's two-launch chain.

The single-pass kernel hands each tile's carry to the next tile through the
workspace; if a wait ever gives up (dsp_chain_status), run() raises
HandoffError after re-zeroing the workspace, so corrupted z never reaches a
caller that checks (the default outside graph capture).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, ops
from .design import (EqPlan, SpectrumPlan, SrcPlan, caller_taps, chunk_len_for, eq_plan,
                     max_chunks_for, spectrum_plan, src_plan, xstate_chunk_len)



# Output row pitch granule in floats (32 = 128 B; DSPCORE_ROW_ALIGN overrides
# it for A/B timing, any multiple of 4).
ROW_ALIGN = int(os.environ.get("DSPCORE_ROW_ALIGN", "32"))

class HandoffError(RuntimeError):
    """A single-pass tile hand-off wait gave up: that call's z is wrong
    (include/dspcore.h, dsp_chain_status).  The workspace has been reset."""


@dataclass(frozen=True)
class ChainConfig:
    n_in: int
    fs: int
    L: int
    M: int
    num_taps: int | None
    gains: dict
    n_fft: int = 2048
    limit_pts: int | None = None     # app.py:202 spectra use sig[:100000]


class Chain:
    """Device-resident plan of the chain for a fixed batch size."""

    def __init__(self, cfg: ChainConfig, batch: int, device: torch.device | str = "cuda",
                 chunk_len: int | None = None, use_table: bool = True,
                 use_xstate: bool = True, plan_batch: int | None = None,
                 keep_y: bool = True, spectra: tuple = ("z",)):
        """plan_batch: the batch size the cascade's chunking is planned for
        (default: `batch`).  Shards of one job pass the job's total batch so
        that every shard runs the same chunking and the rows come out bitwise
        equal to the unsharded run (design.max_chunks_for).
        keep_y=False: run() returns (None, z, mag) and, where the single-pass
        kernel serves the geometry, y is never written (dsp_chain_f32 with
        y = NULL); otherwise y lives in an internal buffer.
        spectra: which magnitude spectra a run() computes, of "x", "y", "z" (z
        always: dsp_chain_f32 produces it).  ("x", "y", "z") is app.py:203-205's
        rerun -- the input's spectrum at fs, the SRC output's and the EQ
        output's at fs' -- each with calcular_espectro_magnitud's segment rule
        on the first limit_pts samples; they land in self.mags[which] and
        self.frequencies(which) gives the rfftfreq axis."""
        ops.require_gpu()
        self.cfg = cfg
        self.B = int(batch)
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.identity_src = cfg.L == 1 and cfg.M == 1
        # SRC bypass (dsp_core.py:144-145): y is x itself.  To the library it
        # is the one-tap SRC y = 1.0 x (K = 1), whose single-pass kernel is
        # the cascade alone: x read once, z written once (include/dspcore.h).
        self.src: SrcPlan = (SrcPlan(1, 1, 1, np.ones(1), 0, cfg.n_in, cfg.n_in, cfg.fs)
                             if self.identity_src else
                             src_plan(cfg.n_in, cfg.fs, cfg.M, cfg.L, cfg.num_taps))
        n_out = cfg.n_in if self.identity_src else self.src.n_out
        self.n_out = n_out
        self.fs_out = cfg.fs if self.identity_src else self.src.fs_out
        self.eq: EqPlan = eq_plan(self.fs_out, cfg.gains)
        spec_len = n_out if cfg.limit_pts is None else min(n_out, cfg.limit_pts)
        self.spec: SpectrumPlan = spectrum_plan(spec_len, cfg.n_fft)
        S = self.eq.sos.shape[0]
        lib = _lib.load()
        self.tile_len = 0 if (self.identity_src and self.eq.bypass) else int(lib.dsp_chain_tile_len(
            cfg.n_in, n_out, self.src.K, self.src.L, self.src.M, self.src.c_offset, S, self.B))
        # Two-launch path (other geometries, or dsp_chain_path(1)): x-domain chunk states (include/dspcore.h, dsp_chain_f32) need a chunk
        # length with chunk_len*M/L a multiple of 4; take it unless it would cut
        # the row into far fewer chunks than the plain rule.
        mc = max_chunks_for(self.B if plan_batch is None else int(plan_batch))
        # a shard of a job runs the single-pass mode the job's batch takes
        # (ops.forced_chain_path; the modes agree to float64 rounding only)
        self._force = ops.forced_chain_path(
            None if plan_batch is None or int(plan_batch) == self.B else int(plan_batch),
            cfg.n_in, n_out, self.src.K, self.src.L, self.src.M, self.src.c_offset, S, self.B)
        plain = chunk_len_for(n_out, mc)
        eligible = (use_xstate and use_table and not self.identity_src and not self.eq.bypass
                    and 1 <= S <= 8 and S != 7)
        if chunk_len is not None:
            T = int(chunk_len)
            self.xstate = eligible and T % 32 == 0 and (T * cfg.M) % (4 * cfg.L) == 0
        else:
            xs_len = xstate_chunk_len(n_out, cfg.L, cfg.M, mc)
            self.xstate = eligible and xs_len <= 2 * plain
            T = xs_len if self.xstate else plain
        self.chunk_len = T
        dev = self.device
        self.taps = ops.taps_tensor(self.src, dev)
        self.window = ops._table("hann", self.spec.n_fft, dev)
        self.tw = ops._table("tw", self.spec.n_fft, dev)
        self.sos = np.ascontiguousarray(self.eq.sos, dtype=np.float64)
        # Rows on 128-byte boundaries (pitch a multiple of ROW_ALIGN floats): the
        # single-pass kernel's float4 stores apply to every n_out and its 1-KB
        # store bursts cover whole cache lines; y and z are [B, n_out] views of
        # the padded buffers.
        ld = -(-n_out // ROW_ALIGN) * ROW_ALIGN
        self._ld = ld
        self.keep_y = bool(keep_y)
        self._zbuf = torch.empty((self.B, ld), dtype=torch.float32, device=dev)
        self.z = self._zbuf[:, :n_out]
        self.mag = torch.empty((self.B, self.spec.n_fft // 2 + 1), dtype=torch.float32,
                               device=dev)
        ws_bytes = lib.dsp_chain_workspace_bytes(self.B, cfg.n_in, n_out, self.src.K, self.src.L,
                                                 self.src.M, self.src.c_offset, S, self.chunk_len)
        # Zero-filled once: the single-pass kernel's hand-off flags start clear
        # and every completed call leaves them clear (include/dspcore.h).
        self.workspace = torch.zeros(max(int(ws_bytes), 256), dtype=torch.uint8, device=dev)
        self.table = ops.state_table(self.sos, self.chunk_len, dev) if use_table else None
        # Single-pass kernel tables (dsp_chain_tile_tables): built once on the
        # host in float64 from the float32 taps and the sos, kept on the device.
        self.tile_tables = None
        self.tile_key = 0
        if self.tile_len > 0:
            nbytes = int(lib.dsp_chain_tile_tables_bytes())
            host = np.zeros(nbytes, dtype=np.uint8)
            taps32 = caller_taps(self.src)
            key = ctypes.c_uint64(0)
            rc = lib.dsp_chain_tile_tables(
                host.ctypes.data, nbytes, cfg.n_in, n_out, taps32.ctypes.data, self.src.K,
                self.src.L, self.src.M, self.src.c_offset, _lib.sos_pointer(self.sos), S,
                ctypes.byref(key))
            if rc < 0:
                _lib.check(rc, "dsp_chain_tile_tables")
            if rc == 0:
                # 256-byte aligned device copy (torch's allocator aligns to 512 B)
                self.tile_tables = torch.from_numpy(host).to(dev)
                self.tile_key = int(key.value)
            else:
                self.tile_len = 0
        # Geometries without a single-pass SRC kernel (e.g. 48 -> 44.1 kHz,
        # L/M = 147/160 at K = 1023): the SRC kernel writes y and the
        # single-pass cascade alone (the one-tap kernel, ops.eq_single_pass)
        # reads it once, instead of the library's two-launch chain (x-domain
        # chunk states, then the cascade's pass 2 over y): 147/160 at 8192
        # channels 1.949 -> 1.659 ms (tools/two_launch_ident.py).
        # dsp_chain_path(1), and a caller that picks a two-launch variant
        # (chunk_len, use_table=False, use_xstate=False), still select the
        # library's two-launch chain.
        self._plan_batch = None if plan_batch is None else int(plan_batch)
        self._split_ws = None
        if (self.tile_len == 0 and not self.identity_src and not self.eq.bypass
                and chunk_len is None and use_table and use_xstate
                and ops._eq_tile_plan(n_out, self.sos, dev) is not None):
            nb = lib.dsp_chain_workspace_bytes(self.B, n_out, n_out, 1, 1, 1, 0, S,
                                               chunk_len_for(n_out, max_chunks_for(self.B)))
            self._split_ws = torch.zeros(max(int(nb), 256), dtype=torch.uint8, device=dev)
        # y: the caller's output, or the two-launch chain's intermediate; with
        # keep_y=False on the single-pass path it is never allocated, and with
        # the SRC bypass it is x.
        if not self.identity_src and (self.keep_y or self.tile_len == 0):
            self._ybuf = torch.empty((self.B, self._ld), dtype=torch.float32, device=dev)
            self.y = self._ybuf[:, :n_out]
        else:
            self._ybuf = self.y = None
        self.xtable, self.xrows = (ops.xstate_table(self.sos, self.src, self.chunk_len, dev)
                                   if self.xstate else (None, 0))
        # Spectra of x and y beside z's (app.py:203-205).
        which = tuple(spectra)
        if "z" not in which or not set(which) <= {"x", "y", "z"}:
            raise ValueError(f"spectra must name 'z' and any of 'x', 'y' (got {which})")
        if "y" in which and not self.keep_y:
            raise ValueError("the y spectrum needs keep_y=True")
        self.spec_plans = {"z": self.spec}
        self.mags = {"z": self.mag}
        for w in ("x", "y"):
            if w in which:
                n = cfg.n_in if w == "x" else n_out
                plan = spectrum_plan(n if cfg.limit_pts is None else min(n, cfg.limit_pts),
                                     cfg.n_fft)
                self.spec_plans[w] = plan
                self.mags[w] = torch.empty((self.B, plan.n_fft // 2 + 1), dtype=torch.float32,
                                           device=dev)

    def frequencies(self, which: str = "z") -> np.ndarray:
        """rfftfreq axis of spectrum `which` (dsp_core.py:94-98): x at fs, y and
        z at fs'."""
        n = self.spec_plans[which].n_fft
        fs = self.cfg.fs if which == "x" else self.fs_out
        return np.fft.rfftfreq(n, 1.0 / fs)[: n // 2 + 1]

    def _extra_spectra(self, x: torch.Tensor, y: torch.Tensor | None) -> None:
        for w, src in (("x", x), ("y", y)):
            if w in self.mags:
                p = self.spec_plans[w]
                ops.spectrum(src, p.seg_start, p.seg_len, p.n_fft, out=self.mags[w])

    # -- algorithmic traffic ---------------------------------
    def algorithmic_bytes(self) -> int:
        """4*N_in + 4*N_out (y) + 4*N_out (z) + 4*(N/2+1) per channel (no y
        with the SRC bypass: y is x)."""
        per = (4 * self.cfg.n_in + (4 if self.identity_src else 8) * self.n_out
               + 4 * (self.spec.n_fft // 2 + 1))
        return per * self.B

    def _status(self, reset: bool) -> int:
        lib = _lib.load()
        total = 0
        for ws in (self.workspace, self._split_ws):
            if ws is None:
                continue
            with torch.cuda.device(self.device):
                rc = lib.dsp_chain_status(ws.data_ptr(), ws.numel(), int(bool(reset)),
                                          torch.cuda.current_stream(self.device).cuda_stream)
            if rc < 0:
                _lib.check(rc, "dsp_chain_status")
            total += rc
        return total

    def handoff_ok(self) -> bool:
        """False if a single-pass call's tile hand-off wait gave up since the
        last reset (dsp_chain_status; synchronises the stream)."""
        return self._status(False) == 0

    def check(self) -> None:
        """Raises HandoffError (after re-zeroing the workspace, so the next
        call starts clean) if a tile hand-off wait gave up since the last
        check; synchronises the stream."""
        if self._status(False):
            self._status(True)
            raise HandoffError("single-pass chain: a tile hand-off wait gave up; z of the "
                               "last call(s) is wrong (workspace reset; rerun the call)")

    def check_input(self, x: torch.Tensor) -> torch.Tensor:
        if x.shape != (self.B, self.cfg.n_in) or x.dtype != torch.float32 or not x.is_cuda:
            raise ValueError(f"expected float32 CUDA [{self.B}, {self.cfg.n_in}], got "
                             f"{x.dtype} {tuple(x.shape)}")
        if x.stride(1) != 1 or (self.B > 1 and x.stride(0) < x.shape[1]):
            x = x.contiguous()
        return x

    def run(self, x: torch.Tensor, check: bool | None = None):
        """One fused-call pass: y = SRC(x), z = EQ(y), mag = |FFT(hann*z[seg])|.

        check: read the hand-off status after the launches and raise
        HandoffError if a wait gave up (synchronises the stream).  None (the
        default) checks unless the stream is being captured into a graph;
        callers that replay graphs or pipeline many calls pass False and call
        check() themselves."""
        x = self.check_input(x)
        if self.identity_src and (self.tile_len == 0 or (self.B > 1 and ops.ld(x) % 4)
                                  or x.data_ptr() % 16 or _lib.chain_path() == 1):
            # SRC bypass (dsp_core.py:144-145) without the single-pass kernel
            # (the EQ bypassed too, dsp_chain_tile_len 0, rows of x not
            # 16-byte aligned, or dsp_chain_path(1)): y is x itself, the
            # cascade runs alone.
            _, z, _ = self.run_stages(x)
            if z is not self.z:
                self.z.copy_(z)         # the EQ bypassed too: z is x (run_stages)
            return (x if self.keep_y else None), self.z, self.mag
        if self._split_ws is not None and _lib.chain_path() != 1:
            # SRC kernel, then the single-pass cascade alone on y (__init__)
            with torch.cuda.device(self.device):
                ops.src_polyphase(x, self.src, self.taps, out=self.y)
                if ops.eq_single_pass(self.y, self.sos, out=self.z, plan_batch=self._plan_batch,
                                      workspace=self._split_ws) is None:
                    raise RuntimeError("single-pass cascade declined the chain's own y / z")
                ops.spectrum(self.z, self.spec.seg_start, self.spec.seg_len, self.spec.n_fft,
                             out=self.mag)
                self._extra_spectra(x, self.y)
            if check is None:
                check = not torch.cuda.is_current_stream_capturing()
            if check:
                self.check()
            return (self.y if self.keep_y else None), self.z, self.mag
        lib = _lib.load()
        sos_ptr = _lib.sos_pointer(self.sos)
        S = self.sos.shape[0]
        clip = 0 if self.eq.bypass else 1
        y_ptr = self.y.data_ptr() if self.y is not None else None
        with torch.cuda.device(self.device), self._force:
            stream = torch.cuda.current_stream(self.device)
            rc = lib.dsp_chain_f32(
                x.data_ptr(), y_ptr, self.z.data_ptr(), self.mag.data_ptr(),
                self.B, self.cfg.n_in, ops.ld(x), self.n_out, ops.ld(self.z),
                self.taps.data_ptr(), self.src.K, self.src.L, self.src.M, self.src.c_offset,
                sos_ptr, S, clip, self.chunk_len, ops._ptr(self.table), ops._ptr(self.xtable),
                self.xrows, ops._ptr(self.tile_tables), self.tile_key, self.spec.seg_start,
                self.spec.seg_len, self.spec.n_fft.bit_length() - 1, ops.ld(self.mag),
                self.window.data_ptr(), self.tw.data_ptr(), self.workspace.data_ptr(),
                self.workspace.numel(), stream.cuda_stream)
            _lib.check(rc, "dsp_chain_f32")
            self._extra_spectra(x, x if self.identity_src else self.y)
            if check is None:
                check = self.tile_len > 0 and not torch.cuda.is_current_stream_capturing()
            if check:
                self.check()
        y = x if self.identity_src else self.y
        return (y if self.keep_y else None), self.z, self.mag

    def run_stages(self, x: torch.Tensor, events: list | None = None):
        """Same pass, one entry point per stage; optional (start, end) event pairs
        around each stage for per-kernel timing on the current stream.  y is
        bitwise that of run(); z may differ from run()'s by rounding when run()
        takes its chunk states from x (both within the EQ tolerance)."""
        x = self.check_input(x)

        def mark(i, which):
            if events is not None:
                events[i][which].record()

        mark(0, 0)
        if self.identity_src:
            y = x
        else:
            y = ops.src_polyphase(x, self.src, self.taps, out=self.y)
        mark(0, 1)
        mark(1, 0)
        if self.eq.bypass:
            z = y                       # dsp_core.py:222-223 returns its input
        else:
            z = ops.biquad_cascade(y, self.sos, True, out=self.z, workspace=self.workspace,
                                   chunk_len=self.chunk_len, use_table=self.table is not None)
        mark(1, 1)
        mark(2, 0)
        ops.spectrum(z, self.spec.seg_start, self.spec.seg_len, self.spec.n_fft, out=self.mag)
        self._extra_spectra(x, y)
        mark(2, 1)
        return y, z, self.mag
