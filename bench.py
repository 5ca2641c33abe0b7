#!/usr/bin/env python3
"""Benchmark of the SRC -> 6-biquad EQ -> FFT chain on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

`--gpus N` without a launcher (WORLD_SIZE unset) starts the N ranks itself: N
fresh child processes with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, created
before this process touches any GPU; the parent only relays rank 0's line.

Workload (default, BASELINE.json configs[3] = SURVEY.md §8(d) config 4):
32768 channels x 48000 samples at 48 kHz, SRC L=3/M=2 with the default 121-tap
sinc x Blackman FIR, the 6-band EQ with gains {+6, -4, +3, -3, +5, -6} dB at
fs' = 72 kHz, and a 4096-point Hann-windowed FFT magnitude of the centre
segment of z; the 32768 channels are sharded over the N ranks (32768/N each,
strong scaling), so every N runs the same job.  `--config c3` is configs[2]
(4096 channels), `--config c5` configs[4] (8192 channels, 44.1 -> 48 kHz,
L/M = 160/147, K = 1023), both sharded the same way.  At N = 1 the default
run also times config 3 (4096 channels, one GPU) and reports it under
"config3".

Input is synthetic uniform(-1, 1) float32 generated on the device (the
reference's example WAVs are missing), resident in HBM before the timed
region.  One step = one pass of the chain over the rank's channels.  Channels
shard with no collective: the only cross-rank calls are the timing barrier and
the max-over-ranks of the elapsed time, over gloo (CPU; RCCL is never
initialised).

Rank 0 prints one JSON line.  Besides the contract fields it carries
`roofline` (dominant kernel: algorithmic bytes per launch / its mean duration
from HIP events the library records around every launch on the launching
stream, against the 8 TB/s spec and against a float4 copy measured in the same
process, and the PMC-measured HBM bytes of that kernel when profiles hold them
for this workload), `chain_roofline` (whole-chain algorithmic bytes /
ms_per_step) and, at N = 1: `cpu_baseline` (the repo's CPU oracle -- same
numpy/scipy calls as the reference's dsp_core.py -- on a bounded channel
sample with one process per usable host core, measured BEFORE the GPU is
initialised), `config3` and `config5` (the other two batched configs on one
GPU), `host_inclusive` (numpy in, H2D, chain, D2H of y/z/|X|, numpy out) and
`copy_ceiling` and `mix_ceiling` (the HBM rate of streaming kernels with the
chain kernel's 1 read : 2 writes mix, tools/ubench_rw_mix in a child
process; roofline.frac_vs_mix_ceiling), `fft_2_28` (the three-pass FFT of
one 2^28-point row: ms and its algorithmic rate; not part of the metric),
`app_rerun` (one channel through the drop-in as app.py calls it, next to the
oracle), `eq_alone` (the sliders' default L = M = 1: the single-pass cascade
alone at 32768 x 48000 and on one 441000-sample channel, against the two-pass
cascade) and `ratio_sweep` (every L/M in 1..8 at 4096 channels: path taken
and Msamples/s against the two-launch chain).  DSP_BENCH_DRYRUN=1 replaces the GPU measurement by a stub
(tests of the rank launcher and sharding on CPU).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "dsp-audio-project_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Msamples/sec SRC→6-biquad EQ→FFT chain at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6    # MI355X fp64 vector peak (FMA = 2 flops)
CONFIG3_GAINS = {"Sub-Bass": 6, "Bass": -4, "Low Mids": 3,
                 "High Mids": -3, "Presence": 5, "Brilliance": -6}

WORKLOADS = {
    "c3": dict(name="config3", n_in=48000, fs=48000, L=3, M=2, num_taps=None, n_fft=4096,
               channels=4096, cpu_per_proc=64,
               desc="config 3: 4096 ch x 48000 @48kHz: SRC L3/M2 K121 -> 6-biquad EQ @72kHz -> "
                    "4096-pt FFT |X| of centre segment"),
    "c4": dict(name="config4", n_in=48000, fs=48000, L=3, M=2, num_taps=None, n_fft=4096,
               channels=32768, cpu_per_proc=64,
               desc="config 4: 32768 ch x 48000 @48kHz sharded over the GPUs: SRC L3/M2 K121 -> "
                    "6-biquad EQ @72kHz -> 4096-pt FFT |X| of centre segment"),
    "c5": dict(name="config5", n_in=48000, fs=44100, L=160, M=147, num_taps=1023, n_fft=4096,
               channels=8192, cpu_per_proc=2,
               desc="config 5: 8192 ch x 48000 @44.1kHz sharded over the GPUs: SRC L160/M147 "
                    "K1023 -> 6-biquad EQ @48kHz -> 4096-pt FFT |X|"),
}


# --------------------------------------------------------------------------- harness
def dist_env():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` with no launcher: starts N fresh `python bench.py` children,
    rank r on LOCAL_RANK r, rendezvous on 127.0.0.1.  This process never
    touches a GPU (no exec from a GPU-initialised process); rank 0 writes the
    JSON line to the shared stdout.  A failing rank ends the others."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


def rank_channels(total: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) of the rank's contiguous channel shard (dspcore.shard)."""
    from dspcore.shard import shard_ranges
    ranges = shard_ranges(total, world)
    return ranges[rank] if rank < len(ranges) else (total, total)


PREHEAT_S = 0.3   # untimed steps before the warmup: GPU clocks settle


def timed_loop(step, steps, warmup, sync, dist=None, preheat_s=PREHEAT_S, same_node=True,
               stats=None):
    """Untimed steps for PREHEAT_S seconds (the MI355X boosts, then throttles,
    then settles over the first ~20-40 ms of a busy GPU: a 1 ms config-3 step
    measured 0.86 -> 1.19 -> 0.89 ms over its first 20 launches), then W untimed
    warmup steps, then K steps bracketed by barrier + sync on both sides.
    Returns the elapsed seconds; with `dist` initialised (a gloo group) the
    job's time over all ranks.  When every rank runs on this node
    (`same_node`, from the gathered host names) that is max(end) - min(start)
    on the host's monotonic clock (perf_counter is CLOCK_MONOTONIC, one clock
    for every process of the node): each rank stamps its start as it leaves
    the start barrier and its end at its own final sync, so skew in leaving the
    barrier counts, and the end barrier's gloo round trips (a sizeable share
    of a ~17 ms N = 8 timed region) do not.  Across nodes the clocks are not
    comparable, and it is the max over ranks of each rank's own elapsed time.
    `stats` (a dict) receives this rank's own elapsed seconds as "local"."""
    t_pre = time.perf_counter()
    while preheat_s > 0:
        step()
        sync()
        if time.perf_counter() - t_pre >= preheat_s:
            break
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    if stats is not None:
        stats["local"] = elapsed
    if dist is not None:
        dist.barrier()
        import torch
        if same_node:
            t_end = torch.tensor([t0 + elapsed], dtype=torch.float64)
            t_start = torch.tensor([t0], dtype=torch.float64)
            dist.all_reduce(t_end, op=dist.ReduceOp.MAX)
            dist.all_reduce(t_start, op=dist.ReduceOp.MIN)
            elapsed = float(t_end.item() - t_start.item())
        else:
            t = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
    return elapsed


# --------------------------------------------------------------------------- CPU baseline
def usable_cores() -> tuple[int, str]:
    """Cores this process may run on: the affinity mask, capped by a cgroup
    CPU quota when one is set (a container's share of a larger host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"affinity {n}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            how += f", cgroup quota {q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, how


def cpu_baseline(wl, procs, per_proc):
    """Times the CPU oracle chain on procs * per_proc channels, one fork-pool
    process per usable core."""
    import multiprocessing as mp

    import numpy as np

    from oracle import dsp_ref_cpu as orc
    sample = procs * per_proc
    rng = np.random.default_rng(1)
    xs = rng.uniform(-1, 1, (sample, wl["n_in"])).astype(np.float32)
    chunks = [xs[i::procs] for i in range(procs)]
    args = [(list(c), wl["fs"], wl["L"], wl["M"], CONFIG3_GAINS, wl["num_taps"], wl["n_fft"])
            for c in chunks if len(c)]
    ctx = mp.get_context("fork")
    with ctx.Pool(len(args)) as pool:
        pool.map(orc.chain_batch_worker, [(a[0][:1],) + a[1:] for a in args])  # warm
        t0 = time.perf_counter()
        pool.map(orc.chain_batch_worker, args)
        wall = time.perf_counter() - t0
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(sample * wl["n_in"] / wall / 1e6, 4),
        "unit": "Msamples/s",
        "cores": len(args),
        "kind": "port",
        "sample": (f"{sample} channels of the {wl['name']} chain (oracle/dsp_ref_cpu.py: "
                   f"np.convolve SRC, scipy lfilter cascade, recursive radix-2 FFT), "
                   f"{len(args)}-process pool ({usable_cores()[1]}), {wall:.2f} s wall, "
                   f"CPU: {cpu_model}"),
    }


# --------------------------------------------------------------------------- per-kernel bytes
def kernel_bytes(chain, name):
    """Algorithmic HBM bytes of one launch of kernel `name`:
    what the kernel must read and write, intermediate re-reads excluded."""
    B, n_in, n_out = chain.B, chain.cfg.n_in, chain.n_out
    return {
        "chain_tile": 4 * B * n_in + 8 * B * n_out,    # x read, y and z written
        "src_poly": 4 * B * (n_in + n_out),
        "iir_xstate": 8 * B * n_out,
        "iir_fused": 8 * B * n_out,
        "iir_apply": 8 * B * n_out,
        "spectrum": 4 * B * (chain.spec.seg_len + chain.spec.n_fft // 2 + 1),
    }.get(name, 0)


def valu_work(chain, mean_ms):
    """float64 FMA work of the single-pass kernel: per output
    sample 24 (pass 2), plus per TS-sample sub-chunk the carry's 210 (the change
    of basis Q e, s = T m and the blocked scan: PMC SQ_INSTS_VALU_FMA_F64 per
    wave is 1362 at TS = 48 and 978 at TS = 32, profiles/r04_m3_*).  Pass 1 and
    the SRC are float32 (v_pk_fma_f32).  None for the two-launch chain."""
    ts = chain.tile_len
    if not ts:
        return None
    per_sample = 24 + 210 / ts
    fma = per_sample * chain.B * chain.n_out
    tflops = 2 * fma / (mean_ms * 1e-3) / 1e12
    return {"kind": "model",
            "model": "fp64 FMA per output sample = 24 (pass 2) + 210 / TS (carry), the static "
                     "counts that SQ_INSTS_VALU_FMA_F64 / SQ_WAVES measured (1362 per wave at "
                     "TS = 48, 978 at TS = 32, profiles/r04_m3_*); achieved = that work / this "
                     "run's HIP-event mean, not a counter of this run",
            "bound": "package power (1400 W cap): fp64 + packed fp32 VALU on top of the HBM stream",
            "fp64_fma_per_output_sample": round(per_sample, 3),
            "achieved": round(tflops, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / FP64_PEAK_TFLOPS, 4),
            "note": "beside the fp64 FMAs the kernel issues 19.7 (L3/M2: SRC 656 + pass 1 288 "
                    "per 48-sample lane sub-chunk) or 10 (generic) v_pk_fma_f32 per sample; it "
                    "runs at the 1400 W package power cap, VALU-issue-bound at the clock that "
                    "leaves (config 4: 89 % of the kernel's cycles issue VALU, PMC, "
                    "profiles/r04_m3_c4_pmc_summary.txt; a pure 1R:2W HBM stream at 5.1 TB/s "
                    "draws ~865 W), and moves ~0.8 of what such a stream reaches "
                    "(mix_ceiling_gbs), DESIGN.md §3.0.2, §3.0.5"}


def load_traffic(wl_name, channels):
    """PMC HBM bytes per launch for this workload and batch, from the summary
    tools/pmc_parse.py --write keeps in pmc_traffic.json (repo root: profiles/ is
    not sent to the GPU box)."""
    path = os.path.join(ROOT, "pmc_traffic.json")  # profiles/ does not travel to the GPU box
    try:
        with open(path) as f:
            ent = json.load(f).get(wl_name, {})
    except (OSError, ValueError):
        return {}, None
    if ent.get("channels") != channels:
        return {}, None
    return ent.get("per_launch", {}), ent.get("source")


def measure(wl, B, steps, warmup, rank, world, dist, eager, device, same_node=True):
    """Builds the chain for B channels of workload wl, times K steps (graph
    replay unless eager) and a traced pass; returns the numbers."""
    import torch

    from dspcore import _lib
    from dspcore.chain import Chain, ChainConfig

    cfg = ChainConfig(wl["n_in"], wl["fs"], wl["L"], wl["M"], wl["num_taps"], CONFIG3_GAINS,
                      n_fft=wl["n_fft"])
    chain = Chain(cfg, B, device, plan_batch=wl["channels"])
    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    x = torch.rand((B, wl["n_in"]), generator=gen, device=device, dtype=torch.float32)
    x.mul_(2).sub_(1)
    torch.cuda.synchronize(device)

    step = lambda: chain.run(x, check=False)  # noqa: E731
    launch = "eager"
    if not eager:
        # One chain step (no host sync, no allocation) captured into a HIP
        # graph and replayed: the timed loop measures the GPU, not Python/ctypes
        # launch overhead.
        try:
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(device)
            cap.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(cap):
                chain.run(x)                      # warm the LUT caches outside capture
                with torch.cuda.graph(graph, stream=cap):
                    chain.run(x, check=False)
            torch.cuda.current_stream(device).wait_stream(cap)
            step = graph.replay
            launch = "hipGraph"
        except Exception as exc:  # noqa: BLE001  (fall back to eager launches)
            print(f"graph capture failed ({exc}); timing eager launches", file=sys.stderr)
    sync = lambda: torch.cuda.synchronize(device)  # noqa: E731
    st = {}
    elapsed = timed_loop(step, steps, warmup, sync, dist, same_node=same_node, stats=st)
    chain.check()      # raises HandoffError if a tile hand-off wait gave up

    # Traced pass: HIP events around every launch, on the kernels' stream.
    _lib.trace_enable(True)
    _lib.trace_read()
    for _ in range(steps):
        chain.run(x, check=False)
    recs = _lib.trace_read()
    _lib.trace_enable(False)
    chain.check()
    per = {}
    for name, ms in recs:
        per.setdefault(name, []).append(ms)
    kernels = {k: round(sum(v) / len(v), 5) for k, v in per.items()}
    dom = max(kernels, key=kernels.get)
    res = dict(chain=chain, elapsed=elapsed, local=st["local"], launch=launch, kernels=kernels,
               dom=dom, dom_bytes=kernel_bytes(chain, dom))
    del x
    return res


def measure_stub(wl, B, steps):
    """DSP_BENCH_DRYRUN=1: the shapes and bookkeeping of measure() without a
    GPU (tests of the rank launcher and sharding; numbers are placeholders)."""
    from types import SimpleNamespace

    from dspcore import design
    src = design.src_plan(wl["n_in"], wl["fs"], wl["M"], wl["L"], wl["num_taps"])
    spec = design.spectrum_plan(src.n_out, wl["n_fft"])
    per = 4 * wl["n_in"] + 8 * src.n_out + 4 * (spec.n_fft // 2 + 1)
    chain = SimpleNamespace(B=B, n_out=src.n_out, tile_len=0, cfg=SimpleNamespace(n_in=wl["n_in"]),
                            spec=spec, algorithmic_bytes=lambda: per * B)
    ms = 1e-6 * B + 1e-3
    return dict(chain=chain, elapsed=steps * ms * 1e-3, local=steps * ms * 1e-3, launch="dry-run",
                kernels={"chain_tile": ms}, dom="chain_tile", dom_bytes=kernel_bytes(chain, "chain_tile"))


def extra_line(wl, r, steps):
    """A second workload on one GPU (config 3 / config 5 next to the default
    config 4): throughput, whole-chain and dominant-kernel HBM fractions."""
    ms = r["elapsed"] / steps * 1e3
    dom_ms = r["kernels"][r["dom"]]
    dom_gbs = r["dom_bytes"] / (dom_ms * 1e-3) / 1e9
    return {
        "workload": wl["desc"], "channels": r["chain"].B,
        "value": round(r["chain"].B * wl["n_in"] / (ms * 1e-3) / 1e6, 2),
        "unit": "Msamples/s", "ms_per_step": round(ms, 4),
        "chain_frac": round(r["chain"].algorithmic_bytes() / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "roofline": {"kernel": r["dom"], "achieved": round(dom_gbs, 1), "unit": "GB/s",
                     "frac": round(dom_gbs / HBM_PEAK_GBS, 4), "mean_ms": dom_ms,
                     "algorithmic_bytes": r["dom_bytes"]},
        "kernels_ms": r["kernels"],
    }


def host_inclusive(device, channels=1024, reps=5):
    """SURVEY.md §8(d)'s host-inclusive rate: numpy x in, H2D, the chain
    (config-3/4 geometry, hand-off status checked), D2H of y, z and |Z|, numpy
    out -- what the drop-in path costs per call.  Never `value`.
    The reported figure is dspcore.host.HostChain (64-channel blocks through
    four slots: pinned staging, the H2D of one block, the chain of the next
    and the D2H of the one before overlap); `single_call` is one Chain.run on
    the whole pageable batch with torch's staged copies, for comparison."""
    import numpy as np
    import torch

    from dspcore.chain import Chain, ChainConfig
    from dspcore.host import HostChain
    wl = WORKLOADS["c4"]
    cfg = ChainConfig(wl["n_in"], wl["fs"], wl["L"], wl["M"], wl["num_taps"], CONFIG3_GAINS,
                      n_fft=wl["n_fft"])
    x = np.random.default_rng(5).uniform(-1, 1, (channels, wl["n_in"])).astype(np.float32)

    def timed(once):
        once()
        torch.cuda.synchronize(device)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            once()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]   # median: host-side stalls hit single calls

    chain = Chain(cfg, channels, device)

    def single():
        y, z, mag = chain.run(torch.from_numpy(x).to(device))
        return y.cpu().numpy(), z.cpu().numpy(), mag.cpu().numpy()

    wall1 = timed(single)
    n_out = chain.n_out
    del chain
    torch.cuda.empty_cache()
    hc = HostChain(cfg, device, block=64, slots=4)
    wall = timed(lambda: hc.run(x))
    hc.close()
    del hc
    torch.cuda.empty_cache()
    moved = x.nbytes + 2 * 4 * channels * n_out + 4 * channels * (wl["n_fft"] // 2 + 1)
    return {"value": round(channels * wl["n_in"] / wall / 1e6, 2), "unit": "Msamples/s",
            "channels": channels, "ms_per_call": round(wall * 1e3, 3),
            "pcie_bytes_per_call": moved, "pcie_gbs": round(moved / wall / 1e9, 2),
            "how": "numpy x -> dspcore.host.HostChain (64-channel blocks, 4 slots: host copy into "
                   "pinned staging, H2D, dsp_chain_f32 (config-4 geometry), D2H of y, z, |Z| into "
                   "pinned numpy outputs, overlapped; staging copies on 4 threads) -> numpy, status "
                   "checked; median of 5 calls after 1 warm",
            "single_call": {"value": round(channels * wl["n_in"] / wall1 / 1e6, 2),
                            "ms_per_call": round(wall1 * 1e3, 3),
                            "how": "pageable numpy -> torch H2D -> Chain.run -> .cpu().numpy() "
                                   "of y, z, |Z|, one call on the whole batch"}}


def copy_ceiling(device, nbytes=1 << 30, reps=20):
    """Measured HBM ceiling in the same process: a contiguous float32 copy of
    1 GiB (torch's vectorized copy kernel: 16-byte loads/stores), read + write
    bytes / time."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=device).uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / reps
    del a, b
    torch.cuda.empty_cache()
    return {"value": round(2 * nbytes / (ms * 1e-3) / 1e9, 1), "unit": "GB/s",
            "how": f"torch contiguous float32 copy_ of {nbytes >> 20} MiB (read + write), "
                   f"mean of {reps} after 3 warm, CUDA events"}


def eq_alone(device, reps=10):
    """The app's default ratio L = M = 1 (app.py:149-150): the SRC returns x
    and sistema_ecualizador (dsp_core.py:216-254) is the whole path, here the
    single-pass one-tap cascade with the config-3 gains and
    no spectrum, graph-replayed: 32768 x 48000 (chained tiles; algorithmic
    bytes 8 per sample, x read and z written, against 8 TB/s) and one
    441000-sample channel (the three-launch mode), each beside the two-pass
    cascade (k_iir_wave) on the same input.  Not the metric."""
    import torch

    from dspcore import ops
    from dspcore.design import eq_plan

    sos = eq_plan(48000, CONFIG3_GAINS).sos

    def graph_ms(fn):
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            fn()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.current_stream(device).wait_stream(s)
        g.replay()
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize(device)
        return e0.elapsed_time(e1) / reps

    out = {}
    with torch.cuda.device(device):
        for tag, B, n in (("32768x48000", 32768, 48000), ("1x441000", 1, 441000)):
            x = torch.rand((B, n), device=device) * 2 - 1
            z = torch.empty_like(x)
            ws = ops.biquad_workspace(B, n, sos.shape[0], device)
            if ops.eq_single_pass(x, sos, out=z) is None:
                return None
            t1 = graph_ms(lambda: ops.eq_single_pass(x, sos, out=z))
            t0 = graph_ms(lambda: ops.biquad_cascade(x, sos, True, out=z, workspace=ws))
            gbs = B * n * 8 / (t1 * 1e-3) / 1e9
            out[tag] = {"single_pass_ms": round(t1, 4), "two_pass_ms": round(t0, 4),
                        "speedup": round(t0 / t1, 2),
                        "msamples_s": round(B * n / (t1 * 1e-3) / 1e6, 1),
                        "algorithmic_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "mode": "three-launch" if _lib_mode(B, n, sos.shape[0]) == 3 else
                                "chained tiles"}
            del x, z, ws
            torch.cuda.empty_cache()
    out["how"] = ("ops.eq_single_pass (dsp_chain_f32 with the one-tap SRC bypass, y and mag NULL) "
                  "vs ops.biquad_cascade, config-3 gains at 48 kHz, HIP graph replays, mean of "
                  f"{reps}; algorithmic bytes 8 per sample")
    return out


def _lib_mode(B, n, S):
    from dspcore import _lib
    return _lib.load().dsp_chain_mode(B, n, n, 1, 1, 1, 0, S)


def fft_large(device, log2n=28, reps=3):
    """The three-pass four-step FFT of one complex row of 2^log2n points
    (fft_diezmado_en_tiempo's size range above one workgroup's LDS): ms per
    transform (HIP events, mean of `reps` after one warm call) and the rate of
    its algorithmic traffic, read + write of N complex64 per pass.  Not part
    of the chain metric; None if it fails."""
    import torch
    from dspcore import ops
    try:
        n = 1 << log2n
        x = torch.randn(1, n, dtype=torch.complex64, device=device)
        out = torch.empty_like(x)
        ops.fft(x, out)
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.fft(x, out)
        e1.record()
        torch.cuda.synchronize(device)
        ms = e0.elapsed_time(e1) / reps
        del x, out
        torch.cuda.empty_cache()
    except (RuntimeError, ValueError) as e:
        return {"error": str(e)[:200]}
    passes = 3
    alg = 2 * n * 8                   # read N complex64, write N complex64
    gbs = alg / (ms * 1e-3) / 1e9
    moved = passes * 2 * n * 8        # what the three passes move (each reads and writes N)
    return {"n": n, "ms": round(ms, 3), "passes": passes,
            "algorithmic_bytes": alg, "achieved_gbs": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "traffic": moved, "traffic_gbs": round(moved / (ms * 1e-3) / 1e9, 1),
            "how": f"ops.fft of one complex64 row of 2^{log2n} (three launches of 8/16-column "
                   f"LDS tiles + twiddle table gather), mean of {reps} after 1 warm, CUDA events "
                   "around the calls (host overhead included); frac = algorithmic bytes (one "
                   "read + one write of the row) / time / 8 TB/s, traffic = the three passes' "
                   "read + write"}


def app_rerun(device, reps=5):
    """The reference app's own call pattern: ONE
    channel per Streamlit rerun through the drop-in module -- app.py:162-167
    (conversion_tasa_muestreo then sistema_ecualizador) and the three spectra
    of :203-205 (x, y and z, each on its first 100000 samples) -- on a
    441000-sample channel (10 s at 44.1 kHz, the config-1 stand-in for the
    missing FastCar.wav) with the config-3 gains, at L/M 1/1 (the sliders'
    default: the SRC returns x, the EQ is the whole path), 2/1 and 3/2.  numpy in,
    numpy out, as app.py calls it; ms per rerun (median of `reps` after one
    warm) next to the oracle (oracle/dsp_ref_cpu.py, the reference's numpy /
    scipy calls) on the same host and input, one process.  Not the metric."""
    import numpy as np
    import torch

    from modules import dsp_core as dc
    from oracle import dsp_ref_cpu as orc
    fs, n, lim = 44100, 441000, 100000
    t = np.arange(n) / fs
    x = (0.6 * np.sin(2 * np.pi * 440.0 * t)
         + 0.3 * np.random.default_rng(7).uniform(-1, 1, n)).astype(np.float32)
    x /= np.max(np.abs(x))

    def rerun_gpu(L, M):
        y, fs2 = dc.conversion_tasa_muestreo(x, fs, M, L)
        z = dc.sistema_ecualizador(y, fs2, CONFIG3_GAINS)
        return (dc.calcular_espectro_magnitud(x[:lim], fs), dc.calcular_espectro_magnitud(y[:lim], fs2),
                dc.calcular_espectro_magnitud(z[:lim], fs2))

    def rerun_cpu(L, M):
        y, fs2 = orc.resample(x, fs, M, L)
        z = orc.equaliser(y, fs2, CONFIG3_GAINS)
        return (orc.spectrum(x[:lim], fs), orc.spectrum(y[:lim], fs2), orc.spectrum(z[:lim], fs2))

    def median_ms(fn, k):
        fn()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(device)
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[len(ts) // 2]

    out = {}
    with torch.cuda.device(device):
        for L, M in ((1, 1), (2, 1), (3, 2)):   # (1/1: the sliders' default, app.py:149-150)
            g = median_ms(lambda: rerun_gpu(L, M), reps)
            c = median_ms(lambda: rerun_cpu(L, M), 3)
            got, ref = rerun_gpu(L, M), rerun_cpu(L, M)
            err = max(float(np.max(np.abs(a[1] - b[1]))) / float(np.max(b[1])) for a, b in zip(got, ref))
            out[f"L{L}M{M}"] = {"gpu_ms_per_rerun": round(g, 3), "oracle_ms_per_rerun": round(c, 2),
                                "speedup": round(c / g, 1), "max_rel_mag_err": float(f"{err:.3g}")}
    out["how"] = ("modules/dsp_core.py drop-in, numpy in/out (H2D, kernels, D2H per call): "
                  "conversion_tasa_muestreo + sistema_ecualizador (app.py:162-167) + three "
                  "calcular_espectro_magnitud on the first 100000 samples of x, y, z "
                  "(app.py:203-205), one 441000-sample channel (10 s @ 44.1 kHz, tone + noise "
                  "stand-in for FastCar.wav), config-3 gains; median of 5 after 1 warm; oracle: "
                  "the same calls through oracle/dsp_ref_cpu.py, 1 process, same host")
    return out


def ratio_sweep(device, channels=4096, steps=8, cases=None, two_launch=True):
    """Every SRC ratio the app's sliders offer (L, M in 1..8, app.py:149-150)
    at the default tap rule K = 40 max(L, M) + 1 (dsp_core.py:158), plus
    config 1's 2/1 at K = 127, on `channels` x 48000 samples at 48 kHz with
    the config-3 gains and the app's spectrum (2048 points of z[:100000],
    app.py:202-205; 4096 points would hit the reference's non-power-of-two
    segment ValueError at M/L = 6, 8): the path dsp_chain_f32 took
    (single-pass kernel or the two-launch chain), Msamples/s of the default
    path and of the two-launch chain (dsp_chain_path(1)) on the same input,
    CUDA events around `steps` eager calls after one warm call."""
    import torch

    from dspcore import _lib
    from dspcore.chain import Chain, ChainConfig
    gen = torch.Generator(device=device).manual_seed(77)
    x = torch.rand((channels, 48000), generator=gen, device=device) * 2 - 1

    def timed(ch):
        ch.run(x)
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            ch.run(x, check=False)
        e1.record()
        torch.cuda.synchronize(device)
        ch.check()
        return e0.elapsed_time(e1) / steps

    rows = []
    if cases is None:
        cases = [(L, M, None) for L in range(1, 9) for M in range(1, 9)] + [(2, 1, 127)]
    for L, M, K in cases:
        ch = Chain(ChainConfig(48000, 48000, L, M, K, CONFIG3_GAINS, n_fft=2048, limit_pts=100000),
                   channels, device)
        _lib.trace_enable(True)
        _lib.trace_read()
        ch.run(x)
        names = sorted({nm for nm, _ in _lib.trace_read()})
        _lib.trace_enable(False)
        ms = timed(ch)
        single = "chain_tile" in names
        ms2 = None
        if single and two_launch:
            prev = _lib.chain_path(1)
            try:
                ms2 = timed(ch)
            finally:
                _lib.chain_path(prev)
        rate = lambda v: round(channels * 48000 / (v * 1e-3) / 1e6, 1)  # noqa: E731
        rows.append({"L": L, "M": M, "K": ch.src.K, "path": "single-pass" if single else
                     ("eq-only (SRC identity)" if ch.identity_src else "two-launch"),
                     **({"note": "SRC bypass: the cascade alone (one-tap single-pass)"}
                        if ch.identity_src and single else {}),
                     "tile_len": ch.tile_len, "ms": round(ms, 4), "msamples_s": rate(ms),
                     **({"two_launch_ms": round(ms2, 4), "two_launch_msamples_s": rate(ms2),
                         "speedup_vs_two_launch": round(ms2 / ms, 3)} if ms2 else {}),
                     "kernels": names})
        del ch
        torch.cuda.empty_cache()
    del x
    torch.cuda.empty_cache()
    sp = [r for r in rows if r["path"] == "single-pass"]
    return {"channels": channels, "n_in": 48000, "fs": 48000, "steps": steps,
            "single_pass_cases": len(sp), "cases": len(rows),
            "min_speedup_vs_two_launch": min((r["speedup_vs_two_launch"] for r in sp
                                              if "speedup_vs_two_launch" in r), default=None),
            "rows": rows}


def mix_ceiling():
    """HBM ceiling for the chain kernel's traffic mix (1 read : 2 writes: x in,
    y and z out), measured by tools/ubench_rw_mix (streaming float4 kernels with
    the chain's nt cache policy, best of three grid sizes) in a child process;
    None when the binary is absent (built by __graft_entry__.build())."""
    exe = os.path.join(ROOT, "tools", "ubench_rw_mix")
    if not os.access(exe, os.X_OK):
        return None
    try:
        out = subprocess.run([exe, "--json"], capture_output=True, text=True, timeout=120,
                             check=True).stdout
        d = json.loads(out.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return None
    return {"value": d["r1w2_gbs"], "unit": "GB/s", "copy_1r1w_gbs": d["r1w1_gbs"],
            "how": "tools/ubench_rw_mix: nt float4 streams, 1 GiB each, 1 read : 2 writes "
                   "(the chain kernel's x : y, z), best of grids 4096/16384/65536 x 256"}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(WORKLOADS), default="c4")
    ap.add_argument("--channels", type=int, default=None,
                    help="total channels over all ranks (default: the config's)")
    ap.add_argument("--cpu-per-proc", type=int, default=None,
                    help="CPU-baseline channels per process (0 = skip; default per config)")
    ap.add_argument("--no-extras", "--no-config3", dest="no_extras", action="store_true",
                    help="skip the config-3/config-5, host-inclusive and copy-ceiling "
                         "measurements at N = 1")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the L/M ratio sweep (every app ratio at 4096 channels)")
    ap.add_argument("--eager", action="store_true",
                    help="launch every step from Python instead of replaying a HIP graph")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    rank, local_rank, world = dist_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    dry = os.environ.get("DSP_BENCH_DRYRUN") == "1"
    wl = dict(WORKLOADS[args.config])
    if args.channels:
        wl["channels"] = args.channels
    total = wl["channels"]
    lo, hi = rank_channels(total, rank, world)
    B = hi - lo

    # CPU baseline first: no GPU context exists yet when the pool forks.
    cpu = None
    per_proc = wl["cpu_per_proc"] if args.cpu_per_proc is None else args.cpu_per_proc
    if rank == 0 and world == 1 and per_proc > 0 and not dry:
        cpu = cpu_baseline(wl, usable_cores()[0], per_proc)

    import torch

    dist = None
    if world > 1:
        import torch.distributed as tdist
        # gloo prints its connection banner on stdout from C++; keep stdout for
        # the one JSON line (the banner goes to stderr).
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            tdist.init_process_group("gloo")  # timing barrier + max only: no RCCL
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        dist = tdist
    same_node = True
    if dist is not None:
        import socket
        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname())
        same_node = len(set(hosts)) == 1
    if dry:
        r = measure_stub(wl, B, args.steps)
        if dist is not None:
            dist.barrier()
        device = None
    else:
        # DSP_BENCH_DEVICE pins every rank to one device: a rehearsal of the
        # multi-rank path on a one-GPU box (the driver's runs leave it unset).
        dev_index = int(os.environ.get("DSP_BENCH_DEVICE", local_rank))
        device = torch.device("cuda", dev_index)
        torch.cuda.set_device(device)
        r = measure(wl, B, args.steps, args.warmup, rank, world, dist, args.eager, device,
                    same_node)
    chain, elapsed, kernels, dom = r["chain"], r["elapsed"], r["kernels"], r["dom"]
    if dist is not None and dry:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    per_rank = None
    if dist is not None:
        # every rank's own timed region, dominant-kernel mean and shard: the
        # N > 1 line shows the spread (a slow or throttled GPU, an imbalance)
        mine = torch.tensor([r["local"] * 1e3 / args.steps, kernels[dom], float(B)],
                            dtype=torch.float64)
        allr = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allr, mine)
        ms_r = [float(t[0]) for t in allr]
        dom_r = [float(t[1]) for t in allr]
        per_rank = {
            "elapsed_ms_min": round(min(ms_r), 4), "elapsed_ms_max": round(max(ms_r), 4),
            f"{dom}_ms_min": round(min(dom_r), 5), f"{dom}_ms_max": round(max(dom_r), 5),
            "channels": [int(t[2]) for t in allr],
            "elapsed_ms": [round(v, 4) for v in ms_r],
            f"{dom}_ms": [round(v, 5) for v in dom_r],
            "timing": ("max(end) - min(start), one node's monotonic clock" if same_node
                       else "max over ranks of each rank's elapsed (ranks on several nodes)"),
            "note": "elapsed_ms: per step, each rank's own timed region; "
                    f"{dom}_ms: its HIP-event mean",
        }
    ms_per_step = elapsed / args.steps * 1e3
    value = total * wl["n_in"] * args.steps / elapsed / 1e6
    mean_ms = kernels[dom]
    achieved = r["dom_bytes"] / (mean_ms * 1e-3) / 1e9
    traffic_map, traffic_src = load_traffic(wl["name"], B)
    traffic = traffic_map.get(dom)
    valu = valu_work(chain, mean_ms) if dom == "chain_tile" else None
    chain_bytes = chain.algorithmic_bytes()
    chain_gbs = chain_bytes / (ms_per_step * 1e-3) / 1e9
    launch, n_out, dom_bytes = r["launch"], chain.n_out, r["dom_bytes"]
    extras = {}
    if world == 1 and not args.no_extras and not dry:
        del chain, r
        torch.cuda.empty_cache()
        for key in ("c3", "c4", "c5"):
            if key == args.config:
                continue
            wlx = WORKLOADS[key]
            rx = measure(wlx, wlx["channels"], args.steps, args.warmup, 0, 1, None, args.eager,
                         device)
            extras[wlx["name"]] = extra_line(wlx, rx, args.steps)
            del rx
            torch.cuda.empty_cache()
        extras["host_inclusive"] = host_inclusive(device)
        extras["app_rerun"] = app_rerun(device)
        extras["eq_alone"] = eq_alone(device)
        if not args.no_sweep:
            extras["ratio_sweep"] = ratio_sweep(device)
        extras["copy_ceiling"] = copy_ceiling(device)
        extras["mix_ceiling"] = mix_ceiling()
        extras["fft_2_28"] = fft_large(device)
    # the copy ceiling is the higher of torch's copy_ and the nt float4 1R:1W
    # stream of tools/ubench_rw_mix (torch's alone flattered)
    ceiling_src = None
    ceiling = (extras.get("copy_ceiling") or {}).get("value")
    if ceiling:
        ceiling_src = "torch copy_"
    nt_copy = (extras.get("mix_ceiling") or {}).get("copy_1r1w_gbs")
    if nt_copy and (not ceiling or nt_copy > ceiling):
        ceiling, ceiling_src = nt_copy, "tools/ubench_rw_mix nt float4 1R:1W"
    mix = (extras.get("mix_ceiling") or {}).get("value")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 (IIR state/coefficients f64)",
            "data": "synthetic uniform(-1,1) float32 generated on device (reference WAVs missing)",
            "config": {
                "workload": wl["desc"], "total_channels": total, "channels_per_gpu": B,
                "n_in": wl["n_in"], "n_out": n_out, "fs_in": wl["fs"],
                "L": wl["L"], "M": wl["M"], "n_fft": wl["n_fft"],
                "parallelism": f"channel-shard x{world} (no collective)",
                "launch": launch,
                "preheat_s": PREHEAT_S,
            },
            "roofline": {
                "bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "frac_algorithmic": round(achieved / HBM_PEAK_GBS, 4),
                "frac_actual": (round(traffic / (mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                if traffic else None),
                "traffic_source": traffic_src if traffic else None,
                "copy_ceiling_gbs": ceiling,
                "copy_ceiling_source": ceiling_src,
                "frac_vs_copy_ceiling": round(achieved / ceiling, 4) if ceiling else None,
                "mix_ceiling_gbs": mix,
                "frac_vs_mix_ceiling": round(achieved / mix, 4) if mix else None,
                "algorithmic_bytes": dom_bytes,
                "mean_ms": mean_ms,
                "valu": valu,
            },
            "chain_roofline": {
                "achieved": round(chain_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(chain_gbs / HBM_PEAK_GBS, 4),
                "frac_vs_copy_ceiling": round(chain_gbs / ceiling, 4) if ceiling else None,
                "algorithmic_bytes_per_gpu_step": chain_bytes,
            },
            "kernels_ms": kernels,
            **({"per_rank": per_rank} if per_rank else {}),
            **{k: extras.get(k) for k in ("config3", "config4", "config5") if k in extras},
            "host_inclusive": extras.get("host_inclusive"),
            "app_rerun": extras.get("app_rerun"),
            "eq_alone": extras.get("eq_alone"),
            **({"ratio_sweep": extras["ratio_sweep"]} if extras.get("ratio_sweep") else {}),
            "copy_ceiling": extras.get("copy_ceiling"),
            "mix_ceiling": extras.get("mix_ceiling"),
            **({"fft_2_28": extras["fft_2_28"]} if extras.get("fft_2_28") else {}),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
