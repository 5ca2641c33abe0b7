"""The N > 1 bench path on CPU: two gloo ranks run bench.timed_loop (barrier +
sync bracketing, max-over-ranks of the elapsed time) and the channel-shard
bookkeeping (config 4's 32768 channels: 16384 per rank).  bench.py's GPU
ranks use the same harness over gloo too (no RCCL)."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from dspcore.shard import shard_ranges
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, lr, w = bench.dist_env()
        assert (r, lr, w) == (rank, rank, world)
        calls = []
        delay = 0.02 * (rank + 1)          # rank 1 is the slow one

        def step():
            calls.append(1)
            time.sleep(delay)

        elapsed = bench.timed_loop(step, steps=3, warmup=2, sync=lambda: None, dist=dist,
                                   preheat_s=0)
        lo, hi = shard_ranges(32768, world)[rank]
        assert bench.rank_channels(bench.WORKLOADS["c4"]["channels"], rank, world) == (lo, hi)
        out[rank] = (elapsed, len(calls), lo, hi)
    finally:
        dist.destroy_process_group()


def test_two_rank_timing_is_max_over_ranks():
    world = 2
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    e0, n0, lo0, hi0 = out[0]
    e1, n1, lo1, hi1 = out[1]
    assert n0 == n1 == 5                       # warmup + timed steps on every rank
    assert e0 == pytest.approx(e1)             # both report the max over ranks
    assert e0 >= 3 * 0.04 * 0.95               # ... which is the slow rank's time
    assert (lo0, hi0, lo1, hi1) == (0, 16384, 16384, 32768)


def _worker_nodes(rank, world, port, out):
    """timed_loop with same_node=False: the max of the ranks' own times."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = {}
        elapsed = bench.timed_loop(lambda: time.sleep(0.01 * (rank + 1)), steps=3, warmup=0,
                                   sync=lambda: None, dist=dist, preheat_s=0, same_node=False,
                                   stats=st)
        out[rank] = (elapsed, st["local"])
    finally:
        dist.destroy_process_group()


def test_timed_loop_across_nodes_is_max_of_local_times():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker_nodes, args=(world, _free_port(), out), nprocs=world, join=True)
    (e0, l0), (e1, l1) = out[0], out[1]
    assert e0 == e1 == pytest.approx(max(l0, l1))
    assert l1 > l0


def test_timed_loop_preheat_then_exact_counts():
    """bench.timed_loop runs untimed steps for preheat_s seconds, then exactly
    W warmup and K timed steps (the timed region covers only the K)."""
    import time as _t

    import bench
    calls = []

    def step():
        calls.append(_t.perf_counter())
        _t.sleep(0.002)

    elapsed = bench.timed_loop(step, steps=3, warmup=2, sync=lambda: None, preheat_s=0.03)
    assert len(calls) >= 2 + 3 + 10          # >= 30 ms of 2 ms pre-heat steps
    assert 0.005 <= elapsed < 0.05           # only the 3 timed steps


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(DSP_BENCH_DRYRUN="1", **extra)
    return env


def test_bench_gpus_flag_launches_the_ranks_itself():
    """`python bench.py --gpus 2` with no launcher starts two ranks (fresh
    processes, gloo rendezvous on 127.0.0.1) that shard config 4's 32768
    channels (0, 16384) and (16384, 32768); rank 0 alone prints the line.
    DSP_BENCH_DRYRUN stubs the GPU measurement (measure_stub)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--steps", "3", "--warmup", "1"], capture_output=True, text=True,
                         timeout=300, env=_bench_env(), cwd=root)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), res.stdout   # stdout: the JSON line only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    assert out["config"]["total_channels"] == 32768
    assert out["config"]["channels_per_gpu"] == 16384
    assert out["config"]["parallelism"] == "channel-shard x2 (no collective)"
    assert out["cpu_baseline"] is None                  # N > 1: rank 0 skips the CPU leg
    pr = out["per_rank"]                                # every rank's own numbers
    assert pr["channels"] == [16384, 16384]
    for k in ("elapsed_ms_min", "elapsed_ms_max", "chain_tile_ms_min", "chain_tile_ms_max"):
        assert pr[k] > 0, k
    assert pr["elapsed_ms_min"] <= pr["elapsed_ms_max"] and len(pr["elapsed_ms"]) == 2
    assert pr["chain_tile_ms_min"] <= pr["chain_tile_ms_max"]
    assert pr["timing"].startswith("max(end) - min(start)")   # both ranks on this host


def test_bench_refuses_gpus_other_than_world_size():
    """Under a launcher, --gpus must equal WORLD_SIZE (one rank per GPU)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4",
                          "--steps", "1"], capture_output=True, text=True, timeout=120,
                         env=_bench_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2"), cwd=root)
    assert res.returncode != 0 and "WORLD_SIZE=2" in res.stderr
