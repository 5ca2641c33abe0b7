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
