"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2): weak-scaling
field assignment (disjoint consecutive 1e9 fields, all inside base 40's range)
and the max-over-ranks timing reduction."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time

    import bench
    field = bench.rank_field(1_916_284_264_916, rank)
    delay = 0.05 * (rank + 1)
    el = bench.timed(lambda: time.sleep(delay), 2, dist.barrier, dist)
    q.put((rank, field, el))
    dist.destroy_process_group()


def test_two_rank_weak_scaling_plumbing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, f0, e0), (r1, f1, e1) = out
    assert f0[1] == f1[0] and f0[1] - f0[0] == 10 ** 9 and f1[1] - f1[0] == 10 ** 9
    assert f1[1] <= 6_553_600_000_000  # inside base 40's range (base_range.rs:86-87)
    # max over ranks: both ranks report the slower rank's time (2 x 0.1 s)
    assert abs(e0 - e1) < 1e-9 and e0 >= 0.2
