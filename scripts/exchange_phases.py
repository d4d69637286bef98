"""Host cost of one PipelinedExchange step under torchrun (no field compute):
median microseconds of each enqueue in submit() and of collecting the
previous field, rank 0.  Run as
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 scripts/exchange_phases.py"""
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nice_amd import dist as D  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
world = dist.get_world_size()
vals = list(range(41)) + [0] * (2 * world)
ex = D.PipelinedExchange(dist, width=len(vals))
phases = {k: [] for k in ("fill", "h2d", "all_reduce", "wait", "d2h", "record", "collect", "submit_total",
                          "finish_both")}
for it in range(300):  # the steps of PipelinedExchange.submit, timed one by one
    t0 = time.perf_counter()
    h_in, d, h_out = ex.bufs[ex.flip]
    ev = ex.events[ex.flip]
    ex.flip ^= 1
    h_in.numpy()[:] = vals
    t1 = time.perf_counter()
    d.copy_(h_in, non_blocking=True)
    t2 = time.perf_counter()
    work = dist.all_reduce(d, op=dist.ReduceOp.SUM, async_op=True)
    t3 = time.perf_counter()
    work.wait()
    t4 = time.perf_counter()
    h_out.copy_(d, non_blocking=True)
    t5 = time.perf_counter()
    ev.record()
    t6 = time.perf_counter()
    prev, ex.pending = ex.pending, (ev, d, h_out, (40, [], [], None))
    got = ex._collect(prev)
    t7 = time.perf_counter()
    D.finish_both(ex, got)
    t8 = time.perf_counter()
    time.sleep(0.002)  # the field's compute would run here
    if it >= 50:
        for k, a, b in (("fill", t0, t1), ("h2d", t1, t2), ("all_reduce", t2, t3), ("wait", t3, t4),
                        ("d2h", t4, t5), ("record", t5, t6), ("collect", t6, t7), ("submit_total", t0, t7),
                        ("finish_both", t7, t8)):
            phases[k].append((b - a) * 1e6)
if dist.get_rank() == 0:
    for k, v in phases.items():
        print(f"{k:14s} {statistics.median(v):8.1f} us", flush=True)
dist.destroy_process_group()
