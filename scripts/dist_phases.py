"""Phase timings of bench.py's N > 1 step under torchrun (rank 0): detailed
shard, niceonly shard, fused exchange — vs the same calls without torch.distributed."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402


def phases(ctx, s, e, reps=20):
    t = {"det": 0.0, "nice": 0.0}
    for _ in range(reps):
        a = time.perf_counter()
        ctx.detailed_raw(s, e, 40)
        b = time.perf_counter()
        ctx.niceonly_raw(s, e, 40)
        c = time.perf_counter()
        t["det"] += b - a
        t["nice"] += c - b
    return {k: v / reps * 1e3 for k, v in t.items()}


use_dist = "WORLD_SIZE" in os.environ
if use_dist:
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
else:
    local = 0
ctx = N.GpuContext([local])
s = N.get_base_range_u128(40).range_start
phases(ctx, s, s + 10 ** 9, 3)
print("dist" if use_dist else "plain", phases(ctx, s, s + 10 ** 9), flush=True)
if use_dist:
    f = N.FieldSize(s, s + 10 ** 9)
    for _ in range(3):
        D.process_field_both_dist(f, 40, ctx)
    a = time.perf_counter()
    for _ in range(20):
        D.process_field_both_dist(f, 40, ctx)
    print("both_dist step ms", (time.perf_counter() - a) / 20 * 1e3, flush=True)
    dist.destroy_process_group()
