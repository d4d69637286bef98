"""Strong-scaling projection of the bench field from one GPU: the b40 1e9
field cut into N contiguous shards exactly as bench.py does at N ranks
(dist.shard_bounds), each rank's detailed shard timed alone (median kernel
time of 7 calls, HIP events) for N = 1, 2, 4, 8.  The N-GPU detailed time
is the slowest shard; efficiency = T_1 / (N x T_N).  What this leaves out:
the per-step histogram all-reduce and the niceonly pass (pipelined beside
the detailed shard in bench.py), so it bounds the kernel side of the
driver's SCALE run, it does not replace it.
    python scripts/shard_projection.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402

f = get_benchmark_field(BM.EXTRA_LARGE)
ctx = N.GpuContext(0)
for _ in range(5):  # warm-up: clocks, code objects, the stride model's table
    ctx.detailed_raw(f.range_start, f.range_end, f.base)
rows = []
t1 = None
for world in (1, 2, 4, 8):
    shards = []
    for r in range(world):
        s, e = D.shard_bounds(f.range_start, f.range_end, r, world)
        ts = []
        for _ in range(7):
            ctx.detailed_raw(s, e, f.base)
            ts.append(ctx.kernel_stats().kernel_ms)
        shards.append(statistics.median(ts))
    tn = max(shards)
    t1 = tn if world == 1 else t1
    row = {"world": world, "shard_numbers": (f.range_end - f.range_start) // world,
           "max_shard_kernel_ms": tn, "min_shard_kernel_ms": min(shards),
           "projected_efficiency": t1 / (world * tn), "shards_ms": shards}
    rows.append(row)
    print(json.dumps(row), flush=True)
ctx.close()
