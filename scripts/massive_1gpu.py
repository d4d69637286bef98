"""Whole massive benchmark field (b50, [start, start + 1e13), niceonly, client
chunking 1e8, device MSD floor 250 or argv[2]) on one GPU: wall time, MSD
leaves, candidates, nice list.  Progress: one line per 1e12 slice.
    python scripts/massive_1gpu.py [slices=10] [floor=250]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402

f = get_benchmark_field(BM.MASSIVE)
ctx = N.GpuContext(0)
slices = int(sys.argv[1]) if len(sys.argv) > 1 else 10
floor = int(sys.argv[2]) if len(sys.argv) > 2 else 250
step = f.range_size // slices
tot = {"ranges": 0, "candidates": 0, "range_numbers": 0, "nice": []}
t0 = time.perf_counter()
for i in range(slices):
    a = f.range_start + i * step
    b = f.range_end if i == slices - 1 else a + step
    t = time.perf_counter()
    lst, st = ctx.niceonly_raw(a, b, 50, chunk_size=10 ** 8, msd_floor=floor, msd_where="device")
    tot["ranges"] += st.ranges
    tot["candidates"] += st.candidates
    tot["range_numbers"] += st.range_numbers
    tot["nice"] += [str(x) for x in lst]
    print(f"slice {i}: {time.perf_counter() - t:.3f} s ranges {st.ranges} cands {st.candidates}",
          flush=True)
wall = time.perf_counter() - t0
tot.update({"config": "massive", "base": 50, "size": f.range_size, "wall_s": wall,
            "numbers_per_sec_1gpu": f.range_size / wall, "chunk": 10 ** 8, "msd_floor": 250,
            "msd_where": "device"})
print(json.dumps(tot), flush=True)
