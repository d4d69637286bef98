"""Massive benchmark field (b50, [start, start + 1e13), niceonly) on one GPU:
the whole field in one call, then each of N ranks' dealt share (chunks
c = r mod N, as dist.niceonly_deal gives rank r), timed one after another.
Prints each share's time and candidates, and the projected N-GPU
efficiency T_1 / (N * max_r T_r) (every rank alone on its own GPU).
    python scripts/massive_deal.py [N=8] [reps=3]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
f = get_benchmark_field(BM.MASSIVE)
ctx = N.GpuContext(0)


def run(**kw):
    ts, out = [], None
    for _ in range(reps):
        t = time.perf_counter()
        out = ctx.niceonly_raw(f.range_start, f.range_end, 50, **kw)
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), out


ctx.niceonly_raw(f.range_start, f.range_start + 10 ** 11, 50)  # warm-up (tables, code objects)
t1, (lst, st) = run()
print(f"whole field: {t1:.4f} s, ranges {st.ranges}, candidates {st.candidates}, nice {len(lst)}",
      flush=True)
shares = []
for r in range(world):
    tr, (l, s) = run(deal_stride=world, deal_offset=r)
    shares.append({"rank": r, "s": tr, "candidates": s.candidates, "ranges": s.ranges, "nice": len(l)})
    print(f"rank {r}/{world}: {tr:.4f} s, ranges {s.ranges}, candidates {s.candidates}", flush=True)
assert sum(x["candidates"] for x in shares) == st.candidates
assert sum(x["ranges"] for x in shares) == st.ranges
tmax = max(x["s"] for x in shares)
cands = [x["candidates"] for x in shares]
print(json.dumps({"config": "massive", "base": 50, "size": f.range_size, "world": world,
                  "t1_s": t1, "max_share_s": tmax, "projected_efficiency": t1 / (world * tmax),
                  "candidate_spread": (max(cands) - min(cands)) / (sum(cands) / world),
                  "shares": shares, "method": "each rank's dealt share timed alone on one GPU"}),
      flush=True)
