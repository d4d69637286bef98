"""Per-rank work of the weak-scaling bench, measured on ONE GPU: for N in
1, 2, 4, 8 the bench field is N x 1e9 at base 40 and rank r owns the r-th
shard (nice_amd/dist.py); this times each shard's detailed + niceonly call
(median of --reps) so the slowest rank — the one the max-over-ranks timing
sees — is known before the driver's 8-GPU run.

  python scripts/shard_balance.py [--reps 5] [--max-n 8]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402
from nice_amd.dist import niceonly_shard_bounds, shard_bounds  # noqa: E402
from nice_amd.types import FieldSize  # noqa: E402


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--max-n", type=int, default=8)
    a = ap.parse_args()
    ctx = N.GpuContext(0)
    f = get_benchmark_field(BM.EXTRA_LARGE)
    for world in (1, 2, 4, 8):
        if world > a.max_n:
            break
        field = FieldSize(f.range_start, f.range_start + world * f.range_size)
        rows = []
        for r in range(world):
            s, e = shard_bounds(field.range_start, field.range_end, r, world)
            ns, ne, chunk = niceonly_shard_bounds(field, r, world)
            det = med(lambda: ctx.detailed_raw(s, e, 40), a.reps)
            nic = med(lambda: ctx.niceonly_raw(ns, ne, 40, chunk_size=chunk), a.reps)
            _, st = ctx.niceonly_raw(ns, ne, 40, chunk_size=chunk)
            rows.append({"rank": r, "detailed_ms": round(det, 3), "niceonly_ms": round(nic, 3),
                         "step_ms": round(det + nic, 3), "msd_ranges": st.ranges,
                         "candidates": st.candidates})
        worst = max(x["step_ms"] for x in rows)
        print(json.dumps({"world": world, "worst_step_ms": worst,
                          "mean_step_ms": round(statistics.mean(x["step_ms"] for x in rows), 3),
                          "ranks": rows}), flush=True)


if __name__ == "__main__":
    main()
