"""Sibling-lane stride per shard of the bench field: for each of the N
contiguous shards of the b40 1e9 field (dist.shard_bounds) the detailed
kernel's median time at the stride the launcher picks and at every forced
odd stride in [lo, hi] (nice_debug_force_sib_stride), so a shard whose pick
is off shows as a gap between `auto` and the best forced stride.

    python3 scripts/ubench/shard_stride_sweep.py [--world 8] [--lo 61 --hi 135] [--reps 5]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--lo", type=int, default=61)
    ap.add_argument("--hi", type=int, default=135)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    f = get_benchmark_field(BM.EXTRA_LARGE)
    ctx = N.GpuContext(0)
    lib = N._lib.lib()
    for _ in range(3):
        ctx.detailed_raw(f.range_start, f.range_end, f.base)

    def timed(s, e):
        ts = []
        for _ in range(a.reps):
            h, _ = ctx.detailed_raw(s, e, f.base)
            assert sum(h) == e - s
            ts.append(ctx.kernel_stats().kernel_ms)
        st = ctx.kernel_stats()
        return statistics.median(ts), st.sib_lanes, st.sib_stride
    try:
        for r in range(a.world):
            s, e = D.shard_bounds(f.range_start, f.range_end, r, a.world)
            lib.nice_debug_force_sib_stride(0)
            auto = timed(s, e)
            sweep = {}
            for L in range(a.lo | 1, a.hi + 1, 2):
                assert lib.nice_debug_force_sib_stride(L) == 0
                sweep[L] = timed(s, e)[0]
            best = min(sweep, key=sweep.get)
            print(json.dumps({"shard": r, "of": a.world, "auto_ms": round(auto[0], 5), "auto_sib": auto[1],
                              "auto_L": auto[2], "best_L": best, "best_ms": round(sweep[best], 5),
                              "sweep": {L: round(v, 5) for L, v in sweep.items()}}), flush=True)
    finally:
        lib.nice_debug_force_sib_stride(0)
    ctx.close()


if __name__ == "__main__":
    main()
