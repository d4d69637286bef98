"""Sibling-lane stride sweep, pipelined, in one process: for each field size
and each odd stride L in [lo, hi] (forced through nice_debug_force_sib_stride;
0 = the launcher's pick) the ms per step of dist.FieldPipeline (both modes,
depth 2, no exchange) over the base range's first SIZE numbers (b40: the
bench field).  The (size, L) cells are visited in a different shuffled order
in each repetition and the median over repetitions is reported, so clock
drift does not line up with L.

    python3 scripts/ubench/stride_sweep_pipe.py --base 40 --sizes 1e9,1.25e8 --lo 61 --hi 131 --reps 3"""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=40)
    ap.add_argument("--sizes", default="1e9,1.25e8")
    ap.add_argument("--lo", type=int, default=61)
    ap.add_argument("--hi", type=int, default=131)
    ap.add_argument("--extra", default="0", help="more strides (comma list; 0 = the pick)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--numbers", type=float, default=6e9, help="numbers per timed cell")
    ap.add_argument("--at", type=float, default=0.0,
                    help="fields start this fraction into the base range (0 = its start, the bench field at b40)")
    a = ap.parse_args()
    lib = N._lib.lib()
    ctx = N.GpuContext(0)
    br = N.get_base_range_u128(a.base)
    start = br.range_start + int((br.range_end - br.range_start) * a.at)
    sizes = [int(float(x)) for x in a.sizes.split(",")]
    Ls = sorted(set(list(range(a.lo | 1, a.hi + 1, 2)) + [int(x) for x in a.extra.split(",") if x]))
    res = {}
    picked = {}
    rng = random.Random(7)
    try:
        for rep in range(a.reps):
            cells = [(sz, L) for sz in sizes for L in Ls]
            rng.shuffle(cells)
            for sz, L in cells:
                assert lib.nice_debug_force_sib_stride(L) == 0
                field = N.FieldSize(start, start + sz)
                steps = max(8, int(a.numbers // sz))
                pipe = D.FieldPipeline(ctx, ctx)
                for _ in range(3):
                    pipe.step(field, a.base)
                pipe.drain()
                ctx.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    pipe.step(field, a.base)
                pipe.drain()
                ctx.synchronize()
                res.setdefault((sz, L), []).append((time.perf_counter() - t0) / steps * 1e3)
                if L == 0:
                    st = ctx.kernel_stats()
                    picked[sz] = (st.sib_lanes, st.sib_stride)
            print(f"# rep {rep} done", file=sys.stderr, flush=True)
    finally:
        lib.nice_debug_force_sib_stride(0)
    for sz in sizes:
        row = {L: statistics.median(res[(sz, L)]) for L in Ls}
        best = min((L for L in Ls if L), key=row.get)
        print(json.dumps({"base": a.base, "at": a.at, "start": str(start), "size": sz, "pick": picked.get(sz), "pick_ms": round(row.get(0, 0), 5),
                          "best_L": best, "best_ms": round(row[best], 5),
                          "ms": {L: round(v, 5) for L, v in row.items()}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
