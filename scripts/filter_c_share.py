#!/usr/bin/env python3
"""Filter C's share of the massive field's MSD pruning.

Filter C (msd_prefix_filter.rs:461-559) drops a range when first / b^2 ==
last / b^2 and the two LSDs of FIRST's square / cube collide with the MSD
prefixes.  That condition fixes the range's high digits, not n mod b^2, so
every other number of the range is judged by first's LSDs: the filter is
sound only for one-number ranges (which return before it).  The GPU path
reproduces it bit for bit (candidate-set parity with the CPU path).

This runs the oracle (CPU, test infrastructure) over sampled 1e8 chunks of
the massive field (b50 1e13, benchmark.rs:62) at MSD floors 250 (the CPU
path's) and 64 (the throughput row), with Filter C as shipped and switched
off (the sound filter), and reports ranges, stride candidates and nice
numbers per variant.  The samples are seeded: 40 chunks from the surviving
part of the field (windows 72..99 of tests/golden/massive_b50.json) and 8
from the pruned part.

    python scripts/filter_c_share.py [--chunks 40] > profiles/r06/filter_c_share.txt
"""
import argparse
import json
import multiprocessing as mp
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(job):
    start, chunk, floor, fc = job
    from oracle import oracle as O
    O.lib().oracle_set_filter_c(fc)
    res, cands, ranges = O.process_field_niceonly_ex(start, start + chunk, 50, 1, chunk, floor)
    return job, cands, ranges, len(res.nice_numbers)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=40)
    ap.add_argument("--pruned", type=int, default=8)
    ap.add_argument("--procs", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "massive_b50.json")) as f:
        m = json.load(f)
    s0, chunk = int(m["start"]), int(m["chunk"])
    per_win = (int(m["end"]) - s0) // chunk // len(m["windows"])  # chunks per window (1000)
    rng = random.Random(20261018)
    live = [rng.randrange(72 * per_win, 100 * per_win) for _ in range(a.chunks)]
    dead = [rng.randrange(0, 72 * per_win) for _ in range(a.pruned)]
    jobs = [(s0 + c * chunk, chunk, floor, fc) for c in live + dead for floor in (250, 64) for fc in (1, 0)]
    with mp.Pool(a.procs) as pool:
        out = pool.map(run, jobs)
    tot = {}
    for (start, _, floor, fc), cands, ranges, nice in out:
        part = "live" if (start - s0) // chunk >= 72 * per_win else "pruned"
        t = tot.setdefault((part, floor, fc), [0, 0, 0])
        t[0] += cands
        t[1] += ranges
        t[2] += nice
    print(f"# massive field b50 [{s0}, {m['end']}), chunks of {chunk:.0e}; seeded sample: "
          f"{a.chunks} chunks of the surviving part (windows 72..99), {a.pruned} of the pruned part")
    print("# Filter C on = as shipped (reference behaviour); off = the sound filter")
    print(f"{'part':7} {'floor':>5} {'filter C':>8} {'candidates':>12} {'ranges':>10} {'nice':>5}")
    for part in ("live", "pruned"):
        for floor in (250, 64):
            for fc in (1, 0):
                c, r, n = tot[(part, floor, fc)]
                print(f"{part:7} {floor:5d} {'on' if fc else 'off':>8} {c:12d} {r:10d} {n:5d}")
    print()
    for floor in (250, 64):
        on, off = tot[("live", floor, 1)], tot[("live", floor, 0)]
        print(f"floor {floor}: Filter C removes {off[0] - on[0]} of {off[0]} sound candidates "
              f"({(off[0] - on[0]) / max(1, off[0]):.1%}); ranges {off[1]} -> {on[1]}")
    on250, on64 = tot[("live", 250, 1)][0], tot[("live", 64, 1)][0]
    off250, off64 = tot[("live", 250, 0)][0], tot[("live", 64, 0)][0]
    print(f"floor 250 -> 64: shipped candidates x{on64 / max(1, on250):.3f}, sound x{off64 / max(1, off250):.3f}; "
          f"of the shipped fall ({on250 - on64}), the sound filter keeps {off250 - off64} "
          f"({(off250 - off64) / max(1, on250 - on64):.1%}), the rest is Filter C firing on more (smaller) nodes")

if __name__ == "__main__":
    main()
