#!/usr/bin/env python3
"""Does Filter C (msd_prefix_filter.rs:461-559, unsound for ranges of more
than one number: scripts/filter_c_share.py) ever drop a nice number?  The
oracle's niceonly path over every base 3..59 whose whole valid range is
under 3e9 numbers, Filter C as shipped vs off: nice lists and candidates.

    python scripts/filter_c_bases.py > profiles/r06/filter_c_bases.txt
"""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def job(args):
    b, fc = args
    from oracle import oracle as O
    O.lib().oracle_set_filter_c(fc)
    r = O.base_range(b)
    if r is None or r[1] - r[0] > 3 * 10 ** 9:
        return b, fc, None
    res, c, rg = O.process_field_niceonly_ex(r[0], r[1], b, 1, 0, 0)
    return b, fc, (sorted(n for n, _ in res.nice_numbers), c, rg)


if __name__ == "__main__":
    with mp.Pool(min(8, os.cpu_count() or 1)) as p:
        out = p.map(job, [(b, fc) for b in range(3, 60) for fc in (1, 0)])
    d = {(b, fc): v for b, fc, v in out}
    print("# whole valid range per base, oracle niceonly (floor 250, k = 2): Filter C on (shipped) / off (sound)")
    print(f"{'base':>4} {'nice on':>7} {'nice off':>8} {'cands on':>10} {'cands off':>10} {'ranges on':>9} {'ranges off':>10}")
    lost = []
    for b in range(3, 60):
        on, off = d[(b, 1)], d[(b, 0)]
        if on is None:
            continue
        print(f"{b:4d} {len(on[0]):7d} {len(off[0]):8d} {on[1]:10d} {off[1]:10d} {on[2]:9d} {off[2]:10d}")
        lost += sorted(set(off[0]) - set(on[0]))
    print(f"nice numbers dropped by Filter C: {lost}")
