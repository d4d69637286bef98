#!/usr/bin/env python3
"""Full-size field fixtures computed with the C oracle (oracle/), for the GPU
parity tests at BASELINE.json's sizes.

The oracle itself is pinned by tests/test_oracle_golden.py (reference golden
vectors + the reference's Python mirror on sub-ranges of the same fields), so
these fixtures inherit that pinning.  Takes a few minutes on 8 cores:

    python tests/golden/gen_oracle_fields.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_fields.json")
THREADS = int(os.environ.get("THREADS", "8"))


def detailed(name, base, start, size, note):
    t = time.time()
    r = O.process_field_detailed_mt(start, start + size, base, THREADS)
    print(f"{name}: {time.time() - t:.1f}s", flush=True)
    return {"name": name, "base": base, "start": str(start), "end": str(start + size),
            "note": note, "distribution": [list(x) for x in r.distribution],
            "near_misses": [[str(n), u] for n, u in r.nice_numbers]}


def niceonly(name, base, start, size, note):
    t = time.time()
    r, cands = O.process_field_niceonly_mt(start, start + size, base, THREADS)
    print(f"{name}: {time.time() - t:.1f}s, {cands} candidates", flush=True)
    return {"name": name, "base": base, "start": str(start), "end": str(start + size),
            "note": note, "candidates": cands, "nice_numbers": [str(n) for n, _ in r.nice_numbers]}


def main():
    s40, _ = O.base_range(40)
    s50, _ = O.base_range(50)
    s80, _ = O.base_range(80)
    out = {"generator": "tests/golden/gen_oracle_fields.py (oracle/ C restatement)",
           "detailed": [], "niceonly": []}
    out["detailed"].append(detailed("b40_extra_large_1e9", 40, s40, 10 ** 9,
                                    "benchmark.rs:60 ExtraLarge (BASELINE metric field)"))
    out["detailed"].append(detailed("b80_hibase_1e8", 80, s80, 10 ** 8, "hi-base prefix"))
    out["detailed"].append(detailed("b50_start_1e8", 50, s50, 10 ** 8, "b50 range start"))
    out["niceonly"].append(niceonly("b40_extra_large_1e9", 40, s40, 10 ** 9,
                                    "reference client chunking, MSD floor 250, k=2"))
    out["niceonly"].append(niceonly("b50_msd_effective_1e11", 50, 26_507_984_537_059_635,
                                    10 ** 11, "benchmark.rs:53 MsdEffective start, 1e11 prefix"))
    out["niceonly"].append(niceonly("b50_msd_ineffective_1e7", 50, 94_760_515_586_064_977,
                                    10 ** 7, "benchmark.rs:54 MsdIneffective"))
    with open(OUT, "w") as f:
        json.dump(out, f)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
