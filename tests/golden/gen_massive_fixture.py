#!/usr/bin/env python3
"""Massive-config fixture: the whole b50 1e13 niceonly field
(common/src/benchmark.rs:62, BenchmarkMode::Massive) computed with the C
oracle, window by window, on the field's own client chunk grid (chunk 1e8 =
client/src/main.rs:158-168 for a 1e13 field) at the CPU path's MSD floor 250.

Each 1e11 window records the stride candidates tested, the MSD-surviving
ranges (get_valid_ranges output length, msd_prefix_filter.rs:665-674) and the
nice list, so the GPU tests can check any window with both MSD placements and
the whole field through sums.  The first ~70 % of the field is pruned by the
MSD filter at the top level; every candidate sits in the last 3e12.

Takes ~25 min on 8 cores; resumable (windows already in the output are kept):

    python tests/golden/gen_massive_fixture.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "massive_b50.json")
THREADS = int(os.environ.get("THREADS", "8"))
BASE = 50
START = 26_507_984_537_059_635   # benchmark.rs:62 (get_base_range_u128(50).start)
SIZE = 10 ** 13
CHUNK = 10 ** 8                  # client chunk rule for a 1e13 field
WINDOW = 10 ** 11


def main():
    assert O.base_range(BASE)[0] == START
    out = {"generator": "tests/golden/gen_massive_fixture.py (oracle/ C restatement)",
           "base": BASE, "start": str(START), "end": str(START + SIZE), "chunk": CHUNK,
           "msd_floor": 250, "stride_k": 2, "windows": []}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out["windows"] = json.load(f)["windows"]
    done = {int(w["start"]) for w in out["windows"]}
    for i in range(SIZE // WINDOW):
        a = START + i * WINDOW
        if a in done:
            continue
        t = time.time()
        r, cands, ranges = O.process_field_niceonly_ex(a, a + WINDOW, BASE, THREADS, chunk=CHUNK)
        out["windows"].append({"start": str(a), "end": str(a + WINDOW), "candidates": cands,
                               "ranges": ranges,
                               "nice_numbers": [str(n) for n, _ in r.nice_numbers]})
        out["windows"].sort(key=lambda w: int(w["start"]))
        with open(OUT + ".tmp", "w") as f:
            json.dump(out, f, indent=0)
        os.replace(OUT + ".tmp", OUT)
        print(f"window {i}: {cands} candidates, {ranges} ranges, {time.time() - t:.1f}s",
              flush=True)
    tot = sum(w["candidates"] for w in out["windows"])
    print("total candidates", tot, "ranges", sum(w["ranges"] for w in out["windows"]))


if __name__ == "__main__":
    main()
