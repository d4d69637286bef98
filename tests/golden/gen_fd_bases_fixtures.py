#!/usr/bin/env python3
"""Whole-field fixtures for the FD kernel's production and hi-base fields at
the CLI sizes, computed with the C oracle (oracle/, pinned by
tests/test_oracle_golden.py): b80 1e9 (benchmark.rs:63 hi-base) and the live
bases b52 / b53 / b54 (CHANGELOG.md:21), 1e9 each from the base's range start.
About 20 minutes on 8 cores:

    python tests/golden/gen_fd_bases_fixtures.py

--more writes fd_bases_more_1e9.json instead: 1e9 fields one third into the
ranges of b42, b49, b59 and b65 -- one base per FD kernel class the first
file does not cover (TCHUNK 80 / 160 / 240 with the side-table low-digit
path / three mask words), each a persistent-grid field, at a position away
from the range start (another limb-count combo than the start's where the
base has one).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

MORE = "--more" in sys.argv
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                   "fd_bases_more_1e9.json" if MORE else "fd_bases_1e9.json")
THREADS = int(os.environ.get("THREADS", "8"))
FIELDS = [("b80_hibase_1e9", 80, "benchmark.rs:63 HiBase (CLI size 1e9)"),
          ("b52_start_1e9", 52, "live base (CHANGELOG.md:21), range start"),
          ("b53_start_1e9", 53, "live base (CHANGELOG.md:21), range start"),
          ("b54_start_1e9", 54, "live base (CHANGELOG.md:21), range start")]
FIELDS_MORE = [("b42_third_1e9", 42, "TCHUNK 80 class, persistent grid, 1/3 into the range"),
               ("b49_third_1e9", 49, "TCHUNK 160 class, persistent grid, 1/3 into the range"),
               ("b59_third_1e9", 59, "TCHUNK 240, side-table low-digit path (LSDX), 1/3 into the range"),
               ("b65_third_1e9", 65, "three mask words (16-byte entries), 1/3 into the range")]


def main():
    out = {"generator": "tests/golden/gen_fd_bases_fixtures.py (oracle/ C restatement)", "detailed": []}
    for name, base, note in (FIELDS_MORE if MORE else FIELDS):
        s, e = O.base_range(base)
        if MORE:
            s = s + (e - s) // 3
        t = time.time()
        r = O.process_field_detailed_mt(s, s + 10 ** 9, base, THREADS)
        print(f"{name}: {time.time() - t:.0f}s", flush=True)
        out["detailed"].append({"name": name, "base": base, "start": str(s), "end": str(s + 10 ** 9),
                                "note": note, "distribution": [list(x) for x in r.distribution],
                                "near_misses": [[str(n), u] for n, u in r.nice_numbers]})
        with open(OUT, "w") as f:
            json.dump(out, f)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
