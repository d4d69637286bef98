#!/usr/bin/env python3
"""Whole-field fixtures for the FD kernel's production and hi-base fields at
the CLI sizes, computed with the C oracle (oracle/, pinned by
tests/test_oracle_golden.py): b80 1e9 (benchmark.rs:63 hi-base) and the live
bases b52 / b53 / b54 (CHANGELOG.md:21), 1e9 each from the base's range start.
About 20 minutes on 8 cores:

    python tests/golden/gen_fd_bases_fixtures.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fd_bases_1e9.json")
THREADS = int(os.environ.get("THREADS", "8"))
FIELDS = [("b80_hibase_1e9", 80, "benchmark.rs:63 HiBase (CLI size 1e9)"),
          ("b52_start_1e9", 52, "live base (CHANGELOG.md:21), range start"),
          ("b53_start_1e9", 53, "live base (CHANGELOG.md:21), range start"),
          ("b54_start_1e9", 54, "live base (CHANGELOG.md:21), range start")]


def main():
    out = {"generator": "tests/golden/gen_fd_bases_fixtures.py (oracle/ C restatement)", "detailed": []}
    for name, base, note in FIELDS:
        s, _ = O.base_range(base)
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
