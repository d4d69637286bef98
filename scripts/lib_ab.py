"""Kernel time of the same fields under two builds of the library, on one
box: `python scripts/lib_ab.py DIR BASE:SIZE[:FRAC] ...` imports nice_amd from
DIR (e.g. ab_old/, a copy of an earlier round's package and library) or from
the repo when DIR is '.', and prints per field the median kernel time (HIP
events) of 9 calls after 2 untimed ones.  Run it alternately for the two
builds (each in its own process: a process loads one library)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = sys.argv[1]
sys.path.insert(0, ROOT if d == "." else os.path.join(ROOT, d))
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
for f in sys.argv[2:]:
    parts = f.split(":")
    base, size = int(parts[0]), int(float(parts[1]))
    r = N.get_base_range_u128(base)
    s = r.range_start + (int((r.range_end - r.range_start) * float(parts[2])) if len(parts) > 2 else 0)
    for _ in range(2):
        ctx.detailed_raw(s, s + size, base)
    t = []
    for _ in range(9):
        ctx.detailed_raw(s, s + size, base)
        t.append(ctx.kernel_stats().kernel_ms)
    print(f"{d} b{base} {size:.0e}@{parts[2] if len(parts) > 2 else 0}: {statistics.median(t) * 1e3:9.1f} us", flush=True)
ctx.close()
