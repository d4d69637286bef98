"""hi-base b80 1e6 (the BASELINE size) and 1e9: median wall / kernel ms of 50
library calls, plus parity of the 1e6 field against the committed vector.
    python scripts/hibase_small.py"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
s = N.get_base_range_u128(80).range_start
for size, reps in ((10 ** 6, 50), (10 ** 9, 5)):
    ctx.detailed_raw(s, s + size, 80)
    w, k = [], []
    for _ in range(reps):
        t = time.perf_counter()
        hist, lst = ctx.detailed_raw(s, s + size, 80)
        w.append(time.perf_counter() - t)
        k.append(ctx.kernel_stats().kernel_ms)
    print(json.dumps({"base": 80, "size": size, "wall_ms": statistics.median(w) * 1e3,
                      "kernel_ms": statistics.median(k), "mass_ok": sum(hist) == size}), flush=True)
