"""Per-repetition wall and kernel times of one detailed field (variance check).
    python scripts/rep_times.py BASE SIZE [REPS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

base, size = int(sys.argv[1]), int(float(sys.argv[2]))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
ctx = N.GpuContext(0)
s = N.get_base_range_u128(base).range_start
for i in range(reps):
    t = time.perf_counter()
    ctx.detailed_raw(s, s + size, base)
    w = (time.perf_counter() - t) * 1e3
    print(f"rep {i}: wall {w:.3f} ms kernel {ctx.kernel_stats().kernel_ms:.3f} ms", flush=True)
