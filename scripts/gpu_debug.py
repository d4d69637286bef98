"""Step-by-step GPU bring-up probe (prints progress, flushes every line)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
t0 = time.time()


def log(*a):
    print(f"[{time.time() - t0:7.2f}s]", *a, flush=True)


import nice_amd as N  # noqa: E402
from oracle import oracle as O  # noqa: E402

log("import ok")
L = N.lib()
import ctypes  # noqa: E402
n = ctypes.c_int()
L.nice_device_count(n)
log("devices", n.value)
ctx = N.GpuContext(0)
log("ctx ok")
step = sys.argv[1] if len(sys.argv) > 1 else "all"
if step in ("all", "generic"):
    h, l = ctx.detailed_raw(47, 100, 10)
    log("generic b10", l)
    h, l = ctx.detailed_raw(1000, 5000, 10)
    w = O.process_range_detailed(1000, 5000, 10)
    log("generic b10 1000..5000 ok?", [(i, h[i]) for i in range(1, 11)] == w.distribution)
if step in ("all", "unique"):
    log("unique", ctx.debug_unique_counts([69, 70, 12345678901234567], 10))
if step in ("all", "fd"):
    s, _ = O.base_range(40)
    for size in (1, 64, 1000, 100000):
        h, l = ctx.detailed_raw(s, s + size, 40)
        w = O.process_range_detailed(s, s + size, 40)
        log("fd b40", size, [(i, h[i]) for i in range(1, 41)] == w.distribution,
            ctx.kernel_stats())
if step in ("all", "nice"):
    log("nice b10", ctx.niceonly_raw(47, 100, 10))
log("done")
if step == "nice40":
    s, _ = O.base_range(40)
    for size in (10 ** 5, 10 ** 6, 10 ** 7):
        log("start nice40", size)
        r = ctx.niceonly_raw(s, s + size, 40)
        log("nice40", size, r)
