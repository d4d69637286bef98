"""Small-field host latency (probe build): median wall of the synchronous
detailed call and of its submit / collect halves, for b40 / b80 at 1e4..1e8,
with collect waiting by polling the published sequence word (NICE_SPIN=1,
default) or by the completion event (NICE_SPIN=0), with the context's kernel
timing on or off (--untimed: nice_ctx_set_kernel_timing(0), no HIP events per
field).  Also the cost of a ctypes no-op call (the Python binding's floor).
Usage:
    NICE_SPIN=0|1 python scripts/latency_probe.py [--product] [--untimed]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
if "--product" not in sys.argv:
    import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402
from nice_amd._lib import lib  # noqa: E402

REPS = 200
L = lib()
t = time.perf_counter()
for _ in range(10000):
    L.nice_gpu_batch_size()
noop_us = (time.perf_counter() - t) / 10000 * 1e6
tag = "product" if "--product" in sys.argv else \
    f"spin={os.environ.get('NICE_SPIN', '1')} nofin={os.environ.get('NICE_FD2_NOFIN', '0')} "\
    f"untimed={int('--untimed' in sys.argv)}"
print(f"[{tag}] ctypes no-op call: {noop_us:.2f} us", flush=True)
ctx = N.GpuContext(0)
if "--untimed" in sys.argv:
    ctx.set_kernel_timing(False)
for base, size in ((40, 10 ** 4), (40, 10 ** 6), (80, 10 ** 6), (40, 10 ** 8)):
    s = N.get_base_range_u128(base).range_start
    ref = ctx.detailed_raw(s, s + size, base)
    wall, sub, col, ker = [], [], [], []
    for _ in range(REPS):
        t0 = time.perf_counter()
        out = ctx.detailed_raw(s, s + size, base)
        wall.append(time.perf_counter() - t0)
        assert out == ref
        ker.append(ctx.kernel_stats().kernel_ms)
        t0 = time.perf_counter()
        tk = ctx.detailed_submit(s, s + size, base)
        t1 = time.perf_counter()
        out = ctx.detailed_collect(tk, base)
        t2 = time.perf_counter()
        sub.append(t1 - t0)
        col.append(t2 - t1)
    med = lambda v: statistics.median(v) * 1e6  # noqa: E731
    print(f"[{tag}] b{base} {size:.0e}: wall {med(wall):.1f} us = submit {med(sub):.1f} + collect "
          f"{med(col):.1f}; kernel {statistics.median(ker) * 1e3:.1f} us", flush=True)
ctx.close()
