"""Phase breakdown of the fd2 detailed kernel on small fields (probe build,
per-workgroup s_memrealtime / s_memtime stamps, fd2_kernel.hpp FD2_STAMP):

    python scripts/fd2_stamps.py [BASE:SIZE ...]     (default 80:1e6 40:1e6)

Phases per workgroup (thread 0): 0 start, 1 lane state built and tables in LDS
(the init overlaps the table DMA), 2 cached high-limb mask done,
3 thread 0's steps done, 4 all waves' steps done (barrier), 5 histogram flushed,
6 end (the last workgroup: after the field finish); the finishing workgroup
also stamps 7 arrival known, 8 copies read and summed, 9 mapped stores
complete (then the release store of the sequence word).  Prints the kernel's event
time, the in-kernel span (first start to last end, 100 MHz real-time counter),
the workgroup start ramp, and per phase the median / max over workgroups in
shader cycles."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_lib  # noqa: E402,F401

import nice_amd as N  # noqa: E402
from nice_amd import _lib  # noqa: E402

L = _lib.lib()
L.nice_probe_fd2_stamps.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
L.nice_probe_fd2_stamps.restype = ctypes.c_int
L.nice_probe_fd2_last.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
GROUPS, WORDS = 65536, 32
cases = sys.argv[1:] or ["80:1e6", "40:1e6"]
ctx = N.GpuContext(0)
names = ["init+tables", "hi mask", "steps(t0)", "wait others", "flush", "finish/end"]
for c in cases:
    base, size = c.split(":")
    base, size = int(base), int(float(size))
    s = N.get_base_range_u128(base).range_start
    for _ in range(5):
        ctx.detailed_raw(s, s + size, base)
    ev = []
    for _ in range(5):
        ctx.detailed_raw(s, s + size, base)
        ev.append(ctx.kernel_stats().kernel_ms)
    assert L.nice_probe_fd2_stamps(1, None, 0) == 0
    ctx.detailed_raw(s, s + size, base)
    k_ms = ctx.kernel_stats().kernel_ms
    geo = (ctypes.c_uint64 * 6)()
    L.nice_probe_fd2_last(geo)
    buf = (ctypes.c_uint64 * (GROUPS * WORDS))()
    assert L.nice_probe_fd2_stamps(0, buf, GROUPS * WORDS) == 0
    wgs = []
    for b in range(GROUPS):
        w = buf[WORDS * b: WORDS * b + 20]
        if w[0] == 0:
            continue
        wgs.append((b, [w[2 * k] for k in range(10)], [w[2 * k + 1] for k in range(10)]))
    rt0 = min(x[1][0] for x in wgs)
    rt_end = max(x[1][6] for x in wgs)
    starts = sorted(x[1][0] - rt0 for x in wgs)
    print(f"b{base} {size:.0e}: {len(wgs)} workgroups; kernel (events) {k_ms * 1e3:.1f} us "
          f"(unstamped runs {statistics.median(ev) * 1e3:.1f} us); in-kernel span "
          f"{(rt_end - rt0) * 10 / 1e3:.1f} us; workgroup starts: median +{statistics.median(starts) * 10 / 1e3:.1f} us, "
          f"last +{starts[-1] * 10 / 1e3:.1f} us")
    print(f"   last launch: grid {geo[0]} x {geo[1]} threads, chunk {geo[2]}, {geo[3]} chunks + "
          f"{geo[4]} tail numbers, {geo[5]} workgroup(s) per CU")
    for k in range(6):
        d = [x[2][k + 1] - x[2][k] for x in wgs if x[2][k + 1] and x[2][k]]
        if not d:
            continue
        print(f"   {names[k]:12s} cycles median {statistics.median(d):9.0f}  max {max(d):9.0f}  "
              f"({statistics.median(d) / 2.4e3:.2f} / {max(d) / 2.4e3:.2f} us at 2.4 GHz)")
    ends = sorted((x[1][5] - rt0) * 10 / 1e3 for x in wgs)
    last = max(wgs, key=lambda x: x[1][6])
    print(f"   flushes done: median +{statistics.median(ends):.1f} us, last +{ends[-1]:.1f} us; "
          f"finishing workgroup {last[0]} ends +{(last[1][6] - rt0) * 10 / 1e3:.1f} us")
    r = last[1]
    if r[7] and r[8] and r[9]:
        us = lambda x, y: (y - x) * 10 / 1e3  # noqa: E731
        print(f"   finish of workgroup {last[0]}: flush -> arrival known {us(r[5], r[7]):.2f} us, "
              f"copies summed {us(r[7], r[8]):.2f} us, mapped stores complete {us(r[8], r[9]):.2f} us, "
              f"release store {us(r[9], r[6]):.2f} us")
ctx.close()
