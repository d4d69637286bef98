"""Wide bases: the big-field FD kernel's workgroup (1024 threads, 4 waves per
SIMD at the 128-VGPR cap, with spills) against 512 threads (2 waves per
SIMD, no spills), probe build NICE_FD2_WG512; 1e9 at the range start, median
kernel ms of 5.
    python scripts/wg512_ab.py 65 67 68 80"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
for b in map(int, sys.argv[1:]):
    s = N.get_base_range_u128(b).range_start
    out = []
    for wg in ("0", "1"):
        os.environ["NICE_FD2_WG512"] = wg
        ctx.detailed_raw(s, s + 10 ** 9, b)
        ks = []
        for _ in range(5):
            ctx.detailed_raw(s, s + 10 ** 9, b)
            ks.append(ctx.kernel_stats().kernel_ms)
        out.append(statistics.median(ks))
    print(f"b{b}: big-field WG {out[0]:.3f} ms, 512 {out[1]:.3f} ms", flush=True)
