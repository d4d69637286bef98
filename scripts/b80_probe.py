"""b80 FD kernel variants (NICE_FD2_PROBE=20: the 512-thread (small-field)
workgroups, 2 waves per SIMD) against production (1024 threads) on the b80
benchmark field (2e8 and 1e9): median kernel ms of 5 calls, results compared
with the first probe's."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401  (knobs exist only in the probe build)
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
s = N.get_base_range_u128(80).range_start
probes = [int(x) for x in sys.argv[1:]] or [0, 20, 0, 20]
ref = {}
for probe in probes:
    os.environ["NICE_FD2_PROBE"] = str(probe)
    for size in (2 * 10 ** 8, 10 ** 9):
        h, l = ctx.detailed_raw(s, s + size, 80)
        res = (list(h), sorted(l))
        ref.setdefault(size, res)
        ks = []
        for _ in range(5):
            ctx.detailed_raw(s, s + size, 80)
            ks.append(ctx.kernel_stats().kernel_ms)
        print(f"probe {probe} b80 {size:.0e}: {statistics.median(ks):.3f} ms  match={res == ref[size]}",
              flush=True)
