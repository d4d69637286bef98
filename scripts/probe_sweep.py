"""Time the production FD kernel against its bottleneck probes
(NICE_FD2_PROBE, fd2_detailed.hip) on the b40 1e9 benchmark field."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
s = N.get_base_range_u128(40).range_start
for probe in (0, 1, 2, 3, 6, 0):
    os.environ["NICE_FD2_PROBE"] = str(probe)
    ctx.detailed_raw(s, s + 10 ** 9, 40)
    ts = []
    for _ in range(3):
        ctx.detailed_raw(s, s + 10 ** 9, 40)
        ts.append(ctx.kernel_stats().kernel_ms)
    print(f"probe {probe}: {sorted(ts)[1]:.3f} ms", flush=True)
