"""b80 detailed kernel time vs field size from the range start (per-n cost
check): median kernel ms of 5 reps for each size, and 1e9 as 5 pieces."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

base = int(sys.argv[1]) if len(sys.argv) > 1 else 80
ctx = N.GpuContext(0)
s = N.get_base_range_u128(base).range_start


def kern(a, n, reps=5):
    ts = []
    for _ in range(reps + 1):
        ctx.detailed_raw(a, a + n, base)
        ts.append(ctx.kernel_stats().kernel_ms)
    return statistics.median(ts[1:])


for n in (5e7, 1e8, 2e8, 4e8, 6e8, 8e8, 1e9):
    t = kern(s, int(n))
    print(f"b{base} {n:.0e}: {t:.3f} ms  {t / n * 1e9:.3f} ms per 1e9", flush=True)
tot = sum(kern(s + i * 2 * 10 ** 8, 2 * 10 ** 8) for i in range(5))
print(f"b{base} 1e9 as 5 x 2e8: {tot:.3f} ms", flush=True)
# (the chunk-length sweep is scripts/gridx_probe.sh, NICE_FD2_TCHUNK)
