"""Small-field latency: wall and kernel time of the default (b40 1e6) and
hi-base (b80 1e6) fields, median of 20 calls (NICE_FD2_MINCHUNK sweeps the FD
chunk floor)."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401  (knobs exist only in the probe build)
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
for base in (40, 80):
    s = N.get_base_range_u128(base).range_start
    ctx.detailed_raw(s, s + 10 ** 6, base)
    w, k = [], []
    for _ in range(20):
        t = time.perf_counter()
        h, _ = ctx.detailed_raw(s, s + 10 ** 6, base)
        w.append((time.perf_counter() - t) * 1e3)
        k.append(ctx.kernel_stats().kernel_ms)
        assert sum(h) == 10 ** 6
    print(f"minchunk={os.environ.get('NICE_FD2_MINCHUNK', '32')} b{base} 1e6: wall {statistics.median(w):.4f} ms "
          f"kernel {statistics.median(k):.4f} ms", flush=True)
