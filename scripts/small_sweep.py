"""Small-field latency sweep (probe build): b40 / b80 1e6 fields, median wall
and kernel time of the library call for small-field workgroup size (512 vs
the base's big size, NICE_FD2_SMALL) x minimum chunk (NICE_FD2_MINCHUNK)."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
for base in (40, 80):
    s = N.get_base_range_u128(base).range_start
    ref = None
    for small in ("10000000", "1"):
        for mc in ("2", "4", "8", "16", "32"):
            os.environ["NICE_FD2_SMALL"] = small
            os.environ["NICE_FD2_MINCHUNK"] = mc
            out = ctx.detailed_raw(s, s + 10 ** 6, base)
            ref = ref or out
            w, k = [], []
            for _ in range(15):
                t = time.perf_counter()
                ctx.detailed_raw(s, s + 10 ** 6, base)
                w.append((time.perf_counter() - t) * 1e3)
                k.append(ctx.kernel_stats().kernel_ms)
            print(f"b{base} 1e6 wg={'512' if small != '1' else 'big'} minchunk={mc}: wall "
                  f"{statistics.median(w):.4f} ms kernel {statistics.median(k):.4f} ms match={out == ref}",
                  flush=True)
