"""b40 1e9 niceonly (client chunk 1e6): the fused per-chunk MSD + candidate
kernel (default for chunk / floor <= 16384) against the wave path (probe
build, NICE_MSD_FCAP=0), wall time of the library call, median of 20.
    python scripts/fused_vs_wave.py"""
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
s = N.get_base_range_u128(40).range_start
for size, tag in ((10 ** 9, "1e9"), (125 * 10 ** 6, "1.25e8 (an 8-way share)")):
    for fcap in ("", "0"):
        if fcap:
            os.environ["NICE_MSD_FCAP"] = fcap
        else:
            os.environ.pop("NICE_MSD_FCAP", None)
        ctx.niceonly_raw(s, s + size, 40)
        ts = []
        for _ in range(20):
            t = time.perf_counter()
            lst, st = ctx.niceonly_raw(s, s + size, 40)
            ts.append(time.perf_counter() - t)
        print(f"b40 {tag} {'wave' if fcap else 'fused'}: {statistics.median(ts) * 1e3:.3f} ms, "
              f"candidates {st.candidates}, square_ok {st.square_ok}, launches {st.launches}", flush=True)
