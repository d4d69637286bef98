"""Fused MSD wave kernel: roots per wave (probe build, NICE_MSD_ROOTS) against
the massive field whole and one 1/8 dealt share (the slowest of ranks 0, 1):
wall times, which must keep the fixture's totals.
    python scripts/roots_sweep.py 8 32 128"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402

f = get_benchmark_field(BM.MASSIVE)
ctx = N.GpuContext(0)
ctx.niceonly_raw(f.range_start, f.range_start + 10 ** 11, 50)


def med(**kw):
    ts, out = [], None
    for _ in range(3):
        t = time.perf_counter()
        out = ctx.niceonly_raw(f.range_start, f.range_end, 50, **kw)
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), out


for r in sys.argv[1:]:
    os.environ["NICE_MSD_ROOTS"] = r
    t1, (lst, st) = med()
    ok = (st.candidates, st.ranges, lst) == (7_480_186_005, 166_585_582, [])
    sh = [med(deal_stride=8, deal_offset=k)[0] for k in range(2)]
    print(f"roots/wave {r}: whole {t1:.4f} s match={ok}; 1/8 shares {sh[0]:.4f} {sh[1]:.4f} s; "
          f"projected eff {t1 / (8 * max(sh)):.3f}", flush=True)
