"""Whole massive field (b50 1e13, device MSD, chunk 1e8) at one MSD floor on
one GPU, per value of a probe-build knob (probe library): median wall time
of 3 calls, candidates, ranges; every value must give the same nice list.
    python scripts/massive_knob.py KNOB V1,V2,... [floor=64]"""
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

knob, values = sys.argv[1], sys.argv[2].split(",")
fl = int(sys.argv[3]) if len(sys.argv) > 3 else 64
f = get_benchmark_field(BM.MASSIVE)
ctx = N.GpuContext(0)
ctx.niceonly_raw(f.range_start, f.range_start + 10 ** 11, 50)
for v in values:
    os.environ[knob] = v
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        lst, st = ctx.niceonly_raw(f.range_start, f.range_end, 50, chunk_size=10 ** 8, msd_floor=fl,
                                   msd_where="device")
        ts.append(time.perf_counter() - t)
    assert lst == []
    print(f"floor {fl} {knob}={v}: {statistics.median(ts) * 1e3:.1f} ms, candidates {st.candidates}, "
          f"ranges {st.ranges}", flush=True)
ctx.close()
