"""Split of the fused wave kernel's time on the massive field (probe build):
NICE_MSD_PROBE=4 skips the candidate test (MSD recursion only; the candidate
count statistic still comes out, the nice list is not searched).
    python scripts/wave_split.py [floors=250]"""
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
floors = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [250]
for fl in floors:
    for probe in ("0", "4"):
        os.environ["NICE_MSD_PROBE"] = probe
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            lst, st = ctx.niceonly_raw(f.range_start, f.range_end, 50, chunk_size=10 ** 8, msd_floor=fl,
                                       msd_where="device")
            ts.append(time.perf_counter() - t)
        print(f"floor {fl} NICE_MSD_PROBE={probe}: {statistics.median(ts):.4f} s, candidates {st.candidates}, "
              f"ranges {st.ranges}", flush=True)
