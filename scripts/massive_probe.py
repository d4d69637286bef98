"""Massive field (b50 1e13 niceonly, one GPU) under device-MSD batching
variants of the probe build (NICE_MSD_CPB chunks per batch, NICE_MSD_FCAP
fused per-chunk level capacity): wall time and totals, which must equal the
fixture's.  Run once per variant (the knobs are read per call)."""
import os
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
tag = f"cpb={os.environ.get('NICE_MSD_CPB', '-')} fcap={os.environ.get('NICE_MSD_FCAP', '-')}"
ts = []
for _ in range(3):
    t = time.perf_counter()
    lst, st = ctx.niceonly_raw(f.range_start, f.range_end, 50)
    ts.append(time.perf_counter() - t)
ok = (st.candidates, st.ranges, lst) == (7_480_186_005, 166_585_582, [])
print(f"{tag}: {min(ts):.4f} s (runs {', '.join(f'{x:.4f}' for x in ts)}), launches {st.launches}, "
      f"candidates {st.candidates}, ranges {st.ranges}, match={ok}", flush=True)
