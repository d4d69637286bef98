"""Massive benchmark field (b50, [start, start + 1e13), niceonly, device MSD,
client chunk 1e8) on one GPU at several MSD recursion floors (VERDICT r04
item 2): per floor the median wall time of `reps` whole-field calls, the
MSD-surviving ranges, the stride candidates, the square survivors and the
nice list.  A floor above 250 checks a superset of the candidates (the
reference GPU path's adaptive floor ranges 250..256 000,
client_process_gpu.rs:82-184), one below it a subset (the recursion
prunes deeper); the nice list must stay [].
    python scripts/massive_floor_sweep.py [reps=3] [floors=250,1000,...]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
floors = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [250, 1000, 4000, 16000, 64000, 256000]
f = get_benchmark_field(BM.MASSIVE)
ctx = N.GpuContext(0)
ctx.niceonly_raw(f.range_start, f.range_start + 10 ** 11, 50)  # warm-up (tables, code objects)
rows = []
base_cands = None
for fl in floors:
    ts, out = [], None
    for _ in range(reps):
        t = time.perf_counter()
        out = ctx.niceonly_raw(f.range_start, f.range_end, 50, chunk_size=10 ** 8, msd_floor=fl,
                               msd_where="device")
        ts.append(time.perf_counter() - t)
    lst, st = out
    if base_cands is None:
        base_cands = st.candidates
    row = {"floor": fl, "wall_s": statistics.median(ts), "wall_all_s": ts, "ranges": st.ranges,
           "candidates": st.candidates, "square_ok": st.square_ok, "nice": [str(x) for x in lst],
           "candidates_vs_floor_250": st.candidates / base_cands}
    rows.append(row)
    print(json.dumps(row), flush=True)
    assert lst == [], "a nice number in the massive field?"
    if fl >= floors[0]:
        assert st.candidates >= base_cands, "a larger floor must check a superset"
print(json.dumps({"config": "massive", "base": 50, "size": f.range_size, "chunk": 10 ** 8,
                  "msd_where": "device", "floors": rows}), flush=True)
