"""Host-side phases of the field pipeline (dist.FieldPipeline) on one GPU:
per step, the time in each library call (submit = enqueue only; collect
includes waiting for the field) and the step total, median over K steps.

    python scripts/pipeline_phases.py [field_size=1.25e8] [steps=60] [depth=2]
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402

size = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ctx = N.GpuContext(0)
s = N.get_base_range_u128(40).range_start
f = N.FieldSize(s, s + size)
T = {}


class Timed:
    def __init__(self, c):
        self.c = c

    def __getattr__(self, name):
        fn = getattr(self.c, name)

        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            T.setdefault(name, []).append((time.perf_counter() - t) * 1e6)
            return r
        return w


for mode in ("both", "detailed", "niceonly"):
    T.clear()
    tc = Timed(ctx)
    pipe = D.FieldPipeline(tc, tc, depth=depth)
    if mode == "detailed":
        pipe.nice = type("S", (), {"niceonly_submit": lambda *a, **k: None})()
    if mode == "niceonly":
        pipe.det = type("S", (), {"detailed_submit": lambda *a, **k: None})()
    for _ in range(5):
        pipe.step(f, 40)
    pipe.drain()
    T.clear()
    st = []
    t0 = time.perf_counter()
    for _ in range(steps):
        t = time.perf_counter()
        pipe.step(f, 40)
        st.append((time.perf_counter() - t) * 1e6)
    pipe.drain()
    wall = (time.perf_counter() - t0) / steps * 1e6
    print(f"[{mode}] size {size:.3g} depth {depth}: wall/step {wall:.1f} us, step median "
          f"{statistics.median(st):.1f} us")
    for k, v in T.items():
        print(f"   {k:18s} median {statistics.median(v):8.1f} us  mean {statistics.mean(v):8.1f}")
