"""Host timestamps of the field pipeline over a strong-scaling shard (a
1.25e8 piece of the b40 field, as one rank of eight): the time each step()
returns and the drain, to locate the fixed cost of a short timed region.
    python scripts/step_trace.py [steps=40]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ctx = N.GpuContext([0])
br = N.get_base_range_u128(40)
field = N.FieldSize(br.range_start, br.range_start + 125 * 10 ** 6)
pipe = D.FieldPipeline(ctx, ctx, None, depth=2)
for rep in range(3):
    for _ in range(5):
        pipe.step(field, 40)
    pipe.drain()
    t0 = time.perf_counter()
    ts = []
    for _ in range(steps):
        pipe.step(field, 40)
        ts.append(time.perf_counter())
    pipe.drain()
    t1 = time.perf_counter()
    d = [(b - a) * 1e3 for a, b in zip([t0] + ts[:-1], ts)]
    print(f"rep {rep}: total {(t1 - t0) * 1e3:.3f} ms = {steps} steps; step ms first 6 "
          f"{[round(x, 3) for x in d[:6]]}, median {sorted(d)[len(d) // 2]:.3f}, last 3 "
          f"{[round(x, 3) for x in d[-3:]]}, drain {(t1 - ts[-1]) * 1e3:.3f}", flush=True)
