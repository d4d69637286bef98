"""The pipelined bench step with the context's per-field HIP-event timing on
(bench.py's default: two timestamped events per detailed field) against off,
alternated in one process: ms per step at 1.25e8 / 2.5e8 / 1e9.

    python3 scripts/ubench/timing_ab.py"""
import sys
import time

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402

ctx = N.GpuContext(0)
br = N.get_base_range_u128(40)
for sz in (1.25e8, 2.5e8, 1e9):
    f = N.FieldSize(br.range_start, br.range_start + int(sz))
    steps = max(20, int(2e10 // sz))
    res = {True: [], False: []}
    for rep in range(3):
        for on in (True, False):
            ctx.set_kernel_timing(on)
            pipe = D.FieldPipeline(ctx, ctx)
            for _ in range(5):
                pipe.step(f, 40)
            pipe.drain()
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                pipe.step(f, 40)
            pipe.drain()
            ctx.synchronize()
            res[on].append((time.perf_counter() - t0) / steps * 1e3)
    print(f"{sz:.3g}: timing on {sorted(res[True])[1]:.4f} ms/step, off {sorted(res[False])[1]:.4f}", flush=True)
ctx.set_kernel_timing(True)
ctx.close()
