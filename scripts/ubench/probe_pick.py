"""Pipelined fields of one size with the launcher's stride pick against the
same stride forced (nice_debug_force_sib_stride), alternated in one process:
ms per step, host time of detailed_submit, and the strides the fields ran.

    python3 scripts/ubench/probe_pick.py [SIZE ...]"""
import collections
import sys
import time

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402

ctx = N.GpuContext(0)
lib = N._lib.lib()
br = N.get_base_range_u128(40)
sub_t = [0.0]
orig = ctx.detailed_submit


def timed_submit(*a, **k):
    t = time.perf_counter()
    try:
        return orig(*a, **k)
    finally:
        sub_t[0] += time.perf_counter() - t


ctx.detailed_submit = timed_submit
for sz in [float(x) for x in sys.argv[1:]] or [2.5e8]:
    f = N.FieldSize(br.range_start, br.range_start + int(sz))
    pipe = D.FieldPipeline(ctx, ctx)
    for _ in range(5):
        pipe.step(f, 40)
    pipe.drain()
    auto_L = ctx.kernel_stats().sib_stride
    for rep in range(3):
        for L in (0, auto_L):
            assert lib.nice_debug_force_sib_stride(L) == 0
            seen = collections.Counter()
            for _ in range(3):
                pipe.step(f, 40)
            pipe.drain()
            ctx.synchronize()
            sub_t[0] = 0.0
            steps = max(10, int(6e9 // sz))
            t0 = time.perf_counter()
            for _ in range(steps):
                if pipe.step(f, 40) is not None:
                    seen[ctx.kernel_stats().sib_stride] += 1
            for _ in pipe.drain():
                seen[ctx.kernel_stats().sib_stride] += 1
            ctx.synchronize()
            el = (time.perf_counter() - t0) / steps * 1e3
            print(f"{sz:.3g} {'forced' if L else 'pick  '} L={L or auto_L}: {el:.4f} ms/step, "
                  f"submit {sub_t[0] / steps * 1e6:.1f} us/step, strides {dict(seen)}", flush=True)
lib.nice_debug_force_sib_stride(0)
ctx.close()
