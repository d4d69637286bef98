"""Sweep the FD kernel variants (NICE_FD_VARIANT) on large in-range fields:
kernel time (HIP events) and bit-exact agreement between variants."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401  (knobs exist only in the probe build)
import nice_amd as N  # noqa: E402

cfg = [(40, 10 ** 9), (50, 10 ** 9), (80, 2 * 10 ** 8)]
if os.environ.get("SWEEP_BASES"):
    keep = {int(b) for b in os.environ["SWEEP_BASES"].split(",")}
    cfg = [c for c in cfg if c[0] in keep]
variants = [int(v) for v in os.environ.get("SWEEP_VARIANTS", "0,1,2,3,8,9,10,11").split(",")]
reps = int(os.environ.get("SWEEP_REPS", "3"))
ctx = N.GpuContext(0)
res = {}
for base, size in cfg:
    s = N.get_base_range_u128(base).range_start
    ref = None
    for v in variants:
        os.environ["NICE_FD_VARIANT"] = str(v)
        out = ctx.detailed_raw(s, s + size, base)  # warm
        times = []
        for _ in range(reps):
            out2 = ctx.detailed_raw(s, s + size, base)
            times.append(ctx.kernel_stats().kernel_ms)
        ok = out == out2 and (ref is None or out == ref)
        if ref is None:
            ref = out
        t = sorted(times)[len(times) // 2]
        res[f"b{base}_v{v}"] = {"kernel_ms": t, "n_per_s": size / t * 1e3, "match": ok}
        print(f"b{base} v{v}: {t:.3f} ms  {size / t * 1e3:.3e} n/s  match={ok}", flush=True)
os.environ["NICE_FD_VARIANT"] = "0"
print(json.dumps(res))
