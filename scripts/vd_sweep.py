"""Sweep the VALU-decoded limb count of the FD kernel (probe build,
NICE_FD2_PROBE 30 + VD: VD % 16 top C limbs, VD / 16 top S limbs) on the
b80 1e9 hi-base field; every variant must reproduce production's results.

    python scripts/vd_sweep.py [probe ...]     (default: 0 31 32 33 34 36 47 48 0)"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

base = int(os.environ.get("VD_BASE", "80"))
ctx = N.GpuContext(0)
s = N.get_base_range_u128(base).range_start
probes = [int(x) for x in sys.argv[1:]] or [0, 31, 32, 33, 34, 36, 47, 48, 0]
ref = None
for probe in probes:
    os.environ["NICE_FD2_PROBE"] = str(probe)
    out = ctx.detailed_raw(s, s + 10 ** 9, base)
    if ref is None:
        ref = out
    ts = []
    for _ in range(5):
        ctx.detailed_raw(s, s + 10 ** 9, base)
        ts.append(ctx.kernel_stats().kernel_ms)
    print(f"b{base} probe {probe}: {statistics.median(ts):.3f} ms  match={out == ref}", flush=True)
