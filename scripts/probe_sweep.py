"""Time the production FD kernel against its bottleneck probes and variants
(NICE_FD2_PROBE, fd2_detailed.hip) on the b40 1e9 benchmark field; variants
that compute real results (0, 6, 8, 9) are checked against probe 0.

  python scripts/probe_sweep.py [probe ...]     (default: 0 1 2 3 6 0)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401  (knobs exist only in the probe build)
import nice_amd as N  # noqa: E402

EXACT = {0, 5, 6, 7, 8, 9}
ctx = N.GpuContext(0)
s = N.get_base_range_u128(40).range_start
probes = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3, 6, 0]
ref = None
for probe in probes:
    os.environ["NICE_FD2_PROBE"] = str(probe)
    out = ctx.detailed_raw(s, s + 10 ** 9, 40)
    res = (list(out[0]), sorted(out[1]))
    if probe == 0 and ref is None:
        ref = res
    ts = []
    for _ in range(5):
        ctx.detailed_raw(s, s + 10 ** 9, 40)
        ts.append(ctx.kernel_stats().kernel_ms)
    match = "" if probe not in EXACT or ref is None else f"  match={res == ref}"
    print(f"probe {probe}: {sorted(ts)[2]:.3f} ms{match}", flush=True)
