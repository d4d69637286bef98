"""Profiling driver: the bench's detailed (and optionally niceonly) hot path on
the 1e9 @ base 40 field, K repetitions, no CPU baseline.  Run under rocprofv3:
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt -- python scripts/prof_detailed.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("NICE_PROBE_LIB"):  # probe build (NICE_MSD_PROBE etc., scripts/gpu_msdprobe.sh)
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = sys.argv[2] if len(sys.argv) > 2 else "detailed"
base = int(sys.argv[3]) if len(sys.argv) > 3 else 40
size = int(float(sys.argv[4])) if len(sys.argv) > 4 else 10 ** 9
ctx = N.GpuContext(0)
s = N.get_base_range_u128(base).range_start
for i in range(reps):
    t = time.perf_counter()
    if mode in ("detailed", "both"):
        h, l = ctx.detailed_raw(s, s + size, base)
        ks = ctx.kernel_stats()
    if mode in ("niceonly", "both"):
        ctx.niceonly_raw(s, s + size, base)
    dt = time.perf_counter() - t
    print(f"rep {i}: {dt * 1e3:.3f} ms wall, kernel {ks.kernel_ms if mode != 'niceonly' else 0:.3f} ms",
          flush=True)
