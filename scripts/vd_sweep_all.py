"""VALU-decoded limb sweep over every FD base (probe build, NICE_FD2_VD =
100 + VD): median kernel ms of the 1e9 field at the range start per variant;
each must reproduce the production library's results.

    python scripts/vd_sweep_all.py [bases...]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

ctx = N.GpuContext(0)
bases = [int(x) for x in sys.argv[1:]] or [b for b in range(2, 129) if N._lib.lib().nice_fd_kernel_base(b)]
for base in bases:
    s = N.get_base_range_u128(base).range_start
    os.environ["NICE_FD2_VD"] = "0"
    ref = ctx.detailed_raw(s, s + 10 ** 9, base)
    row = []
    vds = [int(x) for x in os.environ.get("VDS", "100,101,102,103,117,0").split(",")]
    for vd in vds:
        os.environ["NICE_FD2_VD"] = str(vd)
        out = ctx.detailed_raw(s, s + 10 ** 9, base)
        ts = []
        for _ in range(4):
            ctx.detailed_raw(s, s + 10 ** 9, base)
            ts.append(ctx.kernel_stats().kernel_ms)
        row.append(f"{'prod' if vd == 0 else vd - 100}:{statistics.median(ts):.3f}{'' if out == ref else '!MISMATCH'}")
    print(f"b{base} " + "  ".join(row), flush=True)
