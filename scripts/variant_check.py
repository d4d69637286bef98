"""Probe-build correctness check of FD kernel variants: for each value of a
knob, run fields against the production configuration (knob unset) and
report matches / errors per value (no timing).

    python scripts/variant_check.py KNOB V1,V2,... BASE:SIZE[:OFFSET] ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

knob, values, fields = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
ctx = N.GpuContext(0)
for f in fields:
    parts = f.split(":")
    base, size = int(parts[0]), int(float(parts[1]))
    r = N.get_base_range_u128(base)
    s = r.range_start + int((r.range_end - r.range_start) * float(parts[2])) if len(parts) > 2 else r.range_start
    os.environ.pop(knob, None)
    ref = ctx.detailed_raw(s, s + size, base)
    for v in values:
        os.environ[knob] = v
        try:
            out = ctx.detailed_raw(s, s + size, base)
            ok = out == ref
            diff = "" if ok else f" hist diff bins {[i for i in range(len(ref[0])) if ref[0][i] != out[0][i]]}"
            print(f"b{base} {size:.0e}@{parts[2] if len(parts) > 2 else 0} {knob}={v}: match={ok}{diff}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"b{base} {size:.0e} {knob}={v}: ERROR {e}", flush=True)
    os.environ.pop(knob, None)
ctx.close()
