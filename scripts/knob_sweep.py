"""Sweep one probe-build knob of the FD kernel over values and fields; every
value must reproduce the first value's results (histogram and near-miss list).

    python scripts/knob_sweep.py KNOB V1,V2,... BASE:SIZE[:OFFSET] ...

e.g. NICE_FD2_LG 100000,0,8,12,1000 80:1e9 65:1e9 80:1e6  (OFFSET: fraction of
the base's valid range where the field starts, default 0 = range start).
Prints, per value and field, the median kernel time (HIP events) over
KNOB_ROUNDS (default 3) interleaved rounds of 3 calls, after one untimed call
of every value."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import probe_lib  # noqa: E402,F401
import nice_amd as N  # noqa: E402

knob, values, fields = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
ctx = N.GpuContext(0)
rounds = int(os.environ.get("KNOB_ROUNDS", "3"))
for f in fields:
    parts = f.split(":")
    base, size = int(parts[0]), int(float(parts[1]))
    r = N.get_base_range_u128(base)
    s = r.range_start + int((r.range_end - r.range_start) * float(parts[2])) if len(parts) > 2 else r.range_start
    # every value once, untimed, and checked against the first (the first
    # field of a base runs ~5 % slow whatever the value: a fixed order would
    # charge that to the first value), then KNOB_ROUNDS rounds over the values
    # in turn, 3 timed calls each; the median of a value's calls
    ref = None
    match = {}
    for v in values:
        os.environ[knob] = v
        out = ctx.detailed_raw(s, s + size, base)
        if ref is None:
            ref = out
        match[v] = out == ref
    ts = {v: [] for v in values}
    for _ in range(rounds):
        for v in values:
            os.environ[knob] = v
            for _ in range(3):
                ctx.detailed_raw(s, s + size, base)
                ts[v].append(ctx.kernel_stats().kernel_ms)
    for v in values:
        print(f"b{base} {size:.0e} {knob}={v}: {statistics.median(ts[v]) * 1e3:10.1f} us  "
              f"match={match[v]}", flush=True)
ctx.close()
