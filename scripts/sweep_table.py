"""Tabulate a knob_sweep.py log: one row per knob value, one column per
field, with the change against a baseline value.
    python scripts/sweep_table.py LOG KNOB BASELINE_VALUE"""
import collections
import re
import sys

path, knob, basev = sys.argv[1], sys.argv[2], sys.argv[3]
rows = collections.OrderedDict()
fields = []
for line in open(path):
    m = re.match(r"(b\d+ \S+) " + re.escape(knob) + r"=(\d+):\s+([\d.]+) us\s+match=(\w+)", line)
    if m:
        rows.setdefault(m.group(2), []).append((float(m.group(3)), m.group(4)))
        if m.group(2) == basev:
            fields.append(m.group(1))
base = rows[basev]
print("value " + " ".join(f"{f:>17s}" for f in fields))
for k, v in rows.items():
    print(f"{k:>5s} " + " ".join(f"{t:8.0f}{'' if ok == 'True' else '!'} ({t / b[0] - 1:+6.1%})"
                                 for (t, ok), b in zip(v, base)))
