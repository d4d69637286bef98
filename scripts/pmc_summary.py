"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel-name substring,
sum each counter over dispatches and print per-dispatch averages."""
import collections
import csv
import sys

pat = sys.argv[1]
tot = collections.defaultdict(float)
disp = set()
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        if pat in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add((path, r["Dispatch_Id"]))
n = max(1, len({d for d in disp}) // max(1, len(sys.argv) - 2))
print(f"dispatches per file: {n}")
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v / n:14.4g}")
