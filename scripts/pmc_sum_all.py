"""Sum rocprofv3 --pmc counters over every dispatch of the kernels whose name
contains a substring (whole-run totals; VALUBusy-style ratios averaged,
weighted by dispatch): for runs of many short launches.
    python scripts/pmc_sum_all.py KERNEL_SUBSTRING CSV"""
import collections
import csv
import sys

pat, path = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
disp = set()
for r in csv.DictReader(open(path)):
    if pat in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
        disp.add(r["Dispatch_Id"])
print(f"# {pat}: {len(disp)} dispatches, totals over the run ({path.split('/')[-2]})")
for k, v in sorted(tot.items()):
    avg = k.endswith("Busy") or k.endswith("Utilization")
    print(f"{k:28s} {v / cnt[k] if avg else v:14.4g}{'  (mean per dispatch)' if avg else ''}")
