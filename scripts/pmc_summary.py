"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel-name substring,
sum each counter over dispatches and print per-dispatch averages.  With
--numbers N (numbers per dispatch) also the per-wave-step figures (a
wave-step = 64 numbers): VALU / LDS instructions per wave-step and LDS
cycles (SQ_LDS_IDX_ACTIVE) and bank-conflict cycles per LDS instruction.

    python scripts/pmc_summary.py [--numbers N] KERNEL_SUBSTRING CSV..."""
import collections
import csv
import sys

numbers = 0
if sys.argv[1] == "--numbers":
    numbers = float(sys.argv[2])
    del sys.argv[1:3]
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
if numbers:
    ws = numbers / 64
    per = {k: v / n for k, v in tot.items()}
    if "SQ_INSTS_VALU" in per and "SQ_INSTS_LDS" in per:
        print(f"VALU instr per wave-step (64 n) {per['SQ_INSTS_VALU'] / ws:.1f}; "
              f"LDS instr per wave-step {per['SQ_INSTS_LDS'] / ws:.1f}")
    if "SQ_LDS_IDX_ACTIVE" in per and per.get("SQ_INSTS_LDS"):
        print(f"LDS cycles / LDS instr {per['SQ_LDS_IDX_ACTIVE'] / per['SQ_INSTS_LDS']:.2f} "
              f"(conflict {per.get('SQ_LDS_BANK_CONFLICT', 0) / per['SQ_INSTS_LDS']:.2f}); "
              f"conflict cycles per wave-step {per.get('SQ_LDS_BANK_CONFLICT', 0) / ws:.1f}")
