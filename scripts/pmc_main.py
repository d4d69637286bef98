"""Per-dispatch PMC values of the largest launch of a kernel (rocprofv3 --pmc
CSVs), with derived rates: LDS cycles per LDS instruction, VALU per wave-step."""
import collections
import csv
import sys

pat, files = sys.argv[1], sys.argv[2:]
vals = {}
dur = None
for f in files:
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            d = rows[(int(r["Grid_Size"]), r["Dispatch_Id"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    big = max(rows)
    vals.update(rows[big])
for k, v in sorted(vals.items()):
    print(f"{k:24s} {v:14.4g}")
if "SQ_INSTS_LDS" in vals and "SQ_LDS_IDX_ACTIVE" in vals:
    print(f"LDS cycles / LDS instr   {vals['SQ_LDS_IDX_ACTIVE'] / vals['SQ_INSTS_LDS']:.2f}"
          f"  (conflict {vals['SQ_LDS_BANK_CONFLICT'] / vals['SQ_INSTS_LDS']:.2f})")
