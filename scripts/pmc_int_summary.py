"""Summarise the integer-issue PMC passes (scripts/gpu_pmc_int.sh) for the
main fd2 launch of the b40 1e9 field: counters per dispatch, integer VALU
instructions per wave-step (64 numbers), integer lane-ops per number next to
W_alg = 160, and rocprof's own VALUBusy / VALUUtilization.

    python scripts/pmc_int_summary.py gpurun_out/pmc_int_*/*counter_collection.csv
"""
import collections
import csv
import sys

KERNEL = "fd2_kernel<nice::fd2::Cfg<40, 4, 8, 5"
FIELD = 10 ** 9
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((path, r["Dispatch_Id"]))
per = {k: v / max(1, len(disp[k])) for k, v in tot.items()}
print(f"# b40 1e9 field, main fd2 launch ({KERNEL}...>), per dispatch")
for k in sorted(per):
    print(f"{k:24s} {per[k]:14.4g}   ({len(disp[k])} dispatches)")
steps = FIELD / 64
if "SQ_INSTS_VALU_INT32" in per:
    i32, i64 = per["SQ_INSTS_VALU_INT32"], per.get("SQ_INSTS_VALU_INT64", 0.0)
    print(f"int32 VALU instr per wave-step (64 n)   {i32 / steps:8.2f}")
    print(f"int64 VALU instr per wave-step (64 n)   {i64 / steps:8.2f}")
    print(f"all VALU instr per wave-step (64 n)     {per['SQ_INSTS_VALU'] / steps:8.2f}")
    print(f"integer lane-ops per n (ValuIops / n)   {(i32 + i64) * 64 / FIELD:8.2f}  (W_alg = 160)")
if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per:
    print(f"active lanes per VALU instr             "
          f"{per['SQ_THREAD_CYCLES_VALU'] / per['SQ_ACTIVE_INST_VALU']:8.2f}  (of 64)")
