"""Occupancy and stall shares per FD kernel configuration from the two
rocprofv3 --pmc passes of scripts/ubench/pmc_sib.sh (pmcs_TAG_1, pmcs_TAG_2).

Per kernel (Cfg<...> template arguments), summed over its dispatches:
  waves/SIMD      SQ_WAVE_CYCLES x 4 (quad-cycles) / (kernel cycles x CUs x 4 SIMDs),
                  kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md)
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / barrier)
  wait_inst_any   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (ready, not issued: pipe busy or dependency)
  active_any      SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  wait_inst_lds   SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES   (LDS issue stall, part of wait_inst_any)
  LDS busy        SQ_LDS_IDX_ACTIVE / (CUs x kernel cycles)
  VALU / LDS instr per wave-step (64 numbers) with --numbers N

    python scripts/ubench/occupancy_ab.py --numbers 1e9 gpurun_out/pmcs_TAG_1 gpurun_out/pmcs_TAG_2 ..."""
import collections
import csv
import glob
import os
import re
import sys

CUS = 256
numbers = 0.0
args = sys.argv[1:]
if args and args[0] == "--numbers":
    numbers = float(args[1])
    args = args[2:]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in args:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "fd2_kernel" not in name:
                continue
            m = re.search(r"Cfg<([^>]*)>", name)
            key = m.group(1) if m else name
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[key].add((d, r["Dispatch_Id"]))
for key, c in tot.items():
    nd = max(1, len(disp[key]) // max(1, len(args)))
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 / nd
    wc = c.get("SQ_WAVE_CYCLES", 0)
    print(f"== Cfg<{key}>  ({nd} dispatch(es) per pass)")
    if cyc and wc:
        print(f"  kernel cycles {cyc:.4g}; waves/SIMD {wc / nd * 4 / (cyc * CUS * 4):.2f}")
    if wc:
        fr = {k: c.get(v, 0) / wc for k, v in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                                                ("active_any", "SQ_ACTIVE_INST_ANY"),
                                                ("wait_inst_lds", "SQ_WAIT_INST_LDS"),
                                                ("active_valu", "SQ_ACTIVE_INST_VALU"),
                                                ("active_lds", "SQ_ACTIVE_INST_LDS"))}
        print("  wave-cycle fractions: " + " ".join(f"{k} {v:.3f}" for k, v in fr.items()))
    if cyc and c.get("SQ_LDS_IDX_ACTIVE"):
        print(f"  LDS busy {c['SQ_LDS_IDX_ACTIVE'] / nd / (CUS * cyc):.3f}; LDS cycles per instr "
              f"{c['SQ_LDS_IDX_ACTIVE'] / max(1, c.get('SQ_INSTS_LDS', 0)):.2f} (conflict share "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f})")
    if numbers and c.get("SQ_INSTS_VALU"):
        ws = numbers / 64
        print(f"  per wave-step: VALU {c['SQ_INSTS_VALU'] / nd / ws:.1f} LDS {c.get('SQ_INSTS_LDS', 0) / nd / ws:.1f} "
              f"SALU {c.get('SQ_INSTS_SALU', 0) / nd / ws:.1f}")
