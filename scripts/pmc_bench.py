"""Counter summary of the bench's dominant kernel from rocprofv3 --pmc passes of
the bench command itself (scripts/gpu.sh pmc TAG "COUNTERS" [bench args], one
counter group per pass), for bench.py's roofline.frac_hw:

    python scripts/pmc_bench.py --numbers 1e9 --out profiles/r03/pmc_bench.json \
        gpurun_out/pmc_bench_valu gpurun_out/pmc_bench_lds gpurun_out/pmc_bench_busy

Per-dispatch means over every fd2_kernel dispatch of every pass (warmup, timed
region and the isolated launches alike: the kernel is the same launch each
time).  Derived:
  valu_busy           VALUBusy / 100 (SQ_ACTIVE_INST_VALU over GRBM_GUI_ACTIVE x CUs; the
                      counter charges one cycle per instruction whatever its issue
                      rate, so it is not an issue-slot share and can pass 1)
  valu_issue_busy     the VALU issue-slot share: SQ_INSTS_VALU x (issue cycles per
                      VALU instruction of the kernel's hot-loop mix, --valu-cpi, from
                      scripts/isa/loop_budget.py on its ISA) / (4 SIMDs x CUs x
                      kernel_cycles) -- reconciled: <= 1 by construction of the
                      denominator, the SIMD cycles the kernel spans
  valu_lane_ops_per_n SQ_INSTS_VALU x 64 / numbers per dispatch
  lds_instr_per_n     SQ_INSTS_LDS x 64 / numbers
  lds_conflict_frac   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  kernel_cycles       GRBM_GUI_ACTIVE / XCDs (the CSV sums the 8 XCD instances;
                      VALUBusy's own expression takes their max)
  lds_busy            SQ_LDS_IDX_ACTIVE / CUs / kernel_cycles: the share of the
                      kernel's cycles the CU's one LDS pipe is busy (the counter
                      aggregates the SIMDs of each SE)
                      (the counter agrees with the CU's s_memtime span on the
                      kernel's own index traces for ds_read_b64 and b128:
                      scripts/ubench/lds_trace.hip, profiles/r04/lds_trace.log)
  lds_cycles_per_instr SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS (LDS cycles per wave64
                      LDS instruction; 4 is a conflict-free ds_read_b128)
  traffic_bytes       HBM bytes: FETCH_SIZE x 2 + WRITE_SIZE (KB -> B), separate passes
The output records the sha256 (16 hex digits) of the library profiled
(--lib, default nice_amd/libnice_hip.so): bench.py reports these figures only
while it loads that same library.
"""
import argparse
import collections
import hashlib
import csv
import glob
import json
import os

KERNEL = "fd2_kernel"

ap = argparse.ArgumentParser()
ap.add_argument("--numbers", type=float, required=True, help="numbers per fd2 dispatch")
ap.add_argument("--kernel", default=KERNEL)
ap.add_argument("--out", required=True)
ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "nice_amd", "libnice_hip.so"))
ap.add_argument("--cus", type=int, default=256)
ap.add_argument("--xcds", type=int, default=8)
ap.add_argument("--valu-cpi", type=float, default=None,
                help="issue cycles per VALU instruction of the hot loop (ISA budget)")
ap.add_argument("--valu-cpi-source", default=None, help="file the --valu-cpi figure comes from")
ap.add_argument("dirs", nargs="+", help="pass directories (rocprofv3 -d) or counter_collection CSV files")
a = ap.parse_args()

vals = collections.defaultdict(list)
names = set()
files = []
for d in a.dirs:
    # a pass's output directory, or a committed copy of its counter CSV
    paths = [d] if os.path.isfile(d) else sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                                                             recursive=True))
    for path in paths:
        files.append(path)
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if a.kernel in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                names.add(r["Kernel_Name"])
        for (_, c), v in per.items():
            vals[c].append(v)
if not vals:
    raise SystemExit(f"no {a.kernel} rows under {a.dirs}")
mean = {c: sum(v) / len(v) for c, v in vals.items()}
with open(a.lib, "rb") as fh:
    sha16 = hashlib.sha256(fh.read()).hexdigest()[:16]
out = {"kernel": sorted(names), "numbers_per_dispatch": a.numbers, "lib_sha16": sha16,
       "dispatches": {c: len(v) for c, v in vals.items()},
       "per_dispatch": {c: round(v, 4) for c, v in sorted(mean.items())},
       "files": [os.path.relpath(f) for f in files]}
der = {}
if "VALUBusy" in mean:
    der["valu_busy"] = mean["VALUBusy"] / 100
if "SQ_INSTS_VALU" in mean:
    der["valu_lane_ops_per_n"] = mean["SQ_INSTS_VALU"] * 64 / a.numbers
if "SQ_INSTS_LDS" in mean:
    der["lds_instr_per_n"] = mean["SQ_INSTS_LDS"] * 64 / a.numbers
if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
    der["lds_conflict_frac"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"]
if "GRBM_GUI_ACTIVE" in mean:
    der["kernel_cycles"] = mean["GRBM_GUI_ACTIVE"] / a.xcds
    if "SQ_LDS_IDX_ACTIVE" in mean:
        der["lds_busy"] = mean["SQ_LDS_IDX_ACTIVE"] / a.cus / der["kernel_cycles"]
    if "SQ_INSTS_VALU" in mean and a.valu_cpi:
        der["valu_issue_busy"] = mean["SQ_INSTS_VALU"] * a.valu_cpi / (4 * a.cus * der["kernel_cycles"])
        der["valu_cpi"] = a.valu_cpi
        der["valu_cpi_source"] = a.valu_cpi_source
if "SQ_LDS_IDX_ACTIVE" in mean and mean.get("SQ_INSTS_LDS"):
    der["lds_cycles_per_instr"] = mean["SQ_LDS_IDX_ACTIVE"] / mean["SQ_INSTS_LDS"]
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    # HBM bytes per dispatch: FETCH_SIZE doubled (gfx950 tallies 128-B requests
    # at 64 B, MI355X_MICROARCH.md), WRITE_SIZE as read; both in KB
    der["traffic_bytes"] = int(round((2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024))
out["derived"] = der
with open(a.out, "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(der))
