"""Per-base hardware bound of the FD detailed kernel from rocprofv3 --pmc passes
of `bench.py --base B --mode detailed` (scripts/r05_measure.sh: gpurun_out/
pmc_b{B}_sq and pmc_b{B}_busy), 1e9 at each base's range start:

    python scripts/pmc_bases.py --out profiles/r04/pmc_bases.json gpurun_out 40 52 53 54 64 65 80

Per base (per-dispatch means over every fd2_kernel dispatch of the passes):
  valu_busy           VALUBusy / 100 (can pass 1: the counter's normalisation
                      with fast-issue integer ops)
  lds_busy            SQ_LDS_IDX_ACTIVE / CUs / kernel cycles
  lds_conflict_frac   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  lds_cycles_per_instr SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS
  bound               the busier pipe and its busy fraction, the other pipe,
                      and co_bound when the other is >= 0.85 busy too
  lds_read            the table read of the base (ds_read_b64: 8-byte
                      entries, b40-64; ds_read_b128: 16-byte, b65-80)
The LDS counter is a measurement for both reads: on the kernel's own b40 / b80
index traces (scripts/ubench/lds_trace.hip) it reports 6.08 / 5.93 cycles per
ds_read_b64 and 11.4 per ds_read_b128, and the CU's s_memtime span (first
wave's start to last wave's end) gives 6.12 / 5.95 and 11.56 / 11.45
(profiles/r04/pmc_lds_trace.txt, lds_trace.log).
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--numbers", type=float, default=1e9)
ap.add_argument("--cus", type=int, default=256)
ap.add_argument("--xcds", type=int, default=8)
ap.add_argument("--lib", default=os.path.join(ROOT, "nice_amd", "libnice_hip.so"))
ap.add_argument("dir")
ap.add_argument("bases", nargs="+", type=int)
a = ap.parse_args()


def per_dispatch(paths):
    vals = collections.defaultdict(list)
    for path in paths:
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if "fd2_kernel" in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}, {c: len(v) for c, v in vals.items()}


with open(a.lib, "rb") as fh:
    sha16 = hashlib.sha256(fh.read()).hexdigest()[:16]
res = {"lib_sha16": sha16, "numbers_per_dispatch": a.numbers, "bases": {}}
for b in a.bases:
    paths = sorted(glob.glob(os.path.join(a.dir, f"pmc_b{b}_*", "**", "*counter_collection.csv"),
                             recursive=True))
    m, n = per_dispatch(paths)
    cyc = m["GRBM_GUI_ACTIVE"] / a.xcds
    ws = a.numbers / 64
    vb = m["VALUBusy"] / 100
    lb = m["SQ_LDS_IDX_ACTIVE"] / a.cus / cyc
    b128 = (b + 31) // 32 == 3
    (pipe, busy), (opipe, obusy) = sorted([("valu", vb), ("lds", lb)], key=lambda x: -x[1])
    res["bases"][str(b)] = {
        "valu_busy": round(vb, 4), "lds_busy": round(lb, 4),
        "lds_conflict_frac": round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4),
        "lds_cycles_per_instr": round(m["SQ_LDS_IDX_ACTIVE"] / m["SQ_INSTS_LDS"], 3),
        "valu_instr_per_wave_step": round(m["SQ_INSTS_VALU"] / ws, 2),
        "lds_instr_per_wave_step": round(m["SQ_INSTS_LDS"] / ws, 2),
        "kernel_cycles": round(cyc), "lds_read": "ds_read_b128" if b128 else "ds_read_b64",
        "bound": {"pipe": pipe, "busy": round(busy, 4), "other_pipe": opipe, "other_busy": round(obusy, 4),
                  "co_bound": obusy >= 0.85},
        "dispatches": n, "files": [os.path.relpath(p, ROOT) for p in paths]}
    print(b, json.dumps({k: v for k, v in res["bases"][str(b)].items() if k not in ("files", "dispatches")}))
with open(a.out, "w") as fh:
    json.dump(res, fh, indent=1)
