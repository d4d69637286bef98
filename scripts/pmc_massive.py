"""msd_wave_kernel counters on the whole massive field (scripts/r05_measure.sh:
rocprofv3 --pmc passes of scripts/massive_1gpu.py -> gpurun_out/pmc_massive_sq,
pmc_massive_busy), with the field's totals from tests/golden/massive_b50.json and
its one-GPU wall time from the configs run:

    python scripts/pmc_massive.py --configs gpurun_out/configs.jsonl \
        --out profiles/r04/pmc_massive.json gpurun_out/pmc_massive_sq gpurun_out/pmc_massive_busy
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
ap.add_argument("--configs", required=True)
ap.add_argument("--floor", type=int, default=250, help="the MSD floor the passes ran at")
ap.add_argument("--cus", type=int, default=256)
ap.add_argument("--xcds", type=int, default=8)
ap.add_argument("--lib", default=os.path.join(ROOT, "nice_amd", "libnice_hip.so"))
ap.add_argument("dirs", nargs="+")
a = ap.parse_args()

vals, names, files = collections.defaultdict(list), set(), []
for d in a.dirs:
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        files.append(os.path.relpath(path, ROOT))
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if "msd_wave_kernel" in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                names.add(r["Kernel_Name"])
        for (_, c), v in per.items():
            vals[c].append(v)
m = {c: sum(v) / len(v) for c, v in vals.items()}
# floor 250: the field's totals from the oracle's fixture; other floors: the
# configs run's own row at that floor (massive-floor-F)
name = "massive" if a.floor == 250 else f"massive-floor-{a.floor}"
row = [json.loads(l) for l in open(a.configs) if json.loads(l)["config"] == name][0]
if a.floor == 250:
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "massive_b50.json")))
    cand = sum(w["candidates"] for w in fx["windows"])
    ranges = sum(w["ranges"] for w in fx["windows"])
else:
    cand, ranges = row["candidates"], row["msd_ranges"]
wall = row["wall_ms"]
cyc = m["GRBM_GUI_ACTIVE"] / a.xcds
with open(a.lib, "rb") as fh:
    sha16 = hashlib.sha256(fh.read()).hexdigest()[:16]
der = {"kernel_cycles": cyc, "kernel_ms_at_2_4GHz": cyc / 2.4e6, "valu_busy": m["VALUBusy"] / 100,
       "lds_busy": m["SQ_LDS_IDX_ACTIVE"] / a.cus / cyc,
       "lds_conflict_frac": m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"],
       "valu_lane_instr_per_candidate": m["SQ_INSTS_VALU"] * 64 / cand,
       "lds_instr_per_candidate": m["SQ_INSTS_LDS"] * 64 / cand,
       "whole_field_wall_ms": wall, "candidates_per_sec_whole_field_wall": cand / (wall / 1e3)}
out = {"kernel": sorted(names)[0] if names else None,
       "field": f"massive b50 [start, +1e13), client chunk 1e8, floor {a.floor}, device MSD",
       "lib_sha16": sha16, "candidates": cand, "msd_ranges": ranges,
       "per_dispatch": {c: round(v, 4) for c, v in sorted(m.items())}, "derived": der, "files": files,
       "note": "one dispatch of msd_wave_kernel runs the whole field's MSD recursion below the BFS root "
               "level AND every candidate test (DESIGN 3.3); the per-candidate figures therefore include "
               "the recursion; lds_busy = SQ_LDS_IDX_ACTIVE / CUs / kernel cycles"}
with open(a.out, "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(der))
