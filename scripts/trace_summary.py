"""Dominant-kernel figures from a rocprofv3 --kernel-trace CSV of bench.py
(scripts/gpu.sh prof TAG), next to the bench line the same command printed:

    python scripts/trace_summary.py --isolated 10 --bench gpurun_out/prof_TAG.json \
        gpurun_out/prof_TAG/**/*kernel_trace.csv > profiles/r03/bench_trace_summary.json

  isolated_median_ms   median duration of the LAST `--isolated` fd2 dispatches: the
                       launches bench.py times alone for roofline.kernel_ms
  pipelined_*          the other fd2 dispatches (warmup, timed region, per-mode
                       regions): their mean span (consecutive fields overlap on the
                       slots' streams, so a span holds neighbours' work) and the
                       union of their intervals per dispatch (GPU time the kernel
                       occupies per field, <= the bench's ms_per_step)
"""
import argparse
import csv
import glob
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="fd2_kernel")
ap.add_argument("--isolated", type=int, default=10)
ap.add_argument("--bench", default=None, help="the bench JSON line of the profiled run")
ap.add_argument("csvs", nargs="+")
a = ap.parse_args()

rows = []
for pat in a.csvs:
    for path in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(path)):
            if a.kernel in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort()
if len(rows) <= a.isolated:
    raise SystemExit("not enough dispatches")
iso = rows[-a.isolated:]
pipe = rows[:-a.isolated]
union, cur_s, cur_e = 0, None, None
for s, e in pipe:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
out = {
    "kernel": a.kernel, "dispatches": len(rows),
    "mean_ms_all": statistics.mean((e - s) / 1e6 for s, e in rows),
    "isolated_dispatches": len(iso),
    "isolated_median_ms": statistics.median((e - s) / 1e6 for s, e in iso),
    "pipelined_dispatches": len(pipe),
    "pipelined_mean_span_ms": statistics.mean((e - s) / 1e6 for s, e in pipe),
    "pipelined_union_ms_per_dispatch": union / 1e6 / len(pipe),
}
if a.bench:
    line = json.loads(open(a.bench).read().strip().splitlines()[-1])
    out["bench"] = {"ms_per_step": line["ms_per_step"], "kernel_ms": line["roofline"]["kernel_ms"],
                    "frac": line["roofline"]["frac"]}
print(json.dumps(out, indent=1))
