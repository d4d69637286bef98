"""configs_1gpu.jsonl = the configs run (scripts/bench_configs.py) plus one line
per small config from the C-host latency run (scripts/c_host_latency.sh):

    python scripts/c_host_lines.py gpurun_out/configs.jsonl gpurun_out/c_host_latency.txt \
        > profiles/r04/configs_1gpu.jsonl
"""
import json
import re
import sys

configs, latency = sys.argv[1], sys.argv[2]
txt = open(latency).read()
d = {}
for b, kind, med, mn, k in re.findall(r"== b(\d+) 1e6 (timed|kernel timing off)\nrepeat 300: wall per call "
                                      r"median ([\d.]+) us, min ([\d.]+) us(?:; kernel median ([\d.]+) us)?", txt):
    d.setdefault(int(b), {})[kind] = (float(med), float(mn), float(k) if k else None)
for line in open(configs):
    if line.strip():
        sys.stdout.write(line if line.endswith("\n") else line + "\n")
for b, name in [(40, "default"), (80, "hi-base-1e6")]:
    t, u = d[b]["timed"], d[b]["kernel timing off"]
    print(json.dumps({
        "config": name, "host": "C (examples/nice_field.c --repeat 300, no Python)", "mode": "detailed",
        "base": b, "size": 1000000, "wall_us_median_timed": t[0], "wall_us_min_timed": t[1],
        "kernel_us_median": t[2], "wall_us_median_untimed": u[0], "wall_us_min_untimed": u[1],
        "wall_minus_kernel_us_untimed": round(u[0] - t[2], 2),
        "note": "untimed = nice_ctx_set_kernel_timing(ctx, 0): no HIP events per field; kernel = HIP-event "
                "time of the timed runs; source profiles/r04/c_host_latency.txt"}))
