"""profiles/<round>/traffic.json from the FETCH_SIZE and WRITE_SIZE passes of
scripts/gpu_pmc.sh (separate rocprofv3 --pmc runs): the main fd2 launch's
per-dispatch HBM bytes, FETCH_SIZE doubled as MI355X_MICROARCH.md prescribes
for gfx950 (128-B requests tallied at 64 B), WRITE_SIZE as read; KB units.

  python scripts/traffic_json.py FETCH.csv WRITE.csv > profiles/r01/traffic.json"""
import csv
import json
import statistics
import sys

KERNEL = "fd2::fd2_kernel<nice::fd2::Cfg<40, 4, 8, 5, 0, 1024, 0>"  # the b40 1e9 field's launch


def per_dispatch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {path}")
    return statistics.mean(vals), len(vals)


fetch, nf = per_dispatch(sys.argv[1], "FETCH_SIZE")
write, nw = per_dispatch(sys.argv[2], "WRITE_SIZE")
out = {
    "kernel": "nice::fd2::fd2_kernel<Cfg<40,4,8,5>> (b40 1e9 field: one launch, tail and finish in it)",
    "fetch_size_kb": round(2 * fetch, 3),
    "write_size_kb": round(write, 3),
    "bytes_per_launch": int(round((2 * fetch + write) * 1024)),
    "dispatches": {"fetch": nf, "write": nw},
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
              "(scripts/gpu_pmc.sh), FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies "
              "128-B requests at 64 B); KB per dispatch; scripts/traffic_json.py",
    "source": [sys.argv[1], sys.argv[2]],
}
print(json.dumps(out, indent=1))
