"""Timeline of a rocprofv3 kernel trace (CSV): per kernel name the count and
mean duration, plus the fraction of the traced interval during which at least
one fd2 (detailed) kernel was running, and the gaps between them.

    python scripts/trace_timeline.py gpurun_out/prof/kt_kernel_trace.csv [skip_first_s]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
ks.sort()
t0 = ks[0][0]
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
ks = [k for k in ks if (k[0] - t0) / 1e9 >= skip]
by = defaultdict(list)
for s, e, n in ks:
    short = n.split("(")[0][:90]
    by[short].append((e - s) / 1e3)
for n, v in sorted(by.items(), key=lambda x: -sum(x[1])):
    print(f"{len(v):6d} x {sum(v)/len(v):9.2f} us  total {sum(v)/1e3:9.3f} ms  {n}")
det = [(s, e) for s, e, n in ks if "fd2_kernel" in n or "fd2_tail" in n]
if det:
    # union of detailed busy intervals over the steady part
    lo, hi = det[0][0], max(e for _, e in det)
    busy, cur_s, cur_e = 0, det[0][0], det[0][1]
    gaps = []
    for s, e in det[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e) / 1e3)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"detailed busy {busy/1e6:.3f} ms of {(hi-lo)/1e6:.3f} ms ({busy/(hi-lo):.3f}); "
          f"{len(gaps)} gaps, total {sum(gaps)/1e3:.3f} ms, max {max(gaps) if gaps else 0:.1f} us")
