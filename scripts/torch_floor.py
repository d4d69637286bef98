"""Event-timed floor of a trivial kernel (one-element add) between two HIP
events on the current stream, for comparison with the library's small-field
kernel times (scripts/latency_probe.py)."""
import statistics

import torch

x = torch.zeros(1, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
v = []
for _ in range(300):
    e0.record()
    x.add_(1)
    e1.record()
    e1.synchronize()
    v.append(e0.elapsed_time(e1) * 1e3)
print(f"trivial kernel between two events: {statistics.median(v):.1f} us", flush=True)
