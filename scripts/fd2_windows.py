"""Histogram windows of the FD kernel per base (fd2_kernel.hpp Cfg::W0/W):
the unique-count distribution of in-range n sampled uniformly (the oracle's
num_unique_digits), and for a window width W the start W0 that covers the
most mass with W0 + W <= cutoff + 1 (every near-miss must fall outside the
window: it is recorded on the out-of-window branch).  Prints the table the
kernel's constexpr window() carries.

    python scripts/fd2_windows.py [samples]
"""
import random
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

n_samples = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
rng = random.Random(1)
rows = []
for b in range(40, 81):
    r = O.base_range(b)
    if not r:
        continue
    s, e = r
    h = [0] * (b + 1)
    for _ in range(n_samples):
        h[O.num_unique_digits(s + rng.randrange(e - s), b)] += 1
    cut = O.near_miss_cutoff(b)
    W = 15 if b <= 45 else (18 if b <= 70 else 28)
    best = max(range(0, cut + 2 - W), key=lambda w0: sum(h[w0:w0 + W]))
    out = 1 - sum(h[best:best + W]) / n_samples
    mean = sum(i * c for i, c in enumerate(h)) / n_samples
    rows.append((b, W, best, out, mean))
    print(f"b{b}: mean {mean:.2f} W {W} W0 {best} outside {out:.2e}", file=sys.stderr)
print(" ".join(f"{b}:{W0}/{W}" for b, W, W0, _, _ in rows))
