"""Does the niceonly pass (MSD levels + candidate kernel, latency-bound small
launches) hide under the detailed kernel when the two run on separate
contexts (= separate HIP streams) of one GPU?  Times the bench step
(detailed + niceonly of the b40 1e9 field) sequentially and overlapped."""
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

a, b = N.GpuContext(0), N.GpuContext(0)
s = N.get_base_range_u128(40).range_start
e = s + 10 ** 9


def seq():
    h, near = a.detailed_raw(s, e, 40)
    nice, _ = a.niceonly_raw(s, e, 40)
    return h, nice


class Worker:
    def __init__(self):
        self.go, self.done = threading.Event(), threading.Event()
        self.res = None
        threading.Thread(target=self.run, daemon=True).start()

    def run(self):
        while True:
            self.go.wait()
            self.go.clear()
            self.res = b.niceonly_raw(s, e, 40)
            self.done.set()


w = Worker()


def ovl():
    w.done.clear()
    w.go.set()
    h, near = a.detailed_raw(s, e, 40)
    w.done.wait()
    return h, w.res[0]


def med(fn, reps=15):
    fn()
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e3, r


for name, fn in (("sequential", seq), ("overlapped", ovl), ("sequential", seq), ("overlapped", ovl)):
    ms, r = med(fn)
    print(f"{name}: {ms:.3f} ms  hist_sum={sum(r[0])} nice={r[1]}", flush=True)
