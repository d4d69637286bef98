"""Throughput of detailed 1e9 @ b40 fields with 1 vs 2 host slots (each slot a
thread with its own GpuContext / stream, alternating fields): does keeping a
second field queued hide the host turnaround and the persistent grid's ragged
end?  Also both modes (BothModes per slot)."""
import os
import sys
import threading
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402

s = N.get_base_range_u128(40).range_start
F = 10 ** 9
K = 40


def run(slots, mode):
    runners = []
    for _ in range(slots):
        ctx = N.GpuContext(0)
        runners.append(N.BothModes(0, det_ctx=ctx) if mode == "both" else ctx)

    def work(r, n):
        for _ in range(n):
            if mode == "both":
                (h, _), _ = r.both_raw((s, s + F), (s, s + F), 40)
            else:
                h, _ = r.detailed_raw(s, s + F, 40)
            assert sum(h) == F

    for r in runners:
        work(r, 1)
    t = time.perf_counter()
    th = [threading.Thread(target=work, args=(r, K // slots)) for r in runners]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    for r in runners:
        if mode == "both":
            r.close()
    print(f"{mode} slots={slots}: {dt / K * 1e3:.3f} ms per field", flush=True)


for mode in ("detailed", "both"):
    for slots in (1, 2, 1, 2):
        run(slots, mode)
