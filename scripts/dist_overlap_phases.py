"""bench.py's torchrun step, decomposed (rank 0): BothModes.both_raw alone,
then with the pipelined exchange (process_field_both_pipelined), with and
without torch.distributed initialised.  Run plain and under torchrun."""
import os
import statistics
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

use_dist = "WORLD_SIZE" in os.environ
if use_dist:
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
else:
    local = 0
    if os.environ.get("TORCH_CUDA"):
        import torch
        torch.zeros(1, device="cuda")
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402

ctx = N.GpuContext([local])
both = N.BothModes(local, det_ctx=ctx)
s = N.get_base_range_u128(40).range_start
e = s + 10 ** 9


def med(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    return round(statistics.median(ts) * 1e3, 4)


tag = "dist" if use_dist else ("plain+torch" if os.environ.get("TORCH_CUDA") else "plain")
print(tag, "both_raw", med(lambda: both.both_raw((s, e), (s, e), 40)), flush=True)
print(tag, "detailed", med(lambda: ctx.detailed_raw(s, e, 40)), flush=True)
print(tag, "niceonly", med(lambda: ctx.niceonly_raw(s, e, 40)), flush=True)
print(tag, "sequential", med(lambda: ctx.both_raw((s, e), (s, e), 40)), flush=True)
if use_dist:
    ex = D.PipelinedExchange(dist)
    f = N.FieldSize(s, e)
    print(tag, "pipelined+both", med(lambda: D.process_field_both_pipelined(ex, f, 40, both)), flush=True)
    D.finish_both(ex, ex.drain())
    print(tag, "pipelined+seq", med(lambda: D.process_field_both_pipelined(ex, f, 40, ctx)), flush=True)
    D.finish_both(ex, ex.drain())
    dist.destroy_process_group()
both.close()
