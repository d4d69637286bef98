"""Per-step cost of the rank exchange (nice_amd/dist.py) under torchrun: the
fused all-reduce of [histogram, list counts] in isolation, 200 iterations."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from nice_amd import dist as D  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
vals = list(range(41 + 2 * dist.get_world_size()))
for _ in range(20):
    D._all_reduce_ints(vals, dist, None)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(200):
    D._all_reduce_ints(vals, dist, None)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 200
if dist.get_rank() == 0:
    print(f"all_reduce_ints: {dt * 1e6:.1f} us per call, world {dist.get_world_size()}", flush=True)
dist.destroy_process_group()
