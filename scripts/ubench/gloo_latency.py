"""Latency of one small gloo all-reduce (the field exchange vector, 129 + 2N
int64) among N local CPU processes: blocking, and with two operations in
flight (FieldPipeline's exchange lag 2).  No GPU is touched.

    python3 scripts/ubench/gloo_latency.py [N ...]"""
import sys
import os, time, torch, torch.distributed as dist, torch.multiprocessing as mp
def w(r, n, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=n)
    t = torch.zeros(129 + 2 * n, dtype=torch.int64)
    for _ in range(50): dist.all_reduce(t)
    dist.barrier(); t0 = time.perf_counter()
    for _ in range(500): dist.all_reduce(t)
    el = (time.perf_counter() - t0) / 500
    # async with work in flight
    dist.barrier(); t0 = time.perf_counter(); ws = []
    for _ in range(500):
        ws.append(dist.all_reduce(t, async_op=True))
        if len(ws) > 2: ws.pop(0).wait()
    for x in ws: x.wait()
    el2 = (time.perf_counter() - t0) / 500
    if r == 0: print(n, f"sync {el*1e6:.1f} us  async-lag2 {el2*1e6:.1f} us")
    dist.destroy_process_group()
if __name__ == "__main__":
    for n in [int(a) for a in sys.argv[1:]] or (2, 4, 8):
        mp.spawn(w, args=(n, 29611 + n), nprocs=n)
