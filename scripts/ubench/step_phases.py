"""Host time per pipelined field step, by phase (FieldPipeline of bench.py):
submit / collect of each mode, kernel_stats, the exchange vector, the
exchange itself, finish.  With WORLD_SIZE set in the environment (no
launcher) the process group comes up at world 1 on the exchange backend
given, so the exchange's host and device cost shows against the plain run.

    python3 scripts/ubench/step_phases.py [--exchange nccl|gloo|shm|none] [--lag L]"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--exchange", default="none", choices=["none", "nccl", "gloo", "shm"])
    ap.add_argument("--lag", type=int, default=1)
    ap.add_argument("--field-size", type=float, default=1.25e8)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    dist = group = ex = None
    if a.exchange != "none":
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        if a.exchange == "gloo":
            group = dist.new_group(backend="gloo")
    import nice_amd as N
    from nice_amd import dist as D
    if a.exchange == "shm":
        ex = D.ShmExchange(dist, lag=a.lag)
    T = collections.defaultdict(float)

    def wrap(obj, name, key=None):
        f = getattr(obj, name)

        def g(*args, **kw):
            t = time.perf_counter()
            try:
                return f(*args, **kw)
            finally:
                T[key or name] += time.perf_counter() - t
        setattr(obj, name, g)
    ctx = N.GpuContext([0])
    for m in ("detailed_submit", "detailed_collect", "niceonly_submit", "niceonly_collect", "kernel_stats"):
        wrap(ctx, m)
    wrap(D, "exchange_vector")
    wrap(D, "finish_both")
    br = N.get_base_range_u128(40)
    field = N.FieldSize(br.range_start, br.range_start + int(a.field_size))
    pipe = D.FieldPipeline(ctx, ctx, dist, group=group, lag=a.lag, exchange=ex)
    if pipe.ex is not None:
        wrap(pipe.ex, "submit", "exchange.submit")
    for _ in range(a.warmup):
        pipe.step(field, 40)
    pipe.drain()
    ctx.synchronize()
    T.clear()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pipe.step(field, 40)
    pipe.drain()
    ctx.synchronize()
    el = time.perf_counter() - t0
    print(f"exchange {a.exchange} lag {a.lag}: {el / a.steps * 1e6:.1f} us per step")
    for k, v in sorted(T.items(), key=lambda kv: -kv[1]):
        print(f"  {k:18} {v / a.steps * 1e6:8.1f} us/step")
    if ex is not None:
        ex.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
