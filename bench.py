#!/usr/bin/env python3
"""Benchmark: numbers checked/sec per node, detailed + niceonly, 1e9 @ base 40
(BASELINE.json metric; benchmark.rs:60 ExtraLarge field).

One step = one pass of the hot path over one field in BOTH modes: a detailed
pass (histogram + near-misses) and a niceonly pass (MSD filter + stride
candidates), what the reference client does per field in either mode
(client/src/main.rs:120-208, process_range_*_gpu).  The two passes run at once
on two HIP streams of the GPU (nice_amd.BothModes; --sequential runs them one
after the other).  Inputs are the field bounds only (no host buffers): the
kernels derive every n themselves.

Multi-GPU (one process per GPU, torchrun): weak scaling -- N GPUs process one
N x 1e9 field of base 40, [start, start + N*1e9); rank r takes the r-th
contiguous 1e9 shard (nice_amd/dist.py).  Per step the shard histograms are
combined with one RCCL all-reduce (base + 1 u64 bins) and the near-miss / nice
lists are all-gathered, so every rank ends the step holding the whole field's
results -- the north star's exchange, inside the timed region.
Timing: barrier + device sync on both sides of exactly K steps, max over ranks.

    python bench.py [--gpus N --steps K --warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Hardware queues per process (HIP's default is 4): torch's stream, RCCL's
# stream and the two mode streams of BothModes must not share a queue, or the
# niceonly pass serialises behind the detailed kernel (torchrun 1 rank: 2.86
# ms per step with 4 queues, 2.61 with 8).  Set before HIP initialises; an
# exported value below 8 (the box exports HIP's default, 4) is raised.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FIELD_SIZE = 10 ** 9
BASE = 40
W_ALG = 4 * BASE                    # int32 VALU ops per n
PEAK_INT32_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64 Tops/s per MI355X (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU work for the bounded cpu_baseline sample")
    p.add_argument("--mode", choices=["both", "detailed", "niceonly"], default="both")
    p.add_argument("--msd-floor", type=int, default=0, help="0 = reference CPU-path floor 250")
    p.add_argument("--msd-where", choices=["auto", "host", "device"], default="auto",
                   help="niceonly MSD filter placement (same candidate set either way)")
    p.add_argument("--sequential", action="store_true",
                   help="run the two modes one after the other on one stream (default: at once, "
                        "on two streams of the GPU, nice_amd.BothModes)")
    return p.parse_args()


def pmc_traffic():
    """HBM bytes per main launch of the detailed kernel, from the committed PMC
    pass (scripts/gpu_pmc.sh -> profiles/r01/traffic.json); None if absent."""
    p = os.path.join(ROOT, "profiles", "r01", "traffic.json")
    try:
        with open(p) as f:
            return json.load(f)["bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def rank_field(base_start: int, rank: int):
    """Weak scaling: rank r owns the r-th consecutive 1e9 field of base 40."""
    start = base_start + rank * FIELD_SIZE
    return start, start + FIELD_SIZE


def timed(step, steps: int, sync, dist=None, tail=None):
    """Barrier + device sync on both sides of exactly `steps` steps (plus
    `tail`, e.g. collecting the last step's overlapped exchange); returns the
    max elapsed seconds over ranks (all_reduce MAX)."""
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if tail is not None:
        tail()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def cpu_threads():
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
        if os.environ.get(k, "").isdigit():
            return max(1, int(os.environ[k]))
    return max(1, min(16, os.cpu_count() or 1))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(start, target_s):
    """Reference algorithm (oracle/ C restatement, 'port') on the host cores,
    on a bounded sample of the same workload, extrapolated per number."""
    from oracle import oracle as O
    th = cpu_threads()
    # detailed: size the sample to ~target_s of work
    probe = 4_000_000
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + probe, BASE, th)
    rate = probe / (time.perf_counter() - t)
    n = int(min(FIELD_SIZE, max(probe, rate * target_s)))
    n = max(1_000_000, n // 1_000_000 * 1_000_000)
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + n, BASE, th)
    td = time.perf_counter() - t
    det_rate = n / td
    # niceonly: the whole field (the MSD filter skips most of it at this start)
    t = time.perf_counter()
    O.process_field_niceonly_mt(start, start + FIELD_SIZE, BASE, th)
    tn = time.perf_counter() - t
    nice_rate = FIELD_SIZE / tn
    combined = 2 * FIELD_SIZE / (FIELD_SIZE / det_rate + tn)
    # the reference client's default thread count (--threads 4,
    # client/src/main.rs:94), on a smaller detailed sample
    n4 = max(1_000_000, int(det_rate / th * 4 * target_s / 3) // 1_000_000 * 1_000_000)
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + n4, BASE, 4)
    det4 = n4 / (time.perf_counter() - t)
    t = time.perf_counter()
    O.process_field_niceonly_mt(start, start + FIELD_SIZE, BASE, 4)
    tn4 = time.perf_counter() - t
    return {"value": combined, "unit": "numbers/s", "cores": th, "kind": "port",
            "cpu_model": cpu_model(),
            "threads4": {"value": 2 * FIELD_SIZE / (FIELD_SIZE / det4 + tn4), "cores": 4,
                         "detailed_numbers_per_sec": det4, "niceonly_numbers_per_sec": FIELD_SIZE / tn4,
                         "sample": f"detailed: first {n4:.3g} n; niceonly: whole 1e9 field"},
            "sample": f"detailed: first {n:.3g} n of the field on {th} threads "
                      f"({det_rate:.3e} n/s, extrapolated to 1e9); niceonly: whole 1e9 field "
                      f"({nice_rate:.3e} n/s); reference client chunking, MSD floor 250, k=2",
            "detailed_numbers_per_sec": det_rate, "niceonly_numbers_per_sec": nice_rate}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # The JSON line is the only thing on stdout: runtime banners (RCCL prints
    # its version block to fd 1 when the communicator comes up) go to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    # Any torchrun launch (WORLD_SIZE set, even 1) takes the distributed path:
    # one RCCL communicator, histogram all-reduce + list all-gather per step.
    if "WORLD_SIZE" in os.environ:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import nice_amd as N

    ctx = N.GpuContext([local])
    # Both modes of a field at once: niceonly's launch-bound MSD levels run on
    # a second stream beside the detailed kernel (nice_amd.BothModes).
    runner = N.BothModes(local, det_ctx=ctx) if args.mode == "both" and not args.sequential else ctx
    br = N.get_base_range_u128(BASE)
    start, end = rank_field(br.range_start, rank)
    assert end <= br.range_end

    def barrier_sync():
        # Every library call is synchronous (it returns host results), so the
        # device is idle here; the torch sync/barrier line the ranks up.
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    det_ms, nice_ms, kern_ms, both_ms = [], [], [], []
    last_nice_stats = None
    from nice_amd import dist as D
    whole = N.FieldSize(br.range_start, br.range_start + world * FIELD_SIZE)
    ex = D.PipelinedExchange(dist) if dist is not None else None

    def check_both(done):
        nonlocal last_nice_stats
        if done is None:
            return
        det, _, st = done
        last_nice_stats = st or last_nice_stats
        assert sum(d.count for d in det.distribution) == FIELD_SIZE * world

    def step():
        nonlocal last_nice_stats
        if dist is not None and args.mode == "both":
            # both modes of the rank's shard, then ONE all-reduce, overlapped
            # with the next step's compute (nice_amd/dist.py PipelinedExchange);
            # the previous step's results come back here and are checked.
            t = time.perf_counter()
            done = D.process_field_both_pipelined(ex, whole, BASE, runner, msd_floor=args.msd_floor,
                                                  msd_where=args.msd_where)
            det_ms.append((time.perf_counter() - t) * 1e3)
            kern_ms.append(ctx.kernel_stats().kernel_ms)
            check_both(done)
            return
        if runner is not ctx and dist is None:
            # single GPU, both modes at once: one wall time for the pair
            t = time.perf_counter()
            (hist, _), (_, st) = runner.both_raw((start, end), (start, end), BASE,
                                                 msd_floor=args.msd_floor, msd_where=args.msd_where)
            both_ms.append((time.perf_counter() - t) * 1e3)
            kern_ms.append(ctx.kernel_stats().kernel_ms)
            assert sum(hist) == FIELD_SIZE
            last_nice_stats = st
            return
        if args.mode in ("both", "detailed"):
            t = time.perf_counter()
            if dist is None:
                hist, lst = ctx.detailed_raw(start, end, BASE)
                mass = sum(hist)
            else:
                r = D.process_range_detailed_dist(whole, BASE, ctx=ctx)
                mass = sum(d.count for d in r.distribution)
            det_ms.append((time.perf_counter() - t) * 1e3)
            kern_ms.append(ctx.kernel_stats().kernel_ms)
            assert mass == FIELD_SIZE * world
        if args.mode in ("both", "niceonly"):
            t = time.perf_counter()
            if dist is None:
                _, st = ctx.niceonly_raw(start, end, BASE, msd_floor=args.msd_floor,
                                         msd_where=args.msd_where)
            else:
                def shard(s, e, b, chunk):
                    nonlocal st
                    lst, st = ctx.niceonly_raw(s, e, b, chunk_size=chunk, msd_floor=args.msd_floor,
                                               msd_where=args.msd_where)
                    return lst
                st = None
                D.process_range_niceonly_dist(whole, BASE, shard_fn=shard)
            nice_ms.append((time.perf_counter() - t) * 1e3)
            last_nice_stats = st

    def drain():
        if ex is not None:
            check_both(D.finish_both(ex, ex.drain()))

    for _ in range(args.warmup):
        step()
    drain()
    det_ms.clear(), nice_ms.clear(), kern_ms.clear(), both_ms.clear()

    elapsed = timed(step, args.steps, barrier_sync, dist, tail=drain)

    modes = 2 if args.mode == "both" else 1
    total_numbers = modes * FIELD_SIZE * world * args.steps
    value = total_numbers / elapsed
    if rank != 0:
        if runner is not ctx:
            runner.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    line = {
        "metric": "numbers checked/sec per node, detailed+niceonly, 1e9 @ base 40 field",
        "value": value,
        "unit": "numbers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (the reference's deterministic benchmark field; n derived on device)",
        "config": {
            "workload": "extra-large: 1e9 @ base 40, detailed + niceonly per step "
                        "(benchmark.rs:60); N GPUs: one N x 1e9 field, rank r takes the r-th "
                        "1e9 shard, histogram all-reduce + list all-gather per step",
            "base": BASE, "field_start": start - rank * FIELD_SIZE, "field_size": FIELD_SIZE,
            "mode": args.mode,
            "niceonly_msd_floor": args.msd_floor or 250,
            "niceonly_msd_where": args.msd_where,
            "niceonly_chunking": "reference client (1e6 * clamp(ceil(size/1e11),1,1000))",
            "parallelism": f"weak{world}",
        },
    }
    if dist is not None and args.mode == "both":
        line["rank_step_ms"] = sum(det_ms) / len(det_ms)  # both modes + exchange, rank 0
        line["rank_step_ms_median"] = sorted(det_ms)[len(det_ms) // 2]
        det_ms.clear()  # not split per mode on this path
        line["detailed_kernel_ms"] = sum(kern_ms) / len(kern_ms)
    if kern_ms:
        kms = sum(kern_ms) / len(kern_ms)
        achieved = W_ALG * FIELD_SIZE / (kms / 1e3) / 1e12
        line["roofline"] = {
            "bound": "valu", "kernel": "nice::fd2::fd2_kernel<Cfg<40, 4, 8, 5, 0, 1024>>",
            "achieved": achieved, "peak": PEAK_INT32_TOPS, "unit": "int32 Tops/s",
            "frac": achieved / PEAK_INT32_TOPS, "traffic": pmc_traffic(),
            "kernel_ms": kms,
            "work_per_unit": f"{W_ALG} int32 ops per n (4 per digit x {BASE} digits, SURVEY 8d)",
            "note": "integer-VALU/LDS bound (no HBM stream, no contraction); kernel time from "
                    "HIP events on the launch stream (main + tail launch of one field); traffic: "
                    "HBM bytes per launch from the committed PMC pass (profiles/r01/traffic.json, "
                    "FETCH_SIZE x2 + WRITE_SIZE), the field's bounds are the only input",
        }
    line["modes_overlapped"] = runner is not ctx
    if both_ms:
        line["both_wall_ms"] = sum(both_ms) / len(both_ms)  # detailed + niceonly at once
        line["both_wall_ms_median"] = sorted(both_ms)[len(both_ms) // 2]
    if det_ms:
        line["detailed_numbers_per_sec"] = FIELD_SIZE / (sum(det_ms) / len(det_ms) / 1e3)
        line["detailed_ms"] = sum(det_ms) / len(det_ms)
    if nice_ms:
        line["niceonly_numbers_per_sec"] = FIELD_SIZE / (sum(nice_ms) / len(nice_ms) / 1e3)
        line["niceonly_ms"] = sum(nice_ms) / len(nice_ms)
    st = last_nice_stats
    if st is not None and (nice_ms or both_ms or dist is not None):
        line["niceonly"] = {"ranges": st.ranges, "range_numbers": st.range_numbers,
                            "candidates": st.candidates, "launches": st.launches,
                            "msd_seconds": st.msd_seconds, "total_seconds": st.total_seconds}
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(br.range_start, args.cpu_seconds)
    print(json.dumps(line), file=json_out, flush=True)
    if runner is not ctx:
        runner.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
