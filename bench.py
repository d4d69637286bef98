#!/usr/bin/env python3
"""Benchmark: numbers checked/sec per node, detailed+niceonly, 1e9 @ base 40
(BASELINE.json metric; benchmark.rs:60 ExtraLarge field).

One step = one pass of the hot path over one field in BOTH modes: a detailed
pass (histogram + near-misses) and a niceonly pass (MSD filter + stride
candidates), what the reference client does per field in either mode
(client/src/main.rs:120-208, process_range_*_gpu).  Inputs are the field
bounds only (no host buffers): the kernels derive every n themselves.

Fields are pipelined (nice_amd.dist.FieldPipeline): each step submits its
field to the GPU -- detailed on one stream, niceonly on a second -- before the
previous field's results are collected, so the GPU never waits for the host
between steps.  Every field's results come back and are checked (histogram
mass = field size); the last ones are collected inside the timed region.
`--sync` runs the synchronous library calls instead (both modes at once on two
streams, nice_amd.BothModes; no cross-field overlap).

Multi-GPU (one process per GPU, torchrun; --scaling, default strong):
  strong  the ONE 1e9 field of the metric is split N ways: rank r takes the
          r-th contiguous detailed shard and is dealt every N-th niceonly chunk
          of the field's chunk grid (nice_amd/dist.py);
  weak    N GPUs process one N x 1e9 field, split the same way.
Per step the shard histograms and list lengths are combined with one RCCL
all-reduce (overlapped with the next step's compute) and the near-miss / nice
lists are all-gathered when non-empty, so every rank ends holding the whole
field's results -- the north star's exchange, inside the timed region.  Under
strong scaling rank 0 then times the whole field alone on its GPU (the other
ranks wait) and reports strong_efficiency = T1 / (N * T_N) from the same run.
Timing: barrier + device sync on both sides of exactly K steps, max over ranks.

    python bench.py [--gpus N --steps K --warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

# Hardware queues per process: HIP's default (4, what the GPU box exports and
# what a Rust client linking libnice_hip.so gets), also under torchrun when
# the field exchange runs in shared memory (the default on one node: no device
# work besides the library's six slot streams).  With the exchange over RCCL
# the process also holds torch's stream and RCCL's, and on 4 queues the
# exchange's copies and collective wait behind queued field kernels: a 1/8
# shard's step is 0.281 ms at 4 queues, 0.264 at 8, 0.263 at 16 (plain
# process: 0.259; profiles/r03/dist_hw_queues.log), so that path asks for 8.
# --hw-queues N overrides (A/B runs).  Set before HIP initialises; the value
# used and the exported one are recorded in the JSON line's config.
HW_QUEUES_EXPORTED = os.environ.get("GPU_MAX_HW_QUEUES")


def _argv(flag, default):
    return sys.argv[sys.argv.index(flag) + 1] if flag in sys.argv[:-1] else default


if "--hw-queues" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = _argv("--hw-queues", "4")
elif "WORLD_SIZE" in os.environ:
    _ex = _argv("--exchange-backend", "auto")
    _one_node = os.environ.get("LOCAL_WORLD_SIZE", os.environ["WORLD_SIZE"]) == os.environ["WORLD_SIZE"]
    if _ex == "nccl" or (_ex == "auto" and not _one_node and _argv("--dist-backend", "nccl") == "nccl"):
        os.environ["GPU_MAX_HW_QUEUES"] = "8"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PROBE_LIB = "--probe-lib" in sys.argv  # A/B experiments only (scripts/probe_lib.py)
if PROBE_LIB:
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import probe_lib  # noqa: E402,F401

FIELD_SIZE = 10 ** 9
BASE = 40
PEAK_INT32_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64 Tops/s per MI355X (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="target CPU work for the bounded cpu_baseline sample")
    p.add_argument("--mode", choices=["both", "detailed", "niceonly"], default="both")
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="N > 1: split the one 1e9 field N ways (strong) or run an N x 1e9 field (weak)")
    p.add_argument("--base", type=int, default=BASE, help="(config lines) base of the field")
    p.add_argument("--field-size", type=float, default=FIELD_SIZE, help="(config lines) field size")
    p.add_argument("--msd-floor", type=int, default=0, help="0 = reference CPU-path floor 250")
    p.add_argument("--msd-where", choices=["auto", "host", "device"], default="auto",
                   help="niceonly MSD filter placement (same candidate set either way)")
    p.add_argument("--depth", type=int, default=2, choices=[1, 2],
                   help="fields kept in flight behind the one being collected")
    p.add_argument("--exchange-lag", type=int, default=2, choices=[1, 2, 3],
                   help="N > 1: field exchanges kept in flight (PipelinedExchange lag)")
    p.add_argument("--exchange-backend", choices=["auto", "shm", "nccl", "gloo"], default="auto",
                   help="N > 1: the per-field exchange in node-local shared memory (shm), over "
                        "the process group's RCCL on device buffers (nccl), or over a gloo group "
                        "on host tensors (gloo); auto = shm when every rank is on this node")
    p.add_argument("--probe-lib", action="store_true",
                   help="A/B experiments: load the probe build (env tuning knobs live only there)")
    p.add_argument("--two-ctx", action="store_true",
                   help="A/B: detailed and niceonly on separate contexts")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="N > 1: RCCL over xGMI (nccl, default) or gloo on host tensors (tests)")
    p.add_argument("--hw-queues", type=int, default=None,
                   help="GPU_MAX_HW_QUEUES for this process (default: HIP's 4 at N = 1, 8 under "
                        "torchrun)")
    p.add_argument("--sync", action="store_true",
                   help="synchronous library calls (no cross-field pipelining)")
    return p.parse_args()


PMC_BENCH_FILE = "profiles/r06/pmc_bench.json"


def lib_sha16() -> str:
    """First 16 hex digits of sha256 of the library this process loads."""
    import hashlib
    from nice_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_bench():
    """Counter-derived figures of the fd2 kernel from the committed rocprofv3
    --pmc passes of this bench command (scripts/pmc_bench.py): (derived, file,
    status).  The passes record the sha256 of the library they profiled;
    status is "current" only when it equals the loaded library's, else
    "stale" and derived is None (counter figures of another build are not
    reported as this one's)."""
    try:
        with open(os.path.join(ROOT, PMC_BENCH_FILE)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, PMC_BENCH_FILE, "missing"
    if d.get("lib_sha16") != lib_sha16():
        return None, PMC_BENCH_FILE, f"stale (profiled library {d.get('lib_sha16')}, loaded {lib_sha16()})"
    return d.get("derived"), PMC_BENCH_FILE, "current"


def rank_field(base_start: int, rank: int, size: int = FIELD_SIZE):
    """Rank r's 1e9 shard of an N x 1e9 weak-scaling field (kept for the
    plumbing tests; the pipeline computes shards itself)."""
    start = base_start + rank * size
    return start, start + size


def timed(step, steps: int, sync, dist=None, tail=None):
    """Barrier + device sync on both sides of exactly `steps` steps (plus
    `tail`, e.g. collecting the pipeline's last fields); returns the max
    elapsed seconds over ranks (all_reduce MAX).  Python's cyclic garbage
    collector is paused inside the region (as timeit does): a collection
    pass over the interpreter's objects stalls the host that feeds the
    pipeline, and at a strong-scaling shard's ~0.25 ms per step one such
    stall is several steps' worth of GPU time."""
    gc.collect()
    gc_was = gc.isenabled()
    gc.disable()
    try:
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if tail is not None:
            tail()
        sync()
        elapsed = time.perf_counter() - t0
    finally:
        if gc_was:
            gc.enable()
    if dist is not None:
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def cpu_share() -> tuple:
    """CPUs this process may actually use: the cgroup CPU quota (the GPU box
    grants 16 per GPU through cpu.max while os.cpu_count() shows every logical
    CPU of the host), else the affinity mask.  Returns (cpus, how)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            return max(1, int(int(quota) // int(period))), "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    try:
        return len(os.sched_getaffinity(0)), "affinity mask"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(start, target_s, base=BASE, field=FIELD_SIZE):
    """Reference algorithm (oracle/ C restatement, 'port') on every CPU the
    box grants this process, on a bounded sample of the same workload: the
    detailed leg on the first n of the field (sized to ~target_s, per-number
    rate extrapolated to the field), the niceonly leg on the whole field."""
    from oracle import oracle as O
    th, how = cpu_share()
    probe = 20_000_000  # long enough that thread start-up does not skew the rate
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + probe, base, th)
    rate = probe / (time.perf_counter() - t)
    n = int(min(field, max(probe, rate * target_s)))
    n = max(1_000_000, n // 1_000_000 * 1_000_000)
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + n, base, th)
    td = time.perf_counter() - t
    det_rate = n / td
    t = time.perf_counter()
    O.process_field_niceonly_mt(start, start + field, base, th)
    tn = time.perf_counter() - t
    nice_rate = field / tn
    combined = field / (field / det_rate + tn)  # one field, both modes (as `value`)
    # the reference client's default thread count (--threads 4,
    # client/src/main.rs:94), on a smaller detailed sample
    n4 = max(1_000_000, int(det_rate / th * 4 * target_s / 3) // 1_000_000 * 1_000_000)
    t = time.perf_counter()
    O.process_field_detailed_mt(start, start + n4, base, 4)
    det4 = n4 / (time.perf_counter() - t)
    t = time.perf_counter()
    O.process_field_niceonly_mt(start, start + field, base, 4)
    tn4 = time.perf_counter() - t
    return {"value": combined, "unit": "numbers/s", "cores": th, "kind": "port",
            "nproc": th, "cores_source": how, "host_logical_cpus": os.cpu_count(),
            "cpu_model": cpu_model(),
            "threads4": {"value": field / (field / det4 + tn4), "cores": 4,
                         "detailed_numbers_per_sec": det4, "niceonly_numbers_per_sec": field / tn4,
                         "sample": f"detailed: first {n4:.3g} n; niceonly: whole field"},
            "sample": f"detailed: first {n:.3g} n of the field on {th} threads ({td:.1f} s, "
                      f"{det_rate:.3e} n/s, extrapolated per number to {field:.0e}); niceonly: "
                      f"whole field ({tn:.1f} s, {nice_rate:.3e} n/s); reference client "
                      f"chunking, MSD floor 250, k=2",
            "detailed_numbers_per_sec": det_rate, "niceonly_numbers_per_sec": nice_rate}


def fixture_check(field, base, mode, res, world=1):
    """The last timed field's results against the committed oracle fixture of
    this exact field (tests/golden/oracle_fields.json, data only -- the
    oracle is not run here): the detailed distribution and near-miss list,
    and the niceonly stride-candidate count and nice list.  None when no
    fixture holds this field (non-default configs).  Over N > 1 ranks the
    histogram and the lists are the exchanged whole-field ones; the candidate
    count is rank 0's dealt share, so it is not compared there."""
    path = os.path.join(ROOT, "tests", "golden", "oracle_fields.json")
    try:
        with open(path) as f:
            fx = json.load(f)
    except OSError:
        return None
    key = (str(field.range_start), str(field.range_end), base)
    det_fx = [d for d in fx["detailed"] if (d["start"], d["end"], d["base"]) == key]
    nice_fx = [d for d in fx["niceonly"] if (d["start"], d["end"], d["base"]) == key]
    _, det, nic, st = res
    out = {"fixture": "tests/golden/oracle_fields.json"}
    ok = True
    if mode in ("both", "detailed"):
        if not det_fx:
            return None
        d = det_fx[0]
        dist_ok = [(x.num_uniques, x.count) for x in det.distribution] == [tuple(v) for v in d["distribution"]]
        near_ok = [(n.number, n.num_uniques) for n in det.nice_numbers] == [(int(n), u) for n, u in d["near_misses"]]
        out["detailed"] = {"name": d["name"], "distribution": dist_ok, "near_misses": near_ok,
                           "near_miss_count": len(d["near_misses"])}
        ok = ok and dist_ok and near_ok
    if mode in ("both", "niceonly"):
        if not nice_fx or st is None:
            return None
        d = nice_fx[0]
        cand_ok = st.candidates == d["candidates"] if world == 1 else None
        list_ok = [str(n.number) for n in nic.nice_numbers] == d["nice_numbers"]
        out["niceonly"] = {"name": d["name"], "candidates": st.candidates, "candidates_match": cand_ok,
                           "nice_numbers": list_ok}
        ok = ok and cand_ok is not False and list_ok
    out["verified"] = ok
    return out


def main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    base, field_size = args.base, int(args.field_size)
    w_alg = 4 * base                    # int32 VALU ops per n
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
        # one GPU per rank; more ranks than GPUs (the 2-rank gloo test on a
        # one-GPU box) share devices round-robin
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    # The per-field exchange: its vector (~1 KiB) is host
    # data at both ends, so on one node the ranks sum it in shared memory; over
    # RCCL every step queues an H2D copy, the collective and a D2H copy behind
    # the field kernels for CU slots.
    ex_group, ex_kind = None, None
    if dist is not None:
        ex_kind = args.exchange_backend
        if ex_kind == "auto":
            ex_kind = "shm" if int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world else args.dist_backend
        if ex_kind == "gloo" and args.dist_backend != "gloo":
            ex_group = dist.new_group(backend="gloo")
        if ex_kind == "nccl" and args.dist_backend != "nccl":
            raise SystemExit("bench.py: --exchange-backend nccl needs --dist-backend nccl")

    import nice_amd as N
    from nice_amd import dist as D
    shm_ex = None
    if ex_kind == "shm":
        try:
            shm_ex = D.ShmExchange(dist, lag=args.exchange_lag)
        except D.ShmUnavailable as e:  # raised on every rank alike
            print(f"bench.py: shared-memory exchange unavailable ({e}); exchanging over "
                  f"{args.dist_backend}", file=sys.stderr)
            ex_kind = args.dist_backend + " (shm unavailable)"

    br = N.get_base_range_u128(base)
    strong = args.scaling == "strong" or world == 1
    job_size = field_size if strong else field_size * world
    field = N.FieldSize(br.range_start, br.range_start + job_size)
    assert field.range_end <= br.range_end
    # One context runs both modes: per in-flight field a detailed stream and a
    # high-priority niceonly stream (the MSD chain of short dependent launches
    # cuts in ahead of queued detailed workgroups).  --sync uses two contexts.
    det_ctx = N.GpuContext([local])
    nice_ctx = N.GpuContext([local]) if args.sync or args.two_ctx else det_ctx
    nice_opts = {"msd_floor": args.msd_floor, "msd_where": args.msd_where}
    modes = {"both": (True, True), "detailed": (True, False), "niceonly": (False, True)}[args.mode]

    def barrier_sync():
        # the library's streams (torch is not initialised on the device at N = 1:
        # the process's HIP runtime belongs to libnice_hip.so there)
        det_ctx.synchronize()
        if nice_ctx is not det_ctx:
            nice_ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
            det_ctx.synchronize()

    last_stats = [None]
    last_res = [None]  # the last field's whole results (fixture_check after the timed region)
    checked = [0]  # fields whose whole-field results came back and were checked

    def check(res):
        _, det, _, st = res
        if modes[0]:
            assert sum(d.count for d in det.distribution) == job_size
        checked[0] += 1
        last_stats[0] = st or last_stats[0]
        last_res[0] = res

    def make_pipeline(d):
        # detailed-only / niceonly-only runs pass a context that skips the other mode
        return D.FieldPipeline(det_ctx if modes[0] else _Skip(), nice_ctx if modes[1] else _Skip(),
                               d, group=ex_group if d is not None else None,
                               exchange=shm_ex if d is not None else None,
                               depth=args.depth, lag=args.exchange_lag, **nice_opts)

    if args.sync:
        runner = N.BothModes(local, det_ctx=det_ctx, nice_ctx=nice_ctx)
        ex = shm_ex or (D.PipelinedExchange(dist, ex_group) if dist is not None else None)
        kern = []

        def step():
            if dist is None:
                (hist, _), (_, st) = runner.both_raw(
                    (field.range_start, field.range_end) if modes[0] else None,
                    (field.range_start, field.range_end) if modes[1] else None, base, **nice_opts)
                kern.append(det_ctx.kernel_stats().kernel_ms)
                if modes[0]:
                    assert sum(hist) == job_size
                last_stats[0] = st or last_stats[0]
            else:
                done = D.process_field_both_pipelined(ex, field, base, runner, **nice_opts)
                kern.append(det_ctx.kernel_stats().kernel_ms)
                if done is not None:
                    check((field,) + tuple(done))

        def tail():
            if ex is not None:
                done = D.finish_both(ex, ex.drain())
                if done is not None:
                    check((field,) + tuple(done))
        kernel_ms = kern
    else:
        pipe = make_pipeline(dist)

        def step():
            r = pipe.step(field, base)
            if r is not None:
                check(r)

        def tail():
            for r in pipe.drain():
                check(r)
        kernel_ms = pipe.kernel_ms

    for _ in range(args.warmup):
        step()
    tail()
    kernel_ms.clear()

    checked[0] = 0
    elapsed = timed(step, args.steps, barrier_sync, dist, tail=tail)
    fields_checked = checked[0]  # every field of the timed region came back whole and was checked
    # the timed region's last field against the oracle fixture of this field
    fixture = fixture_check(field, base, args.mode, last_res[0], world) if last_res[0] is not None else None
    # Event spans of the detailed launches inside the timed region: consecutive
    # fields run on different slots' streams and overlap at their edges by
    # design (a field's first workgroups fill the CUs the previous field's last
    # ones leave idle), so a span holds its neighbours' work too; reported as
    # pipelined_launch_span_ms, not used as a launch duration.
    pipelined_kms = sum(kernel_ms) / len(kernel_ms) if kernel_ms else None

    # Each mode alone over the same field, same pipeline, same timing rules
    # (BOTH modes check every n of the field; these are the per-mode rates).
    per_mode = {}
    if args.mode == "both" and not args.sync:
        for name, sel in (("detailed", (True, False)), ("niceonly", (False, True))):
            p1 = D.FieldPipeline(det_ctx if sel[0] else _Skip(), nice_ctx if sel[1] else _Skip(),
                                 dist, group=ex_group, exchange=shm_ex, depth=args.depth,
                                 lag=args.exchange_lag, **nice_opts)

            def step1(p1=p1):
                r = p1.step(field, base)
                if r is not None and sel[0]:
                    assert sum(d.count for d in r[1].distribution) == job_size

            def tail1(p1=p1):
                for r in p1.drain():
                    if sel[0]:
                        assert sum(d.count for d in r[1].distribution) == job_size
            for _ in range(args.warmup):
                step1()
            tail1()
            per_mode[name] = timed(step1, args.steps, barrier_sync, dist, tail=tail1)

    # The dominant kernel's launch duration: this rank's detailed shard
    # launched back to back with the host waiting in between (no overlap), HIP
    # events on the launch stream; the same dispatches are the last fd2 ones in
    # a rocprofv3 kernel trace of this command (scripts/trace_summary.py).
    iso_ms = []
    if modes[0]:
        s_r, e_r = D.shard_bounds(field.range_start, field.range_end, rank, world)
        for _ in range(max(3, min(10, args.steps))):
            hist, _ = det_ctx.detailed_raw(s_r, e_r, base)
            assert sum(hist) == e_r - s_r
            iso_ms.append(det_ctx.kernel_stats().kernel_ms)
    kms = sorted(iso_ms)[len(iso_ms) // 2] if iso_ms else None

    # Strong scaling: the whole field on rank 0's GPU alone, same run (T1).
    t1 = None
    if dist is not None and strong and world > 1:
        if rank == 0:
            solo = make_pipeline(None)

            def solo_step():
                r = solo.step(field, base)
                if r is not None:
                    check(r)

            def solo_tail():
                for r in solo.drain():
                    check(r)
            for _ in range(args.warmup):
                solo_step()
            solo_tail()
            t1 = timed(solo_step, args.steps, det_ctx.synchronize, None, tail=solo_tail) / args.steps
        dist.barrier()

    # the metric: field numbers / elapsed, one field per step --
    # every n of it checked in both modes (detailed AND niceonly)
    value = job_size * args.steps / elapsed
    if rank != 0:
        if args.sync:
            runner.close()
        if shm_ex is not None:
            shm_ex.close()
        dist.destroy_process_group()
        return

    default_cfg = base == BASE and field_size == FIELD_SIZE
    line = {
        "metric": "numbers checked/sec per node, detailed+niceonly, 1e9 @ base 40 field"
        if default_cfg else f"numbers checked/sec per node, {args.mode}, {field_size:.0e} @ base {base} field",
        "value": value,
        "unit": "numbers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "value_definition": "field numbers x steps / elapsed; one step = ONE field, every n checked in "
                            "both modes (detailed AND niceonly), as BASELINE.md defines the metric",
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (the reference's deterministic benchmark field; n derived on device)",
        "config": {
            "workload": (f"extra-large: {field_size:.0e} @ base {base}, detailed + niceonly per step "
                         f"(benchmark.rs:60)" if default_cfg else
                         f"{field_size:.0e} @ base {base}, {args.mode} per step") +
                        (f"; ONE field sharded {world} ways (rank r: r-th contiguous detailed shard, "
                         f"every {world}-th niceonly chunk), histogram all-reduce + list all-gather "
                         f"per step" if world > 1 and strong else
                         f"; one {world} x field, split {world} ways" if world > 1 else ""),
            "base": base, "field_start": field.range_start, "field_size": field_size,
            "job_numbers_per_step": job_size, "mode": args.mode,
            "niceonly_msd_floor": args.msd_floor or 250,
            "niceonly_msd_where": args.msd_where,
            "niceonly_chunking": "reference client (1e6 * clamp(ceil(size/1e11),1,1000))",
            "parallelism": f"{'strong' if strong else 'weak'}{world}",
            "dist_backend": args.dist_backend if dist is not None else None,
            "pipelined": not args.sync,
            "pipeline_depth": None if args.sync else args.depth,
            "exchange_lag": args.exchange_lag if dist is not None else None,
            "exchange_backend": ex_kind,
            "probe_lib": PROBE_LIB,
            "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            "gpu_max_hw_queues_exported": HW_QUEUES_EXPORTED,
        },
    }
    line["fields_checked"] = fields_checked
    line["verified_against_fixture"] = bool(fixture and fixture["verified"])
    if fixture is not None:
        line["fixture_check"] = fixture
    for name, el in per_mode.items():
        line[f"{name}_numbers_per_sec"] = job_size * args.steps / el
        line[f"{name}_ms_per_step"] = el / args.steps * 1e3
    if t1 is not None:
        line["t1_ms_per_step"] = t1 * 1e3
        line["strong_efficiency"] = t1 / (world * elapsed / args.steps)
    if kms is not None and modes[0]:
        shard = job_size // world
        achieved = w_alg * shard / (kms / 1e3) / 1e12
        step_rate = w_alg * shard / (elapsed / args.steps) / 1e12
        line["roofline"] = {
            "bound": "valu", "kernel": f"nice::fd2::fd2_kernel<Cfg<{base}, ...>>",
            "achieved": achieved, "peak": PEAK_INT32_TOPS, "unit": "int32 Tops/s",
            "frac": achieved / PEAK_INT32_TOPS,
            "traffic": None,
            "kernel_ms": kms, "numbers_per_launch": shard,
            "work_per_unit": f"{w_alg} int32 ops per n (4 per digit x {base} digits, SURVEY 8d)",
            "frac_is": "W_alg model (SURVEY 8d charges a division-per-digit kernel 4 int32 ops per "
                       "digit); this kernel does the digit work in fewer instructions, partly as LDS "
                       "table lookups, so frac is NOT a hardware utilisation and can pass 1. The "
                       "hardware bound is hw_bound: the busier of the VALU and LDS pipes, from the "
                       "rocprofv3 --pmc passes of this command on this library",
            "step_frac": step_rate / PEAK_INT32_TOPS,
            "pipelined_launch_span_ms": pipelined_kms,
            "note": "integer-VALU/LDS bound (no HBM stream, no contraction). kernel_ms = median "
                    "duration of this rank's detailed shard launched alone (HIP events on its "
                    "launch stream, after the timed region; the same dispatches close the rocprofv3 "
                    "trace of this command). step_frac = the same work per timed step, both modes "
                    "and the pipeline's overlap of consecutive fields included. traffic: HBM bytes "
                    "per launch (FETCH_SIZE x2 + WRITE_SIZE); the field's bounds are the only input",
        }
        if default_cfg and world == 1:
            der, src, status = pmc_bench()
            line["roofline"]["hw_source"] = src
            line["roofline"]["hw_status"] = status
            if der is not None:
                vb, lb = der.get("valu_issue_busy", der.get("valu_busy")), der.get("lds_busy")
                line["roofline"]["traffic"] = der.get("traffic_bytes")
                line["roofline"]["hw"] = {
                    "valu_issue_busy": der.get("valu_issue_busy"), "valu_busy_counter": der.get("valu_busy"),
                    "valu_cpi": der.get("valu_cpi"), "valu_cpi_source": der.get("valu_cpi_source"),
                    "lds_busy": lb,
                    "lds_conflict_frac": der.get("lds_conflict_frac"),
                    "lds_cycles_per_instr": der.get("lds_cycles_per_instr"),
                    "valu_lane_ops_per_n": der.get("valu_lane_ops_per_n"),
                    "lds_instr_per_n": der.get("lds_instr_per_n"),
                    "kernel_cycles": der.get("kernel_cycles"),
                    "note": "valu_issue_busy = SQ_INSTS_VALU x valu_cpi / (4 SIMDs x CUs x kernel "
                            "cycles): the share of the kernel's SIMD cycles its VALU instructions "
                            "occupy the issue port, valu_cpi = issue cycles per instruction of the "
                            "hot loop's opcode mix at the measured gfx950 rates (valu_cpi_source; "
                            "profiles/r01/isa_issue_rates_gfx950.log) -- <= 1 by construction; "
                            "valu_busy_counter = VALUBusy/100 (SQ_ACTIVE_INST_VALU / CUs / kernel "
                            "cycles), one count per instruction whatever its rate, so not a "
                            "share and it can pass 1; lds_busy = SQ_LDS_IDX_ACTIVE / CUs / kernel "
                            "cycles (the CU's one LDS pipe; the counter matches the CU's s_memtime "
                            "span on the kernel's own index trace, profiles/r04/lds_trace.log); "
                            "both pipes near 1 = co-bound; lds_conflict_frac = SQ_LDS_BANK_CONFLICT / "
                            "SQ_LDS_IDX_ACTIVE; kernel cycles = GRBM_GUI_ACTIVE / XCDs"}
                if vb is not None and lb is not None:
                    (pipe, busy), other = sorted([("valu", vb), ("lds", lb)], key=lambda x: -x[1])
                    line["roofline"]["hw_bound"] = {"pipe": pipe, "busy": busy,
                                                    "other_pipe": other[0], "other_busy": other[1],
                                                    "co_bound": other[1] >= 0.85}
                    line["roofline"]["frac_hw"] = busy
    st = last_stats[0]
    if st is not None:
        line["niceonly"] = {"ranges": st.ranges, "range_numbers": st.range_numbers,
                            "candidates": st.candidates, "launches": st.launches,
                            "rank0_dealt_chunks": f"every {world}-th" if world > 1 else "all"}
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(br.range_start, args.cpu_seconds, base, field_size)
    print(json.dumps(line), file=json_out, flush=True)
    if args.sync:
        runner.close()
    if shm_ex is not None:
        shm_ex.close()
    if dist is not None:
        dist.destroy_process_group()


class _Skip:
    """A context that runs nothing (single-mode bench runs)."""

    def detailed_submit(self, *a, **k):
        return None

    def niceonly_submit(self, *a, **k):
        return None


def spawn_ranks(n: int) -> int:
    """`--gpus N` (N > 1) without a distributed launcher: start one -- as a
    CHILD process, before this process has touched a GPU (bench.py initialises
    HIP only inside main()) -- running this same command line with N ranks,
    one per GPU, on 127.0.0.1 and a free port.  Rank 0's JSON line reaches
    stdout through the inherited descriptor; the exit status is the child's."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def entry() -> int:
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return spawn_ranks(args.gpus)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
              f"{os.environ['WORLD_SIZE']} ranks", file=sys.stderr)
        return 2
    main(args)
    return 0


if __name__ == "__main__":
    sys.exit(entry())
