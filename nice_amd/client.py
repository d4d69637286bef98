"""nice_client drop-in for the offline path (client/src/main.rs).

Supports the reference client's flag surface for field processing
(main.rs:60-116): mode (detailed | niceonly, env NICE_MODE), --benchmark,
--gpu, --gpu-device (extended: a list "0,1,2" or "all" shards one field over
several GPUs), --threads (host MSD workers for niceonly), --no-progress,
--log-level, --username, --repeat.  Fields come from --benchmark or from an
explicit --range/--base; the reference's HTTP claim/submit/validate transport
(client_api_*.rs) is out of scope, so --validate
compares against a JSON file of a canonical submission instead of the server.

With --gpu a field runs on the HIP path (process_range_*_gpu, one call per
field).  Without it, the reference's CPU mode (main.rs:154-207): the field is
cut into client chunks (1e6 * clamp(ceil(size / 1e11), 1, 1000)), the chunks
are processed by --threads workers through the library's CPU API
(nice_cpu_process_range_detailed / _niceonly, the reference's
process_range_detailed / process_range_niceonly), and the per-chunk results are
merged in chunk order (compile_results).  No GPU is touched in that mode.

    python -m nice_amd detailed --benchmark extra-large --gpu
    python -m nice_amd --benchmark base-ten            # CPU mode
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

from . import api
from .benchmark import BenchmarkMode, get_benchmark_field
from .types import DataToClient, DataToServer, SearchMode

log = logging.getLogger("nice_client")


def _msd_floor(v: str):
    return v if v == "adaptive" else int(v)


def parse_args(argv=None):
    env = os.environ.get
    p = argparse.ArgumentParser(prog="nice_client", description=__doc__.split("\n")[0])
    p.add_argument("mode", nargs="?", default=env("NICE_MODE", "detailed"),
                   choices=["detailed", "niceonly"])
    p.add_argument("--api-base", default=env("NICE_API_BASE", "https://api.nicenumbers.net"))
    p.add_argument("--api-max-retries", type=int, default=int(env("NICE_API_MAX_RETRIES", 10)))
    p.add_argument("-u", "--username", default=env("NICE_USERNAME", "anonymous"))
    p.add_argument("-r", "--repeat", action="store_true", default=bool(env("NICE_REPEAT")))
    p.add_argument("-n", "--no-progress", action="store_true", default=bool(env("NICE_NO_PROGRESS")))
    p.add_argument("-t", "--threads", type=int, default=int(env("NICE_THREADS", 4)))
    p.add_argument("-b", "--benchmark", default=env("NICE_BENCHMARK"),
                   choices=[m.value for m in BenchmarkMode])
    p.add_argument("--validate", default=env("NICE_VALIDATE"),
                   help="JSON file with the canonical submission to compare against")
    p.add_argument("--gpu", action="store_true", default=bool(env("NICE_GPU")))
    p.add_argument("--gpu-device", default=env("NICE_GPU_DEVICE", "0"),
                   help="device ordinal, comma list, or 'all'")
    p.add_argument("-l", "--log-level", default=env("NICE_LOG_LEVEL", "info"),
                   choices=["off", "error", "warn", "info", "debug", "trace"])
    p.add_argument("--base", type=int, help="explicit field: base")
    p.add_argument("--range", nargs=2, type=int, metavar=("START", "END"),
                   help="explicit field: half-open [START, END)")
    p.add_argument("--hi-base-size", type=int, default=None,
                   help="hi-base field size (code: 1e9, doc/BASELINE: 1e6)")
    p.add_argument("--msd-floor", type=_msd_floor, default=0,
                   help="niceonly MSD floor: a number (0 = 250, or NICE_GPU_MSD_FLOOR), or "
                        "'adaptive' for the reference GPU path's adaptive floor "
                        "(client_process_gpu.rs:96-184)")
    return p.parse_args(argv)


def _devices(spec: str):
    if spec == "all":
        import ctypes
        n = ctypes.c_int()
        api.lib().nice_device_count(n)
        return list(range(max(1, n.value)))
    return [int(x) for x in str(spec).split(",") if x.strip() != ""]


def compile_results(results, claim: DataToClient, username: str, mode: SearchMode) -> DataToServer:
    """compile_results (client/src/main.rs:212-254)."""
    nice = [n for r in results for n in r.nice_numbers]
    if mode is SearchMode.NICEONLY:
        dist = None
    else:
        acc = {}
        for r in results:
            for d in r.distribution:
                acc[d.num_uniques] = acc.get(d.num_uniques, 0) + d.count
        from .types import UniquesDistributionSimple
        dist = [UniquesDistributionSimple(k, v) for k, v in sorted(acc.items())]
    return DataToServer(claim.claim_id, username, api.CLIENT_VERSION, dist, nice)


def validate_results(submit: DataToServer, canon: dict, mode: SearchMode) -> bool:
    """validate_results (client/src/main.rs:258-292), against a canonical JSON."""
    ok = True
    ours = sorted((n.number, n.num_uniques) for n in submit.nice_numbers)
    theirs = sorted((int(n["number"]), int(n["num_uniques"])) for n in canon["nice_numbers"])
    if ours != theirs:
        log.error("VALIDATION FAILED: Semi-nice numbers don't match!")
        ok = False
    if mode is SearchMode.DETAILED and submit.unique_distribution is not None:
        a = sorted((d.num_uniques, d.count) for d in submit.unique_distribution)
        b = sorted((int(d["num_uniques"]), int(d["count"])) for d in canon["unique_distribution"])
        if a != b:
            log.error("VALIDATION FAILED: Distribution doesn't match!")
            ok = False
    return ok


def process_field_sync(claim: DataToClient, mode: SearchMode, args, ctx=None):
    """process_field_sync (client/src/main.rs:120-208): the GPU call for the
    whole field with --gpu, else the CPU path per client chunk on --threads
    workers (rayon par_iter in the reference), results in chunk order."""
    field = claim.field()
    if args.gpu:
        if mode is SearchMode.DETAILED:
            return [api.process_range_detailed_gpu(ctx, field, claim.base)]
        return [api.process_range_niceonly_gpu(ctx, field, claim.base, threads=args.threads,
                                               msd_floor=args.msd_floor)]
    from concurrent.futures import ThreadPoolExecutor
    from .dist import client_chunk_size
    from .types import FieldSize
    chunk = client_chunk_size(field.range_size)
    chunks = [FieldSize(a, min(field.range_end, a + chunk))
              for a in range(field.range_start, field.range_end, chunk)]
    if mode is SearchMode.DETAILED:
        def work(c):
            return api.process_range_detailed_cpu(c, claim.base)
    else:
        # main.rs:173-180: one stride table for the field (k = 2, main.rs:19)
        table = api.StrideTable.new(claim.base, 2)

        def work(c):
            return api.process_range_niceonly_cpu(c, claim.base, table)
    # ctypes releases the GIL inside the library call, so the workers run the
    # chunks in parallel on the host cores
    with ThreadPoolExecutor(max(1, args.threads)) as pool:
        return list(pool.map(work, chunks))


def run_once(args, ctx) -> int:
    mode = SearchMode.DETAILED if args.mode == "detailed" else SearchMode.NICEONLY
    if args.benchmark:
        claim = get_benchmark_field(BenchmarkMode(args.benchmark), args.hi_base_size)
        log.info("Beginning benchmark:  %s", args.benchmark)
    elif args.range and args.base:
        s, e = args.range
        claim = DataToClient(0, args.base, s, e, e - s)
        log.info("Processing field: base %d [%d, %d)", args.base, s, e)
    else:
        log.error("no field: the server claim path is out of scope offline; "
                  "use --benchmark or --base/--range")
        return 2
    t0 = time.perf_counter()
    results = process_field_sync(claim, mode, args, ctx)
    elapsed = time.perf_counter() - t0
    # The reference prints this line with --no-progress or --gpu (main.rs:358-371);
    # this client has no progress bar, so it always does.
    log.info("✓ Processed %.2e numbers in %.2fs (%.2e numbers/sec)",
             claim.range_size, elapsed, claim.range_size / elapsed)
    submit = compile_results(results, claim, args.username, mode)
    log.debug("Submit Data: %s", json.dumps(submit.to_json()))
    for n in submit.nice_numbers:
        log.info("Nice number: %d (%d uniques)", n.number, n.num_uniques)
    if args.validate:
        with open(args.validate) as f:
            canon = json.load(f)
        if validate_results(submit, canon, mode):
            print("\nValidation passed! Results match the canoncical submission.")
        else:
            print("\nValidation failed! Results do not match the canoncical submission.")
            return 1
    return 0


def main(argv=None) -> int:
    args = parse_args(argv)
    level = {"off": logging.CRITICAL + 10, "error": logging.ERROR, "warn": logging.WARNING,
             "info": logging.INFO, "debug": logging.DEBUG, "trace": logging.DEBUG}[args.log_level]
    logging.basicConfig(level=level, format="%(asctime)s %(levelname)s %(message)s")
    ctx = None
    if args.gpu:  # main.rs:592-625: the GPU context only in GPU mode
        log.info("GPU_BATCH_SIZE = %d", api.GPU_BATCH_SIZE)
        try:
            ctx = api.GpuContext(_devices(args.gpu_device))
        except api._lib.NiceError as e:
            log.error("GPU processing error: %s", e)
            return 1
    else:
        log.info("CPU mode: %d threads", args.threads)
    while True:
        rc = run_once(args, ctx)
        if rc or not args.repeat:
            return rc


if __name__ == "__main__":
    sys.exit(main())
