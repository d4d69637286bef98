"""Measure every BASELINE.json config on one GPU (the bench.py line covers the
headline extra-large config; these are the others).  One JSON line per config:
numbers/s = field size / median wall seconds of the library call (same
definition as the reference's log line, client/src/main.rs:363-370).

  python scripts/bench_configs.py [--massive-sample 1e11] [--reps 5]

massive (b50, 1e13, niceonly) runs on a bounded prefix of the field with the
full field's client chunk (1e8, client/src/main.rs:159-168), so MSD leaves
and candidates are the ones the whole field would produce there."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--massive-sample", type=float, default=1e11)
    ap.add_argument("--bases", default="", help="also: detailed 1e9 at the range start of these "
                    "bases ('all' = every FD base), with the W_alg roofline fraction")
    ap.add_argument("--nice-bases", default="", help="also: niceonly 1e10 at 1/3 of the range "
                    "of these bases")
    ap.add_argument("--only-bases", action="store_true")
    a = ap.parse_args()
    ctx = N.GpuContext(0)
    out = []

    def det(name, f, note=""):
        sec, (hist, lst) = timed(lambda: ctx.detailed_raw(f.range_start, f.range_end, f.base), a.reps)
        ks = ctx.kernel_stats()
        out.append({"config": name, "mode": "detailed", "base": f.base, "size": f.range_size,
                    "numbers_per_sec": f.range_size / sec, "wall_ms": sec * 1e3,
                    "kernel_ms": ks.kernel_ms, "fd_kernel": ks.fd_kernel,
                    "near_misses": len(lst), "note": note})

    def nice(name, f, chunk=0, reps=None, note=""):
        sec, (lst, st) = timed(lambda: ctx.niceonly_raw(f.range_start, f.range_end, f.base,
                                                       chunk_size=chunk), reps or a.reps)
        out.append({"config": name, "mode": "niceonly", "base": f.base, "size": f.range_size,
                    "numbers_per_sec": f.range_size / sec, "wall_ms": sec * 1e3,
                    "msd_ranges": st.ranges, "candidates": st.candidates,
                    "candidates_per_sec": st.candidates / sec, "nice": [str(x) for x in lst],
                    "chunk": chunk or "client rule", "note": note})

    peak = 256 * 4 * 32 * 2.4e9  # int32 lane-ops/s
    bases = []
    if a.bases == "all":
        bases = [b for b in range(2, 129) if N._lib.lib().nice_fd_kernel_base(b)]
    elif a.bases:
        bases = [int(x) for x in a.bases.split(",")]
    for b in bases:
        r = N.get_base_range_u128(b)
        f = type(get_benchmark_field(BM.DEFAULT))(claim_id=0, base=b, range_start=r.range_start,
                                                 range_end=r.range_start + 10 ** 9, range_size=10 ** 9)
        det(f"production-b{b}-1e9", f, "range start, 1e9")
        k = out[-1]["kernel_ms"]
        out[-1]["roofline_frac"] = 4 * b * 10 ** 9 / (k / 1e3) / peak
        out[-1]["w_alg_ops_per_n"] = 4 * b
    for b in [int(x) for x in a.nice_bases.split(",") if x]:
        r = N.get_base_range_u128(b)
        st = r.range_start + (r.range_end - r.range_start) // 3
        f = type(get_benchmark_field(BM.DEFAULT))(claim_id=0, base=b, range_start=st,
                                                 range_end=st + 10 ** 10, range_size=10 ** 10)
        nice(f"production-b{b}-niceonly-1e10", f, note="1/3 into the range, 1e10, client chunking")
    if a.only_bases:
        for r in out:
            print(json.dumps(r), flush=True)
        return
    det("base-ten", get_benchmark_field(BM.BASE_TEN), "b10 [47,100): must list (69, 10)")
    det("default", get_benchmark_field(BM.DEFAULT), "latency-dominated (SURVEY 8d)")
    det("large", get_benchmark_field(BM.LARGE))
    xl = get_benchmark_field(BM.EXTRA_LARGE)
    det("extra-large", xl)
    nice("extra-large", xl)
    det("hi-base-1e6", get_benchmark_field(BM.HI_BASE, hi_base_size=10 ** 6), "BASELINE size")
    det("hi-base-1e9", get_benchmark_field(BM.HI_BASE), "benchmark.rs:63 size")
    m = get_benchmark_field(BM.MASSIVE)
    size = int(a.massive_sample)
    sample = type(m)(claim_id=0, base=50, range_start=m.range_start,
                     range_end=m.range_start + size, range_size=size)
    nice("massive-sample", sample, chunk=10 ** 8, reps=3,
         note=f"first {size:.0e} n of the 1e13 b50 field, client chunk 1e8; "
              f"full field on 8 GPUs ~ 1e13 / (8 x numbers_per_sec)")
    nice("msd-effective", get_benchmark_field(BM.MSD_EFFECTIVE), reps=3)
    nice("msd-ineffective", get_benchmark_field(BM.MSD_INEFFECTIVE))
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
