"""Measure every BASELINE.json config on one GPU (the bench.py line covers the
headline extra-large config; these are the others).  One JSON line per config:
numbers/s = field size / median wall seconds of the library call (same
definition as the reference's log line, client/src/main.rs:363-370).

  python scripts/bench_configs.py [--reps 5] [--massive-world 8]

massive (b50, 1e13, niceonly) runs the WHOLE field with its client chunk
(1e8, client/src/main.rs:159-168) on one GPU, its candidate and range totals
asserted against tests/golden/massive_b50.json (the oracle's fixture), then
each of the --massive-world ranks' dealt shares (chunks c = r mod N, what
rank r of an N-GPU job processes, nice_amd/dist.py) timed alone: the
N-GPU time of the field is the slowest share, not an extrapolation."""
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


THROUGHPUT_FLOOR = 64


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
    ap.add_argument("--massive-world", type=int, default=8)
    ap.add_argument("--bases", default="", help="also: detailed 1e9 at the range start of these "
                    "bases ('all' = every FD base), with the W_alg roofline fraction")
    ap.add_argument("--nice-bases", default="", help="also: niceonly 1e10 at 1/3 of the range "
                    "of these bases")
    ap.add_argument("--only-bases", action="store_true")
    a = ap.parse_args()
    ctx = N.GpuContext(0)
    out = []
    # Warm the GPU up before the first timed config: the first fields after
    # an idle spell run ~5 % slow (clocks ramping; profiles/r04/
    # vd_below_top_order.log), which would charge the first row.
    w = get_benchmark_field(BM.EXTRA_LARGE)
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        ctx.detailed_raw(w.range_start, w.range_end, w.base)

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
    with open(os.path.join(ROOT, "tests", "golden", "massive_b50.json")) as fh:
        fx = json.load(fh)
    want = (sum(w["candidates"] for w in fx["windows"]), sum(w["ranges"] for w in fx["windows"]))
    nice("massive", m, chunk=10 ** 8, reps=3, note="whole 1e13 b50 field on one GPU, client chunk 1e8")
    assert (out[-1]["candidates"], out[-1]["msd_ranges"]) == want, (out[-1], want)
    t1 = out[-1]["wall_ms"]
    W = a.massive_world
    shares = []
    for r in range(W):
        sec, (lst, st) = timed(lambda: ctx.niceonly_raw(m.range_start, m.range_end, 50, chunk_size=10 ** 8,
                                                         deal_stride=W, deal_offset=r), 3)
        shares.append({"rank": r, "wall_ms": sec * 1e3, "candidates": st.candidates, "msd_ranges": st.ranges,
                       "nice": len(lst)})
    assert (sum(x["candidates"] for x in shares), sum(x["msd_ranges"] for x in shares)) == want
    tmax = max(x["wall_ms"] for x in shares)
    out.append({"config": f"massive-dealt-{W}", "mode": "niceonly", "base": 50, "size": m.range_size,
                "world": W, "max_share_wall_ms": tmax, "t1_wall_ms": t1,
                "numbers_per_sec": m.range_size / (tmax / 1e3),
                "projected_efficiency": t1 / (W * tmax), "shares": shares,
                "note": f"each of {W} ranks' dealt share of the whole field timed alone on one GPU; "
                        f"numbers_per_sec = field / slowest share (the {W}-GPU field time without "
                        f"the exchange)"})
    # The same field at the throughput floor: MSD recursion down to nodes of
    # <= 2 * 64 numbers (depth 20 of its 1e8 chunks) instead of < 500 (depth
    # 18), trading 7.5e9 stride candidates for 1.9e9 and deeper recursion
    # (scripts/massive_floor_sweep.py: the fastest floor on one GPU,
    # profiles/r05/massive_floor_low.log).  The nice list is floor-independent
    # and must equal the fixture's; ranges / candidates are this floor's own.
    # Reference-quirk dependent: Filter C (msd_prefix_filter.rs:461-559) judges
    # a range by its first number's two LSDs, which is unsound for ranges of
    # more than one number, and it is what prunes at this floor -- 93 % of the
    # sound filter's candidates at floor 64, 78 % at floor 250
    # (scripts/filter_c_share.py, profiles/r06/filter_c_share.txt).
    sec, (lst, st) = timed(lambda: ctx.niceonly_raw(m.range_start, m.range_end, 50, chunk_size=10 ** 8,
                                                     msd_floor=THROUGHPUT_FLOOR, msd_where="device"), 3)
    assert [str(x) for x in lst] == [str(x) for w in fx["windows"] for x in w["nice_numbers"]], lst
    out.append({"config": f"massive-floor-{THROUGHPUT_FLOOR}", "mode": "niceonly", "base": 50,
                "size": m.range_size, "numbers_per_sec": m.range_size / sec, "wall_ms": sec * 1e3,
                "msd_floor": THROUGHPUT_FLOOR, "msd_ranges": st.ranges, "candidates": st.candidates,
                "nice": [str(x) for x in lst], "chunk": 10 ** 8,
                "note": "whole field, throughput MSD floor (parity row: 'massive', floor 250); "
                        "reference-quirk dependent: Filter C (unsound for ranges of > 1 number) removes "
                        "93 % of the sound filter's candidates at this floor (profiles/r06/filter_c_share.txt)"})
    t1f = sec * 1e3
    shares = []
    for r in range(W):
        sec, (lst, st) = timed(lambda: ctx.niceonly_raw(m.range_start, m.range_end, 50, chunk_size=10 ** 8,
                                                         msd_floor=THROUGHPUT_FLOOR, msd_where="device",
                                                         deal_stride=W, deal_offset=r), 3)
        shares.append({"rank": r, "wall_ms": sec * 1e3, "candidates": st.candidates, "msd_ranges": st.ranges,
                       "nice": len(lst)})
    tmax = max(x["wall_ms"] for x in shares)
    out.append({"config": f"massive-floor-{THROUGHPUT_FLOOR}-dealt-{W}", "mode": "niceonly", "base": 50,
                "size": m.range_size, "world": W, "msd_floor": THROUGHPUT_FLOOR, "max_share_wall_ms": tmax,
                "t1_wall_ms": t1f, "numbers_per_sec": m.range_size / (tmax / 1e3),
                "projected_efficiency": t1f / (W * tmax), "shares": shares})
    nice("msd-effective", get_benchmark_field(BM.MSD_EFFECTIVE), reps=3)
    nice("msd-ineffective", get_benchmark_field(BM.MSD_INEFFECTIVE))
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
