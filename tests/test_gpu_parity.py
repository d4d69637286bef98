"""GPU parity: the HIP path (through the C ABI) against the oracle and the
committed golden fixtures.  Bit-exact: histograms, near-miss lists, nice lists.

Run on the MI355X box:  python -m pytest tests -m gpu -x -q
"""
import json
import os
import random

import pytest

import nice_amd as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    c = N.GpuContext(0)
    yield c
    c.close()


def _dist(hist):
    return [(i, hist[i]) for i in range(1, len(hist))]


def check_detailed(ctx, start, end, base, want=None):
    hist, lst = ctx.detailed_raw(start, end, base)
    if want is None:
        want = O.process_range_detailed(start, end, base, cap=end - start)
    assert hist[0] == 0
    assert _dist(hist) == want.distribution, (base, start, end)
    assert lst == want.nice_numbers, (base, start, end)
    return hist, lst


# --- reference golden vectors (client_process.rs:473-1053) -------------------
def test_reference_detailed_vectors(ctx, golden):
    for c in golden["reference"]["detailed"]:
        b = c["base"]
        s, e = O.base_range(b)
        if c["size"]:
            e = s + c["size"]
        hist, lst = ctx.detailed_raw(s, e, b)
        assert _dist(hist) == [tuple(x) for x in c["distribution"]], c["source"]
        assert lst == [tuple(x) for x in c["nice_numbers"]], c["source"]


# --- reference-Python-mirror vectors (tests/golden/python_vectors.json) -------
def test_python_detailed_vectors(ctx, golden):
    for c in golden["python"]["detailed"]:
        hist, lst = ctx.detailed_raw(int(c["start"]), int(c["end"]), c["base"])
        assert _dist(hist) == [tuple(x) for x in c["distribution"]], c["name"]
        assert lst == [(int(n), u) for n, u in c["near_misses"]], c["name"]


def test_reference_gpu_test_ranges(ctx):
    # client_process_gpu.rs:1478-1498: (b10, [1e6, +1e4)) and (b40, [2e12, +1e5))
    check_detailed(ctx, 1_000_000, 1_010_000, 10)
    check_detailed(ctx, 2_000_000_000_000, 2_000_000_100_000, 40)


@pytest.mark.parametrize("base", [40, 50, 80])
def test_fd_kernel_segments(ctx, base):
    """FD kernel over in-range segments, including both range edges and
    segments straddling them (generic kernel outside, FD inside)."""
    s, e = O.base_range(base)
    check_detailed(ctx, s, s + 300_000, base)
    check_detailed(ctx, e - 300_000, e, base)
    check_detailed(ctx, s - 5_000, s + 5_000, base)
    check_detailed(ctx, e - 5_000, e + 5_000, base)
    mid = s + (e - s) // 3
    check_detailed(ctx, mid, mid + 1_000_003, base)
    # tiny and ragged sizes
    for size in (1, 2, 3, 63, 64, 65, 255, 257, 4097):
        check_detailed(ctx, mid + 7, mid + 7 + size, base)


def _fd2_cuts(base):
    """n where the production FD kernel's limb counts (D1 = 2e+1, E1 =
    3e^2+3e+1, E2 = 6e+6 in radix b^2 at a segment end e) change inside the
    valid range -- the host splits launches there (fd2_detailed.hip)."""
    B = base * base

    def limbs(x):
        k = 0
        while x >= B ** k:
            k += 1
        return k

    def combo(e):
        return (limbs(2 * e + 1), limbs(3 * e * e + 3 * e + 1), limbs(6 * e + 6))

    s, e = O.base_range(base)
    cuts, a = [], s
    while combo(a + 1) != combo(e):
        lo, hi, cur = a + 1, e, combo(a + 1)
        while lo < hi:
            mid = (lo + hi) // 2
            if combo(mid) == cur:
                lo = mid + 1
            else:
                hi = mid
        cuts.append(lo - 1)
        a = lo - 1
    return cuts


@pytest.mark.parametrize("base", [40, 50, 80])
def test_fd_kernel_limb_count_cuts(ctx, base):
    """Segments ending on, just past and straddling each limb-count cut use
    neighbouring kernel instantiations; all must agree with the oracle."""
    cuts = _fd2_cuts(base)
    assert len(cuts) == 2
    lib = N._lib.lib()
    buf = (N._lib.ctypes.c_uint64 * 16)()
    n = N._lib.ctypes.c_size_t()
    lib.nice_fd_segment_cuts(base, buf, 8, n)
    assert [buf[2 * i] | (buf[2 * i + 1] << 64) for i in range(n.value)] == cuts
    for c in cuts:
        check_detailed(ctx, c - 200_000, c + 200_000, base)
        check_detailed(ctx, c - 70_001, c, base)
        check_detailed(ctx, c, c + 70_001, base)
        check_detailed(ctx, c - 1, c + 2, base)


FD_BASES_NEW = [42, 43, 44, 45, 47, 48, 49, 52, 53, 54, 55, 57, 58, 59, 60, 62, 63, 64, 65, 67, 68]


@pytest.mark.parametrize("base", FD_BASES_NEW)
def test_fd_kernel_production_bases(ctx, base):
    """The FD kernel for every base 42..68 with a range (live fields are at
    b52-54, CHANGELOG.md:21; the reference specialises a kernel per base,
    client_process_gpu.rs:318-381): both range edges, segments straddling
    them (generic kernel outside), every limb-count cut, a random 2e6 window
    and ragged sizes, all against the oracle."""
    assert N._lib.lib().nice_fd_kernel_base(base) == 1
    s, e = O.base_range(base)
    check_detailed(ctx, s, s + 100_000, base)
    assert ctx.kernel_stats().fd_kernel
    check_detailed(ctx, e - 100_000, e, base)
    check_detailed(ctx, s - 3_000, s + 3_000, base)
    check_detailed(ctx, e - 3_000, e + 3_000, base)
    for c in _fd2_cuts(base):
        check_detailed(ctx, c - 50_001, c + 50_000, base)
        check_detailed(ctx, c - 1, c + 2, base)
    rng = random.Random(base)
    a = s + rng.randrange(e - s - 3 * 10 ** 6)
    check_detailed(ctx, a, a + 2 * 10 ** 6, base,
                   want=O.process_field_detailed_mt(a, a + 2 * 10 ** 6, base, 8))
    for size in (1, 2, 63, 65, 257, 4097):
        check_detailed(ctx, a + 11, a + 11 + size, base)


def test_fd_kernel_random_windows(ctx):
    rng = random.Random(7)
    for base in (40, 50, 80):
        s, e = O.base_range(base)
        for _ in range(4):
            a = s + rng.randrange(e - s - 200_000)
            check_detailed(ctx, a, a + rng.randrange(1, 200_000), base)


def test_generic_kernel_bases(ctx):
    rng = random.Random(11)
    for base in (2, 3, 7, 10, 12, 16, 25, 31, 32, 33, 45, 57, 62, 63, 64, 65, 68, 70, 94, 97,
                 100, 127, 128):
        r = O.base_range(base) if base <= 97 else None
        if r:
            s = r[0] + rng.randrange(max(1, r[1] - r[0]))
        else:
            s = rng.randrange(1, 1 << 100)
        check_detailed(ctx, s, s + 3_000, base)


def test_out_of_range_large_lists(ctx):
    # near-miss list much larger than typical (SURVEY hazard 9) and huge n
    check_detailed(ctx, 1_000_000, 1_200_000, 10)
    big = (1 << 127) + 12345
    check_detailed(ctx, big, big + 2_000, 97)
    check_detailed(ctx, (1 << 128) - 1_000, (1 << 128) - 1, 128)


def test_device_unique_counts_samples(ctx, golden):
    for c in golden["python"]["samples"]:
        ns = [int(n) for n in c["n"]]
        assert ctx.debug_unique_counts(ns, c["base"]) == c["num_uniques"], c["base"]
    wild = golden["python"]["wild"]
    for n, b, u in wild:
        assert ctx.debug_unique_counts([int(n)], b) == [u], (n, b)


def test_device_is_nice(ctx, golden):
    assert ctx.debug_is_nice([69, 70, 47, 99], 10) == [True, False, False, False]
    rng = random.Random(3)
    for base in (10, 12, 25, 40, 45, 50, 62, 80, 97):
        s, e = O.base_range(base)
        ns = [s + rng.randrange(e - s) for _ in range(500)] + list(range(s, s + 500))
        want = [O.is_nice(n, base) for n in ns]
        assert ctx.debug_is_nice(ns, base) == want, base
    # out-of-range small n: reference CPU semantics (no repeat => "nice")
    ns = list(range(1, 200))
    assert ctx.debug_is_nice(ns, 10) == [O.is_nice(n, 10) for n in ns]


@pytest.mark.parametrize("base", [40, 50, 52, 53, 54, 80])
def test_device_unique_fast_path(ctx, golden, base):
    """The niceonly kernel's in-range test is "the digit union of n^2 and n^3
    has b members" (radix_fast.hpp is_nice_limbs).  No nice number is known at
    these bases, so its True branch is pinned through the count itself: the
    device limb path's unique counts equal the oracle's on both range ends,
    random n, and the Python-mirror samples of this base."""
    rng = random.Random(11 * base)
    s, e = O.base_range(base)
    ns = [s, s + 1, e - 2, e - 1] + [rng.randrange(s, e) for _ in range(3000)]
    want = [O.num_unique_digits(n, base) for n in ns]
    for c in golden["python"]["samples"]:
        if c["base"] == base:
            ins = [(int(n), u) for n, u in zip(c["n"], c["num_uniques"]) if s <= int(n) < e]
            ns += [n for n, _ in ins]
            want += [u for _, u in ins]
    assert ctx.debug_unique_fast(ns, base) == want


# --- niceonly ---------------------------------------------------------------
def test_niceonly_reference_vectors(ctx, golden):
    for c in golden["reference"]["niceonly"]:
        b = c["base"]
        s, e = O.base_range(b)
        if c["size"]:
            e = s + c["size"]
        r = N.process_range_niceonly_gpu(ctx, N.FieldSize(s, e), b)
        assert [(x.number, x.num_uniques) for x in r.nice_numbers] == \
            [tuple(x) for x in c["nice_numbers"]], c["source"]


MSD_WHERE = ["host", "device"]


@pytest.mark.parametrize("where", MSD_WHERE)
@pytest.mark.parametrize("base", [10, 12, 25, 40, 45, 52, 53, 54, 62, 97])
def test_niceonly_matches_oracle(ctx, base, where):
    # client_process_gpu.rs:1500-1534: first 5e6 of each base's range
    s, e = O.base_range(base)
    e = min(e, s + 5_000_000)
    lst, st = ctx.niceonly_raw(s, e, base, msd_where=where)
    want, cands = O.process_field_niceonly_mt(s, e, base, threads=8)
    assert [(n, base) for n in lst] == want.nice_numbers
    assert st.candidates == cands, "candidate set differs from the CPU path"


@pytest.mark.parametrize("where", MSD_WHERE)
def test_niceonly_candidate_counts(ctx, where):
    rng = random.Random(5)
    for base in (40, 50, 52, 53, 54, 80):
        s, e = O.base_range(base)
        for _ in range(3):
            a = s + rng.randrange(e - s - 10 ** 8)
            size = rng.choice([10 ** 6, 10 ** 7, 3 * 10 ** 7])
            lst, st = ctx.niceonly_raw(a, a + size, base, msd_where=where)
            want, cands = O.process_field_niceonly_mt(a, a + size, base, threads=8)
            assert st.candidates == cands and [(n, base) for n in lst] == want.nice_numbers


def test_niceonly_coarse_floor_superset(ctx):
    # Coarser MSD floors (reference GPU path, client_process_gpu.rs:82-123) check
    # a superset of candidates and find the same nice numbers.
    lst, st = ctx.niceonly_raw(47, 10 ** 5, 10, msd_floor=4000)
    assert 69 in lst
    s, _ = O.base_range(40)
    a, b = ctx.niceonly_raw(s, s + 10 ** 8, 40)
    c, d = ctx.niceonly_raw(s, s + 10 ** 8, 40, msd_floor=64000)
    assert a == c and d.candidates >= b.candidates


def test_niceonly_device_msd_edges(ctx):
    # Ragged / tiny ranges, custom chunking, deep recursion (floor 1 -> depth
    # limit 22), chunk boundaries: the device MSD must reproduce the host MSD
    # candidate set exactly.
    rng = random.Random(11)
    cases = []
    for base in (40, 50, 80, 10, 33):
        s, e = O.base_range(base)
        for size in (1, 2, 63, 250, 499, 500, 501, 10 ** 4 + 7):
            a = s + rng.randrange(max(1, e - s - size))
            cases.append((base, a, min(e, a + size), {}))
    s40 = O.base_range(40)[0]
    cases += [
        (40, s40 + 12345, s40 + 12345 + 3_000_001, {"chunk_size": 999_983}),
        (40, s40, s40 + 2_000_000, {"msd_floor": 1}),
        (40, s40 + 5, s40 + 40_000_000, {"msd_floor": 7, "chunk_size": 5_000_000}),
        (50, O.base_range(50)[0], O.base_range(50)[0] + 10 ** 7, {"msd_floor": 1000}),
    ]
    for base, a, b, kw in cases:
        h_l, h_st = ctx.niceonly_raw(a, b, base, msd_where="host", **kw)
        d_l, d_st = ctx.niceonly_raw(a, b, base, msd_where="device", **kw)
        assert d_l == h_l and d_st.candidates == h_st.candidates, (base, a, b, kw)
        if not kw:
            want, cands = O.process_field_niceonly_mt(a, b, base, threads=8)
            assert d_st.candidates == cands and [(n, base) for n in d_l] == want.nice_numbers


def test_niceonly_multi_device_context():
    import torch
    n = torch.cuda.device_count()
    devs = [0, 0] if n < 2 else [0, 1]
    c = N.GpuContext(devs)
    s = O.base_range(40)[0]
    # 3e8 at chunk 1e6, floor 4 -> 5 device-MSD batches alternating over devices
    for where in MSD_WHERE:
        lst, st = c.niceonly_raw(s, s + 3 * 10 ** 8, 40, msd_where=where, chunk_size=10 ** 6,
                                 msd_floor=4)
        one, st1 = N.GpuContext([0]).niceonly_raw(s, s + 3 * 10 ** 8, 40, msd_where=where,
                                                  chunk_size=10 ** 6, msd_floor=4)
        assert lst == one and st.candidates == st1.candidates
        assert (st.ranges, st.square_ok) == (st1.ranges, st1.square_ok)
    # the wave path on a massive window with candidates: one batch per device
    a = int(_massive()["start"]) + 8 * 10 ** 12
    lst, st = c.niceonly_raw(a, a + 16 * 10 ** 8, 50, chunk_size=10 ** 8, msd_where="device")
    one, st1 = N.GpuContext([0]).niceonly_raw(a, a + 16 * 10 ** 8, 50, chunk_size=10 ** 8,
                                              msd_where="device")
    assert lst == one and st.square_ok > 0 and st.launches == 2
    assert (st.candidates, st.ranges, st.square_ok) == (st1.candidates, st1.ranges, st1.square_ok)
    c.close()


@pytest.mark.parametrize("where", MSD_WHERE)
@pytest.mark.parametrize("path", ["fused", "wave"])
def test_niceonly_below_range_windows(ctx, where, path):
    """Windows below a base's valid range, where get_is_nice lists every n
    whose n^2 and n^3 digits are merely distinct (no digit-count test,
    client_process.rs:258-290; process_range_niceonly lists them, :439-465):
    b10 [1, 47) -> 3, 8, 9, 24; b40 [1, 1e5) -> 265 numbers.  Nice list,
    candidates and MSD ranges against the oracle on the same chunk grid, for
    both MSD placements, through the fused per-chunk kernel (client chunking)
    and the wave kernel (1e8 chunks)."""
    chunk = 10 ** 8 if path == "wave" else 0
    cases = [(10, 1, 47, 4), (16, 1, 60, 5), (25, 1, 10 ** 4, 19), (40, 1, 10 ** 5, 265),
             (12, 1, 2_000, None), (64, 10 ** 6, 10 ** 6 + 5 * 10 ** 5, None)]
    for base, a, b, count in cases:
        res, cands, ranges, _ = O.process_field_niceonly_sq(a, b, base, 4, chunk)
        want = [n for n, _ in res.nice_numbers]
        if count is not None:
            assert len(want) == count, base
        lst, st = ctx.niceonly_raw(a, b, base, chunk_size=chunk, msd_where=where)
        assert lst == want, (base, a, b)
        assert (st.candidates, st.ranges) == (cands, ranges), (base, a, b)
    assert ctx.niceonly_raw(1, 47, 10, chunk_size=chunk, msd_where=where)[0] == [3, 8, 9, 24]


def test_slots_reused_after_out_of_order_collect(ctx):
    """Tickets are collected in any order (nice_hip.h): after submit t0, t1, t2
    and collect t1, a new submit takes the free slot instead of failing."""
    s40 = O.base_range(40)[0]
    fields = [(s40 + k * 10 ** 6, s40 + (k + 1) * 10 ** 6) for k in range(4)]
    want = [ctx.detailed_raw(a, b, 40) for a, b in fields]
    t = [ctx.detailed_submit(a, b, 40) for a, b in fields[:3]]
    assert ctx.detailed_collect(t[1], 40) == want[1]
    t3 = ctx.detailed_submit(*fields[3], 40)
    assert t3 == t[1]
    assert [ctx.detailed_collect(x, 40) for x in (t[0], t[2], t3)] == [want[0], want[2], want[3]]
    nice_want = [ctx.niceonly_raw(a, b, 40) for a, b in fields]
    t = [ctx.niceonly_submit(a, b, 40) for a, b in fields[:3]]
    got2 = ctx.niceonly_collect(t[2])
    t3 = ctx.niceonly_submit(*fields[3], 40)
    got = [ctx.niceonly_collect(x) for x in (t[0], t[1], t3)]
    for (l, st), (wl, wst) in zip([got[0], got[1], got2, got[2]], nice_want):
        assert l == wl and st.candidates == wst.candidates and st.ranges == wst.ranges


def test_residue_empty_base(ctx):
    assert ctx.niceonly_raw(100, 200, 11)[0] == []


# --- full BASELINE-size fields against the committed oracle fixtures --------
def _oracle_fields():
    p = os.path.join(ROOT, "tests", "golden", "oracle_fields.json")
    if not os.path.exists(p):
        pytest.skip("oracle_fields.json not generated")
    with open(p) as f:
        return json.load(f)


def test_full_fields_detailed(ctx):
    for c in _oracle_fields()["detailed"]:
        hist, lst = ctx.detailed_raw(int(c["start"]), int(c["end"]), c["base"])
        assert _dist(hist) == [tuple(x) for x in c["distribution"]], c["name"]
        assert lst == [(int(n), u) for n, u in c["near_misses"]], c["name"]


@pytest.mark.parametrize("where", MSD_WHERE)
def test_full_fields_niceonly(ctx, where):
    for c in _oracle_fields()["niceonly"]:
        lst, st = ctx.niceonly_raw(int(c["start"]), int(c["end"]), c["base"], msd_where=where)
        assert st.candidates == c["candidates"], c["name"]
        assert [str(n) for n in lst] == c["nice_numbers"], c["name"]


def test_size_independent_properties(ctx):
    # Whole b40 extra-large field: histogram mass = field size, split invariance
    # (two halves sum to the whole), near-miss bins consistent with the list.
    s = O.base_range(40)[0]
    e = s + 10 ** 9
    h, l = ctx.detailed_raw(s, e, 40)
    assert sum(h) == 10 ** 9
    m = s + 333_333_337
    h1, l1 = ctx.detailed_raw(s, m, 40)
    h2, l2 = ctx.detailed_raw(m, e, 40)
    assert [a + b for a, b in zip(h1, h2)] == h and l1 + l2 == l
    cutoff = O.near_miss_cutoff(40)
    assert sum(h[cutoff + 1:]) == len(l)
    assert all(O.num_unique_digits(n, 40) == u for n, u in l)
    # determinism
    assert ctx.detailed_raw(s, e, 40) == (h, l)


@pytest.mark.parametrize("base", [40, 65, 67, 68, 80])
def test_big_field_kernel_equals_small_field_kernel(ctx, base):
    """Fields >= 1e7 run the big-field instantiation (1024-thread workgroups,
    the three-mask-word bases with lookup groups, 64 histogram copies); fields
    < 1e7 the 512-thread one (16 copies), pinned against the oracle by
    test_fd_kernel_production_bases.  A 2e7 window 1/4 into the range must
    equal the sum of its twenty 1e6 sub-windows (histogram) and their
    concatenation (near-miss list); every near-miss recomputes by the oracle."""
    r0, r1 = O.base_range(base)
    s = r0 + (r1 - r0) // 4
    h, l = ctx.detailed_raw(s, s + 2 * 10 ** 7, base)
    assert sum(h) == 2 * 10 ** 7
    hs, ls = [0] * len(h), []
    for k in range(20):
        a = s + k * 10 ** 6
        hk, lk = ctx.detailed_raw(a, a + 10 ** 6, base)
        hs = [x + y for x, y in zip(hs, hk)]
        ls += lk
    assert h == hs and l == ls
    assert sum(h[O.near_miss_cutoff(base) + 1:]) == len(l)
    assert all(O.num_unique_digits(n, base) == u for n, u in l)


@pytest.mark.parametrize("base", [42, 45, 49, 55, 58, 59, 64, 65, 67, 68])
def test_persistent_grid_equals_rounds(ctx, base):
    """Bases whose big-field kernel holds one workgroup per CU run segments of
    >= 2 rounds (2 x TCHUNK x resident lanes: 4.2e7 numbers at TCHUNK 80,
    8.4e7 at 160, 1.26e8 at 240 on 256 CUs) on the persistent grid (waves
    pull strided 64-unit batches; 1024-thread workgroups).  2.5e7 windows
    are below every base's threshold, so they run in rounds of workgroups
    (b42..50 and b59..64 at 512 threads).  A 1e9 field must equal the sum of
    its forty 2.5e7 windows, and every near-miss recomputes by the oracle.
    (b52-54 and b80 1e9 are pinned to oracle fixtures in
    test_fd_bases_whole_fields_1e9.)"""
    r0, r1 = O.base_range(base)
    s = r0 + (r1 - r0) // 3
    h, l = ctx.detailed_raw(s, s + 10 ** 9, base)
    w = 25 * 10 ** 6
    hs, ls = [0] * len(h), []
    for k in range(40):
        hk, lk = ctx.detailed_raw(s + k * w, s + (k + 1) * w, base)
        hs = [x + y for x, y in zip(hs, hk)]
        ls += lk
    assert h == hs and l == ls and sum(h) == 10 ** 9
    assert all(O.num_unique_digits(n, base) == u for n, u in l)


@pytest.mark.parametrize("base,size", [(40, 32 * 10 ** 9), (80, 16 * 10 ** 9)])
def test_detailed_field_longer_than_one_launch(ctx, base, size):
    """launch_cfg (fd2_kernel.hpp) splits a segment into launches of at most
    60 000 numbers per resident lane: 3.1e10 at b40 (two 1024-thread
    workgroups per CU), 1.6e10 at b80 (one, persistent grid); the field's
    finish rides on its last launch.  The reference batches any field size
    (client_process_gpu.rs:832-856).  A field above one launch must report
    more than one launch, hold exactly its size in the histogram, equal the
    sum of two halves that each fit one launch, and every near-miss must
    recompute by the oracle."""
    r0, r1 = O.base_range(base)
    s = r0 + (r1 - r0) // 5
    h, l = ctx.detailed_raw(s, s + size, base)
    assert ctx.kernel_stats().launches >= 2
    assert sum(h) == size
    m = s + size // 2 + 12_345
    h1, l1 = ctx.detailed_raw(s, m, base)
    assert ctx.kernel_stats().launches == 1
    h2, l2 = ctx.detailed_raw(m, s + size, base)
    assert [a + b for a, b in zip(h1, h2)] == h and l1 + l2 == l
    assert sum(h[O.near_miss_cutoff(base) + 1:]) == len(l)
    assert all(O.num_unique_digits(n, base) == u for n, u in l)


# Where the per-layout VALU-decode choice of fields >= 1e7 (valu_limbs_big,
# fd2_kernel.hpp) changes the kernel: b40 on its 8-limb n^3 layouts and
# b50/53/60 (below-top decode), b65/67/68
# (limb 0 + two / three below the top), b80 on its 16-limb layouts (the first
# ~40 % of the range) and on the 17-limb one (four below the top).
BIG_VD_CASES = [(40, 0.0), (40, 0.1), (40, 0.35), (40, 0.7), (50, 0.0), (50, 0.6), (53, 0.3), (60, 0.0), (60, 0.7), (65, 0.0), (65, 0.5), (67, 0.4),
                (68, 0.0), (68, 0.8), (80, 0.0), (80, 0.05), (80, 0.2), (80, 0.33), (80, 0.6), (80, 0.95)]


@pytest.mark.parametrize("base,frac", BIG_VD_CASES)
def test_big_field_valu_decode_variants(ctx, base, frac):
    """A 2e7 field takes the >= 1e7 kernel (1024-thread persistent grid, its
    valu_limbs_big choice); its four 5e6 quarters take the small-field
    kernel (512 threads, the base's other VALU-decode choice), which the
    oracle fuzz pins.  The histograms must add up and the near-miss lists
    concatenate exactly, and every near-miss must recompute by the oracle."""
    r0, r1 = O.base_range(base)
    s = r0 + int((r1 - r0) * frac)
    size, q = 2 * 10 ** 7, 5 * 10 ** 6
    h, l = ctx.detailed_raw(s, s + size, base)
    assert sum(h) == size
    hs, ls = [0] * len(h), []
    for k in range(4):
        hk, lk = ctx.detailed_raw(s + k * q, s + (k + 1) * q, base)
        hs = [a + b for a, b in zip(hs, hk)]
        ls += lk
    assert hs == h and ls == l, (base, frac)
    assert all(O.num_unique_digits(n, base) == u for n, u in l)


@pytest.mark.parametrize("where", MSD_WHERE)
@pytest.mark.parametrize("chunk", [0, 10 ** 8])
def test_niceonly_list_longer_than_device_capacity(ctx, where, chunk):
    """b100 [1, 1e7) lies below b100's valid range, where get_is_nice lists
    every n whose n^2 and n^3 digits are merely distinct
    (client_process.rs:222-253): 70 636 numbers on the client's 1e6 chunk
    grid, 72 207 as ONE chunk (the CPU API's whole-range call,
    client_process.rs:439-465; Filter C makes the two differ).  Both exceed
    the device list's initial 2^16 entries, so the library grows the list
    to the count the kernels report and re-runs the field.  Nice list,
    candidates and MSD ranges against the oracle (cap 2^22), for both MSD
    placements; then the same field through submit / collect with a caller
    list too small (NICE_ERR_CAPACITY with the true length, results kept for
    the retry)."""
    res, cands, ranges, _ = O.process_field_niceonly_sq(1, 10 ** 7, 100, 8, chunk, 0, cap=1 << 22)
    want = [n for n, _ in res.nice_numbers]
    assert len(want) == (72_207 if chunk else 70_636)
    lst, st = ctx.niceonly_raw(1, 10 ** 7, 100, chunk_size=chunk, msd_where=where)
    assert lst == want
    assert (st.candidates, st.ranges) == (cands, ranges)
    lib = N._lib.lib()
    ct = N._lib.ctypes
    t = ctx.niceonly_submit(1, 10 ** 7, 100, chunk_size=chunk, msd_where=where)
    out = (N._lib.nice_number * 16)()
    n = ct.c_size_t()
    st2 = N._lib.nice_niceonly_stats()
    assert lib.nice_niceonly_collect(ctx._h, t, out, 16, n, st2) == N._lib.NICE_ERR_CAPACITY
    assert n.value == len(want)
    got, st3 = ctx.niceonly_collect(t, cap=n.value)
    assert got == want and st3.candidates == cands


def test_collect_waits_without_holding_the_context(ctx):
    """A collect waits for its field outside the context lock: while thread
    A collects a long b80 field, thread B submits (and collects) a detailed
    and a niceonly field on the same context -- the pipelined loop of the
    reference client (client/src/main.rs:411-562) with one thread per stage.
    B's submits must return before A's collect does, and every result must
    equal the synchronous call's.  Raw ABI calls with per-thread buffers."""
    import threading
    import time
    lib = N._lib.lib()
    ct = N._lib.ctypes
    s40, s80 = O.base_range(40)[0], O.base_range(80)[0]
    big = (s80, s80 + 5 * 10 ** 9)  # ~35 ms
    small = (s40 + 7 * 10 ** 6, s40 + 8 * 10 ** 6)
    want_big = ctx.detailed_raw(*big, 80)
    want_small = ctx.detailed_raw(*small, 40)
    want_nice = ctx.niceonly_raw(*small, 40)[0]

    def submit_det(a, b, base):
        t = ct.c_int()
        assert lib.nice_detailed_submit(ctx._h, *N.api._split(a), *N.api._split(b), base, t) == 0
        return t.value

    def collect_det(t, base):
        hist = (ct.c_uint64 * (base + 1))()
        out = (N._lib.nice_number * 4096)()
        n = ct.c_size_t()
        assert lib.nice_detailed_collect(ctx._h, t, hist, out, 4096, n) == 0, lib.nice_last_error()
        return list(hist), [(out[i].number_lo | (out[i].number_hi << 64), out[i].num_uniques)
                            for i in range(n.value)]

    res = {}
    t_big = submit_det(*big, 80)

    def a_thread():
        res["big"] = collect_det(t_big, 80)
        res["big_done"] = time.perf_counter()

    th = threading.Thread(target=a_thread)
    th.start()
    time.sleep(0.003)  # A is inside its collect
    t_small = submit_det(*small, 40)
    tn = ct.c_int()
    opts = N.GpuContext._nice_opts()
    assert lib.nice_niceonly_submit(ctx._h, *N.api._split(small[0]), *N.api._split(small[1]), 40,
                                    opts, tn) == 0
    submitted = time.perf_counter()
    got_small = collect_det(t_small, 40)
    out = (N._lib.nice_number * 16)()
    n = ct.c_size_t()
    assert lib.nice_niceonly_collect(ctx._h, tn.value, out, 16, n, None) == 0
    th.join()
    assert submitted < res["big_done"], "submit waited for the other thread's collect"
    assert res["big"] == want_big and got_small == want_small
    assert [out[i].number_lo | (out[i].number_hi << 64) for i in range(n.value)] == want_nice


def test_untimed_fields_match_timed():
    """With kernel timing off (nice_ctx_set_kernel_timing) a detailed field
    records no HIP events; its completion comes from the published sequence
    word and the slot's stream.  Results must equal the timed context's,
    including fields with near-miss lists (read after the stream drains),
    generic-kernel fields (finish kernel) and asynchronous tickets; kernel_ms
    reads 0."""
    c = N.GpuContext(0)
    c.set_kernel_timing(False)
    s40, s80 = O.base_range(40)[0], O.base_range(80)[0]
    cases = [(s40, s40 + 10 ** 6, 40), (s80, s80 + 10 ** 6, 80), (10 ** 6, 10 ** 6 + 10 ** 4, 10),
             (s40 - 5000, s40 + 5000, 40), (s40, s40 + 10 ** 9, 40)]
    for a, b, base in cases:
        want = O.process_range_detailed(a, b, base, cap=b - a) if b - a <= 10 ** 6 else None
        got = c.detailed_raw(a, b, base)
        if want is not None:
            assert got == ([0] + [n for _, n in want.distribution], want.nice_numbers), (base, a, b)
        else:
            assert got == ctx_timed_detailed(a, b, base)
        assert c.kernel_stats().kernel_ms == 0
    t = [c.detailed_submit(a, b, base) for a, b, base in cases[:3]]
    assert [c.detailed_collect(x, base) for x, (_, _, base) in zip(t, cases[:3])] == \
        [c.detailed_raw(a, b, base) for a, b, base in cases[:3]]
    c.set_kernel_timing(True)
    c.detailed_raw(*cases[0])
    assert c.kernel_stats().kernel_ms > 0
    c.close()


def ctx_timed_detailed(a, b, base):
    c = N.GpuContext(0)
    try:
        return c.detailed_raw(a, b, base)
    finally:
        c.close()


def test_multi_device_context_sharding():
    import torch
    n = torch.cuda.device_count()
    devs = [0, 0] if n < 2 else [0, 1]
    c = N.GpuContext(devs)
    s = O.base_range(40)[0]
    want = O.process_range_detailed(s, s + 100_001, 40)
    hist, lst = c.detailed_raw(s, s + 100_001, 40)
    assert _dist(hist) == want.distribution and lst == want.nice_numbers
    c.close()


def test_both_modes_overlapped_matches_fixtures(ctx):
    # BothModes (bench.py's default): niceonly on a second stream beside the
    # detailed kernel; both results must equal the committed full-field
    # fixtures, repeatedly (the two streams share the device).
    fields = _oracle_fields()
    det = {c["name"]: c for c in fields["detailed"]}
    b = N.BothModes(0, det_ctx=ctx)
    try:
        for c in fields["niceonly"]:
            s, e, base = int(c["start"]), int(c["end"]), c["base"]
            d = next((x for x in det.values() if (int(x["start"]), int(x["end"]), x["base"])
                      == (s, e, base)), None)
            for _ in range(2):
                (hist, near), (nice, st) = b.both_raw((s, e), (s, e), base)
                assert st.candidates == c["candidates"], c["name"]
                assert [str(n) for n in nice] == c["nice_numbers"], c["name"]
                assert sum(hist) == e - s
                if d is not None:
                    assert _dist(hist) == [tuple(x) for x in d["distribution"]], c["name"]
                    assert near == [(int(n), u) for n, u in d["near_misses"]], c["name"]
        (hist, near), (nice, _) = b.both_raw((47, 100), (47, 100), 10)
        assert near == [(69, 10)] and nice == [69]
    finally:
        b.close()


@pytest.mark.parametrize("where", MSD_WHERE)
def test_niceonly_dealt_chunks_partition_the_field(ctx, where):
    """deal_stride / deal_offset (the N-way niceonly split, nice_amd/dist.py):
    the N dealt runs together are the single run -- same candidates, same
    ranges, same nice list -- for several N and chunkings, and each dealt run
    equals the oracle over exactly its chunks."""
    from nice_amd.dist import dealt_chunks
    s10 = 47
    cases = [(10, s10, 10 ** 5, 997, 3), (40, O.base_range(40)[0], O.base_range(40)[0] + 10 ** 8,
                                          10 ** 6, 8)]
    s50 = O.base_range(50)[0] + 7_372_000_000_000
    cases.append((50, s50, s50 + 2 * 10 ** 9, 10 ** 7, 8))
    for base, a, b, chunk, world in cases:
        whole, st = ctx.niceonly_raw(a, b, base, chunk_size=chunk, msd_where=where)
        got, cands, ranges = [], 0, 0
        for r in range(world):
            lst, sr = ctx.niceonly_raw(a, b, base, chunk_size=chunk, msd_where=where,
                                       deal_stride=world, deal_offset=r)
            got += lst
            cands += sr.candidates
            ranges += sr.ranges
            if r == 1:
                want = sum((O.process_field_niceonly_ex(cs, ce, base, 8, chunk=chunk)[1]
                            for cs, ce in dealt_chunks(a, b, chunk, world, r)), 0)
                assert sr.candidates == want, (base, r)
        assert sorted(got) == whole and cands == st.candidates and ranges == st.ranges, base
    assert ctx.niceonly_raw(47, 100, 10, chunk_size=10, deal_stride=8, deal_offset=7)[0] == []


def test_env_msd_floor_pins_the_floor():
    """NICE_GPU_MSD_FLOOR (client_process_gpu.rs:161-172) pins the MSD floor
    when the caller passes none; an invalid value is ignored."""
    import subprocess
    import sys
    s = O.base_range(40)[0]
    code = ("import sys; sys.path.insert(0, %r); import nice_amd as N; c = N.GpuContext(0); "
            "print(c.niceonly_raw(%d, %d, 40)[1].candidates)" % (ROOT, s, s + 10 ** 8))
    def run(env_val):
        env = dict(os.environ)
        env.pop("NICE_GPU_MSD_FLOOR", None)
        if env_val is not None:
            env["NICE_GPU_MSD_FLOOR"] = env_val
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                             text=True, timeout=120, check=True)
        return int(out.stdout.strip().splitlines()[-1])
    pinned = run("64000")
    assert pinned == ctx_free_candidates(s, s + 10 ** 8, 64000)
    assert run("bogus") == run(None) == ctx_free_candidates(s, s + 10 ** 8, 250)


def test_adaptive_msd_floor_host_path():
    """msd_floor="adaptive" (AdaptiveFloor, client_process_gpu.rs:96-184,
    551-568) on the host-MSD path, in a fresh process: each field's floor is
    the seed for the 3 warmup fields, then follows the reference's step of the
    previous field's msd / gpu-tail seconds; the candidates are a superset of
    the floor-250 set and the nice list is the oracle's."""
    import subprocess
    import sys
    s40 = O.base_range(40)[0]
    fields = [(47, 100, 10)] + [(s40 + k * 5 * 10 ** 7, s40 + (k + 1) * 5 * 10 ** 7, 40) for k in range(5)]
    code = ("import sys, json; sys.path.insert(0, %r); import nice_amd as N; c = N.GpuContext(0); "
            "f0 = N.adaptive_floor(); out = []\n"
            "for a, b, base in %r:\n"
            "    lst, st = c.niceonly_raw(a, b, base, msd_floor='adaptive', msd_where='host')\n"
            "    out.append([lst, st.msd_floor, st.msd_seconds, st.total_seconds, st.candidates])\n"
            "print(json.dumps([f0, out, N.adaptive_floor()]))" % (ROOT, fields))
    env = dict(os.environ)
    env.pop("NICE_GPU_MSD_FLOOR", None)
    res = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         timeout=300, check=True)
    (floor, warm), rows, last = json.loads(res.stdout.strip().splitlines()[-1])
    assert warm == 3
    for k, ((a, b, base), (lst, used, msd, total, cands)) in enumerate(zip(fields, rows)):
        assert used == int(floor), (k, used, floor)
        if k >= 3:
            floor = N.adaptive_floor_step(floor, msd, total)
        want, _ = O.process_range_niceonly(a, b, base)
        assert lst == [n for n, _ in want.nice_numbers]
        assert cands >= ctx_free_candidates(a, b, 250, base)
    assert last[0] == pytest.approx(floor) and last[1] == 0


def ctx_free_candidates(a, b, floor, base=40):
    c = N.GpuContext(0)
    try:
        return c.niceonly_raw(a, b, base, msd_floor=floor)[1].candidates
    finally:
        c.close()


def test_async_fields_match_sync(ctx):
    """nice_detailed/niceonly_submit + _collect: three fields in flight per
    mode, collected in any order, equal the synchronous calls; a fourth submit
    is refused; a too-small list keeps the results for a retry."""
    s40 = O.base_range(40)[0]
    fa, fb = (s40, s40 + 3 * 10 ** 7), (s40 + 10 ** 9, s40 + 10 ** 9 + 2 * 10 ** 7 + 17)
    fc = (s40 + 77, s40 + 77 + 5 * 10 ** 6)
    want_a, want_b, want_c = (ctx.detailed_raw(*f, 40) for f in (fa, fb, fc))
    ta = ctx.detailed_submit(*fa, 40)
    tb = ctx.detailed_submit(*fb, 40)
    tc = ctx.detailed_submit(*fc, 40)
    with pytest.raises(N.NiceError):
        ctx.detailed_submit(*fa, 40)
    assert ctx.detailed_collect(tb, 40) == want_b
    assert ctx.detailed_collect(tc, 40) == want_c
    assert ctx.detailed_collect(ta, 40) == want_a
    # near-miss lists through the async path (b10 out of range: 5 395 entries)
    t = ctx.detailed_submit(10 ** 6, 10 ** 6 + 10 ** 4, 10)
    lib = N._lib.lib()
    hist = (N._lib.ctypes.c_uint64 * 11)()
    out = (N._lib.nice_number * 10)()
    n = N._lib.ctypes.c_size_t()
    assert lib.nice_detailed_collect(ctx._h, t, hist, out, 10, n) == N._lib.NICE_ERR_CAPACITY
    assert n.value == 5395
    want = O.process_range_detailed(10 ** 6, 10 ** 6 + 10 ** 4, 10, cap=10 ** 4)
    h, lst = ctx.detailed_collect(t, 10, cap=n.value)
    assert lst == want.nice_numbers and [(i, h[i]) for i in range(1, 11)] == want.distribution
    # niceonly, device and host MSD, interleaved with detailed fields
    n1 = ctx.niceonly_submit(*fa, 40)
    d1 = ctx.detailed_submit(*fb, 40)
    n2 = ctx.niceonly_submit(47, 100, 10, msd_where="host")
    assert ctx.niceonly_collect(n2)[0] == [69]
    lst, st = ctx.niceonly_collect(n1)
    wl, wst = ctx.niceonly_raw(*fa, 40)
    assert lst == wl and st.candidates == wst.candidates and st.ranges == wst.ranges
    assert ctx.detailed_collect(d1, 40) == want_b


def test_field_pipeline_on_gpu():
    """dist.FieldPipeline (bench.py's step) on one GPU: results one field late,
    every field equal to the committed fixture."""
    from nice_amd import dist as D
    c = _oracle_fields()
    det = next(x for x in c["detailed"] if x["name"] == "b40_extra_large_1e9")
    nic = next(x for x in c["niceonly"] if x["name"] == "b40_extra_large_1e9")
    a, b = N.GpuContext(0), N.GpuContext(0)
    try:
        pipe = D.FieldPipeline(a, b)
        f = N.FieldSize(int(det["start"]), int(det["end"]))
        got = [pipe.step(f, 40) for _ in range(4)]
        got = [g for g in got if g is not None] + pipe.drain()
        assert len(got) == 4
        for r, d, n, st in got:
            assert r == f
            assert [(x.num_uniques, x.count) for x in d.distribution] == \
                [tuple(x) for x in det["distribution"]]
            assert [(x.number, x.num_uniques) for x in d.nice_numbers] == \
                [(int(n_), u) for n_, u in det["near_misses"]]
            assert st.candidates == nic["candidates"] and [x.number for x in n.nice_numbers] == []
    finally:
        a.close()
        b.close()


def test_fd_bases_whole_fields_1e9(ctx):
    """The CLI hi-base field (b80 1e9, benchmark.rs:63) and the live bases
    52 / 53 / 54 (1e9 from each range start): the whole field's distribution
    and near-miss list against the oracle fixture (gen_fd_bases_fixtures.py)."""
    p = os.path.join(ROOT, "tests", "golden", "fd_bases_1e9.json")
    with open(p) as f:
        fx = json.load(f)
    assert [c["base"] for c in fx["detailed"]] == [80, 52, 53, 54]
    for c in fx["detailed"]:
        hist, lst = ctx.detailed_raw(int(c["start"]), int(c["end"]), c["base"])
        assert _dist(hist) == [tuple(x) for x in c["distribution"]], c["name"]
        assert lst == [(int(n), u) for n, u in c["near_misses"]], c["name"]
        assert ctx.kernel_stats().fd_kernel == 1


def test_fd_bases_more_whole_fields_1e9(ctx):
    """One 1e9 field per FD kernel class the CLI fields do not cover (b42:
    TCHUNK 80; b49: 160; b59: 240 with the side-table low-digit path; b65:
    three mask words), one third into each range, all on the persistent grid:
    distribution and near-miss list against the oracle fixture
    (gen_fd_bases_fixtures.py --more)."""
    p = os.path.join(ROOT, "tests", "golden", "fd_bases_more_1e9.json")
    with open(p) as f:
        fx = json.load(f)
    for c in fx["detailed"]:
        hist, lst = ctx.detailed_raw(int(c["start"]), int(c["end"]), c["base"])
        assert _dist(hist) == [tuple(x) for x in c["distribution"]], c["name"]
        assert lst == [(int(n), u) for n, u in c["near_misses"]], c["name"]
        assert ctx.kernel_stats().fd_kernel == 1


# --- massive config (benchmark.rs:62): b50 [start, +1e13), niceonly ----------
def _massive():
    p = os.path.join(ROOT, "tests", "golden", "massive_b50.json")
    with open(p) as f:
        return json.load(f)


@pytest.mark.parametrize("where", MSD_WHERE)
def test_massive_windows_with_candidates(ctx, where):
    """Windows of the massive field where its candidates are (the last 3e12;
    the MSD filter prunes the first ~70 %), on the field's own chunk grid
    (1e8), against the oracle fixture: stride candidates, MSD-surviving
    ranges and the nice list, for both MSD placements."""
    m = _massive()
    w = {int(x["start"]) - int(m["start"]): x for x in m["windows"]}
    picks = [85 * 10 ** 11] if where == "host" else [72 * 10 ** 11, 73 * 10 ** 11, 85 * 10 ** 11,
                                                     99 * 10 ** 11]
    for off in picks:
        x = w[off]
        lst, st = ctx.niceonly_raw(int(x["start"]), int(x["end"]), 50, chunk_size=m["chunk"],
                                   msd_where=where)
        assert (st.candidates, st.ranges) == (x["candidates"], x["ranges"]), off
        assert [str(n) for n in lst] == x["nice_numbers"]


def test_square_survivors_match_oracle(ctx):
    """No nice number is known at these bases, so a wrong digit test or a
    wrong candidate enumeration would pass every nice-list comparison.  This
    pins both: the number of stride candidates whose square alone has no
    repeated digit (the device's square-survivor queue; the oracle's
    get_is_nice reaching the cube scan) must match, with candidates and ranges,
    on
      * the b40 1e9 field (fused per-chunk MSD + candidate kernel),
      * a 64-chunk window of the massive b50 field where its candidates are
        (level BFS to the root level, then the wave kernel's own recursion,
        lane walk, stepped limbs),
      * 1e9 windows of the live bases 52 / 53 on 1e8 chunks (wave kernel)."""
    m = _massive()
    s50 = int(m["start"])
    s40 = O.base_range(40)[0]
    cases = [(s40, s40 + 10 ** 9, 40, 0), (s50 + 8 * 10 ** 12, s50 + 8 * 10 ** 12 + 64 * 10 ** 8, 50, 10 ** 8)]
    for b in (52, 53):
        lo, hi = O.base_range(b)
        a = lo + (hi - lo) // 3
        cases.append((a, a + 10 ** 9, b, 10 ** 8))
    for a, e, b, chunk in cases:
        res, cands, ranges, sq = O.process_field_niceonly_sq(a, e, b, 16, chunk)
        lst, st = ctx.niceonly_raw(a, e, b, chunk_size=chunk, msd_where="device")
        assert (st.candidates, st.ranges, st.square_ok) == (cands, ranges, sq), (b, a)
        assert lst == [n for n, _ in res.nice_numbers]
        assert sq > 0


def test_wave_path_other_bases(ctx):
    """The wave kernel (large chunks) beyond the lane walk: the packed
    candidate groups with a VALU digit decode (b80, three-word masks), the
    generic kernels (b45, b62: no compile-time base), and the out-of-range
    path (b10 [47, 100): generic MSD test inside the wave kernel, must find
    69).  Candidates, ranges and nice lists against the oracle at 1e8 chunks
    (square survivors too where the in-range fast path counts them)."""
    cases = [(47, 100, 10)]
    for b, fr, size in ((80, 0.9, 10 ** 10), (45, 0.5, 10 ** 9), (62, 0.5, 10 ** 9)):
        s, e = O.base_range(b)
        a = s + int((e - s) * fr)
        cases.append((a, a + size, b))
    for a, e, b in cases:
        res, cands, ranges, sq = O.process_field_niceonly_sq(a, e, b, 16, 10 ** 8)
        lst, st = ctx.niceonly_raw(a, e, b, chunk_size=10 ** 8, msd_where="device")
        assert (st.candidates, st.ranges) == (cands, ranges), (b, a)
        assert lst == [n for n, _ in res.nice_numbers], (b, a)
        if b == 80:
            assert st.square_ok == sq > 0
    assert ctx.niceonly_raw(47, 100, 10, chunk_size=10 ** 8, msd_where="device")[0] == [69]


def test_massive_whole_field_sums():
    """The whole 1e13 field on the device MSD: totals equal the sum of the
    oracle windows (7 480 186 005 candidates, 166 585 582 ranges, no nice
    numbers), and ten 1e12 slices sum to the same, slice by slice."""
    m = _massive()
    s, e = int(m["start"]), int(m["end"])
    c = N.GpuContext(0)
    try:
        lst, st = c.niceonly_raw(s, e, 50)  # client chunking of a 1e13 field = 1e8
        tot_c = sum(x["candidates"] for x in m["windows"])
        tot_r = sum(x["ranges"] for x in m["windows"])
        assert (st.candidates, st.ranges, lst) == (tot_c, tot_r, [])
        assert tot_c == 7_480_186_005 and tot_r == 166_585_582
        for k in range(10):
            a = s + k * 10 ** 12
            l2, s2 = c.niceonly_raw(a, a + 10 ** 12, 50, chunk_size=m["chunk"])
            ws = [x for x in m["windows"] if a <= int(x["start"]) < a + 10 ** 12]
            assert (s2.candidates, s2.ranges) == (sum(x["candidates"] for x in ws),
                                                  sum(x["ranges"] for x in ws)), k
            assert l2 == []
        # dealt 8 ways (the N = 8 split): the same totals
        got_c = got_r = 0
        for r in range(8):
            l3, s3 = c.niceonly_raw(s, e, 50, deal_stride=8, deal_offset=r)
            got_c += s3.candidates
            got_r += s3.ranges
            assert l3 == []
        assert (got_c, got_r) == (tot_c, tot_r)
    finally:
        c.close()


def test_c_host_example_gpu():
    """A plain C host (examples/nice_field.c: include/nice_hip.h + the .so, no
    Python in the process) through the GPU entry points: the default b40 and
    hi-base b80 1e6 fields against the oracle, b10 niceonly, and an
    out-of-range b10 field whose 5 395 near-misses outgrow the host's first
    list capacity (the NICE_ERR_CAPACITY retry the header prescribes)."""
    from test_abi import run_c_example
    for base in (40, 80):
        s, _ = O.base_range(base)
        rc, dist, nice, err = run_c_example("--gpu", "detailed", base, "range", 10 ** 6)
        assert rc == 0, err
        want = O.process_range_detailed(s, s + 10 ** 6, base)
        assert (dist, nice) == (want.distribution, want.nice_numbers), base
    rc, dist, nice, err = run_c_example("--gpu", "detailed", 10, 10 ** 6, 10 ** 6 + 10 ** 4)
    assert rc == 0, err
    want = O.process_range_detailed(10 ** 6, 10 ** 6 + 10 ** 4, 10, cap=10 ** 4)
    assert (dist, nice) == (want.distribution, want.nice_numbers) and len(nice) == 5395
    rc, _, nice, err = run_c_example("--gpu", "niceonly", 10, "range")
    assert rc == 0 and nice == [(69, 10)], err


def test_fd_kernel_fuzz_windows(ctx):
    """Seeded fuzz over every FD base: 64 windows at random offsets inside
    the valid range with sizes spread log-uniformly over 1 .. 3e6 (tails,
    single rounds, several rounds, the small-field chunking), each against
    the oracle (client-chunked, 8 threads)."""
    rng = random.Random(20261017)
    bases = list(range(40, 69)) + [80]
    bases = [b for b in bases if N._lib.lib().nice_fd_kernel_base(b) == 1]
    for i in range(64):
        base = bases[i % len(bases)] if i < len(bases) else rng.choice(bases)
        s, e = O.base_range(base)
        size = max(1, int(10 ** rng.uniform(0, 6.48)))
        a = s + rng.randrange(e - s - size)
        want = O.process_field_detailed_mt(a, a + size, base, 8, cap=size)
        check_detailed(ctx, a, a + size, base, want=want)


def test_niceonly_fuzz_every_base(ctx):
    """Seeded niceonly fuzz over every base 3..97 with a valid range (and the
    residue-empty ones, which must return nothing): per base a window at a
    random offset of its range, size log-uniform over 1 .. 3e7, through both
    MSD placements; nice list, stride candidates and MSD ranges against the
    oracle on the same client chunk grid (client_process.rs:439-465 per chunk,
    client/src/main.rs:158-168 chunking)."""
    rng = random.Random(4_20261017)
    checked = 0
    for base in range(3, 98):
        r = O.base_range(base)
        if r is None:
            continue
        s, e = r
        size = min(e - s, max(1, int(10 ** rng.uniform(0, 7.48))))
        a = s + rng.randrange(e - s - size + 1)
        res, cands, ranges, _ = O.process_field_niceonly_sq(a, a + size, base, 8, 0, 0, cap=1 << 20)
        want = [n for n, _ in res.nice_numbers]
        for where in MSD_WHERE:
            lst, st = ctx.niceonly_raw(a, a + size, base, msd_where=where)
            assert lst == want, (base, a, size, where)
            if O.residue_filter(base):
                assert (st.candidates, st.ranges) == (cands, ranges), (base, a, size, where)
        checked += 1
    assert checked > 60


def test_threads_share_a_context():
    """Four host threads drive ONE context at once, each submitting and
    collecting its own detailed and niceonly fields (raw ABI calls, per-thread
    buffers): with collects waiting outside the context lock the submits,
    waits and gathers interleave freely, and every result must equal the
    single-threaded one.  (The reference shares its GpuContext as an Arc
    across the client's tasks, client/src/main.rs:622.)"""
    import threading
    import time
    lib = N._lib.lib()
    ct = N._lib.ctypes
    c = N.GpuContext(0)
    s40, s80 = O.base_range(40)[0], O.base_range(80)[0]
    jobs = [(s40 + k * 3 * 10 ** 6, s40 + (k * 3 + 1) * 10 ** 6, 40) for k in range(6)] + \
           [(s80 + k * 10 ** 6, s80 + k * 10 ** 6 + 5 * 10 ** 5, 80) for k in range(4)] + \
           [(10 ** 6, 10 ** 6 + 10 ** 4, 10)]
    want_det = [c.detailed_raw(a, b, base) for a, b, base in jobs]
    want_nice = [c.niceonly_raw(a, b, base)[0] for a, b, base in jobs]
    errors, got = [], {}

    def worker(w):
        try:
            for rep in range(3):
                for i, (a, b, base) in enumerate(jobs):
                    if (i + w + rep) % 4:
                        continue
                    t, tn = ct.c_int(), ct.c_int()
                    # three fields per mode in flight per context: a full
                    # context answers NICE_ERR_BUSY (only that is retried: a
                    # bad argument would fail at once)
                    for _ in range(100000):
                        rc = lib.nice_detailed_submit(c._h, *N.api._split(a), *N.api._split(b), base, t)
                        if rc != N._lib.NICE_ERR_BUSY:
                            break
                        time.sleep(0.0002)
                    assert rc == 0, lib.nice_last_error()
                    for _ in range(100000):
                        rn = lib.nice_niceonly_submit(c._h, *N.api._split(a), *N.api._split(b), base,
                                                      N.GpuContext._nice_opts(), tn)
                        if rn != N._lib.NICE_ERR_BUSY:
                            break
                        time.sleep(0.0002)
                    assert rn == 0, lib.nice_last_error()
                    hist = (ct.c_uint64 * (base + 1))()
                    cap = 1 << 14
                    out = (N._lib.nice_number * cap)()
                    n = ct.c_size_t()
                    assert lib.nice_detailed_collect(c._h, t.value, hist, out, cap, n) == 0, lib.nice_last_error()
                    det = (list(hist), [(out[q].number_lo | (out[q].number_hi << 64), out[q].num_uniques)
                                        for q in range(n.value)])
                    assert lib.nice_niceonly_collect(c._h, tn.value, out, cap, n, None) == 0
                    nice = [out[q].number_lo | (out[q].number_hi << 64) for q in range(n.value)]
                    got.setdefault(i, []).append((det, nice))
        except BaseException as e:  # reported on the main thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    c.close()
    assert not errors, errors[0]
    assert len(got) == len(jobs)
    for i, results in got.items():
        for det, nice in results:
            assert det == want_det[i], jobs[i]
            assert nice == want_nice[i], jobs[i]


# --- round 5: shared-context blocking, BUSY, host MSD pool, 8 shards ---------
def _raw_detailed(lib, ct, h, a, b, base, cap=1 << 14):
    hist = (ct.c_uint64 * (base + 1))()
    out = (N._lib.nice_number * cap)()
    n = ct.c_size_t()
    rc = lib.nice_process_range_detailed(h, *N.api._split(a), *N.api._split(b), base, hist, out, cap, n)
    return rc, (list(hist), [(out[q].number_lo | (out[q].number_hi << 64), out[q].num_uniques)
                             for q in range(min(n.value, cap))])


def test_synchronous_calls_wait_for_a_slot():
    """Eight host threads call the SYNCHRONOUS entry points on one context
    with no retry loop (the reference shares one GpuContext across the
    client's tasks and blocks behind its Mutex, client/src/main.rs:622,
    client_process_gpu.rs:199-200): with three slots per mode, five threads
    at a time find every slot in flight and must wait for another thread's
    collect, never fail; every result equals the single-threaded one."""
    import threading
    lib = N._lib.lib()
    ct = N._lib.ctypes
    c = N.GpuContext(0)
    s40, s80 = O.base_range(40)[0], O.base_range(80)[0]
    jobs = [(s40 + k * 10 ** 7, s40 + k * 10 ** 7 + 2 * 10 ** 6, 40) for k in range(5)] + \
           [(s80 + k * 10 ** 6, s80 + k * 10 ** 6 + 3 * 10 ** 5, 80) for k in range(3)]
    want = [c.detailed_raw(a, b, base) for a, b, base in jobs]
    want_nice = [c.niceonly_raw(a, b, base)[0] for a, b, base in jobs]
    errors, got = [], []

    def worker(w):
        try:
            for rep in range(4):
                i = (w + rep) % len(jobs)
                a, b, base = jobs[i]
                rc, res = _raw_detailed(lib, ct, c._h, a, b, base)
                assert rc == 0, (rc, lib.nice_last_error())
                cap = 64
                out = (N._lib.nice_number * cap)()
                n = ct.c_size_t()
                rn = lib.nice_process_range_niceonly_ex(c._h, *N.api._split(a), *N.api._split(b), base, None,
                                                        out, cap, n, None)
                assert rn == 0, (rn, lib.nice_last_error())
                got.append((i, res, [out[q].number_lo | (out[q].number_hi << 64) for q in range(n.value)]))
        except BaseException as e:
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    c.close()
    assert not errors, errors[0]
    assert len(got) == 32
    for i, res, nice in got:
        assert res == want[i], jobs[i]
        assert nice == want_nice[i], jobs[i]


def test_busy_and_invalid_statuses():
    """A full context answers NICE_ERR_BUSY to a submit (and to a synchronous
    call from the thread that holds every slot, which no other thread could
    free); a bad argument answers NICE_ERR_INVALID at once, busy or not."""
    lib = N._lib.lib()
    ct = N._lib.ctypes
    c = N.GpuContext(0)
    s = O.base_range(40)[0]
    try:
        tick = [c.detailed_submit(s + k * 10 ** 6, s + (k + 1) * 10 ** 6, 40) for k in range(3)]
        t = ct.c_int()
        assert lib.nice_detailed_submit(c._h, *N.api._split(s), *N.api._split(s + 10), 40, t) == N._lib.NICE_ERR_BUSY
        rc, _ = _raw_detailed(lib, ct, c._h, s, s + 10, 40)
        assert rc == N._lib.NICE_ERR_BUSY
        assert lib.nice_detailed_submit(c._h, *N.api._split(s + 10), *N.api._split(s), 40, t) == N._lib.NICE_ERR_INVALID
        assert lib.nice_detailed_submit(c._h, *N.api._split(s), *N.api._split(s + 10), 1, t) == N._lib.NICE_ERR_INVALID
        ntick = [c.niceonly_submit(s + k * 10 ** 6, s + (k + 1) * 10 ** 6, 40) for k in range(3)]
        assert lib.nice_niceonly_submit(c._h, *N.api._split(s), *N.api._split(s + 10), 40, None, t) == \
            N._lib.NICE_ERR_BUSY
        assert lib.nice_niceonly_submit(c._h, *N.api._split(s), *N.api._split(s + 10), 2, None, t) == \
            N._lib.NICE_ERR_INVALID
        got = [c.detailed_collect(x, 40) for x in tick]
        assert got == [c.detailed_raw(s + k * 10 ** 6, s + (k + 1) * 10 ** 6, 40) for k in range(3)]
        for x in ntick:
            c.niceonly_collect(x)
        # free again: the synchronous call goes through
        rc, res = _raw_detailed(lib, ct, c._h, s, s + 10, 40)
        assert rc == 0 and sum(res[0]) == 10
    finally:
        c.close()


def test_synchronous_calls_of_two_ticket_holders_do_not_deadlock():
    """Thread A holds two asynchronous detailed tickets and thread B one, so
    every slot is in flight; then both call the SYNCHRONOUS entry point.  The
    first to enter waits for the other's slot; the second must see that the
    only thread that could free a slot is itself blocked and answer
    NICE_ERR_BUSY (nice_hip.h), not wait forever.  Once it collects its
    ticket, the waiting call goes through."""
    import threading
    lib = N._lib.lib()
    ct = N._lib.ctypes
    c = N.GpuContext(0)
    s = O.base_range(40)[0]
    go = threading.Barrier(2)
    rcs, errors = {}, []

    def worker(name, k0, nt):
        try:
            tick = [c.detailed_submit(s + (k0 + k) * 10 ** 6, s + (k0 + k + 1) * 10 ** 6, 40) for k in range(nt)]
            go.wait()
            rc, res = _raw_detailed(lib, ct, c._h, s, s + 1000, 40)
            rcs[name] = rc
            for x in tick:
                c.detailed_collect(x, 40)
            if rc == 0:
                assert sum(res[0]) == 1000
        except BaseException as e:
            errors.append(e)

    threads = [threading.Thread(target=worker, args=("A", 0, 2)), threading.Thread(target=worker, args=("B", 2, 1))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=60)
    alive = any(th.is_alive() for th in threads)
    if not alive:
        c.close()
    assert not alive, "synchronous calls deadlocked"
    assert not errors, errors[0]
    assert sorted(rcs.values()) == [N._lib.NICE_OK, N._lib.NICE_ERR_BUSY], rcs


def test_host_msd_pool_is_available_parallelism(ctx):
    """threads = 0 sizes the host MSD pool with available_parallelism() (the
    affinity mask capped by the cgroup quota), as client_process_gpu.rs:598
    does -- not hardware_concurrency (256 on the box's 16-CPU cgroup)."""
    s = O.base_range(40)[0]
    want = N.api.host_threads()
    assert 1 <= want <= (os.cpu_count() or want)
    lst, st = ctx.niceonly_raw(s, s + 10 ** 8, 40, msd_where="host")
    assert st.msd_threads == min(want, 100)  # 100 chunks of 1e6
    lst, st = ctx.niceonly_raw(s, s + 10 ** 8, 40, msd_where="host", threads=3)
    assert st.msd_threads == 3
    lst, st = ctx.niceonly_raw(s, s + 10 ** 8, 40, msd_where="device")
    assert st.msd_threads == 0


def test_eight_shard_context():
    """The C-ABI multi-device context at a node's width: nice_ctx_create with
    eight devices (all device 0 here: 8 shards, 24 slots of streams), as a
    Rust client passing --gpu-device for all eight GPUs would create it
    (client/src/main.rs:109-111; north_star's 8-way contiguous split).  The
    whole extra-large field against the oracle fixture; an out-of-range b10
    field whose every shard lists thousands of near-misses (merged across 8
    lists, each shard's list self-checked on its own device); a massive
    window with candidates on both MSD placements (the host producer deals
    its batches over the 8 devices); and a 3-field submit/collect pipeline
    collected out of order."""
    c = N.GpuContext([0] * 8)
    try:
        f = _oracle_fields()
        x = {d["name"]: d for d in f["detailed"]}["b40_extra_large_1e9"]
        hist, lst = c.detailed_raw(int(x["start"]), int(x["end"]), 40)
        assert _dist(hist) == [tuple(v) for v in x["distribution"]]
        assert lst == [(int(n), u) for n, u in x["near_misses"]]
        for y in f["niceonly"]:
            nice, st = c.niceonly_raw(int(y["start"]), int(y["end"]), y["base"])
            assert st.candidates == y["candidates"] and [str(n) for n in nice] == y["nice_numbers"], y["name"]
        want = O.process_range_detailed(10 ** 6, 12 * 10 ** 5, 10, cap=2 * 10 ** 5)
        hist, lst = c.detailed_raw(10 ** 6, 12 * 10 ** 5, 10)
        assert _dist(hist) == want.distribution and lst == want.nice_numbers
        assert len(lst) > 8 * 1000
        m = _massive()
        w = {int(v["start"]) - int(m["start"]): v for v in m["windows"]}[85 * 10 ** 11]
        for where in ("device", "host"):
            nice, st = c.niceonly_raw(int(w["start"]), int(w["end"]), 50, chunk_size=m["chunk"], msd_where=where)
            assert (st.candidates, st.ranges) == (w["candidates"], w["ranges"]), where
            assert [str(n) for n in nice] == w["nice_numbers"]
        s = O.base_range(40)[0]
        fields = [(s + k * 10 ** 8, s + k * 10 ** 8 + 3 * 10 ** 7 + k, 40) for k in range(3)]
        td = [c.detailed_submit(a, b, base) for a, b, base in fields]
        tn = [c.niceonly_submit(a, b, base) for a, b, base in fields]
        got_d = {k: c.detailed_collect(td[k], 40) for k in (2, 0, 1)}
        got_n = {k: c.niceonly_collect(tn[k])[0] for k in (1, 2, 0)}
        for k, (a, b, base) in enumerate(fields):
            assert got_d[k] == ctx_timed_detailed(a, b, base)
            want_n, cands = O.process_field_niceonly_mt(a, b, base, 4)
            assert got_n[k] == [n for n, _ in want_n.nice_numbers]
    finally:
        c.close()


@pytest.mark.parametrize("base,frac", [(40, 0.0), (40, 0.1), (40, 0.2926), (40, 0.45), (40, 0.97),
                                       (42, 0.0), (43, 0.6), (44, 0.3), (45, 0.0), (45, 0.8),
                                       (47, 0.0), (48, 0.5), (49, 0.3), (50, 0.5), (52, 0.2),
                                       (53, 0.5), (54, 0.6), (55, 0.0), (55, 0.8)])
def test_sibling_kernel_equals_small_fields(ctx, base, frac):
    """b40 fields of >= ~1e8 numbers (1.5 rounds of the resident lanes'
    units, launch_sib's NICE_FD2_SIBROUNDS default 15 / 10) run the
    sibling-lane kernel (Cfg::SIB = 3, fd2_kernel.hpp: a
    lane steps n, n + B^2 and n + 2 B^2 together, sharing limbs 0 and 1;
    super-blocks, edge units where the lane stride does not divide B^2, and
    the regular remainder in one launch; the lane stride from the
    bank-conflict model).  Shorter fields run the round-4 kernel (512 threads
    below 1e7).  A field of ragged size at several points of the range
    (b40 0.2926: across the limb-count cut at 2n + 1 = 40^8) must equal the
    sum of its sub-1e7 pieces, and every near-miss must recompute by the
    oracle.  b42..45 run the same kernel (per-sibling lookup groups), b47..55
    two lanes (Cfg::SIB = 2) over the short low-digit table (Cfg::LDE: lane
    strides capped at 255)."""
    r0, r1 = O.base_range(base)
    s = r0 + int((r1 - r0) * frac) + 12345
    m = 3 if base <= 45 else 2
    n = 26 * m * (base * base) ** 2 + 2_345_677  # 26 super-blocks + a remainder
    if s + n > r1:
        s = r1 - n
    h, l = ctx.detailed_raw(s, s + n, base)
    assert sum(h) == n
    st = ctx.kernel_stats()
    assert (st.sib_lanes, st.fd_kernel) == (m, True), st  # the sibling kernel ran (not its fallback)
    piece = 9_000_001
    hs, ls = [0] * len(h), []
    a = s
    while a < s + n:
        b = min(s + n, a + piece)
        hk, lk = ctx.detailed_raw(a, b, base)
        hs = [x + y for x, y in zip(hs, hk)]
        ls += lk
        a = b
    assert h == hs and l == ls
    assert all(O.num_unique_digits(m, base) == u for m, u in l)
    # a window of the same field against the oracle itself
    want = O.process_range_detailed(s, s + 200_003, base)
    hw, lw = ctx.detailed_raw(s, s + 200_003, base)
    assert _dist(hw) == want.distribution and lw == want.nice_numbers


# --- round 6: every lane stride the sibling pickers can return --------------
_STRIDE_FIELDS = {}


def _stride_field(base, frac):
    """A field of 4 super-blocks + a ragged remainder (so edge units, whole
    super-blocks and the regular remainder part all run) at a fraction of the
    base's range, and its oracle result (computed once per module)."""
    key = (base, frac)
    if key not in _STRIDE_FIELDS:
        m = 3 if base <= 45 else 2
        r0, r1 = O.base_range(base)
        s = r0 + int((r1 - r0) * frac) + 777
        n = 4 * m * (base * base) ** 2 + 1_234_567
        want = O.process_field_detailed_mt(s, s + n, base, min(16, os.cpu_count() or 1))
        _STRIDE_FIELDS[key] = (m, s, n, want)
    return _STRIDE_FIELDS[key]


@pytest.mark.parametrize("base,frac,strides", [
    (40, 0.0, range(45, 211, 2)),                 # the bench layout: pipelined walk, VALU-decoded C2
    (40, 0.5, (45, 61, 79, 81, 97, 119, 143, 181, 209)),  # the per-sibling lookup-group walk
    (52, 0.2, range(45, 241, 2)),                 # two lanes over the short low-digit table
])
def test_every_sibling_lane_stride(ctx, base, frac, strides):
    """the sibling kernels pick their lane stride L per
    launch (pick_lane_stride over odd L in [0.75, 1.5] T -- T = 140 for the
    pipelined walk, else TCHUNK: 80 at b40, 160 at b52 -- pick_small_stride
    over [0.75, 1.25] TCHUNK, fd2_kernel.hpp), and every L that does not divide
    B^2 leaves an edge unit per super-block.  With the stride forced through
    nice_debug_force_sib_stride, each odd L of those ranges ([45, 210] on the
    b40 bench layout, M = 3; [45, 240] on b52, M = 2; a sample on b40's other
    walk) runs a field of 4 super-blocks plus a ragged remainder -- whole
    super-blocks, one edge unit each, the regular remainder part -- and must
    equal the oracle's histogram and near-miss list bit for bit; the kernel
    stats must show the sibling kernel ran at that L."""
    lib = N._lib.lib()
    m, s, n, want = _stride_field(base, frac)
    bad = []
    try:
        for L in strides:
            assert lib.nice_debug_force_sib_stride(L) == 0
            h, lst = ctx.detailed_raw(s, s + n, base)
            st = ctx.kernel_stats()
            if (st.sib_lanes, st.sib_stride) != (m, L):
                bad.append((L, "ran", st.sib_lanes, st.sib_stride))
            elif _dist(h) != want.distribution or lst != want.nice_numbers:
                bad.append((L, "result"))
    finally:
        lib.nice_debug_force_sib_stride(0)
    assert not bad, bad
    assert lib.nice_debug_force_sib_stride(2) == N._lib.NICE_ERR_INVALID
    assert lib.nice_debug_force_sib_stride(257) == N._lib.NICE_ERR_INVALID
    # production pick restored: the same field, the model's stride
    h, lst = ctx.detailed_raw(s, s + n, base)
    assert _dist(h) == want.distribution and lst == want.nice_numbers
