"""The CPU API (nice_cpu_process_range_detailed / _niceonly, cpu_path.cpp):
the reference's process_range_detailed / process_range_niceonly on the host
cores.  No device is involved, so these run in the CPU suite: against the
reference's own vectors (client_process.rs tests), its known answers, and
the oracle on windows in and out of every base's valid range."""
import random

import pytest

import nice_amd as N
from oracle import oracle as O


def _range_for(case, base):
    s, e = O.base_range(base)
    if case["range"] == "base_range":
        return s, e
    return s, s + case["size"]


def _dist(r):
    return [(d.num_uniques, d.count) for d in r.distribution]


def _nice(r):
    return [(x.number, x.num_uniques) for x in r.nice_numbers]


@pytest.mark.parametrize("threads", [1, 3])
def test_cpu_detailed_reference_vectors(golden, threads):
    # client_process.rs:473-1053 (process_detailed_b10 / b40 / b80)
    for c in golden["reference"]["detailed"]:
        s, e = _range_for(c, c["base"])
        r = N.process_range_detailed_cpu(N.FieldSize(s, e), c["base"], threads=threads)
        assert _dist(r) == [tuple(x) for x in c["distribution"]], c["source"]
        assert _nice(r) == [tuple(x) for x in c["nice_numbers"]], c["source"]


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_niceonly_reference_vectors(golden, threads):
    # client_process.rs:1055-1168 (StrideTable k from the test)
    for c in golden["reference"]["niceonly"]:
        s, e = _range_for(c, c["base"])
        r = N.process_range_niceonly_cpu(N.FieldSize(s, e), c["base"], N.StrideTable.new(c["base"], c["k"]),
                                         threads=threads)
        assert r.distribution == []
        assert _nice(r) == [tuple(x) for x in c["nice_numbers"]], c["source"]


def test_cpu_known_answers(golden):
    for c in golden["reference"]["known_answers"]:  # web/index.html
        n, b = c["n"], c["base"]
        r = N.process_range_detailed_cpu(N.FieldSize(n, n + 1), b)
        assert sum(d.count for d in r.distribution) == 1
        assert [d.num_uniques for d in r.distribution if d.count] == [c["num_uniques"]]


def test_cpu_detailed_matches_oracle_every_base():
    # windows at each base's range start, inside, at the end, and outside it
    rng = random.Random(2024)
    for b in range(2, 129):
        try:
            r = O.base_range(b)
        except OverflowError:
            r = (10 ** 30, 10 ** 30 + 10 ** 6)
        s, e = r if r and r[0] < r[1] else (10 ** 6, 2 * 10 ** 6)
        starts = {s, max(0, e - 300), s + rng.randrange(max(1, e - s)), rng.randrange(1, 1 << 100)}
        for a in sorted(starts):
            size = 300 if b > 60 else 600
            want = O.process_range_detailed(a, a + size, b)
            got = N.process_range_detailed_cpu(N.FieldSize(a, a + size), b, threads=2)
            assert _dist(got) == [tuple(x) for x in want.distribution], (b, a)
            assert _nice(got) == [(n, u) for n, u in want.nice_numbers], (b, a)


def test_cpu_detailed_out_of_range_lists():
    # b10 [1e6, 1e6 + 1e4): 5 395 listed numbers, ascending
    r = N.process_range_detailed_cpu(N.FieldSize(10 ** 6, 10 ** 6 + 10 ** 4), 10, threads=3)
    want = O.process_range_detailed(10 ** 6, 10 ** 6 + 10 ** 4, 10)
    assert _dist(r) == [tuple(x) for x in want.distribution]
    assert _nice(r) == [(n, u) for n, u in want.nice_numbers]
    assert len(r.nice_numbers) == 5395


@pytest.mark.parametrize("base,start,size,k", [
    (40, None, 10 ** 6, 2),                      # default benchmark field
    (50, 94_760_515_586_064_977, 10 ** 6, 2),     # msd-ineffective field prefix
    (45, None, 2 * 10 ** 6, 1),
    (12, None, None, 2),                          # whole small base range
    (30, None, 10 ** 6, 2),
])
def test_cpu_niceonly_matches_oracle(base, start, size, k):
    s, e = O.base_range(base)
    a = s if start is None else start
    b = e if size is None else min(e, a + size) if start is None else a + size
    want, _ = O.process_range_niceonly(a, b, base, k)
    for threads in (1, 4):
        got = N.process_range_niceonly_cpu(N.FieldSize(a, b), base, N.StrideTable.new(base, k), threads=threads)
        assert _nice(got) == [(n, u) for n, u in want.nice_numbers], (base, threads)


@pytest.mark.parametrize("base,start,end,count", [
    (10, 1, 47, 4),         # below b10's range: [(3,10),(8,10),(9,10),(24,10)]
    (16, 1, 60, 5),
    (25, 1, 10 ** 4, 19),
    (40, 1, 10 ** 5, 265),
    (12, 1, 200, None),
    (64, 10 ** 6, 10 ** 6 + 5 * 10 ** 5, None),
])
def test_cpu_niceonly_below_range_matches_oracle(base, start, end, count):
    # get_is_nice has no digit-count test (client_process.rs:258-290): below a
    # base's valid range every n whose n^2 and n^3 digits are all distinct is
    # listed by process_range_niceonly (:439-465)
    want, _ = O.process_range_niceonly(start, end, base, 2)
    want = [(n, u) for n, u in want.nice_numbers]
    if count is not None:
        assert len(want) == count
    if base == 10:
        assert want == [(3, 10), (8, 10), (9, 10), (24, 10)]
    for threads in (1, 4):
        got = N.process_range_niceonly_cpu(N.FieldSize(start, end), base, N.StrideTable.new(base, 2),
                                           threads=threads)
        assert _nice(got) == want, (base, threads)


def test_cpu_errors_and_capacity():
    with pytest.raises(N.NiceError):
        N.process_range_detailed_cpu(N.FieldSize(10, 20), 129)
    with pytest.raises(N.NiceError):
        N.process_range_niceonly_cpu(N.FieldSize(10, 20), 1)
    # through the C ABI: an empty range gives an all-zero histogram and no
    # list; a list longer than cap reports the required capacity
    import ctypes
    from nice_amd import _lib
    L = _lib.lib()
    hist = (ctypes.c_uint64 * 11)(*([7] * 11))
    n = ctypes.c_size_t(99)
    assert L.nice_cpu_process_range_detailed(100, 0, 100, 0, 10, 1, hist, None, 0, n) == _lib.NICE_OK
    assert list(hist) == [0] * 11 and n.value == 0
    assert L.nice_cpu_process_range_niceonly(100, 0, 100, 0, 10, 1, 1, None, 0, n) == _lib.NICE_OK
    assert n.value == 0
    out = (_lib.nice_number * 4)()
    rc = L.nice_cpu_process_range_detailed(10 ** 6, 0, 10 ** 6 + 10 ** 4, 0, 10, 2, hist, out, 4, n)
    assert rc == _lib.NICE_ERR_CAPACITY and n.value == 5395
    assert L.nice_cpu_process_range_detailed(20, 0, 10, 0, 10, 1, hist, out, 4, n) == _lib.NICE_ERR_INVALID
