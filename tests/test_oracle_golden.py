"""Pin the CPU oracle (oracle/) to the reference's golden vectors.

The oracle is the checker for every GPU parity test, so it is itself checked
first: against the reference's inline Rust unit-test vectors
(tests/golden/reference_vectors.json) and against vectors produced by the
reference's Python mirror scripts/inspect_number.py
(tests/golden/python_vectors.json).
"""
import pytest

from oracle import oracle as O


def _range_for(case, base):
    s, e = O.base_range(base)
    if case["range"] == "base_range":
        return s, e
    return s, s + case["size"]


def test_reference_detailed_vectors(golden):
    # common/src/client_process.rs:473-1053
    for case in golden["reference"]["detailed"]:
        b = case["base"]
        s, e = _range_for(case, b)
        r = O.process_range_detailed(s, e, b)
        assert r.distribution == [tuple(x) for x in case["distribution"]], case["source"]
        assert r.nice_numbers == [tuple(x) for x in case["nice_numbers"]], case["source"]


def test_reference_niceonly_vectors(golden):
    # common/src/client_process.rs:1055-1127 (k = 1 in those tests)
    for case in golden["reference"]["niceonly"]:
        b = case["base"]
        s, e = _range_for(case, b)
        r, _ = O.process_range_niceonly(s, e, b, k=case["k"])
        assert r.nice_numbers == [tuple(x) for x in case["nice_numbers"]], case["source"]
        r2, _ = O.process_range_niceonly(s, e, b, k=2)
        assert r2.nice_numbers == r.nice_numbers


def test_reference_base_ranges(golden):
    # common/src/base_range.rs:98-224
    for c in golden["reference"]["base_range"]["cases"]:
        b = c["base"]
        if c["range"] is None:
            assert O.base_range(b) is None, b
        elif c["range"][1] < (1 << 128):
            assert O.base_range(b) == tuple(c["range"]), b
        else:
            with pytest.raises(OverflowError):
                O.base_range(b)


def test_python_base_ranges(golden):
    for b, r in golden["python"]["base_ranges"].items():
        got = O.base_range(int(b))
        assert got == (None if r is None else (int(r[0]), int(r[1]))), b


def test_reference_residue_filter(golden):
    # common/src/residue_filter.rs:26-76
    for c in golden["reference"]["residue_filter"]["cases"]:
        assert O.residue_filter(c["base"]) == c["residues"], c["base"]


def test_reference_lsd(golden):
    # common/src/lsd_filter.rs:244-583
    for c in golden["reference"]["lsd"]["valid_lsds"]:
        bm = O.lsd_bitmap(c["base"], 1)
        assert [i for i, v in enumerate(bm) if v] == c["lsds"], c["source"]
    for c in golden["reference"]["lsd"]["bitmap_points"]:
        bm = O.lsd_bitmap(c["base"], c["k"])
        for k, v in c["points"].items():
            assert bm[int(k)] == v, c["source"]
    # extract_digits break-on-zero quirk (lsd_filter.rs:142-144): suffix 10 in base
    # 10 with k=2 -> sq=00 {0}, cb=00 {0} -> collision; suffix 2 -> sq 04 gives {4}
    # only (no phantom 0), cb 08 gives {8}: valid.
    bm = O.lsd_bitmap(10, 2)
    assert bm[2] is True and bm[10] is False


def test_reference_stride(golden):
    # common/src/stride_filter.rs:162-246
    for c in golden["reference"]["stride"]:
        M, res = O.stride_residues(c["base"], c["k"])
        assert M == c["modulus"]
        gaps = [res[i + 1] - res[i] for i in range(len(res) - 1)] + [M - res[-1] + res[0]]
        assert sum(gaps) == M and all(g > 0 for g in gaps)
    # SURVEY.md section 8 table (restated this session; nice_kernels.cu:72 fallback says 4992)
    assert len(O.stride_residues(40, 2)[1]) == 4996
    assert len(O.stride_residues(50, 2)[1]) == 14336
    assert len(O.stride_residues(80, 2)[1]) == 10594


def test_reference_msd(golden):
    m = golden["reference"]["msd"]
    for c in m["early_exit"]:
        assert O.has_duplicate_msd_prefix(*c["range"], c["base"]) == c["skip"], c["source"]
    for c in m["whole_range_no_skip"]:
        s, e = O.base_range(c["base"])
        assert not O.has_duplicate_msd_prefix(s, e, c["base"]), c["source"]
    for c in m["segments"]:
        b = c["base"]
        s, e = O.base_range(b)
        chunk = (e - s) // c["divisor"]
        for seg, want in c["expect"]:
            ss = s + seg * chunk
            se = min(ss + chunk, e)
            assert O.has_duplicate_msd_prefix(ss, se, b) == want, (c["source"], seg)


def test_known_answers(golden):
    for c in golden["reference"]["known_answers"]:
        assert O.num_unique_digits(c["n"], c["base"]) == c["num_uniques"], c["source"]
    assert O.is_nice(69, 10)
    assert not O.is_nice(70, 10)


def test_python_detailed_vectors(golden):
    for c in golden["python"]["detailed"]:
        b = c["base"]
        r = O.process_range_detailed(int(c["start"]), int(c["end"]), b)
        assert r.distribution == [tuple(x) for x in c["distribution"]], c["name"]
        assert r.nice_numbers == [(int(n), u) for n, u in c["near_misses"]], c["name"]


def test_python_samples(golden):
    for c in golden["python"]["samples"]:
        b = c["base"]
        got = [O.num_unique_digits(int(n), b) for n in c["n"]]
        assert got == c["num_uniques"], b


def test_python_wild(golden):
    for n, b, u in golden["python"]["wild"]:
        assert O.num_unique_digits(int(n), b) == u, (n, b)


def test_mt_driver_matches_single():
    s, _ = O.base_range(40)
    a = O.process_range_detailed(s, s + 300_000, 40)
    b = O.process_field_detailed_mt(s, s + 300_000, 40, threads=4)
    assert a == b
    r1, c1 = O.process_range_niceonly(47, 100, 10)
    r2, c2 = O.process_field_niceonly_mt(47, 100, 10, threads=2)
    assert r1 == r2 and r1.nice_numbers == [(69, 10)]


def _digits(v, b):
    out = []
    while v:
        v, d = divmod(v, b)
        out.append(d)
    return out


def test_square_survivor_statistic():
    """oracle_process_field_niceonly_sq's test statistic (candidates whose
    square alone has no repeated digit) restated in Python on a b40 window
    with MSD survivors: walk the oracle's valid ranges with the stride
    residues and test n^2's digits directly."""
    s, _ = O.base_range(40)
    a = s + 10 ** 9 - 3 * 10 ** 6          # inside the extra-large field, ranges survive
    e = a + 2 * 10 ** 6
    res, cands, ranges, sq = O.process_field_niceonly_sq(a, e, 40, 4, 10 ** 6)
    M, residues = O.stride_residues(40, 2)
    want_c = want_sq = want_r = 0
    for c0 in range(a, e, 10 ** 6):
        for lo, hi in O.valid_ranges(c0, min(c0 + 10 ** 6, e), 40):
            want_r += 1
            for base_ in range(lo - lo % M, hi, M):
                for r in residues:
                    n = base_ + r
                    if lo <= n < hi:
                        want_c += 1
                        d = _digits(n * n, 40)
                        want_sq += len(set(d)) == len(d)
    assert (cands, ranges, sq) == (want_c, want_r, want_sq)
    assert want_c > 1000 and 0 < want_sq < want_c


def test_scan_depth_consistent():
    # scan depth == total digits iff is_nice (no repeat anywhere)
    s, _ = O.base_range(40)
    for n in range(s, s + 2000):
        d = O.scan_depth(n, 40)
        assert (d == 40) == O.is_nice(n, 40) or d == 40
    assert O.scan_depth(69, 10) == 10 and O.is_nice(69, 10)


def test_massive_fixture_consistent():
    """tests/golden/massive_b50.json (gen_massive_fixture.py): 100 windows of
    1e11 tile the massive field exactly; the first 72 are pruned entirely by
    the MSD filter; one window re-checked here with the oracle."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "massive_b50.json")
    m = json.load(open(p))
    s = int(m["start"])
    assert s == O.base_range(50)[0] and int(m["end"]) == s + 10 ** 13 and m["chunk"] == 10 ** 8
    w = m["windows"]
    assert [int(x["start"]) for x in w] == [s + i * 10 ** 11 for i in range(100)]
    assert all(x["candidates"] == 0 for x in w[:72]) and all(x["candidates"] > 0 for x in w[73:])
    assert sum(x["candidates"] for x in w) == 7_480_186_005
    assert all(x["nice_numbers"] == [] for x in w)
    # window 72 (the survival onset: 86 candidates) recomputed exactly
    x = w[72]
    r, c, rg = O.process_field_niceonly_ex(int(x["start"]), int(x["end"]), 50, 8, chunk=10 ** 8)
    assert (c, rg) == (x["candidates"], x["ranges"]) == (86, x["ranges"]) and r.nice_numbers == []


def test_fd_bases_fixture_consistent():
    """tests/golden/fd_bases_1e9.json: each field is 1e9 from its base's range
    start, the distribution sums to 1e9, and the near-miss list matches the
    bins above the cutoff; a 1e5 prefix of the b80 field re-checked against
    the oracle's distribution shape (the same n have at most the whole
    field's counts)."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fd_bases_1e9.json")
    fx = json.load(open(p))
    for c in fx["detailed"]:
        b = c["base"]
        s = int(c["start"])
        assert s == O.base_range(b)[0] and int(c["end"]) == s + 10 ** 9
        hist = dict((u, n) for u, n in c["distribution"])
        assert [u for u, _ in c["distribution"]] == list(range(1, b + 1))
        assert sum(hist.values()) == 10 ** 9
        cut = O.near_miss_cutoff(b)
        assert sum(n for u, n in hist.items() if u > cut) == len(c["near_misses"])
        assert all(u > cut for _, u in c["near_misses"])
    b80 = fx["detailed"][0]
    s = int(b80["start"])
    pre = O.process_range_detailed(s, s + 10 ** 5, 80)
    full = dict((u, n) for u, n in b80["distribution"])
    assert all(n <= full[u] for u, n in pre.distribution)


def test_fd_bases_more_fixture_consistent():
    """tests/golden/fd_bases_more_1e9.json (gen_fd_bases_fixtures.py --more):
    1e9 fields one third into the ranges of b42 / b49 / b59 / b65, each
    distribution summing to 1e9 with the near-miss list matching the bins above
    the cutoff, and every near-miss recomputing by the oracle."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fd_bases_more_1e9.json")
    fx = json.load(open(p))
    assert [c["base"] for c in fx["detailed"]] == [42, 49, 59, 65]
    for c in fx["detailed"]:
        b = c["base"]
        r0, r1 = O.base_range(b)
        s = int(c["start"])
        assert s == r0 + (r1 - r0) // 3 and int(c["end"]) == s + 10 ** 9
        assert [u for u, _ in c["distribution"]] == list(range(1, b + 1))
        assert sum(n for _, n in c["distribution"]) == 10 ** 9
        cut = O.near_miss_cutoff(b)
        assert sum(n for u, n in c["distribution"] if u > cut) == len(c["near_misses"])
        assert all(O.num_unique_digits(int(n), b) == u > cut for n, u in c["near_misses"])
