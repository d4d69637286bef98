"""CPU tests of the product library's boundary and host logic (no GPU needed).

- libnice_hip.so loads and exports every function include/nice_hip.h declares;
- host-side number theory (base ranges, cutoff, residue/LSD/stride tables, the
  MSD prefix filter that feeds the niceonly kernel) matches the oracle and the
  reference's golden vectors bit for bit;
- without a GPU, context creation fails loudly (no CPU fallback).
"""
import os
import random
import re

import pytest

import nice_amd as N
from nice_amd import _lib
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    with open(os.path.join(ROOT, "include", "nice_hip.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^\s*(?:int|void|const char|uint32_t|uint64_t)\s*\*?\s*(nice_\w+)\(",
                              hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(_lib.EXPORTS)
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name


def test_constants():
    assert N.api._const("nice_gpu_batch_size") == 50_000_000      # client_process_gpu.rs:59
    assert N.api._const("nice_processing_chunk_size") == 1_000_000  # :54
    assert all(N.gpu_supports_base(b) for b in range(2, 129))
    assert not N.gpu_supports_base(129)


def test_base_ranges_match_oracle(golden):
    for b in range(2, 129):
        try:
            want = O.base_range(b)
        except OverflowError:
            with pytest.raises(OverflowError):
                N.get_base_range_u128(b)
            continue
        got = N.get_base_range_u128(b)
        assert (None if got is None else (got.range_start, got.range_end)) == want, b
    for c in golden["reference"]["base_range"]["cases"]:
        if c["range"] and c["range"][1] < (1 << 128):
            r = N.get_base_range_u128(c["base"])
            assert (r.range_start, r.range_end) == tuple(c["range"])


def test_cutoff_matches_oracle():
    for b in range(2, 129):
        assert N.get_near_miss_cutoff(b) == O.near_miss_cutoff(b)


@pytest.mark.parametrize("base,k", [(10, 1), (10, 2), (12, 2), (25, 2), (40, 2), (45, 2),
                                    (50, 2), (62, 2), (80, 2), (97, 2)])
def test_stride_table_matches_oracle(base, k):
    t = N.StrideTable.new(base, k)
    M, res = O.stride_residues(base, k)
    assert t.modulus == M and t.valid_residues == res


def test_msd_skippable_matches_oracle(golden):
    rng = random.Random(1234)
    for b in (10, 12, 20, 25, 40, 45, 50, 57, 62, 70, 80, 94, 97):
        s, e = O.base_range(b)
        for _ in range(60):
            a = s + rng.randrange(e - s)
            size = 1 + rng.randrange(max(1, min(e - a, 10 ** rng.randrange(1, 12))))
            assert N.has_duplicate_msd_prefix(N.FieldSize(a, a + size), b) == \
                O.has_duplicate_msd_prefix(a, a + size, b), (b, a, size)
    for c in golden["reference"]["msd"]["early_exit"]:
        assert N.has_duplicate_msd_prefix(N.FieldSize(*c["range"]), c["base"]) == c["skip"]


def test_valid_ranges_match_oracle():
    rng = random.Random(99)
    for b in (10, 40, 45, 50, 62, 80):
        s, e = O.base_range(b)
        for _ in range(6):
            a = s + rng.randrange(max(1, e - s - 10 ** 7))
            size = min(e - a, rng.choice([10 ** 4, 10 ** 5, 10 ** 6, 10 ** 7]))
            got = [(r.range_start, r.range_end) for r in N.get_valid_ranges(N.FieldSize(a, a + size), b)]
            assert got == O.valid_ranges(a, a + size, b), (b, a, size)
    s, _ = O.base_range(40)
    got = N.get_valid_ranges(N.FieldSize(s, s + 10 ** 8), 40, floor_size=4000)
    assert [(r.range_start, r.range_end) for r in got] == O.valid_ranges(s, s + 10 ** 8, 40, 4000)


def test_benchmark_fields():
    f = N.get_benchmark_field(N.BenchmarkMode.EXTRA_LARGE)
    assert (f.base, f.range_start, f.range_size) == (40, 1_916_284_264_916, 10 ** 9)
    f = N.get_benchmark_field(N.BenchmarkMode.BASE_TEN)
    assert (f.base, f.range_start, f.range_end) == (10, 47, 100)
    f = N.get_benchmark_field(N.BenchmarkMode.HI_BASE)
    assert f.base == 80 and f.range_size == 10 ** 9  # benchmark.rs:63 (doc says 1e6)
    f = N.get_benchmark_field(N.BenchmarkMode.MASSIVE)
    assert f.base == 50 and f.range_size == 10 ** 13


def test_field_size_semantics():
    with pytest.raises(ValueError):
        N.FieldSize(5, 5)
    f = N.FieldSize(100, 105)
    assert (f.first(), f.last(), f.size()) == (100, 104, 5)
    assert [(c.start(), c.end()) for c in f.chunks(2)] == [(100, 102), (102, 104), (104, 105)]


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(N.NiceError):
        N.GpuContext(0)
