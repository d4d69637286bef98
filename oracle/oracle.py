"""ctypes wrapper over oracle/liboracle.so -- the CPU restatement of the
reference's field processing.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  The product (nice_amd/) never
imports it.  Reference citations live on the C functions (oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
# NICE_ORACLE_LIB_PATH: a sanitizer build of the same source (scripts/sanitize.sh)
_LIB_PATH = os.environ.get("NICE_ORACLE_LIB_PATH") or os.path.join(_HERE, "liboracle.so")
_lib = None

MASK64 = (1 << 64) - 1


def build() -> str:
    """Compile liboracle.so from oracle.c (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.environ.get("NICE_ORACLE_LIB_PATH") and (
                not os.path.exists(_LIB_PATH) or
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, u32, i32, sz = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
        P64, P32, P8 = ctypes.POINTER(u64), ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_uint8)
        L.oracle_base_range.argtypes = [u32, P64, P64, P64, P64]
        L.oracle_base_range.restype = i32
        L.oracle_near_miss_cutoff.argtypes = [u32]
        L.oracle_near_miss_cutoff.restype = u32
        L.oracle_num_unique_digits.argtypes = [u64, u64, u32]
        L.oracle_num_unique_digits.restype = u32
        L.oracle_is_nice.argtypes = [u64, u64, u32]
        L.oracle_is_nice.restype = i32
        L.oracle_scan_depth.argtypes = [u64, u64, u32]
        L.oracle_scan_depth.restype = u32
        L.oracle_process_range_detailed.argtypes = [u64, u64, u64, u64, u32, P64, P64, P32, sz,
                                                    ctypes.POINTER(sz)]
        L.oracle_process_range_detailed.restype = i32
        L.oracle_process_field_detailed_mt.argtypes = [u64, u64, u64, u64, u32, i32, P64, P64,
                                                       P32, sz, ctypes.POINTER(sz)]
        L.oracle_process_field_detailed_mt.restype = i32
        L.oracle_residue_filter.argtypes = [u32, P32]
        L.oracle_residue_filter.restype = u32
        L.oracle_lsd_bitmap.argtypes = [u32, u32, P8]
        L.oracle_lsd_bitmap.restype = ctypes.c_int64
        L.oracle_stride_residues.argtypes = [u32, u32, P64, P64, u64]
        L.oracle_stride_residues.restype = u64
        L.oracle_set_filter_c.argtypes = [i32]
        L.oracle_set_filter_c.restype = None
        L.oracle_has_duplicate_msd_prefix.argtypes = [u64, u64, u64, u64, u32]
        L.oracle_has_duplicate_msd_prefix.restype = i32
        L.oracle_valid_ranges.argtypes = [u64, u64, u64, u64, u32, u64, P64, u64]
        L.oracle_valid_ranges.restype = u64
        L.oracle_process_range_niceonly.argtypes = [u64, u64, u64, u64, u32, u32, u64, P64, u64,
                                                    P64]
        L.oracle_process_range_niceonly.restype = u64
        L.oracle_process_field_niceonly_mt.argtypes = [u64, u64, u64, u64, u32, i32, P64, u64,
                                                       P64]
        L.oracle_process_field_niceonly_mt.restype = u64
        L.oracle_process_field_niceonly_ex.argtypes = [u64, u64, u64, u64, u32, i32, u64, u64,
                                                       P64, u64, P64, P64]
        L.oracle_process_field_niceonly_ex.restype = u64
        L.oracle_process_field_niceonly_sq.argtypes = [u64, u64, u64, u64, u32, i32, u64, u64,
                                                       P64, u64, P64, P64, P64]
        L.oracle_process_field_niceonly_sq.restype = u64
        _lib = L
    return _lib


def _split(n: int):
    return n & MASK64, n >> 64


@dataclass
class FieldResults:
    """Mirror of FieldResults (common/src/lib.rs:319-323)."""
    distribution: list  # [(num_uniques, count)] for 1..=base (detailed) or []
    nice_numbers: list  # [(number, num_uniques)] ascending


def base_range(base: int):
    a, b, c, d = (ctypes.c_uint64() for _ in range(4))
    rc = lib().oracle_base_range(base, a, b, c, d)
    if rc < 0:
        raise OverflowError(f"base {base} range does not fit in u128")
    if rc == 0:
        return None
    return (a.value | (b.value << 64), c.value | (d.value << 64))


def near_miss_cutoff(base: int) -> int:
    return lib().oracle_near_miss_cutoff(base)


def num_unique_digits(n: int, base: int) -> int:
    return lib().oracle_num_unique_digits(*_split(n), base)


def is_nice(n: int, base: int) -> bool:
    return bool(lib().oracle_is_nice(*_split(n), base))


def scan_depth(n: int, base: int) -> int:
    return lib().oracle_scan_depth(*_split(n), base)


def _detailed(fn, start, end, base, *extra, cap=None):
    size = end - start
    if cap is None:
        cap = min(size, 1 << 22)
    hist = (ctypes.c_uint64 * (base + 1))()
    miss_n = (ctypes.c_uint64 * (2 * max(cap, 1)))()
    miss_u = (ctypes.c_uint32 * max(cap, 1))()
    n_miss = ctypes.c_size_t()
    rc = fn(*_split(start), *_split(end), base, *extra, hist, miss_n, miss_u, cap, n_miss)
    if rc != 0:
        raise OverflowError("near-miss list exceeded capacity")
    dist = [(i, hist[i]) for i in range(1, base + 1)]
    nice = [(miss_n[2 * i] | (miss_n[2 * i + 1] << 64), miss_u[i]) for i in range(n_miss.value)]
    return FieldResults(dist, nice)


def process_range_detailed(start: int, end: int, base: int, cap=None) -> FieldResults:
    """client_process.rs:150-191 on [start, end)."""
    return _detailed(lib().oracle_process_range_detailed, start, end, base, cap=cap)


def process_field_detailed_mt(start: int, end: int, base: int, threads: int,
                              cap=None) -> FieldResults:
    """client/src/main.rs:120-254 (detailed) on `threads` threads."""
    return _detailed(lib().oracle_process_field_detailed_mt, start, end, base, threads, cap=cap)


def residue_filter(base: int) -> list:
    out = (ctypes.c_uint32 * max(base, 1))()
    n = lib().oracle_residue_filter(base, out)
    return list(out[:n])


def lsd_bitmap(base: int, k: int) -> list:
    m = base ** k
    buf = (ctypes.c_uint8 * m)()
    if lib().oracle_lsd_bitmap(base, k, buf) < 0:
        raise OverflowError("base^k overflows u32")
    return [bool(x) for x in buf]


def stride_residues(base: int, k: int):
    M = ctypes.c_uint64()
    n = lib().oracle_stride_residues(base, k, M, None, 0)
    buf = (ctypes.c_uint64 * max(n, 1))()
    lib().oracle_stride_residues(base, k, M, buf, n)
    return M.value, list(buf[:n])


def has_duplicate_msd_prefix(start: int, end: int, base: int) -> bool:
    return bool(lib().oracle_has_duplicate_msd_prefix(*_split(start), *_split(end), base))


def valid_ranges(start: int, end: int, base: int, floor_size: int = 250) -> list:
    args = (*_split(start), *_split(end), base, floor_size)
    n = lib().oracle_valid_ranges(*args, None, 0)
    buf = (ctypes.c_uint64 * (4 * max(n, 1)))()
    lib().oracle_valid_ranges(*args, buf, n)
    return [(buf[4 * i] | (buf[4 * i + 1] << 64), buf[4 * i + 2] | (buf[4 * i + 3] << 64))
            for i in range(n)]


def process_range_niceonly(start: int, end: int, base: int, k: int = 2,
                           floor_size: int = 250, cap: int = 1 << 16):
    """client_process.rs:439-465 with StrideTable::new(base, k).
    Returns (FieldResults, stride candidates tested)."""
    buf = (ctypes.c_uint64 * (2 * cap))()
    cands = ctypes.c_uint64()
    n = lib().oracle_process_range_niceonly(*_split(start), *_split(end), base, k, floor_size,
                                            buf, cap, cands)
    if n > cap:
        raise OverflowError("nice list exceeded capacity")
    nice = [(buf[2 * i] | (buf[2 * i + 1] << 64), base) for i in range(n)]
    return FieldResults([], nice), cands.value


def process_field_niceonly_mt(start: int, end: int, base: int, threads: int,
                              cap: int = 1 << 16):
    """client/src/main.rs:120-254 (niceonly, k=2, floor 250) on `threads` threads.
    Returns (FieldResults, stride candidates tested)."""
    buf = (ctypes.c_uint64 * (2 * cap))()
    cands = ctypes.c_uint64()
    n = lib().oracle_process_field_niceonly_mt(*_split(start), *_split(end), base, threads,
                                               buf, cap, cands)
    if n > cap:
        raise OverflowError("nice list exceeded capacity")
    nice = [(buf[2 * i] | (buf[2 * i + 1] << 64), base) for i in range(n)]
    return FieldResults([], nice), cands.value


def process_field_niceonly_ex(start: int, end: int, base: int, threads: int, chunk: int = 0,
                              floor_size: int = 0, cap: int = 1 << 16):
    """process_field_niceonly_mt with an explicit MSD chunk size (0 = client
    rule) and floor (0 = 250).  Returns (FieldResults, candidates, ranges)."""
    buf = (ctypes.c_uint64 * (2 * cap))()
    cands, ranges = ctypes.c_uint64(), ctypes.c_uint64()
    n = lib().oracle_process_field_niceonly_ex(*_split(start), *_split(end), base, threads, chunk,
                                               floor_size, buf, cap, cands, ranges)
    if n > cap:
        raise OverflowError("nice list exceeded capacity")
    nice = [(buf[2 * i] | (buf[2 * i + 1] << 64), base) for i in range(n)]
    return FieldResults([], nice), cands.value, ranges.value


def process_field_niceonly_sq(start: int, end: int, base: int, threads: int, chunk: int = 0,
                              floor_size: int = 0, cap: int = 1 << 16):
    """process_field_niceonly_ex plus the number of stride candidates whose
    square alone has no repeated digit (get_is_nice reached the cube scan): a
    test statistic for the GPU's square-survivor count.  Returns
    (FieldResults, candidates, ranges, square_ok)."""
    buf = (ctypes.c_uint64 * (2 * cap))()
    cands, ranges, sq = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    n = lib().oracle_process_field_niceonly_sq(*_split(start), *_split(end), base, threads, chunk,
                                               floor_size, buf, cap, cands, ranges, sq)
    if n > cap:
        raise OverflowError("nice list exceeded capacity")
    nice = [(buf[2 * i] | (buf[2 * i + 1] << 64), base) for i in range(n)]
    return FieldResults([], nice), cands.value, ranges.value, sq.value
