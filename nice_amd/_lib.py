"""ctypes binding of libnice_hip.so (include/nice_hip.h).

The library is built in-tree (nice_amd/Makefile, hipcc --offload-arch=gfx950)
and is the only compute path: there is no CPU fallback.  If the library is
missing or fails to load, every entry point raises NiceLibraryError.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# NICE_LIB_PATH: a CPU-only sanitizer build of the same sources
# (make -C nice_amd sanitize; scripts/sanitize.sh)
LIB_PATH = os.environ.get("NICE_LIB_PATH") or os.path.join(_HERE, "libnice_hip.so")

NICE_OK = 0
NICE_ERR_INVALID = 1
NICE_ERR_HIP = 2
NICE_ERR_CAPACITY = 3
NICE_ERR_NO_DEVICE = 4
NICE_ERR_MSD_OVERFLOW = 5
NICE_ERR_BUSY = 6  # *_submit: every slot of the context is in flight
NICE_MSD_FLOOR_ADAPTIVE = (1 << 64) - 1  # msd_floor: the reference GPU path's AdaptiveFloor

# Every symbol include/nice_hip.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "nice_ctx_create", "nice_ctx_destroy", "nice_ctx_synchronize", "nice_device_count", "nice_last_error",
    "nice_process_range_detailed", "nice_process_range_niceonly",
    "nice_process_range_niceonly_ex", "nice_last_kernel_stats", "nice_base_range",
    "nice_near_miss_cutoff", "nice_gpu_batch_size", "nice_processing_chunk_size",
    "nice_gpu_supports_base", "nice_fd_kernel_base", "nice_msd_valid_ranges",
    "nice_msd_skippable", "nice_stride_table", "nice_debug_unique_counts",
    "nice_debug_is_nice", "nice_debug_unique_fast", "nice_check_is_nice_inrange", "nice_check_unique_inrange", "nice_check_msd_skippable_inrange",
    "nice_fd_segment_cuts", "nice_validate_detailed", "nice_detailed_submit",
    "nice_detailed_collect", "nice_niceonly_submit", "nice_niceonly_collect",
    "nice_cpu_process_range_detailed", "nice_cpu_process_range_niceonly",
    "nice_adaptive_floor_step", "nice_adaptive_floor", "nice_ctx_set_kernel_timing",
    "nice_host_threads", "nice_debug_cgroup_cpus", "nice_debug_force_sib_stride",
)


class NiceLibraryError(RuntimeError):
    pass


class NiceError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class nice_number(ctypes.Structure):
    _fields_ = [("number_lo", ctypes.c_uint64), ("number_hi", ctypes.c_uint64),
                ("num_uniques", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class nice_niceonly_opts(ctypes.Structure):
    _fields_ = [("msd_floor", ctypes.c_uint64), ("chunk_size", ctypes.c_uint64),
                ("threads", ctypes.c_int32), ("stride_k", ctypes.c_uint32),
                ("msd_where", ctypes.c_int32), ("deal_stride", ctypes.c_uint32),
                ("deal_offset", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class nice_niceonly_stats(ctypes.Structure):
    _fields_ = [("ranges", ctypes.c_uint64), ("range_numbers", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("launches", ctypes.c_uint32),
                ("square_ok", ctypes.c_uint32), ("msd_seconds", ctypes.c_double),
                ("total_seconds", ctypes.c_double), ("msd_floor", ctypes.c_uint64),
                ("msd_threads", ctypes.c_uint32), ("reruns", ctypes.c_uint32)]


class nice_kernel_stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("launches", ctypes.c_uint32),
                ("fd_kernel", ctypes.c_uint32), ("numbers", ctypes.c_uint64),
                ("sib_lanes", ctypes.c_uint32), ("sib_stride", ctypes.c_uint32)]


_lib = None


def build(force: bool = False) -> str:
    """Compile libnice_hip.so in-tree (hipcc, gfx950)."""
    cmd = ["make", "-s", "-C", _HERE] + (["-B"] if force else [])
    subprocess.run(cmd, check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NiceLibraryError(
            f"{LIB_PATH} is missing: build it with `make -C nice_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NiceLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    u64, u32, i32, sz = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
    P64, P32, PSZ = ctypes.POINTER(u64), ctypes.POINTER(u32), ctypes.POINTER(sz)
    PN = ctypes.POINTER(nice_number)
    vp = ctypes.c_void_p
    sig = {
        "nice_ctx_create": ([ctypes.POINTER(ctypes.c_int), i32, ctypes.POINTER(vp)], i32),
        "nice_ctx_destroy": ([vp], None),
        "nice_ctx_synchronize": ([vp], i32),
        "nice_device_count": ([ctypes.POINTER(ctypes.c_int)], i32),
        "nice_last_error": ([], ctypes.c_char_p),
        "nice_process_range_detailed": ([vp, u64, u64, u64, u64, u32, P64, PN, sz, PSZ], i32),
        "nice_process_range_niceonly": ([vp, u64, u64, u64, u64, u32, PN, sz, PSZ], i32),
        "nice_process_range_niceonly_ex": ([vp, u64, u64, u64, u64, u32,
                                            ctypes.POINTER(nice_niceonly_opts), PN, sz, PSZ,
                                            ctypes.POINTER(nice_niceonly_stats)], i32),
        "nice_last_kernel_stats": ([vp, i32, ctypes.POINTER(nice_kernel_stats)], i32),
        "nice_ctx_set_kernel_timing": ([vp, i32], i32),
        "nice_base_range": ([u32, P64, P64, P64, P64], i32),
        "nice_near_miss_cutoff": ([u32], u32),
        "nice_gpu_batch_size": ([], u64),
        "nice_processing_chunk_size": ([], u64),
        "nice_gpu_supports_base": ([u32], i32),
        "nice_fd_kernel_base": ([u32], i32),
        "nice_msd_valid_ranges": ([u64, u64, u64, u64, u32, u64, P64, sz, PSZ], i32),
        "nice_msd_skippable": ([u64, u64, u64, u64, u32], i32),
        "nice_stride_table": ([u32, u32, P64, P32, sz, PSZ], i32),
        "nice_debug_unique_counts": ([vp, P64, u32, u32, P32], i32),
        "nice_debug_is_nice": ([vp, P64, u32, u32, P32], i32),
        "nice_debug_unique_fast": ([vp, P64, u32, u32, P32], i32),
        "nice_check_is_nice_inrange": ([u32, u64, u64], i32),
        "nice_check_unique_inrange": ([u32, u64, u64], i32),
        "nice_check_msd_skippable_inrange": ([u32, u64, u64, u64, u64], i32),
        "nice_fd_segment_cuts": ([u32, P64, sz, PSZ], i32),
        "nice_validate_detailed": ([u32, u64, u64, P64, PN, sz], i32),
        "nice_detailed_submit": ([vp, u64, u64, u64, u64, u32, ctypes.POINTER(i32)], i32),
        "nice_detailed_collect": ([vp, i32, P64, PN, sz, PSZ], i32),
        "nice_niceonly_submit": ([vp, u64, u64, u64, u64, u32, ctypes.POINTER(nice_niceonly_opts),
                                  ctypes.POINTER(i32)], i32),
        "nice_niceonly_collect": ([vp, i32, PN, sz, PSZ, ctypes.POINTER(nice_niceonly_stats)], i32),
        "nice_cpu_process_range_detailed": ([u64, u64, u64, u64, u32, i32, P64, PN, sz, PSZ], i32),
        "nice_cpu_process_range_niceonly": ([u64, u64, u64, u64, u32, u32, i32, PN, sz, PSZ], i32),
        "nice_adaptive_floor_step": ([ctypes.c_double, ctypes.c_double, ctypes.c_double], ctypes.c_double),
        "nice_adaptive_floor": ([ctypes.POINTER(ctypes.c_double), P32], i32),
        "nice_host_threads": ([], u32),
        "nice_debug_cgroup_cpus": ([ctypes.c_char_p, ctypes.c_char_p], u32),
        "nice_debug_force_sib_stride": ([u32], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int):
    if rc != NICE_OK:
        msg = lib().nice_last_error()
        raise NiceError(rc, msg.decode() if msg else "")
