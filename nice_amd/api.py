"""Host-side mirror of the reference's field-processing API over the C ABI.

Names, argument meaning and error behaviour follow
common/src/client_process_gpu.rs (GpuContext, process_range_detailed_gpu,
process_range_niceonly_gpu, process_detailed_gpu, process_niceonly_gpu) and
common/src/client_process.rs (process_range_detailed, process_range_niceonly,
which here run on the GPU through a default context -- the drop-in the
north star asks for).  All compute happens in libnice_hip.so.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from . import _lib
from ._lib import check, lib
from .types import (DataToClient, DataToServer, FieldResults, FieldSize, NiceNumberSimple,
                    UniquesDistributionSimple)

CLIENT_VERSION = "3.2.15-mi355x"
MASK64 = (1 << 64) - 1


def _split(n: int):
    if n < 0 or n >> 128:
        raise ValueError("value must fit in u128")
    return n & MASK64, n >> 64


# pub const GPU_BATCH_SIZE / PROCESSING_CHUNK_SIZE (client_process_gpu.rs:54, 59)
def _const(name):
    try:
        return int(getattr(lib(), name)())
    except _lib.NiceLibraryError:
        return None


GPU_BATCH_SIZE = 50_000_000
PROCESSING_CHUNK_SIZE = 1_000_000


def get_base_range_u128(base: int) -> Optional[FieldSize]:
    """get_base_range_u128 (common/src/base_range.rs:43-54)."""
    a, b, c, d = (ctypes.c_uint64() for _ in range(4))
    rc = lib().nice_base_range(base, a, b, c, d)
    if rc < 0:
        raise OverflowError(f"base {base}: range does not fit in u128")
    if rc == 0:
        return None
    return FieldSize(a.value | (b.value << 64), c.value | (d.value << 64))


def get_near_miss_cutoff(base: int) -> int:
    """get_near_miss_cutoff (common/src/number_stats.rs:15-17)."""
    return int(lib().nice_near_miss_cutoff(base))


def gpu_supports_base(base: int) -> bool:
    return bool(lib().nice_gpu_supports_base(base))


@dataclass
class StrideTable:
    """StrideTable (common/src/stride_filter.rs:20-87), host-built by the library."""
    base: int
    k: int
    modulus: int
    valid_residues: List[int]

    @classmethod
    def new(cls, base: int, k: int) -> "StrideTable":
        m = ctypes.c_uint64()
        n = ctypes.c_size_t()
        check(lib().nice_stride_table(base, k, m, None, 0, n))
        buf = (ctypes.c_uint32 * max(n.value, 1))()
        check(lib().nice_stride_table(base, k, m, buf, n.value, n))
        return cls(base, k, m.value, list(buf[: n.value]))


def get_valid_ranges(range_: FieldSize, base: int, floor_size: int = 250) -> List[FieldSize]:
    """get_valid_ranges_recursive (common/src/msd_prefix_filter.rs:583-674)."""
    s, e = range_.range_start, range_.range_end
    n = ctypes.c_size_t()
    rc = lib().nice_msd_valid_ranges(*_split(s), *_split(e), base, floor_size, None, 0, n)
    if rc not in (_lib.NICE_OK, _lib.NICE_ERR_CAPACITY):
        check(rc)
    buf = (ctypes.c_uint64 * (4 * max(n.value, 1)))()
    check(lib().nice_msd_valid_ranges(*_split(s), *_split(e), base, floor_size, buf, n.value, n))
    return [FieldSize(buf[4 * i] | (buf[4 * i + 1] << 64), buf[4 * i + 2] | (buf[4 * i + 3] << 64))
            for i in range(n.value)]


def has_duplicate_msd_prefix(range_: FieldSize, base: int) -> bool:
    """has_duplicate_msd_prefix (common/src/msd_prefix_filter.rs:382-563)."""
    rc = lib().nice_msd_skippable(*_split(range_.range_start), *_split(range_.range_end), base)
    if rc < 0 or rc > 1:
        check(rc)
    return bool(rc)


@dataclass
class NiceonlyStats:
    ranges: int
    range_numbers: int
    candidates: int
    launches: int
    msd_seconds: float
    total_seconds: float
    # device MSD, in-range fast bases: candidates whose square alone has no
    # repeated digit (mod 2^32; 0 where not counted)
    square_ok: int = 0
    # the MSD recursion floor the field used (msd_floor="adaptive": the
    # adaptive floor's value at submit)
    msd_floor: int = 0
    # host MSD worker threads the field ran (0: the MSD ran on the device)
    msd_threads: int = 0
    # times the field re-ran with grown device lists
    reruns: int = 0


def _stats(st) -> NiceonlyStats:
    return NiceonlyStats(st.ranges, st.range_numbers, st.candidates, st.launches,
                         st.msd_seconds, st.total_seconds, st.square_ok, st.msd_floor,
                         st.msd_threads, st.reruns)


def host_threads() -> int:
    """std::thread::available_parallelism() as the library computes it (the
    affinity mask capped by the cgroup cpu.max quota): the host MSD pool's
    size when threads=0 (client_process_gpu.rs:598)."""
    return int(lib().nice_host_threads())


def adaptive_floor_step(floor: float, msd_seconds: float, total_seconds: float) -> float:
    """AdaptiveFloor::update's step (client_process_gpu.rs:130-157)."""
    return lib().nice_adaptive_floor_step(floor, msd_seconds, total_seconds)


def adaptive_floor() -> Tuple[float, int]:
    """The process-wide adaptive MSD floor and its warmup fields left
    (0xffffffff: pinned by NICE_GPU_MSD_FLOOR)."""
    f, w = ctypes.c_double(), ctypes.c_uint32()
    check(lib().nice_adaptive_floor(f, w))
    return f.value, w.value


@dataclass
class KernelStats:
    kernel_ms: float
    launches: int
    fd_kernel: bool
    numbers: int
    sib_lanes: int = 0   # sibling lanes of the FD kernel's last sibling launch (0: none)
    sib_stride: int = 0  # ... and its lane stride


class GpuContext:
    """GpuContext (client_process_gpu.rs:196-306).  `devices` extends the
    reference's single ordinal: a field is sharded across the listed GPUs."""

    def __init__(self, devices: Sequence[int] | int = 0):
        if isinstance(devices, int):
            devices = [devices]
        arr = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(lib().nice_ctx_create(arr, len(devices), ctypes.byref(h)))
        self._h = h
        self.devices = list(devices)
        # Reused host output buffer (grown on NICE_ERR_CAPACITY): allocating a
        # zeroed 64K-entry ctypes array per call cost ~0.1 ms of host time.
        self._out = None
        self._out_cap = 0
        self._hist = {}

    @classmethod
    def new(cls, device_ordinal: int = 0) -> "GpuContext":
        return cls([device_ordinal])

    def close(self):
        if getattr(self, "_h", None):
            lib().nice_ctx_destroy(self._h)
            self._h = None

    def synchronize(self):
        """Wait until every stream of this context is idle (nice_ctx_synchronize)."""
        check(lib().nice_ctx_synchronize(self._h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _out_buf(self, cap):
        if cap > self._out_cap:
            self._out = (_lib.nice_number * cap)()
            self._out_cap = cap
        return self._out

    def set_kernel_timing(self, enable: bool):
        """HIP-event timing of later detailed fields (default on; off saves two
        runtime calls per field, and kernel_stats().kernel_ms reads 0)."""
        check(lib().nice_ctx_set_kernel_timing(self._h, 1 if enable else 0))

    def kernel_stats(self, device_index: int = 0) -> KernelStats:
        s = _lib.nice_kernel_stats()
        check(lib().nice_last_kernel_stats(self._h, device_index, s))
        return KernelStats(s.kernel_ms, s.launches, bool(s.fd_kernel), s.numbers, s.sib_lanes, s.sib_stride)

    # -- detailed -------------------------------------------------------------
    def detailed_raw(self, start: int, end: int, base: int, cap: int = 0):
        """Histogram (base+1 bins) and near-miss list [(n, u)] ascending."""
        hist = self._hist.get(base)
        if hist is None:
            hist = self._hist[base] = (ctypes.c_uint64 * (base + 1))()
        cap = max(cap, self._out_cap, 1024)
        while True:
            out = self._out_buf(cap)
            n = ctypes.c_size_t()
            rc = lib().nice_process_range_detailed(self._h, *_split(start), *_split(end), base,
                                                   hist, out, cap, n)
            if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
                cap = n.value
                continue
            check(rc)
            lst = [(out[i].number_lo | (out[i].number_hi << 64), out[i].num_uniques)
                   for i in range(n.value)]
            return list(hist), lst

    def detailed_submit(self, start: int, end: int, base: int) -> int:
        """Enqueue a detailed field and return at once (a ticket for
        detailed_collect); at most three fields in flight per context."""
        t = ctypes.c_int()
        check(lib().nice_detailed_submit(self._h, *_split(start), *_split(end), base, t))
        return t.value

    def detailed_collect(self, ticket: int, base: int, cap: int = 0):
        """(hist, near-misses) of a submitted field, as detailed_raw returns."""
        hist = self._hist.get(base)
        if hist is None:
            hist = self._hist[base] = (ctypes.c_uint64 * (base + 1))()
        cap = max(cap, self._out_cap, 1024)
        while True:
            out = self._out_buf(cap)
            n = ctypes.c_size_t()
            rc = lib().nice_detailed_collect(self._h, ticket, hist, out, cap, n)
            if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
                cap = n.value
                continue
            check(rc)
            return list(hist), [(out[i].number_lo | (out[i].number_hi << 64), out[i].num_uniques)
                                for i in range(n.value)]

    # -- niceonly -------------------------------------------------------------
    def niceonly_raw(self, start: int, end: int, base: int, msd_floor: int = 0,
                     chunk_size: int = 0, threads: int = 0, stride_k: int = 0,
                     msd_where: str = "auto", cap: int = 0, deal_stride: int = 0,
                     deal_offset: int = 0):
        """Nice numbers of [start, end) ascending, and NiceonlyStats.  With
        deal_stride N > 1 only the field's chunks c with c % N == deal_offset
        are processed (rank deal_offset of an N-way job, nice_amd/dist.py)."""
        opts = self._nice_opts(msd_floor, chunk_size, threads, stride_k, msd_where, deal_stride,
                               deal_offset)
        st = _lib.nice_niceonly_stats()
        cap = max(cap, self._out_cap, 1024)
        while True:
            out = self._out_buf(cap)
            n = ctypes.c_size_t()
            rc = lib().nice_process_range_niceonly_ex(self._h, *_split(start), *_split(end), base,
                                                      opts, out, cap, n, st)
            if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
                cap = n.value
                continue
            check(rc)
            lst = [out[i].number_lo | (out[i].number_hi << 64) for i in range(n.value)]
            return lst, _stats(st)

    @staticmethod
    def _nice_opts(msd_floor=0, chunk_size=0, threads=0, stride_k=0, msd_where="auto",
                   deal_stride=0, deal_offset=0):
        where = {"auto": 0, "host": 1, "device": 2}[msd_where]
        if msd_floor == "adaptive":  # client_process_gpu.rs:96-184
            msd_floor = _lib.NICE_MSD_FLOOR_ADAPTIVE
        return _lib.nice_niceonly_opts(msd_floor, chunk_size, threads, stride_k, where,
                                       deal_stride, deal_offset, 0)

    def niceonly_submit(self, start: int, end: int, base: int, **opts) -> int:
        """Enqueue a niceonly field (options as niceonly_raw) and return a
        ticket for niceonly_collect."""
        t = ctypes.c_int()
        check(lib().nice_niceonly_submit(self._h, *_split(start), *_split(end), base,
                                         self._nice_opts(**opts), t))
        return t.value

    def niceonly_collect(self, ticket: int, cap: int = 0):
        """(nice numbers, NiceonlyStats) of a submitted field."""
        st = _lib.nice_niceonly_stats()
        cap = max(cap, self._out_cap, 1024)
        while True:
            out = self._out_buf(cap)
            n = ctypes.c_size_t()
            rc = lib().nice_niceonly_collect(self._h, ticket, out, cap, n, st)
            if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
                cap = n.value
                continue
            check(rc)
            return ([out[i].number_lo | (out[i].number_hi << 64) for i in range(n.value)],
                    _stats(st))

    # -- both modes of one field ---------------------------------------------
    def both_raw(self, det_range, nice_range, base: int, **nice_opts):
        """Detailed of det_range and niceonly of nice_range (either None to
        skip), one after the other on this context's stream.  Returns
        ((hist, near_misses), (nice, stats)); BothModes runs the two at once."""
        det = self.detailed_raw(*det_range, base) if det_range else (None, [])
        nice = self.niceonly_raw(*nice_range, base, **nice_opts) if nice_range else ([], None)
        return det, nice

    def debug_unique_counts(self, ns: Sequence[int], base: int) -> List[int]:
        arr = (ctypes.c_uint64 * (2 * max(len(ns), 1)))()
        for i, n in enumerate(ns):
            arr[2 * i], arr[2 * i + 1] = _split(n)
        out = (ctypes.c_uint32 * max(len(ns), 1))()
        check(lib().nice_debug_unique_counts(self._h, arr, len(ns), base, out))
        return list(out[: len(ns)])

    def debug_unique_fast(self, ns: Sequence[int], base: int) -> List[int]:
        """Unique-digit counts by the niceonly kernel's in-range limb path
        (radix_fast.hpp); every n must lie in the base's valid range."""
        arr = (ctypes.c_uint64 * (2 * max(len(ns), 1)))()
        for i, n in enumerate(ns):
            arr[2 * i], arr[2 * i + 1] = _split(n)
        out = (ctypes.c_uint32 * max(len(ns), 1))()
        check(lib().nice_debug_unique_fast(self._h, arr, len(ns), base, out))
        return list(out[: len(ns)])

    def debug_is_nice(self, ns: Sequence[int], base: int) -> List[bool]:
        arr = (ctypes.c_uint64 * (2 * max(len(ns), 1)))()
        for i, n in enumerate(ns):
            arr[2 * i], arr[2 * i + 1] = _split(n)
        out = (ctypes.c_uint32 * max(len(ns), 1))()
        check(lib().nice_debug_is_nice(self._h, arr, len(ns), base, out))
        return [bool(x) for x in out[: len(ns)]]


class BothModes:
    """Detailed and niceonly of one field at the same time on one GPU.

    Each mode gets its own context, i.e. its own HIP stream, and the niceonly
    pass is driven from a worker thread (ctypes releases the GIL for the
    call), so its launch-latency-bound MSD levels and candidate kernel run
    beside the detailed kernel instead of after it: the b40 1e9 bench step
    goes from 2.63 to 2.48 ms (scripts/overlap_probe.py).  Same results as
    GpuContext.both_raw, which runs the two in sequence."""

    def __init__(self, device: int = 0, det_ctx: Optional[GpuContext] = None,
                 nice_ctx: Optional[GpuContext] = None):
        self.det = det_ctx if det_ctx is not None else GpuContext([device])
        self.nice = nice_ctx if nice_ctx is not None else GpuContext([device])
        self._own_nice = nice_ctx is None
        self._go = threading.Event()
        self._done = threading.Event()
        self._job = None
        self._res = None
        self._closed = False
        self._thread = threading.Thread(target=self._serve, name="nice-niceonly", daemon=True)
        self._thread.start()

    def _serve(self):
        while True:
            self._go.wait()
            self._go.clear()
            if self._closed:
                return
            args, kw = self._job
            try:
                self._res = (True, self.nice.niceonly_raw(*args, **kw))
            except BaseException as e:  # re-raised on the calling thread
                self._res = (False, e)
            self._done.set()

    def kernel_stats(self, device_index: int = 0) -> KernelStats:
        """The detailed pass's kernel statistics."""
        return self.det.kernel_stats(device_index)

    def detailed_raw(self, *a, **kw):
        return self.det.detailed_raw(*a, **kw)

    def niceonly_raw(self, *a, **kw):
        return self.nice.niceonly_raw(*a, **kw)

    def both_raw(self, det_range, nice_range, base: int, **nice_opts):
        if self._closed:
            raise RuntimeError("BothModes is closed")
        if not nice_range:
            return (self.det.detailed_raw(*det_range, base) if det_range else (None, [])), ([], None)
        self._job = ((*nice_range, base), nice_opts)
        self._done.clear()
        self._go.set()
        try:
            det = self.det.detailed_raw(*det_range, base) if det_range else (None, [])
        finally:
            self._done.wait()
        ok, nice = self._res
        self._res = None
        if not ok:
            raise nice
        return det, nice

    def close(self):
        if not self._closed:
            self._closed = True
            self._go.set()
            self._thread.join()
            if self._own_nice:
                self.nice.close()


def process_range_detailed_gpu(ctx: GpuContext, range_: FieldSize, base: int) -> FieldResults:
    """process_range_detailed_gpu (client_process_gpu.rs:812-897)."""
    hist, lst = ctx.detailed_raw(range_.range_start, range_.range_end, base)
    return FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in lst])


def process_range_niceonly_gpu(ctx: GpuContext, range_: FieldSize, base: int,
                               **opts) -> FieldResults:
    """process_range_niceonly_gpu (client_process_gpu.rs:515-557)."""
    lst, _ = ctx.niceonly_raw(range_.range_start, range_.range_end, base, **opts)
    return FieldResults(distribution=[], nice_numbers=[NiceNumberSimple(n, base) for n in lst])


def process_detailed_gpu(ctx: GpuContext, claim: DataToClient, username: str) -> DataToServer:
    """process_detailed_gpu (client_process_gpu.rs:907-922)."""
    r = process_range_detailed_gpu(ctx, claim.field(), claim.base)
    return DataToServer(claim.claim_id, username, CLIENT_VERSION, r.distribution, r.nice_numbers)


def process_niceonly_gpu(ctx: GpuContext, claim: DataToClient, username: str) -> DataToServer:
    """process_niceonly_gpu (client_process_gpu.rs:924-941)."""
    r = process_range_niceonly_gpu(ctx, claim.field(), claim.base)
    return DataToServer(claim.claim_id, username, CLIENT_VERSION, None, r.nice_numbers)


_default_ctx: Optional[GpuContext] = None
_default_lock = threading.Lock()


def default_context() -> GpuContext:
    global _default_ctx
    with _default_lock:
        if _default_ctx is None:
            _default_ctx = GpuContext(0)
        return _default_ctx


def process_range_detailed(range_: FieldSize, base: int) -> FieldResults:
    """Drop-in for process_range_detailed (client_process.rs:150-191), on the GPU."""
    return process_range_detailed_gpu(default_context(), range_, base)


def process_range_niceonly(range_: FieldSize, base: int,
                           stride_table: Optional[StrideTable] = None) -> FieldResults:
    """Drop-in for process_range_niceonly (client_process.rs:439-465), on the GPU,
    with the CPU path's candidate set (MSD floor 250 over the whole range, stride
    table k from `stride_table`, default 2)."""
    k = stride_table.k if stride_table is not None else 2
    size = range_.range_size
    return process_range_niceonly_gpu(default_context(), range_, base, stride_k=k,
                                      chunk_size=min(size, (1 << 64) - 1))


def _cpu_out(cap: int):
    return (_lib.nice_number * max(cap, 1))()


def process_range_detailed_cpu(range_: FieldSize, base: int, threads: int = 1) -> FieldResults:
    """process_range_detailed (client_process.rs:150-191) on the host cores
    (nice_cpu_process_range_detailed): no device, for callers without a GPU.
    threads = 1 is the reference's single-threaded call."""
    hist = (ctypes.c_uint64 * (base + 1))()
    cap = 1024
    while True:
        out, n = _cpu_out(cap), ctypes.c_size_t()
        rc = lib().nice_cpu_process_range_detailed(*_split(range_.range_start), *_split(range_.range_end),
                                                    base, threads, hist, out, cap, n)
        if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
            cap = n.value
            continue
        check(rc)
        break
    return FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(out[i].number_lo | (out[i].number_hi << 64), out[i].num_uniques)
                      for i in range(n.value)])


def process_range_niceonly_cpu(range_: FieldSize, base: int,
                               stride_table: Optional[StrideTable] = None,
                               threads: int = 1) -> FieldResults:
    """process_range_niceonly (client_process.rs:439-465) on the host cores
    (nice_cpu_process_range_niceonly): MSD floor 250 over the whole range,
    stride table k from `stride_table` (default 2)."""
    k = stride_table.k if stride_table is not None else 2
    cap = 256
    while True:
        out, n = _cpu_out(cap), ctypes.c_size_t()
        rc = lib().nice_cpu_process_range_niceonly(*_split(range_.range_start), *_split(range_.range_end),
                                                    base, k, threads, out, cap, n)
        if rc == _lib.NICE_ERR_CAPACITY and n.value > cap:  # retry only with more room
            cap = n.value
            continue
        check(rc)
        break
    return FieldResults(distribution=[], nice_numbers=[
        NiceNumberSimple(out[i].number_lo | (out[i].number_hi << 64), base) for i in range(n.value)])
