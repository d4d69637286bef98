"""One field across the ranks of a torch.distributed group.

North star (BASELINE.json): "Fields shard naturally by contiguous n-range across
the 8 GPUs of one node; the tiny histograms are combined with an RCCL
all-reduce over xGMI, and nice-number lists are gathered to the host."

One process per GPU.  Rank r takes the r-th contiguous shard of [start, end)
and runs the library on its own device; the only exchange is ONE all-reduce
(SUM, int64) of [the (base + 1)-bin histogram, every rank's list length] —
a rank writes its own length into its slot of a one-hot block — followed by
an all-gather of the padded (lo, hi, num_uniques) rows only when some list is
non-empty (near-misses and nice numbers are rare: usually no second
collective).  `process_field_both_dist` does detailed and niceonly of a field
with that single all-reduce.

Detailed shards are contiguous and ordered by rank, so concatenating the
gathered near-miss lists in rank order is already ascending.  Niceonly work is
DEALT, not sliced: the whole field is cut on its client chunk grid
(client/src/main.rs:158-168) and rank r processes chunks c with c % N == r.
MSD survival is very uneven along a field (the b50 massive field's first 70 %
is pruned entirely), so contiguous slabs would leave most ranks idle; dealt
chunks give every rank a sample of the whole field, the way the reference
feeds descriptors from a shared channel (client_process_gpu.rs:589-709).  Each
chunk's MSD recursion is exactly the single-process CPU path's, so the
candidate set is unchanged; the gathered nice list is sorted (the reference
sorts after the fact too, client_process_gpu.rs:792).  A rank whose detailed
shard is empty (a field smaller than the world) contributes zeros to the
collective instead of calling the library.

With the nccl backend the collectives are RCCL over xGMI on device tensors;
with gloo (the CPU tests) they run on host tensors.  The per-field SUM of a
pipelined run has two transports: PipelinedExchange (the group's collective)
and ShmExchange (node-local shared memory, no device work; bench.py's default
when every rank is on one node).  `shard_fn` lets tests
substitute a shard processor; the default is the HIP library.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .types import FieldResults, FieldSize, NiceNumberSimple, UniquesDistributionSimple

MASK64 = (1 << 64) - 1


def client_chunk_size(size: int) -> int:
    """client/src/main.rs:158-168: 1e6 * clamp(ceil(size / 1e11), 1, 1000)."""
    mult = -(-size // (10 ** 6 * 10 ** 5))
    return 10 ** 6 * max(1, min(mult, 1000))


def shard_bounds(start: int, end: int, rank: int, world: int, grain: int = 1) -> Tuple[int, int]:
    """Contiguous shard r of [start, end), cut on multiples of `grain` from start
    (the last shard takes the ragged tail)."""
    if not 0 <= rank < world or start >= end:
        raise ValueError("bad shard request")
    units = -(-(end - start) // grain)
    per, extra = divmod(units, world)
    u0 = rank * per + min(rank, extra)
    u1 = u0 + per + (1 if rank < extra else 0)
    return min(end, start + u0 * grain), min(end, start + u1 * grain)


def dealt_chunks(start: int, end: int, chunk: int, stride: int, offset: int):
    """The chunks [c_s, c_e) of [start, end)'s chunk grid with index c %
    stride == offset, ascending (what nice_process_range_niceonly_ex processes
    with deal_stride / deal_offset)."""
    c = offset
    while start + c * chunk < end:
        a = start + c * chunk
        yield a, min(end, a + chunk)
        c += stride


def _device(dist, group):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _to_i64(v: int) -> int:
    return v - (1 << 64) if v >> 63 else v


def _all_reduce_ints(vals: Sequence[int], dist, group) -> List[int]:
    """One SUM all-reduce of an int64 vector (one H2D, one collective, one D2H)."""
    import torch
    t = torch.tensor(list(vals), dtype=torch.int64).to(_device(dist, group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().tolist()


def _onehot(rank: int, world: int, v: int) -> List[int]:
    out = [0] * world
    out[rank] = v
    return out


def _gather_rows(rows: Sequence[Tuple[int, int]], dist, group,
                 counts: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """all_gather of variable-length (number, aux) lists, in rank order.  With
    `counts` (every rank's list length, already exchanged) no count collective
    is issued, and nothing at all when every list is empty."""
    if counts is not None and not any(counts):
        return []  # every list empty (the usual case): no collective, no device work
    import torch
    dev = _device(dist, group)
    world = dist.get_world_size(group)
    if counts is None:
        counts = _all_reduce_ints(_onehot(dist.get_rank(group), world, len(rows)), dist, group)
    counts = [int(c) for c in counts]
    width = max(counts)
    if width == 0:
        return []
    buf = torch.zeros((width, 3), dtype=torch.int64)
    for i, (n, u) in enumerate(rows):
        buf[i, 0] = _to_i64(n & MASK64)
        buf[i, 1] = _to_i64(n >> 64)
        buf[i, 2] = u
    buf = buf.to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = []
    for c, p in zip(counts, parts):
        p = p[:c].cpu().tolist()
        out.extend((((hi & MASK64) << 64) | (lo & MASK64), u) for lo, hi, u in p)
    return out


def process_range_detailed_dist(range_: FieldSize, base: int, ctx=None, group=None,
                                shard_fn: Optional[Callable] = None) -> FieldResults:
    """process_range_detailed over a process group: every rank returns the
    whole field's FieldResults (identical to the single-process result).  One
    all-reduce carries the histogram and every rank's near-miss count; the
    lists are all-gathered only when some rank has entries."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    s, e = shard_bounds(range_.range_start, range_.range_end, rank, world)
    if shard_fn is None:
        shard_fn = ctx.detailed_raw
    hist, lst = shard_fn(s, e, base) if s < e else ([0] * (base + 1), [])
    red = _all_reduce_ints(list(hist[: base + 1]) + _onehot(rank, world, len(lst)), dist, group)
    hist, counts = red[: base + 1], red[base + 1:]
    rows = _gather_rows(lst, dist, group, counts=counts)
    return FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in rows])


def niceonly_deal(range_: FieldSize, rank: int, world: int, chunk: int = 0):
    """Rank r's niceonly work: the whole field's chunk grid, every world-th
    chunk from r.  Returns the library options that select it, or None when
    the field has fewer chunks than r + 1."""
    chunk = chunk or client_chunk_size(range_.range_size)
    if range_.range_start + rank * chunk >= range_.range_end:
        return None
    return {"chunk_size": chunk, "deal_stride": world, "deal_offset": rank}


def _zeros(base: int):
    return [0] * (base + 1)


def _both_shards(range_: FieldSize, base: int, ctx, rank: int, world: int, nice_opts):
    """This rank's detailed shard and niceonly deal of `range_`, through
    ctx.both_raw when the context has it (GpuContext: in sequence; BothModes:
    at once, on two streams), else detailed_raw then niceonly_raw."""
    s, e = shard_bounds(range_.range_start, range_.range_end, rank, world)
    det_range = (s, e) if s < e else None
    nice_opts = dict(nice_opts)
    deal = niceonly_deal(range_, rank, world, nice_opts.pop("chunk_size", 0))
    nice_range = (range_.range_start, range_.range_end) if deal else None
    if deal:
        nice_opts.update(deal)
    if hasattr(ctx, "both_raw"):
        (hist, near), nice = ctx.both_raw(det_range, nice_range, base, **nice_opts)
    else:
        hist, near = ctx.detailed_raw(s, e, base) if det_range else (None, [])
        nice = ctx.niceonly_raw(*nice_range, base, **nice_opts) if nice_range else ([], None)
    return (hist if hist is not None else _zeros(base), near), nice


def process_field_both_dist(range_: FieldSize, base: int, ctx, group=None,
                            **nice_opts):
    """Detailed AND niceonly of one field over a process group with ONE
    exchange: a single all-reduce of [histogram, near-miss counts per rank,
    nice counts per rank]; the lists are all-gathered only if non-empty.
    Returns (detailed FieldResults, niceonly FieldResults, this rank's
    niceonly statistics or None)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    (hist, near), (nice, stats) = _both_shards(range_, base, ctx, rank, world, nice_opts)
    red = _all_reduce_ints(list(hist[: base + 1]) + _onehot(rank, world, len(near))
                           + _onehot(rank, world, len(nice)), dist, group)
    hist = red[: base + 1]
    near_rows = _gather_rows(near, dist, group, counts=red[base + 1: base + 1 + world])
    nice_rows = sorted(_gather_rows([(n, base) for n in nice], dist, group,
                                    counts=red[base + 1 + world:]))
    det = FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in near_rows])
    return det, FieldResults(distribution=[],
                             nice_numbers=[NiceNumberSimple(n, u) for n, u in nice_rows]), stats


class PipelinedExchange:
    """Overlap each field's exchange with the next field's compute: submit()
    starts the all-reduce of this field's [histogram, counts] vector
    asynchronously (RCCL runs it while the ranks process the next field) and
    returns the reduced vector of the field submitted `lag` calls earlier (the
    previous one by default); drain() / drain_all() return the rest.
    The lists of a field are gathered when its vector is collected (only if
    non-empty, which is rare).  lag+1 preallocated device vectors rotate, fed
    from / read back into pinned host memory; on a GPU the read-back is queued
    behind the collective at submit time and marked by an event, so a step
    costs three asynchronous enqueues and collecting the previous field only
    waits on an event that has long fired (no synchronous copy on the
    launching thread)."""

    def __init__(self, dist, group=None, width: int = 0, lag: int = 1):
        # lag: submissions between a field's submit() and the one that returns
        # its vector (1 = the next one); lag+1 buffer sets rotate
        if lag < 1:
            raise ValueError("PipelinedExchange: lag must be >= 1")
        self.dist, self.group = dist, group
        self.lag = lag
        self.pending = []
        self.width = 0
        self.bufs = []
        self.flip = 0
        if width:
            self._alloc(width)

    def _alloc(self, width: int):
        import torch
        dev = _device(self.dist, self.group)
        pin = dev.type == "cuda"
        self.bufs = [(torch.zeros(width, dtype=torch.int64, pin_memory=pin),
                      torch.zeros(width, dtype=torch.int64, device=dev),
                      torch.zeros(width, dtype=torch.int64, pin_memory=pin)) for _ in range(self.lag + 1)]
        self.events = [torch.cuda.Event() for _ in range(self.lag + 1)] if pin else None
        self.width = width

    def submit(self, vals: Sequence[int], payload):
        if len(vals) != self.width:
            self.drain_check()
            self._alloc(len(vals))
        h_in, d, h_out = self.bufs[self.flip]
        ev = self.events[self.flip] if self.events is not None else None
        self.flip = (self.flip + 1) % (self.lag + 1)
        h_in.numpy()[:] = vals
        d.copy_(h_in, non_blocking=True)
        work = self.dist.all_reduce(d, op=self.dist.ReduceOp.SUM, group=self.group, async_op=True)
        if ev is not None:
            # device: the current stream waits for the collective (no host
            # block), then the read-back is queued and marked
            work.wait()
            h_out.copy_(d, non_blocking=True)
            ev.record()
            work = ev
        self.pending.append((work, d, h_out, payload))
        return self._collect(self.pending.pop(0)) if len(self.pending) > self.lag else None

    def drain_check(self):
        if self.pending:
            raise RuntimeError("PipelinedExchange: drain() before changing the vector width")

    def drain(self):
        """The oldest pending field's (vector, payload), or None."""
        return self._collect(self.pending.pop(0)) if self.pending else None

    def drain_all(self):
        out = []
        while self.pending:
            out.append(self._collect(self.pending.pop(0)))
        return out

    def _collect(self, p):
        if p is None:
            return None
        work, d, h_out, payload = p
        if self.events is not None:
            work.synchronize()  # the read-back queued at submit time
        else:
            work.wait()
            h_out.copy_(d)
        return h_out.tolist(), payload


class ShmUnavailable(RuntimeError):
    """Raised on EVERY rank when some rank cannot map the shared array."""


class ShmExchange:
    """PipelinedExchange's interface (submit / drain / drain_all) with the SUM
    done in node-local shared memory: the field's exchange vector is host data
    at both ends (the histogram comes back through the library's mapped
    result words, the counts are list lengths), so when every rank of the
    group runs on this host the ranks write their vectors into their rows of
    one /dev/shm array and each sums the column block itself.  No device copy
    and no collective kernel is queued behind the field kernels, and no
    transport latency is paid; the rare near-miss / nice lists still go
    through the group's collective (_gather_rows).

    Layout: int64 [2*lag + 2 sets][world][1 + width]; a rank writes its row's
    values, then the row's sequence word (= submission index + 1).  A set is
    rewritten 2*lag + 2 submissions later, and a rank can only be that far
    ahead of the slowest reader after that reader has published (its collect
    of s - lag waits for every row of s - lag), so no row is overwritten
    while it can still be read; collect checks the sequence words anyway.
    x86 stores are seen in program order, so a row whose sequence word is
    current holds that submission's values."""

    def __init__(self, dist, group=None, width: int = 0, lag: int = 1, timeout_s: float = 300.0):
        import platform
        import secrets
        if lag < 1:
            raise ValueError("ShmExchange: lag must be >= 1")
        if platform.machine() not in ("x86_64", "AMD64"):
            raise RuntimeError("ShmExchange relies on x86 store ordering")
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.lag, self.sets = lag, 2 * lag + 2
        self.width = width or MAX_BINS + 2 * self.world
        self.timeout_s = timeout_s
        name = [f"/dev/shm/nice_ex_{os.getpid()}_{secrets.token_hex(6)}" if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        self.path = name[0]
        shape = (self.sets, self.world, 1 + self.width)
        self.buf, err = None, None
        if self.rank == 0:
            try:
                self.buf = np.memmap(self.path, dtype=np.int64, mode="w+", shape=shape)
                self.buf[:] = 0
                self.buf.flush()
            except OSError as e:
                err = f"rank 0: {e}"
        dist.barrier(group=group)
        if self.rank != 0:
            try:
                self.buf = np.memmap(self.path, dtype=np.int64, mode="r+", shape=shape)
            except OSError as e:  # another host, or no /dev/shm
                err = f"rank {self.rank}: {e}"
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=group)
        if self.rank == 0 and self.buf is not None:
            os.unlink(self.path)  # the mappings stay; nothing is left behind in /dev/shm
        if any(errs):
            self.buf = None
            raise ShmUnavailable("; ".join(e for e in errs if e))
        self.step = 0
        self.pending = []

    def submit(self, vals: Sequence[int], payload):
        if len(vals) != self.width:
            raise ValueError(f"ShmExchange: vector of {len(vals)} values, the exchange holds {self.width}")
        row = self.buf[self.step % self.sets, self.rank]
        row[1:] = vals  # non-negative counts below 2**63 (numpy raises on anything else)
        row[0] = self.step + 1
        self.pending.append((self.step, payload))
        self.step += 1
        return self._collect(self.pending.pop(0)) if len(self.pending) > self.lag else None

    def drain(self):
        return self._collect(self.pending.pop(0)) if self.pending else None

    def drain_all(self):
        out = []
        while self.pending:
            out.append(self._collect(self.pending.pop(0)))
        return out

    def drain_check(self):
        if self.pending:
            raise RuntimeError("ShmExchange: drain() first")

    def _collect(self, p):
        import time
        step, payload = p
        blk = self.buf[step % self.sets]
        seq = blk[:, 0]
        deadline = None
        spins = 0
        while True:
            if (seq == step + 1).all():
                break
            if (seq > step + 1).any():
                raise RuntimeError("ShmExchange: a row was overwritten before it was read")
            spins += 1
            if spins > 64:
                now = time.monotonic()
                deadline = deadline or now + self.timeout_s
                if now > deadline:
                    raise TimeoutError(f"ShmExchange: ranks {list(np.flatnonzero(seq != step + 1))} "
                                       f"never published submission {step}")
                time.sleep(20e-6)
        red = blk[:, 1:].sum(axis=0).tolist()
        if not (seq == step + 1).all():
            raise RuntimeError("ShmExchange: a row was overwritten while it was read")
        return red, payload

    def close(self):
        """Drop this rank's mapping (no collective: the other ranks' mappings
        keep the memory until the last one is closed)."""
        self.pending = []
        self.buf = None


def process_field_both_pipelined(ex: PipelinedExchange, range_: FieldSize, base: int, ctx,
                                 **nice_opts):
    """process_field_both_dist with the exchange overlapped (see
    PipelinedExchange): computes this rank's shards of `range_`, starts their
    exchange, and returns the PREVIOUS submitted field's (detailed, niceonly,
    stats) results (None on the first call); ex.drain() + finish_both() give
    the last field's."""
    dist, group = ex.dist, ex.group
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    (hist, near), (nice, stats) = _both_shards(range_, base, ctx, rank, world, nice_opts)
    vec = exchange_vector(hist, base, rank, world, len(near), len(nice))
    return finish_both(ex, ex.submit(vec, (base, near, nice, stats)))


MAX_BINS = 129  # histogram bins of the widest base (128) -- the exchange vector's fixed head


def exchange_vector(hist, base: int, rank: int, world: int, n_near: int, n_nice: int) -> List[int]:
    """A field's pipelined exchange vector: the histogram zero-padded to the
    widest base's 129 bins, then every rank's near-miss and nice counts (one-hot
    blocks).  Its length depends only on the world size, so consecutive fields
    of different bases share the exchange's buffers (no drain in between)."""
    head = list(hist[: base + 1]) + [0] * (MAX_BINS - base - 1)
    return head + _onehot(rank, world, n_near) + _onehot(rank, world, n_nice)


def finish_both(ex: PipelinedExchange, collected):
    """Turn a collected (vector, payload) pair into (detailed, niceonly, stats)."""
    if collected is None:
        return None
    red, (base, near, nice, stats) = collected
    world = ex.dist.get_world_size(ex.group)
    hist = red[: base + 1]
    near_rows = _gather_rows(near, ex.dist, ex.group, counts=red[MAX_BINS: MAX_BINS + world])
    nice_rows = sorted(_gather_rows([(n, base) for n in nice], ex.dist, ex.group,
                                    counts=red[MAX_BINS + world:]))
    det = FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in near_rows])
    return det, FieldResults(distribution=[],
                             nice_numbers=[NiceNumberSimple(n, u) for n, u in nice_rows]), stats


def process_range_niceonly_dist(range_: FieldSize, base: int, ctx=None, group=None,
                                shard_fn: Optional[Callable] = None, **opts) -> FieldResults:
    """process_range_niceonly over a process group: rank r is dealt every
    world-th chunk of the field's chunk grid (see module doc).  shard_fn(start,
    end, base, **deal) stands in for ctx.niceonly_raw in the CPU tests."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    deal = niceonly_deal(range_, rank, world, opts.pop("chunk_size", 0))
    lst = []
    if deal:
        if shard_fn is None:
            lst, _ = ctx.niceonly_raw(range_.range_start, range_.range_end, base, **deal, **opts)
        else:
            lst = shard_fn(range_.range_start, range_.range_end, base, **deal)
    rows = sorted(_gather_rows([(n, base) for n in lst], dist, group))
    return FieldResults(distribution=[], nice_numbers=[NiceNumberSimple(n, u) for n, u in rows])


class FieldPipeline:
    """Both modes of a stream of fields with the GPU never waiting for the
    host: field i is submitted (detailed and niceonly on their own streams,
    nice_*_submit) before field i-depth is collected, and -- over a
    process group -- that field's exchange (one all-reduce, PipelinedExchange)
    is in flight while the later fields compute.  step() returns the results of an
    earlier field as (range, detailed FieldResults, niceonly FieldResults,
    this rank's niceonly stats), or None while the pipeline fills; drain()
    returns the rest.  The reference client overlaps fetch / process / submit
    across fields the same way (client/src/main.rs:411-562).

    Rank r (of N) processes the r-th contiguous detailed shard of each field
    and is dealt every N-th niceonly chunk of it (see module doc); with
    dist=None the whole field runs on this process's contexts."""

    def __init__(self, det_ctx, nice_ctx, dist=None, group=None, depth: int = 2, lag: int = 1,
                 exchange=None, **nice_opts):
        # depth: fields kept in flight behind the one being collected (the
        # library holds up to 3 per mode and context)
        self.depth = depth
        self.det, self.nice = det_ctx, nice_ctx
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group) if dist is not None else 0
        self.world = dist.get_world_size(group) if dist is not None else 1
        # exchange: a PipelinedExchange / ShmExchange to use (drained by every
        # drain()), else a PipelinedExchange over `group` with `lag`
        # exchanges kept in flight
        self.ex = exchange if exchange is not None or dist is None else \
            PipelinedExchange(dist, group, lag=lag)
        self.nice_opts = dict(nice_opts)
        self.inflight = []  # (range, base, det ticket or None, nice ticket or None)
        self.kernel_ms = []  # detailed kernel time of each collected field (HIP events)

    def _submit(self, range_: FieldSize, base: int):
        s, e = shard_bounds(range_.range_start, range_.range_end, self.rank, self.world)
        opts = dict(self.nice_opts)
        deal = niceonly_deal(range_, self.rank, self.world, opts.pop("chunk_size", 0))
        td = self.det.detailed_submit(s, e, base) if s < e else None
        tn = None
        if deal:
            opts.update(deal)
            tn = self.nice.niceonly_submit(range_.range_start, range_.range_end, base, **opts)
        self.inflight.append((range_, base, td, tn))

    def _collect_oldest(self):
        range_, base, td, tn = self.inflight.pop(0)
        if td is not None:
            hist, near = self.det.detailed_collect(td, base)
            self.kernel_ms.append(self.det.kernel_stats().kernel_ms)
        else:
            hist, near = _zeros(base), []
        nice, stats = self.nice.niceonly_collect(tn) if tn is not None else ([], None)
        if self.ex is None:
            return (range_, _results(hist, near, base), FieldResults(
                distribution=[], nice_numbers=[NiceNumberSimple(n, base) for n in nice]), stats)
        vec = exchange_vector(hist, base, self.rank, self.world, len(near), len(nice))
        return self._finish(self.ex.submit(vec, (base, near, nice, stats, range_)))

    def _finish(self, collected):
        if collected is None:
            return None
        red, (base, near, nice, stats, range_) = collected
        det, nic, st = finish_both(self.ex, (red, (base, near, nice, stats)))
        return range_, det, nic, st

    def step(self, range_: FieldSize, base: int):
        self._submit(range_, base)
        if len(self.inflight) <= self.depth:
            return None
        return self._collect_oldest()

    def drain(self):
        out = []
        while self.inflight:
            r = self._collect_oldest()
            if r is not None:
                out.append(r)
        if self.ex is not None:
            out.extend(self._finish(c) for c in self.ex.drain_all())
        return out


def _results(hist, near, base):
    return FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in near])
