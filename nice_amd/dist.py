"""One field across the ranks of a torch.distributed group.

North star (BASELINE.json): "Fields shard naturally by contiguous n-range across
the 8 GPUs of one node; the tiny histograms are combined with an RCCL
all-reduce over xGMI, and nice-number lists are gathered to the host."

One process per GPU.  Rank r takes the r-th contiguous shard of [start, end)
and runs the library on its own device; the only exchange is

  detailed:  all_reduce(SUM) of the (base + 1)-bin u64 histogram, then an
             all_gather of the near-miss lists (count first, then the padded
             (lo, hi, num_uniques) rows);
  niceonly:  the same all_gather of the nice lists.

Shards are contiguous and ordered by rank, so concatenating the gathered lists
in rank order is already ascending (the reference sorts after the fact,
client_process_gpu.rs:792, 873).  Niceonly shards are cut on the client chunk
grid of the WHOLE field (client/src/main.rs:158-168) and each rank is told
that chunk size, so the MSD recursion sees exactly the chunks the single-
process CPU path would, and the candidate set is unchanged by sharding.

With the nccl backend the collectives are RCCL over xGMI on device tensors;
with gloo (the CPU tests) they run on host tensors.  `shard_fn` lets tests
substitute a shard processor; the default is the HIP library.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

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


def _device(dist, group):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _to_i64(v: int) -> int:
    return v - (1 << 64) if v >> 63 else v


def _gather_rows(rows: Sequence[Tuple[int, int]], dist, group) -> List[Tuple[int, int]]:
    """all_gather of variable-length (number, aux) lists, in rank order."""
    import torch
    dev = _device(dist, group)
    world = dist.get_world_size(group)
    cnt = torch.tensor([len(rows)], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
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
    whole field's FieldResults (identical to the single-process result)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    s, e = shard_bounds(range_.range_start, range_.range_end, rank, world)
    if shard_fn is None:
        shard_fn = ctx.detailed_raw
    hist, lst = shard_fn(s, e, base)
    h = torch.tensor(list(hist[: base + 1]), dtype=torch.int64, device=_device(dist, group))
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    hist = [int(x) for x in h.cpu().tolist()]
    rows = _gather_rows(lst, dist, group)
    return FieldResults(
        distribution=[UniquesDistributionSimple(i, hist[i]) for i in range(1, base + 1)],
        nice_numbers=[NiceNumberSimple(n, u) for n, u in rows])


def process_range_niceonly_dist(range_: FieldSize, base: int, ctx=None, group=None,
                                shard_fn: Optional[Callable] = None, **opts) -> FieldResults:
    """process_range_niceonly over a process group (shards on the whole
    field's client chunk grid, see module doc)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    chunk = opts.pop("chunk_size", 0) or client_chunk_size(range_.range_size)
    s, e = shard_bounds(range_.range_start, range_.range_end, rank, world, grain=chunk)
    if s < e:
        if shard_fn is None:
            lst, _ = ctx.niceonly_raw(s, e, base, chunk_size=chunk, **opts)
        else:
            lst = shard_fn(s, e, base, chunk)
    else:
        lst = []
    rows = _gather_rows([(n, base) for n in lst], dist, group)
    return FieldResults(distribution=[], nice_numbers=[NiceNumberSimple(n, u) for n, u in rows])
