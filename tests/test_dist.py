"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2; one 8-rank
rehearsal of the N = 8 path): weak-scaling
field assignment (disjoint consecutive 1e9 fields, all inside base 40's range)
and the max-over-ranks timing reduction."""
import contextlib
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time

    import bench
    field = bench.rank_field(1_916_284_264_916, rank)
    delay = 0.05 * (rank + 1)
    el = bench.timed(lambda: time.sleep(delay), 2, dist.barrier, dist)
    q.put((rank, field, el))
    dist.destroy_process_group()


def test_two_rank_weak_scaling_plumbing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, f0, e0), (r1, f1, e1) = out
    assert f0[1] == f1[0] and f0[1] - f0[0] == 10 ** 9 and f1[1] - f1[0] == 10 ** 9
    assert f1[1] <= 6_553_600_000_000  # inside base 40's range (base_range.rs:86-87)
    # max over ranks: both ranks report the slower rank's time (2 x 0.1 s)
    assert abs(e0 - e1) < 1e-9 and e0 >= 0.2


# --- one field across ranks: histogram all-reduce + list all-gather ----------
def _oracle_detailed_shard(s, e, base):
    from oracle import oracle as O
    r = O.process_range_detailed(s, e, base)
    hist = [0] * (base + 1)
    for u, c in r.distribution:
        hist[u] = c
    return hist, list(r.nice_numbers)


def _oracle_niceonly_shard(s, e, base, chunk_size, deal_stride=1, deal_offset=0):
    """The oracle over the chunks nice_process_range_niceonly_ex processes
    with these deal options (every deal_stride-th chunk of [s, e)'s grid)."""
    from oracle import oracle as O
    from nice_amd.dist import dealt_chunks
    out = []
    for a, b in dealt_chunks(s, e, chunk_size, deal_stride or 1, deal_offset):
        out += [n for n, _ in O.process_range_niceonly(a, b, base)[0].nice_numbers]
    return out


class _OracleCtx:
    """Stands in for nice_amd.GpuContext in the CPU tests (oracle-backed),
    including the asynchronous submit / collect pair (two fields in flight)."""

    def __init__(self):
        self.jobs = {}
        self.next = 0

    def _ticket(self, job):
        t = self.next
        assert t not in self.jobs, "more than three fields in flight"
        self.jobs[t] = job
        self.next = (t + 1) % 3
        return t

    def detailed_submit(self, s, e, base):
        return self._ticket(("d", s, e, base))

    def detailed_collect(self, t, base):
        _, s, e, b = self.jobs.pop(t)
        assert b == base
        return self.detailed_raw(s, e, base)

    def niceonly_submit(self, s, e, base, **kw):
        return self._ticket(("n", s, e, base, kw))

    def niceonly_collect(self, t):
        _, s, e, base, kw = self.jobs.pop(t)
        return self.niceonly_raw(s, e, base, **kw)

    def kernel_stats(self):
        class _K:
            kernel_ms = 0.0
        return _K()

    def detailed_raw(self, s, e, base):
        assert s < e, "empty detailed shard must not reach the library"
        return _oracle_detailed_shard(s, e, base)

    def niceonly_raw(self, s, e, base, chunk_size=0, deal_stride=1, deal_offset=0, **_):
        from nice_amd.dist import client_chunk_size
        return _oracle_niceonly_shard(s, e, base, chunk_size or client_chunk_size(e - s),
                                      deal_stride, deal_offset), None


def _field_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nice_amd import dist as D
    from nice_amd.types import FieldSize
    res = {}
    s40 = 1_916_284_264_916
    for name, f, b in [("b40", FieldSize(s40, s40 + 200_001), 40),
                       ("b10_oob", FieldSize(10 ** 6, 10 ** 6 + 10 ** 4), 10)]:
        r = D.process_range_detailed_dist(f, b, shard_fn=_oracle_detailed_shard)
        res[name] = ([(d.num_uniques, d.count) for d in r.distribution],
                     [(n.number, n.num_uniques) for n in r.nice_numbers])
    r = D.process_range_niceonly_dist(FieldSize(47, 100), 10, shard_fn=_oracle_niceonly_shard)
    res["nice_b10"] = [(n.number, n.num_uniques) for n in r.nice_numbers]
    r = D.process_range_niceonly_dist(FieldSize(s40, s40 + 10 ** 6), 40, chunk_size=99_991,
                                      shard_fn=_oracle_niceonly_shard)
    res["nice_b40"] = [(n.number, n.num_uniques) for n in r.nice_numbers]
    # both modes with one exchange (bench.py's N > 1 step), oracle-backed context
    det, nic, _ = D.process_field_both_dist(FieldSize(10 ** 6 - 53, 10 ** 6 + 3_000), 10,
                                            _OracleCtx(), chunk_size=1_013)
    res["both_b10"] = ([(d.num_uniques, d.count) for d in det.distribution],
                       [(n.number, n.num_uniques) for n in det.nice_numbers],
                       [n.number for n in nic.nice_numbers])
    # the pipelined exchange returns each field's results one call later
    ex = D.PipelinedExchange(dist)
    fields = [FieldSize(a, a + 2_000) for a in (47, 10 ** 6 - 53, 2 * 10 ** 6)]
    got = [D.process_field_both_pipelined(ex, f, 10, _OracleCtx(), chunk_size=997) for f in fields]
    got.append(D.finish_both(ex, ex.drain()))
    assert got[0] is None
    res["pipelined"] = [([(d.num_uniques, d.count) for d in r[0].distribution],
                         [(n.number, n.num_uniques) for n in r[0].nice_numbers],
                         [n.number for n in r[1].nice_numbers]) for r in got[1:]]
    # the same through BothModes (the two modes at once, bench.py's default)
    from nice_amd import BothModes
    both = BothModes(det_ctx=_OracleCtx(), nice_ctx=_OracleCtx())
    got = [D.process_field_both_pipelined(ex, f, 10, both, chunk_size=997) for f in fields]
    got.append(D.finish_both(ex, ex.drain()))
    both.close()
    res["pipelined_both"] = [([(d.num_uniques, d.count) for d in r[0].distribution],
                              [(n.number, n.num_uniques) for n in r[0].nice_numbers],
                              [n.number for n in r[1].nice_numbers]) for r in got[1:]]
    # a field smaller than the world: rank 1's detailed shard is empty and
    # must contribute zeros instead of calling the library (no hang)
    r = D.process_range_detailed_dist(FieldSize(69, 70), 10, shard_fn=_oracle_detailed_shard)
    res["tiny"] = ([(d.num_uniques, d.count) for d in r.distribution],
                   [(n.number, n.num_uniques) for n in r.nice_numbers])
    det, nic, _ = D.process_field_both_dist(FieldSize(69, 70), 10, _OracleCtx())
    res["tiny_both"] = ([(d.num_uniques, d.count) for d in det.distribution],
                        [(n.number, n.num_uniques) for n in det.nice_numbers],
                        [n.number for n in nic.nice_numbers])
    # the field pipeline (bench.py's step): two fields in flight, exchange overlapped
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, chunk_size=997)
    got = [pipe.step(f, 10) for f in fields + [FieldSize(69, 70)]]
    got = [g for g in got if g is not None] + pipe.drain()
    res["field_pipeline"] = [((r.range_start, r.range_end),
                              [(d.num_uniques, d.count) for d in det.distribution],
                              [(n.number, n.num_uniques) for n in det.nice_numbers],
                              [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    # fields of different bases back to back (the client's field stream can
    # change base): the exchange vector keeps its width, nothing drains early
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, chunk_size=997)
    mixed = [(FieldSize(47, 2_047), 10), (FieldSize(1, 3_000), 12), (FieldSize(10 ** 6, 10 ** 6 + 900), 40),
             (FieldSize(69, 70), 10)]
    got = [pipe.step(f, b) for f, b in mixed]
    got = [g for g in got if g is not None] + pipe.drain()
    res["field_pipeline_mixed"] = [((r.range_start, r.range_end), len(det.distribution),
                                    [(d.num_uniques, d.count) for d in det.distribution],
                                    [(n.number, n.num_uniques) for n in det.nice_numbers],
                                    [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    # two exchanges in flight (bench.py --exchange-lag 2): the same results, in order
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, lag=2, chunk_size=997)
    got = [pipe.step(f, b) for f, b in mixed]
    assert got == [None] * 4  # depth 2 + lag 2: a field's results come back 4 steps later
    got = [g for g in got if g is not None] + pipe.drain()
    res["field_pipeline_lag2"] = [((r.range_start, r.range_end), len(det.distribution),
                                   [(d.num_uniques, d.count) for d in det.distribution],
                                   [(n.number, n.num_uniques) for n in det.nice_numbers],
                                   [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    # the node-local shared-memory exchange (bench.py --exchange-backend shm), lag 1 and 2
    for lag in (1, 2):
        ex = D.ShmExchange(dist, lag=lag)
        pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, exchange=ex, chunk_size=997)
        got = [pipe.step(f, b) for f, b in mixed]
        got = [g for g in got if g is not None] + pipe.drain()
        ex.close()
        res[f"field_pipeline_shm{lag}"] = [((r.range_start, r.range_end), len(det.distribution),
                                           [(d.num_uniques, d.count) for d in det.distribution],
                                           [(n.number, n.num_uniques) for n in det.nice_numbers],
                                           [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    # one rank unable to map the array: every rank raises ShmUnavailable (no hang)
    import unittest.mock
    import numpy
    with unittest.mock.patch.object(numpy, "memmap", side_effect=OSError("no /dev/shm")) \
            if rank == 1 else contextlib.nullcontext():
        try:
            D.ShmExchange(dist)
            res["shm_unavailable"] = None
        except D.ShmUnavailable as e:
            res["shm_unavailable"] = str(e)
    q.put((rank, res))
    dist.destroy_process_group()


def test_two_rank_field_sharding_matches_single_process():
    from oracle import oracle as O
    from nice_amd import dist as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_field_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1]  # every rank holds the whole field's results
    s40 = 1_916_284_264_916
    w = O.process_range_detailed(s40, s40 + 200_001, 40)
    assert out[0]["b40"] == (w.distribution, w.nice_numbers)
    w = O.process_range_detailed(10 ** 6, 10 ** 6 + 10 ** 4, 10)
    assert out[0]["b10_oob"] == (w.distribution, w.nice_numbers)
    assert len(w.nice_numbers) == 5395  # lists gathered in ascending order
    assert out[0]["nice_b10"] == [(69, 10)]
    assert out[0]["nice_b40"] == []
    w = O.process_range_detailed(10 ** 6 - 53, 10 ** 6 + 3_000, 10)
    want_nice = _oracle_niceonly_shard(10 ** 6 - 53, 10 ** 6 + 3_000, 10, 1_013)
    assert out[0]["both_b10"] == (w.distribution, w.nice_numbers, want_nice)
    assert len(w.nice_numbers) > 1000
    for (a, r) in zip((47, 10 ** 6 - 53, 2 * 10 ** 6), out[0]["pipelined"]):
        w = O.process_range_detailed(a, a + 2_000, 10)
        assert r == (w.distribution, w.nice_numbers, _oracle_niceonly_shard(a, a + 2_000, 10, 997))
    assert out[0]["pipelined"][0][2] == [69]
    assert out[0]["pipelined_both"] == out[0]["pipelined"]
    fields = [(47, 2_047), (10 ** 6 - 53, 10 ** 6 + 1_947), (2 * 10 ** 6, 2 * 10 ** 6 + 2_000),
              (69, 70)]
    assert [r[0] for r in out[0]["field_pipeline"]] == fields
    for (a, b), d, near, nice in [r for r in out[0]["field_pipeline"]]:
        w = O.process_range_detailed(a, b, 10)
        assert (d, near) == (w.distribution, w.nice_numbers)
        assert nice == _oracle_niceonly_shard(a, b, 10, 997)
    mixed = out[0]["field_pipeline_mixed"]
    assert [(r[0], r[1]) for r in mixed] == [((47, 2_047), 10), ((1, 3_000), 12),
                                             ((10 ** 6, 10 ** 6 + 900), 40), ((69, 70), 10)]
    for (a, b), base, d, near, nice in mixed:
        w = O.process_range_detailed(a, b, base)
        assert (d, near) == (w.distribution, w.nice_numbers), base
        assert nice == _oracle_niceonly_shard(a, b, base, 997), base
    assert out[0]["field_pipeline_lag2"] == mixed
    assert out[0]["field_pipeline_shm1"] == mixed and out[0]["field_pipeline_shm2"] == mixed
    assert out[0]["shm_unavailable"] == "rank 1: no /dev/shm"
    w = O.process_range_detailed(69, 70, 10)
    assert out[0]["tiny"] == (w.distribution, [(69, 10)])
    assert out[0]["tiny_both"] == (w.distribution, [(69, 10)], [69])
    # niceonly is dealt on the whole field's chunk grid
    from nice_amd.types import FieldSize
    assert D.niceonly_deal(FieldSize(0, 10 ** 6), 1, 2, 99_991) == \
        {"chunk_size": 99_991, "deal_stride": 2, "deal_offset": 1}
    assert D.niceonly_deal(FieldSize(0, 5), 1, 2) is None
    assert list(D.dealt_chunks(0, 10, 3, 2, 1)) == [(3, 6), (9, 10)]
    assert D.shard_bounds(0, 10, 1, 3) == (4, 7)
    assert D.client_chunk_size(10 ** 9) == 10 ** 6 and D.client_chunk_size(10 ** 13) == 10 ** 8


def _eight_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nice_amd import dist as D
    from nice_amd.types import FieldSize
    res = {}
    r = D.process_range_detailed_dist(FieldSize(10 ** 6, 10 ** 6 + 4_001), 10, shard_fn=_oracle_detailed_shard)
    res["b10_oob"] = ([(d.num_uniques, d.count) for d in r.distribution],
                      [(n.number, n.num_uniques) for n in r.nice_numbers])
    r = D.process_range_niceonly_dist(FieldSize(47, 100), 10, shard_fn=_oracle_niceonly_shard)
    res["nice_b10"] = [(n.number, n.num_uniques) for n in r.nice_numbers]
    # bench.py's step at N = 8: the field pipeline, exchange overlapped, with
    # fields smaller than the world (most ranks' shards empty) between others
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, chunk_size=97)
    fields = [(FieldSize(47, 1_047), 10), (FieldSize(69, 70), 10), (FieldSize(1, 5), 12),
              (FieldSize(10 ** 6, 10 ** 6 + 1_003), 40), (FieldSize(2 * 10 ** 6, 2 * 10 ** 6 + 777), 10)]
    got = [pipe.step(f, b) for f, b in fields]
    got = [g for g in got if g is not None] + pipe.drain()
    res["field_pipeline"] = [((r.range_start, r.range_end),
                              [(d.num_uniques, d.count) for d in det.distribution],
                              [(n.number, n.num_uniques) for n in det.nice_numbers],
                              [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    # the same over the shared-memory exchange (bench.py's default at N > 1 on one node)
    ex = D.ShmExchange(dist, lag=2)
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx(), dist, exchange=ex, chunk_size=97)
    got = [pipe.step(f, b) for f, b in fields]
    got = [g for g in got if g is not None] + pipe.drain()
    ex.close()
    res["field_pipeline_shm"] = [((r.range_start, r.range_end),
                                  [(d.num_uniques, d.count) for d in det.distribution],
                                  [(n.number, n.num_uniques) for n in det.nice_numbers],
                                  [n.number for n in nic.nice_numbers]) for r, det, nic, _ in got]
    q.put((rank, res))
    dist.destroy_process_group()


def test_eight_rank_rehearsal():
    """The N = 8 code path (the driver's scaling run) rehearsed on CPU: eight
    gloo ranks shard detailed fields, deal niceonly chunks and run bench.py's
    field pipeline, including fields smaller than the world; every rank ends
    with the whole field's results, equal to the oracle's."""
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_eight_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] == out[0] for r in range(8))
    w = O.process_range_detailed(10 ** 6, 10 ** 6 + 4_001, 10)
    assert out[0]["b10_oob"] == (w.distribution, w.nice_numbers)
    assert out[0]["nice_b10"] == [(69, 10)]
    want = [((47, 1_047), 10), ((69, 70), 10), ((1, 5), 12), ((10 ** 6, 10 ** 6 + 1_003), 40),
            ((2 * 10 ** 6, 2 * 10 ** 6 + 777), 10)]
    assert [r[0] for r in out[0]["field_pipeline"]] == [f for f, _ in want]
    for ((a, b), base), (_, d, near, nice) in zip(want, out[0]["field_pipeline"]):
        w = O.process_range_detailed(a, b, base)
        assert (d, near) == (w.distribution, w.nice_numbers), (a, base)
        assert nice == _oracle_niceonly_shard(a, b, base, 97), (a, base)
    assert out[0]["field_pipeline_shm"] == out[0]["field_pipeline"]


def test_both_modes_runner_matches_sequential_and_propagates_errors():
    """BothModes (nice_amd/api.py): niceonly on a worker thread beside the
    detailed call; same results as the two calls in sequence, and an error
    raised by the niceonly pass surfaces on the calling thread."""
    from nice_amd import BothModes
    both = BothModes(det_ctx=_OracleCtx(), nice_ctx=_OracleCtx())
    try:
        for a in (47, 10 ** 6 - 53):
            (h, near), (nice, _) = both.both_raw((a, a + 1_500), (a, a + 1_500), 10, chunk_size=500)
            ref = _OracleCtx()
            assert (h, near) == ref.detailed_raw(a, a + 1_500, 10)
            assert nice == ref.niceonly_raw(a, a + 1_500, 10, chunk_size=500)[0]
        (h, _), (nice, st) = both.both_raw((47, 100), None, 10)
        assert nice == [] and st is None and sum(h) == 53

        class Boom(_OracleCtx):
            def niceonly_raw(self, *a, **k):
                raise ValueError("boom")
        bad = BothModes(det_ctx=_OracleCtx(), nice_ctx=Boom())
        with pytest.raises(ValueError, match="boom"):
            bad.both_raw((47, 100), (47, 100), 10)
        bad.close()
    finally:
        both.close()


def test_niceonly_dealing_balances_survival_skew():
    """Per-rank niceonly work under dealing (dist.niceonly_deal), on a scaled
    b50 window across the massive field's survival onset (the MSD filter
    prunes everything before it): with 8 ranks every rank's candidate count
    is within 10 % of the mean, while contiguous slabs would give rank 0
    almost nothing; the dealt chunks together are the single-process run."""
    from concurrent.futures import ThreadPoolExecutor

    from nice_amd import dist as D
    from nice_amd.types import FieldSize
    from oracle import oracle as O
    a = O.base_range(50)[0] + 7_372_000_000_000
    e, chunk, world = a + 2 * 10 ** 9, 10 ** 6, 8

    def cands(c):
        return O.process_field_niceonly_ex(c[0], c[1], 50, 1, chunk=chunk)[1]

    with ThreadPoolExecutor(8) as pool:
        per_rank = []
        for r in range(world):
            deal = D.niceonly_deal(FieldSize(a, e), r, world, chunk)
            per_rank.append(sum(pool.map(cands, D.dealt_chunks(a, e, **{
                "chunk": deal["chunk_size"], "stride": deal["deal_stride"],
                "offset": deal["deal_offset"]}))))
        slabs = [sum(pool.map(cands, D.dealt_chunks(*D.shard_bounds(a, e, r, world, chunk),
                                                    chunk, 1, 0))) for r in (0,)]
    mean = sum(per_rank) / world
    assert all(abs(c - mean) <= 0.1 * mean for c in per_rank), per_rank
    assert slabs[0] < 0.01 * mean  # the contiguous first slab is pruned
    assert sum(per_rank) == O.process_field_niceonly_ex(a, e, 50, 8, chunk=chunk)[1]


def test_field_pipeline_single_process():
    """FieldPipeline without a process group (bench.py at N = 1): results come
    back `depth` fields late, in submission order, equal to the oracle."""
    from nice_amd import dist as D
    from nice_amd.types import FieldSize
    from oracle import oracle as O
    pipe = D.FieldPipeline(_OracleCtx(), _OracleCtx())
    fields = [FieldSize(a, a + 3_000) for a in (47, 5 * 10 ** 5, 10 ** 6)]
    got = [pipe.step(f, 10) for f in fields]
    assert got[0] is None and got[1] is None and got[2][0] == fields[0]
    got = got[2:] + pipe.drain()
    assert [g[0] for g in got] == fields
    for f, det, nic, _ in got:
        w = O.process_range_detailed(f.range_start, f.range_end, 10)
        assert [(d.num_uniques, d.count) for d in det.distribution] == w.distribution
        assert [(n.number, n.num_uniques) for n in det.nice_numbers] == w.nice_numbers
        assert [n.number for n in nic.nice_numbers] == \
            [n for n, _ in O.process_field_niceonly_mt(f.range_start, f.range_end, 10, 2)[0].nice_numbers]


class _OneRank:
    """The slice of torch.distributed ShmExchange uses, for a 1-rank group."""

    def get_rank(self, group=None):
        return 0

    def get_world_size(self, group=None):
        return 1

    def broadcast_object_list(self, objs, src=0, group=None):
        pass

    def barrier(self, group=None):
        pass

    def all_gather_object(self, out, obj, group=None):
        out[0] = obj


def test_shm_exchange_order_lag_and_guards():
    """ShmExchange on one rank: each submit returns the vector submitted `lag`
    calls earlier (summed over the ranks: itself here), drain_all returns the
    rest in order, the /dev/shm file is gone once mapped, and a wrong width,
    a lag below 1 and a row overwritten before it was read all raise."""
    from nice_amd import dist as D
    d = _OneRank()
    with pytest.raises(ValueError):
        D.ShmExchange(d, lag=0)
    for lag in (1, 2, 3):
        ex = D.ShmExchange(d, lag=lag)
        assert not os.path.exists(ex.path)
        w = ex.width
        vecs = [[k * 1000 + i for i in range(w)] for k in range(7)]
        got = [ex.submit(v, k) for k, v in enumerate(vecs)]
        assert got[:lag] == [None] * lag
        got = [g for g in got[lag:]] + ex.drain_all()
        assert [k for _, k in got] == list(range(7))
        assert all(red == vecs[k] for red, k in got)
        with pytest.raises(ValueError):
            ex.submit([0] * (w - 1), None)
        # a row rewritten past its set's reuse distance is detected, not read
        ex.submit(vecs[0], "a")
        step = ex.step - 1
        ex.buf[step % ex.sets, 0, 0] = step + 1 + ex.sets
        with pytest.raises(RuntimeError):
            ex.drain()
        ex.close()


def test_bench_refuses_a_world_size_other_than_gpus():
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus exits
    non-zero before touching a device (a run that would time another number
    of GPUs than it reports); --gpus 0 likewise."""
    import subprocess
    import sys
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    for world, gpus in (("3", "2"), ("1", "8"), ("2", "1")):
        out = subprocess.run([sys.executable, bench, "--gpus", gpus], capture_output=True, text=True,
                             timeout=60, env=dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0"))
        assert out.returncode == 2 and "WORLD_SIZE" in out.stderr and out.stdout == ""
    out = subprocess.run([sys.executable, bench, "--gpus", "0"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 2 and out.stdout == ""
