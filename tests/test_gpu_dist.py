"""Two ranks on the GPU (gloo collectives, both ranks on device 0): the
strong-scaling field pipeline of bench.py end to end -- the b40 1e9 field
split two ways (contiguous detailed shards, dealt niceonly chunks), results
exchanged and compared with the committed oracle fixtures on every rank; and
the massive field's niceonly dealt over the two ranks, whose candidate and
range totals must equal the oracle fixture's.  (RCCL needs one GPU per rank;
gloo exercises the same code path on a one-GPU box.)"""
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import nice_amd as N
    from nice_amd import dist as D
    out = {}
    ctx = N.GpuContext(0)
    try:
        s = N.get_base_range_u128(40).range_start
        f = N.FieldSize(s, s + 10 ** 9)
        pipe = D.FieldPipeline(ctx, ctx, dist)
        got = [pipe.step(f, 40) for _ in range(3)]
        got = [g for g in got if g is not None] + pipe.drain()
        out["fields"] = [([(d.num_uniques, d.count) for d in det.distribution],
                          [(n.number, n.num_uniques) for n in det.nice_numbers],
                          [str(n.number) for n in nic.nice_numbers], st.candidates, st.ranges)
                         for _, det, nic, st in got]
        with open(os.path.join(ROOT, "tests", "golden", "massive_b50.json")) as fh:
            m = json.load(fh)
        lst, st = ctx.niceonly_raw(int(m["start"]), int(m["end"]), 50, deal_stride=world,
                                   deal_offset=rank)
        out["massive"] = (st.candidates, st.ranges, lst)
    finally:
        ctx.close()
    q.put((rank, out))
    dist.destroy_process_group()


def test_two_rank_strong_pipeline_on_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    with open(os.path.join(ROOT, "tests", "golden", "oracle_fields.json")) as fh:
        fx = json.load(fh)
    det = next(c for c in fx["detailed"] if c["name"] == "b40_extra_large_1e9")
    nic = next(c for c in fx["niceonly"] if c["name"] == "b40_extra_large_1e9")
    # every rank holds the whole field's results, every field equal to the fixture
    assert len(res[0]["fields"]) == 3 and [r[:3] for r in res[0]["fields"]] == [r[:3] for r in res[1]["fields"]]
    for r in range(2):
        for dist_, near, nice, _, _ in res[r]["fields"]:
            assert dist_ == [tuple(x) for x in det["distribution"]]
            assert near == [(int(n), u) for n, u in det["near_misses"]]
            assert nice == nic["nice_numbers"]
    # dealt niceonly: the two ranks' candidate counts sum to the whole field's
    assert all(a[3] + b[3] == nic["candidates"] for a, b in zip(res[0]["fields"], res[1]["fields"]))
    with open(os.path.join(ROOT, "tests", "golden", "massive_b50.json")) as fh:
        m = json.load(fh)
    c = res[0]["massive"][0] + res[1]["massive"][0]
    r_ = res[0]["massive"][1] + res[1]["massive"][1]
    assert (c, r_) == (sum(w["candidates"] for w in m["windows"]), sum(w["ranges"] for w in m["windows"]))
    assert res[0]["massive"][2] == [] and res[1]["massive"][2] == []


@pytest.mark.parametrize("launcher,exchange", [("torchrun", "auto"), ("self", "auto"), ("torchrun", "gloo")])
def test_bench_two_ranks_strong_scaling_branch(launcher, exchange):
    """bench.py's N > 1 path end to end, with gloo collectives so two ranks can
    share the one GPU of the test box -- as the driver's scaling run launches
    it (torch.distributed.run, one process per rank), and as a bare
    `bench.py --gpus 2`, which starts that launcher itself as a child process:
    the line carries n_gpus 2 and the strong-scaling fields (t1_ms_per_step,
    strong_efficiency, parallelism strong2) and every field of the timed
    region came back whole and was checked (fields_checked == steps).  The
    per-field sum runs in shared memory (auto: both ranks on this node) and,
    in the last case, over the process group's collective."""
    import subprocess
    import sys
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
            "--no-cpu-baseline", "--dist-backend", "gloo", "--exchange-backend", exchange]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                         env=dict(env, OMP_NUM_THREADS="4"))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints the one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "strong2"
    assert line["config"]["dist_backend"] == "gloo"
    assert line["config"]["exchange_backend"] == ("shm" if exchange == "auto" else exchange)
    assert line["config"]["exchange_lag"] == 2
    assert line["fields_checked"] == 6
    assert line["t1_ms_per_step"] > 0 and 0 < line["strong_efficiency"] < 2
    assert line["value"] > 0 and line["roofline"]["numbers_per_launch"] == 5 * 10 ** 8
    assert line["detailed_numbers_per_sec"] > 0 and line["niceonly_numbers_per_sec"] > 0
