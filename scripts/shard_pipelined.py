"""Strong-scaling projection from one GPU, pipelined: rank r's whole step of
an N-way bench.py run -- its detailed shard of the b40 1e9 field and its
dealt niceonly chunks, through dist.FieldPipeline exactly as at N ranks --
timed for every r of N = 2, 4, 8 on this one GPU, one rank after the other.
The exchange is a loopback (this rank's vector comes back as the sum), so
what is left out is only the cross-rank part of the exchange (DESIGN.md
section 5 measures the shared-memory exchange's own cost under torchrun).
T_N = the slowest rank's ms per step; T_1 = the whole field the same way;
efficiency = T_1 / (N x T_N).

    python3 scripts/shard_pipelined.py [--steps 200 --warmup 20] [--mode both|detailed|niceonly]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nice_amd as N  # noqa: E402
from nice_amd import dist as D  # noqa: E402
from nice_amd.benchmark import BenchmarkMode as BM, get_benchmark_field  # noqa: E402


class _Rank:
    """The slice of torch.distributed FieldPipeline and finish_both use, for
    rank r of `world` with nothing on the other ranks."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def get_rank(self, group=None):
        return self.rank

    def get_world_size(self, group=None):
        return self.world

    def get_backend(self, group=None):
        return "gloo"

    def all_gather(self, parts, buf, group=None):
        for i, p in enumerate(parts):
            p.copy_(buf if i == self.rank else 0 * buf)


class _Loopback:
    def __init__(self, dist):
        self.dist, self.group, self.pending = dist, None, []

    def submit(self, vals, payload):
        self.pending.append((list(vals), payload))
        return self.pending.pop(0) if len(self.pending) > 1 else None

    def drain_all(self):
        out, self.pending = self.pending, []
        return out


class _Skip:
    """A context that runs nothing (one mode alone)."""

    def detailed_submit(self, *a, **k):
        return None

    def niceonly_submit(self, *a, **k):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mode", choices=["both", "detailed", "niceonly"], default="both")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--field-size", type=float, default=0, help="the field's first numbers only (0 = all 1e9)")
    ap.add_argument("--base", type=int, default=40,
                    help="another base: its range's first --field-size numbers (default 1e9)")
    ap.add_argument("--force-L", type=int, default=0,
                    help="sibling-lane stride forced through nice_debug_force_sib_stride (0 = the pick)")
    a = ap.parse_args()
    f = get_benchmark_field(BM.EXTRA_LARGE)
    if a.base != f.base:
        import types
        br = N.get_base_range_u128(a.base)
        f = types.SimpleNamespace(range_start=br.range_start, range_end=br.range_start + 10 ** 9, base=a.base)
    field = N.FieldSize(f.range_start, f.range_start + int(a.field_size) if a.field_size else f.range_end)
    ctx = N.GpuContext(0)
    if a.force_L:
        assert N._lib.lib().nice_debug_force_sib_stride(a.force_L) == 0
    t1 = None
    worlds = [int(w) for w in a.worlds.split(",")]
    det = ctx if a.mode != "niceonly" else _Skip()
    nic = ctx if a.mode != "detailed" else _Skip()
    for world in worlds:
        per, strides = [], []
        for r in range(world):
            d = _Rank(r, world)
            pipe = D.FieldPipeline(det, nic, d, exchange=_Loopback(d))
            for _ in range(a.warmup):
                pipe.step(field, f.base)
            pipe.drain()
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                pipe.step(field, f.base)
            pipe.drain()
            ctx.synchronize()
            per.append((time.perf_counter() - t0) / a.steps * 1e3)
            strides.append(ctx.kernel_stats().sib_stride)
        tn = max(per)
        t1 = tn if world == 1 else t1
        st = ctx.kernel_stats()
        print(json.dumps({"mode": a.mode, "base": f.base, "field_size": field.range_end - field.range_start,
                          "sib_lanes": st.sib_lanes, "sib_stride": st.sib_stride,
                          "force_L": a.force_L, "world": world, "max_rank_ms_per_step": round(tn, 5),
                          "min_rank_ms_per_step": round(min(per), 5),
                          "projected_efficiency": round(t1 / (world * tn), 4) if t1 else None,
                          "ranks_ms_per_step": [round(x, 5) for x in per], "ranks_sib_stride": strides}),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
