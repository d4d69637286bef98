"""The client mirror (nice_amd/client.py, client/src/main.rs): argument
surface, compile_results / validate_results on synthetic results (CPU), and a
benchmark run end to end through the GPU library (gpu)."""
import json

import pytest

from nice_amd import client as C
from nice_amd.types import (DataToClient, FieldResults, NiceNumberSimple, SearchMode,
                            UniquesDistributionSimple)


def test_parse_args_env_and_flags(monkeypatch):
    monkeypatch.setenv("NICE_MODE", "niceonly")
    monkeypatch.setenv("NICE_THREADS", "7")
    a = C.parse_args(["--benchmark", "default", "--gpu-device", "0,1"])
    assert a.mode == "niceonly" and a.threads == 7 and a.benchmark == "default"
    assert C._devices(a.gpu_device) == [0, 1]
    a = C.parse_args(["detailed", "--base", "40", "--range", "10", "20"])
    assert a.mode == "detailed" and a.base == 40 and a.range == [10, 20]


def _results():
    d1 = FieldResults(distribution=[UniquesDistributionSimple(1, 2), UniquesDistributionSimple(2, 5)],
                      nice_numbers=[NiceNumberSimple(69, 10)])
    d2 = FieldResults(distribution=[UniquesDistributionSimple(2, 1), UniquesDistributionSimple(3, 4)],
                      nice_numbers=[])
    return [d1, d2]


def test_compile_results_merges_chunks():
    claim = DataToClient(7, 10, 47, 100, 53)
    sub = C.compile_results(_results(), claim, "alice", SearchMode.DETAILED)
    assert sub.claim_id == 7 and sub.username == "alice"
    assert [(d.num_uniques, d.count) for d in sub.unique_distribution] == [(1, 2), (2, 6), (3, 4)]
    assert [(n.number, n.num_uniques) for n in sub.nice_numbers] == [(69, 10)]
    sub = C.compile_results(_results(), claim, "alice", SearchMode.NICEONLY)
    assert sub.unique_distribution is None


def test_validate_results_detects_mismatch():
    claim = DataToClient(0, 10, 47, 100, 53)
    sub = C.compile_results(_results(), claim, "u", SearchMode.DETAILED)
    canon = {"nice_numbers": [{"number": "69", "num_uniques": 10}],
             "unique_distribution": [{"num_uniques": 1, "count": 2}, {"num_uniques": 2, "count": 6},
                                     {"num_uniques": 3, "count": 4}]}
    assert C.validate_results(sub, canon, SearchMode.DETAILED)
    canon["unique_distribution"][0]["count"] = 3
    assert not C.validate_results(sub, canon, SearchMode.DETAILED)
    assert C.validate_results(sub, canon, SearchMode.NICEONLY)  # distribution not compared
    canon["nice_numbers"] = []
    assert not C.validate_results(sub, canon, SearchMode.NICEONLY)


@pytest.mark.gpu
def test_client_benchmark_base_ten_validates(tmp_path, capsys):
    # base-ten (benchmark.rs:40-76): [47, 100) must report (69, 10); the
    # distribution is the reference's process_detailed_b10 vector.
    from oracle import oracle as O
    want = O.process_range_detailed(47, 100, 10)
    canon = {"nice_numbers": [{"number": str(n), "num_uniques": u} for n, u in want.nice_numbers],
             "unique_distribution": [{"num_uniques": u, "count": c} for u, c in want.distribution]}
    p = tmp_path / "canon.json"
    p.write_text(json.dumps(canon))
    assert C.main(["detailed", "--benchmark", "base-ten", "--gpu", "--validate", str(p)]) == 0
    assert "Validation passed" in capsys.readouterr().out
    assert C.main(["niceonly", "--benchmark", "base-ten", "--gpu", "--validate", str(p)]) == 0
    canon["nice_numbers"] = []
    p.write_text(json.dumps(canon))
    assert C.main(["niceonly", "--benchmark", "base-ten", "--gpu", "--validate", str(p)]) == 1


def test_client_cpu_mode_base_ten(tmp_path, capsys):
    """Without --gpu the client runs the reference's CPU mode (main.rs:154-207):
    base-ten lists (69, 10) with the process_detailed_b10 distribution, no
    GPU touched (this runs in the CPU suite)."""
    from oracle import oracle as O
    want = O.process_range_detailed(47, 100, 10)
    canon = {"nice_numbers": [{"number": str(n), "num_uniques": u} for n, u in want.nice_numbers],
             "unique_distribution": [{"num_uniques": u, "count": c} for u, c in want.distribution]}
    assert want.nice_numbers == [(69, 10)]
    p = tmp_path / "canon.json"
    p.write_text(json.dumps(canon))
    assert C.main(["--benchmark", "base-ten", "--validate", str(p)]) == 0
    assert "Validation passed" in capsys.readouterr().out
    assert C.main(["niceonly", "--benchmark", "base-ten", "--validate", str(p)]) == 0
    canon["nice_numbers"] = []
    p.write_text(json.dumps(canon))
    assert C.main(["niceonly", "--benchmark", "base-ten", "--validate", str(p)]) == 1


def test_client_cpu_mode_chunks_merge_like_one_range():
    """CPU mode cuts the field into client chunks and merges them in order:
    a 2.5e6 b40 field (three 1e6 chunks, the last ragged) on 3 workers equals
    the oracle over the whole range; niceonly below b40's range lists the
    265 numbers of [1, 1e5) (get_is_nice has no digit-count test)."""
    from oracle import oracle as O
    s = O.base_range(40)[0]
    claim = DataToClient(0, 40, s, s + 2_500_000, 2_500_000)
    args = C.parse_args(["--threads", "3"])
    res = C.process_field_sync(claim, SearchMode.DETAILED, args)
    assert len(res) == 3
    sub = C.compile_results(res, claim, "u", SearchMode.DETAILED)
    want = O.process_range_detailed(s, s + 2_500_000, 40)
    assert [(d.num_uniques, d.count) for d in sub.unique_distribution if d.count] == \
        [x for x in want.distribution if x[1]]
    assert [(n.number, n.num_uniques) for n in sub.nice_numbers] == want.nice_numbers
    claim = DataToClient(0, 40, 1, 10 ** 5, 10 ** 5 - 1)
    res = C.process_field_sync(claim, SearchMode.NICEONLY, args)
    sub = C.compile_results(res, claim, "u", SearchMode.NICEONLY)
    want, _ = O.process_range_niceonly(1, 10 ** 5, 40)
    assert [(n.number, n.num_uniques) for n in sub.nice_numbers] == want.nice_numbers
    assert len(want.nice_numbers) == 265
