"""bench.py reports counter figures (roofline.hw, hw_bound, frac_hw, traffic)
only from PMC passes of the library it loads: pmc_bench()
returns "current" when the committed summary's lib_sha16 matches the loaded
library, "stale" (and no figures) when it does not, "missing" without a
summary.  CPU only: no device call."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _with_summary(tmp_path, monkeypatch, payload):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    if payload is not None:
        p = tmp_path / bench.PMC_BENCH_FILE
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps(payload))
    return bench.pmc_bench()


def test_current_summary_is_reported(tmp_path, monkeypatch):
    der = {"valu_busy": 0.95, "lds_busy": 0.9}
    d, src, status = _with_summary(tmp_path, monkeypatch, {"lib_sha16": bench.lib_sha16(), "derived": der})
    assert status == "current" and d == der and src == bench.PMC_BENCH_FILE


def test_stale_summary_is_withheld(tmp_path, monkeypatch):
    d, _, status = _with_summary(tmp_path, monkeypatch, {"lib_sha16": "0" * 16, "derived": {"valu_busy": 1}})
    assert d is None and status.startswith("stale")


def test_missing_summary(tmp_path, monkeypatch):
    d, _, status = _with_summary(tmp_path, monkeypatch, None)
    assert d is None and status == "missing"

