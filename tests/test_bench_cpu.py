"""bench.py's host logic on the CPU: the roofline names its binding resource (_finalize_roofline,
VERDICT r05 item 3) and flags any fraction above 1; no GPU needed."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _line(traffic=None, valu=None, step_ratio=0.9):
    r = {"bound": "hbm", "achieved": 0.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.0,
         "effective_launch_ms": 0.7, "avg_launch_ms": 1.2, "segments_per_launch": 23.6e6,
         "algorithmic_bytes_per_launch": 184 * 23.6e6, "kernel_min_bytes_per_launch": 64 * 23.6e6,
         "step_model_ratio": step_ratio}
    if traffic is not None:
        r["traffic"] = traffic
        r["traffic_per_segment"] = traffic / 23.6e6
    if valu is not None:
        r["valu_issue"] = {"instructions_per_launch": valu, "frac": 0.0}
    return r


def test_issue_bound_reports_valu_issue():
    import bench
    r = _line(traffic=67 * 23.6e6, valu=19.3 * 23.6e6, step_ratio=1.08)
    bench._finalize_roofline(r)
    want = 19.3 * 23.6e6 / 0.7e-3 / bench.VALU_PEAK
    assert r["bound"] == "issue" and r["unit"] == "wave64 VALU instr/s"
    assert r["frac"] == pytest.approx(want) and r["peak"] == bench.VALU_PEAK
    h = r["hbm"]
    assert h["model_184B"]["frac"] == pytest.approx(184 * 23.6e6 / 0.7e-3 / 1e9 / 8000.0)
    assert h["kernel_min"]["frac"] == pytest.approx(64 * 23.6e6 / 0.7e-3 / 1e9 / 8000.0)
    assert h["counter_traffic"]["frac"] == pytest.approx(67 * 23.6e6 / 0.7e-3 / 1e9 / 8000.0)
    assert r["fractions_above_1"] == []
    assert list(r["model_ratios_above_1"]) == ["step_model_ratio"]


def test_hbm_bound_when_traffic_reaches_half_the_peak():
    import bench
    traffic = 0.6 * 8000e9 * 0.7e-3
    r = _line(traffic=traffic, valu=5e8)
    bench._finalize_roofline(r)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert r["frac"] == pytest.approx(0.6)


def test_without_counters_the_model_is_labelled():
    import bench
    r = _line()
    bench._finalize_roofline(r)
    assert r["bound"] == "hbm" and "model" in r["definition"]
    assert r["frac"] == pytest.approx(184 * 23.6e6 / 0.7e-3 / 1e9 / 8000.0)
    assert r["model_ratios_above_1"] == {}


def test_fractions_above_one_are_listed():
    import bench
    r = _line(traffic=1e9, valu=1e9)
    r["effective_launch_ms"] = 0.01   # absurdly short: every fraction above 1
    bench._finalize_roofline(r)
    assert "frac" in r["fractions_above_1"] and "hbm.model_184B.frac" in r["fractions_above_1"]
