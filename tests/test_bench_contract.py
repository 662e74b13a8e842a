"""bench.py's accounting on the CPU (no GPU): the algorithmic bytes it
prices the roofline with match BASELINE.md's table, the per-octave split sums
to the pass, the metric label follows BASELINE.json for the metric's
configuration, and the host-core parsing tolerates OpenMP list values."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("W,H,O,gb", [(1920, 1080, 4, 0.669), (3840, 2160, 4, 2.677), (7680, 4320, 6, 10.75)])
def test_alg_bytes_match_baseline_table(W, H, O, gb):
    """BASELINE.md 'MI355X targets': B_alg = 4WH + sum 4P(S+3) + sum 4P(S+2)."""
    b = _bench()
    assert abs(b.alg_bytes(W, H, O, 5, False) / 1e9 - gb) < 0.006


def test_octave_bytes_sum_to_pass():
    b = _bench()
    for skip in (False, True):
        assert sum(b.octave_bytes(3840, 2160, 4, 5, skip)) == b.alg_bytes(3840, 2160, 4, 5, skip)
    assert b.oct0_bytes(3840, 2160, 5, False) == 2023833600


def test_metric_label_is_baselines_for_its_configuration():
    b = _bench()
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    assert b.metric_name(3840, 2160, 4, 5) == metric
    assert "1920x1080" in b.metric_name(1920, 1080, 4, 5, batch=8)


def test_host_cores_parses_openmp_lists(monkeypatch):
    b = _bench()
    monkeypatch.setenv("OMP_NUM_THREADS", "8,2")
    assert 1 <= b.host_cores() <= 8
    monkeypatch.setenv("OMP_NUM_THREADS", "junk")
    assert b.host_cores() >= 1
