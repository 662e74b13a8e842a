"""The single-threaded JS restatement (tools/js_restatement/sift_restated.mjs,
bench.py's `cpu_baseline_js`) against the golden fixtures captured from the
reference itself: it must compute the reference's lists before its time can
stand for the reference's algorithm on one core."""
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from golden_util import Golden, case_names

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "js_restatement", "sift_restated.mjs")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def run_restated(img, O, S, lists=True, blur=(0.8, 0.5, 0.5)):
    H, W = img.shape
    with tempfile.TemporaryDirectory() as td:
        np.ascontiguousarray(img, dtype="<f4").tofile(os.path.join(td, "img.f32"))
        out = os.path.join(td, "o.json")
        args = [NODE, SCRIPT, os.path.join(td, "img.f32"), str(W), str(H), str(O), str(S), out]
        args += ["--lists" if lists else "-"] + [repr(float(b)) for b in blur]
        r = subprocess.run(args, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        with open(out) as f:
            return json.load(f)


@pytest.mark.parametrize("name", case_names())
def test_restatement_matches_reference_goldens(name):
    g = Golden(name)
    p = g.params
    out = run_restated(g.img, p["num_octaves"], p["scales_per_octave"],
                       blur=(p["min_blur"], p["assumed_blur"], p["min_interpixel_distance"]))
    cand = np.array(out["lists"]["candidates"], dtype=np.float64).reshape(-1, 5)
    ref = np.asarray(g.candidates, dtype=np.float64).reshape(-1, 5)
    assert cand.shape == ref.shape
    np.testing.assert_array_equal(cand[:, :4], ref[:, :4])
    np.testing.assert_allclose(cand[:, 4], ref[:, 4], rtol=0, atol=1e-12)
    kp = np.array(out["lists"]["keypoints"], dtype=np.float64).reshape(-1, 8)
    ref_kp = np.asarray(g.refined, dtype=np.float64).reshape(-1, 8)
    assert kp.shape == ref_kp.shape
    np.testing.assert_array_equal(kp[:, :4], ref_kp[:, :4])
    np.testing.assert_allclose(kp[:, 4:], ref_kp[:, 4:], rtol=0, atol=1e-9)
    assert out["lowContrast"] == int(np.asarray(g.z["low_contrast_counts"]).sum())
    assert out["singular"] == 0
