"""Helpers to load the golden fixtures (tests/golden, made by make_golden.py
from the reference itself) and regenerate their inputs."""
import glob
import hashlib
import json
import os

import numpy as np

from sift_amd.synth import blob_image, constant_image

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.json")))


class Golden:
    def __init__(self, name):
        with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.name = name
        self.params = self.meta["params"]
        sp = self.meta["input"]
        if sp["kind"] == "blob":
            self.img = blob_image(sp["width"], sp["height"], seed=sp["seed"], noise=sp["noise"])
        else:
            self.img = constant_image(sp["width"], sp["height"], sp["value"])
        digest = hashlib.sha256(self.img.tobytes()).hexdigest()
        assert digest == self.meta["input_sha256"], "regenerated input differs from the fixture's"

    @property
    def candidates(self):
        return self.z["candidates"]  # (N,5): octave, scale, x, y, value

    @property
    def refined(self):
        return self.z["refined"]  # (M,8)


BIG_DIR = os.path.join(GOLDEN_DIR, "big")


def big_case_names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(BIG_DIR, "*.json")))


class BigGolden:
    """Headline-scale fixtures (make_golden_big.py): the reference's own
    candidate lists, low-contrast counts and keypoints at BASELINE cfg 2 / 3,
    stored compactly (see that script)."""

    def __init__(self, name):
        with open(os.path.join(BIG_DIR, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(BIG_DIR, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.name = name
        self.params = self.meta["params"]
        sp = self.meta["input"]
        self.img = blob_image(sp["width"], sp["height"], seed=sp["seed"], noise=sp["noise"])
        digest = hashlib.sha256(self.img.tobytes()).hexdigest()
        assert digest == self.meta["input_sha256"], "regenerated input differs from the fixture's"

    @property
    def candidates(self):
        """(N,5) octave, scale, x, y, value (value rounded to fp32)."""
        z = self.z
        return np.concatenate([z["cand_os"].astype(np.float64), z["cand_xy"].astype(np.float64),
                               z["cand_value"].astype(np.float64)[:, None]], axis=1)

    @property
    def refined(self):
        """(M,8) in the reference's record order; x, y rebuilt from the stored
        sub-pixel offsets (fp32, |error| < 3e-7 delta)."""
        z = self.z
        o = z["kp_os"][:, 0].astype(np.float64)
        lx, ly = z["kp_xy"][:, 0].astype(np.float64), z["kp_xy"][:, 1].astype(np.float64)
        delta = 2.0 ** (o - 1)
        return np.stack([o, z["kp_os"][:, 1].astype(np.float64), lx, ly, z["kp_sigma"].astype(np.float64),
                         delta * lx + z["kp_dx"], delta * ly + z["kp_dy"], z["kp_value"].astype(np.float64)],
                        axis=1)

    @property
    def low_contrast_counts(self):
        return self.z["low_contrast_counts"]
