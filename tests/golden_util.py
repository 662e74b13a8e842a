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
