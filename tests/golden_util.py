"""Load the committed golden fixtures (tests/golden/*.json) and rebuild their inputs."""
from __future__ import annotations

import glob
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def fixtures(pattern: str = "cdc_*.json"):
    return sorted(glob.glob(os.path.join(GOLDEN, pattern)))


def load(path: str):
    with open(path) as f:
        return json.load(f)


def make_input(spec: dict) -> np.ndarray:
    from oracle import cdc_ref as P
    kind = spec["kind"]
    if kind == "zeros":
        return np.zeros(spec["len"], np.uint8)
    if kind == "synth":
        return P.synth(spec["seed"], spec.get("offset", 0), spec["len"])
    if kind == "synth_zero_runs":
        d = P.synth(spec["seed"], 0, spec["len"])
        for a, b in spec["zero_runs"]:
            d[a:b] = 0
        return d
    if kind == "synth_repeat":
        base = P.synth(spec["seed"], 0, spec["period"])
        reps = -(-spec["len"] // spec["period"])
        return np.tile(base, reps)[: spec["len"]].copy()
    raise ValueError(kind)


def params(doc):
    p = doc["params"]
    return int(p["pol"], 16), int(p["min"]), int(p["max"]), int(p["avg_bits"])


def expected(doc):
    return [(int(s), int(l), int(c, 16), i) for s, l, c, i in doc["chunks"]]
