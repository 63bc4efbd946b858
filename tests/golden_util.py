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


def rsync_pair(spec: dict):
    """(basis, source) byte arrays for an rsync fixture spec (make_golden_rsync.py)."""
    from oracle import cdc_ref as P
    from oracle import rsync_ref as R
    from tests import oracle_lib as O
    kind = spec["kind"]
    n = spec["basis_len"]
    if kind == "dup_blocks":
        unit = P.synth(spec["seed"], 0, spec["period"])
        basis = np.tile(unit, -(-n // spec["period"]))[:n].copy()
    else:
        basis = P.synth(spec["seed"], 0, n)
    if kind in ("mutate", "dup_blocks"):
        bl = O.rsync_sizes(n, spec.get("block_size", 0))[0]
        src = R.mutate(basis, bl, spec["edit_seed"], spec["frac"])
        if spec.get("shift"):
            src = np.concatenate([P.synth(99, 0, spec["shift"]), src])
    elif kind == "identical":
        src = basis.copy()
    elif kind == "disjoint":
        src = P.synth(spec["seed"] + 1000, 0, spec["src_len"])
    elif kind == "prefix":
        src = basis[: spec["src_len"]].copy()
    else:
        raise ValueError(kind)
    if "src_len" in spec and kind == "mutate":
        src = src[: spec["src_len"]]
    return basis, src


def params(doc):
    p = doc["params"]
    return int(p["pol"], 16), int(p["min"]), int(p["max"]), int(p["avg_bits"])


def expected(doc):
    return [(int(s), int(l), int(c, 16), i) for s, l, c, i in doc["chunks"]]
