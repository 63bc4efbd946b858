"""Generate the committed golden fixtures for restic CDC + SHA-256 blob IDs.

Run from the repo root:  python tests/golden/make_golden.py [--big]

Outputs come from oracle/cdc_ref.py (closed-form fingerprint restatement +
hashlib SHA-256), i.e. NOT from the C oracle the tests check, so every fixture
is a cross-implementation check.  Inputs are described by generator specs
(synthetic splitmix64 stream, zeros, zero runs) so the files stay small:
a fixture is data -- inputs and expected outputs.

Pinned by upstream: the `zeros_4min` case restates the zero-data known answer
of github.com/restic/chunker@v0.4.0 chunker_test.go (4 x MinSize zero bytes
-> four MinSize chunks, Cut 0, SHA-256 07854d2f...).  Everything else is
"parity partially pinned" (DESIGN.md section 5).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import cdc_ref as P  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MIN, MAX = P.MIN_SIZE, P.MAX_SIZE


def make_input(spec: dict) -> np.ndarray:
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
        # a period-`period` pattern: candidates repeat with the period
        base = P.synth(spec["seed"], 0, spec["period"])
        reps = -(-spec["len"] // spec["period"])
        return np.tile(base, reps)[: spec["len"]].copy()
    raise ValueError(kind)


def find_pol(seed: int) -> int:
    """A deterministic random irreducible degree-53 polynomial (restic init draws one)."""
    rng = np.random.default_rng(seed)
    while True:
        p = int(rng.integers(0, 1 << 53, dtype=np.uint64)) | (1 << 53) | 1
        if P.pol_irreducible(p):
            return p


def case(name, spec, pol=P.TEST_POL, mn=MIN, mx=MAX, ab=P.AVG_BITS, note=""):
    data = make_input(spec)
    chunks = P.chunk(data, pol, mn, mx, ab)
    doc = {
        "name": name,
        "note": note,
        "input": spec,
        "params": {"pol": hex(pol), "min": mn, "max": mx, "avg_bits": ab},
        "generator": "tests/golden/make_golden.py (oracle/cdc_ref.py + hashlib)",
        "chunks": [[s, l, hex(c), i] for (s, l, c, i) in chunks],
    }
    with open(os.path.join(OUT, f"cdc_{name}.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(name, len(chunks), "chunks", flush=True)


def main(big: bool):
    case("zeros_4min", {"kind": "zeros", "len": 4 * MIN},
         note="upstream chunker_test.go zero-data known answer")
    case("synth1_8m", {"kind": "synth", "seed": 1, "len": 8 << 20})
    case("synth1_64m", {"kind": "synth", "seed": 1, "len": 64 << 20})
    case("synth7_off_16m", {"kind": "synth", "seed": 7, "offset": 12345, "len": (16 << 20) + 777})
    case("small_params_forced", {"kind": "synth", "seed": 2, "len": 3 << 20},
         mn=1024, mx=2048, ab=14, note="max close to min: many forced MaxSize cuts")
    case("small_params", {"kind": "synth", "seed": 1, "len": 4 << 20},
         mn=4096, mx=16384, ab=12)
    case("avg16", {"kind": "synth", "seed": 9, "len": 8 << 20}, ab=16)
    case("zero_runs", {"kind": "synth_zero_runs", "seed": 5, "len": 16 << 20,
                       "zero_runs": [[2 << 20, 5 << 20], [9 << 20, (9 << 20) + 700000],
                                     [(12 << 20) + 3, (12 << 20) + 70]]},
         note="dense candidates inside zero runs")
    case("repeat_period", {"kind": "synth_repeat", "seed": 11, "period": 4099, "len": 6 << 20},
         mn=2048, mx=65536, ab=8, note="periodic data")
    case("pol_random", {"kind": "synth", "seed": 3, "len": 8 << 20}, pol=find_pol(2024),
         note="random irreducible degree-53 polynomial (restic init style)")
    for n in [0, 1, 63, 64, 100, MIN - 64, MIN - 63, MIN - 10, MIN - 1, MIN, MIN + 1,
              MIN + 4097, MAX - 1, MAX, MAX + 1]:
        case(f"eof_{n}", {"kind": "synth", "seed": 3, "len": n},
             note="EOF Cut semantics for short/boundary lengths")
    if big:
        case("synth1_1g", {"kind": "synth", "seed": 1, "len": 1 << 30},
             note="config C1: 1 GiB synthetic, default parameters")


if __name__ == "__main__":
    main("--big" in sys.argv)
