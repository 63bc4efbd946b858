"""Generate golden fixtures for rsync 3.2.3 delta matching (R1-R6).

Run from the repo root:  python tests/golden/make_golden_rsync.py

Outputs come from oracle/rsync_ref.py (closed-form weak sums + greedy walk,
xxhash / hashlib strong sums) and every case is cross-checked against the C
restatement (oracle/rsync_ref.c, the rolling hash_search loop) before it is
written.  Inputs are generator specs (synthetic basis + seeded edits), so the
files hold data: parameters, signature table and match list.

Parity note: no rsync binary or source is available
offline; the weak/strong checksums are pinned by the system libxxhash /
hashlib and by closed-form identities, the match list by two independent
restatements.  "Parity partially pinned."
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import cdc_ref as P  # noqa: E402
from oracle import rsync_ref as R  # noqa: E402
from tests import oracle_lib as O  # noqa: E402
from tests.golden_util import rsync_pair as make_pair  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED5EED


def case(name, spec, csum_type=R.CSUM_XXH3_128, seed=SEED, note=""):
    basis, src = make_pair(spec)
    bs = spec.get("block_size", 0)
    blength, s2length, count, remainder = R.sum_sizes(len(basis), bs)
    assert (blength, s2length, count, remainder) == O.rsync_sizes(len(basis), bs)
    s1, s2 = R.signatures(basis, blength, s2length, csum_type, seed)
    c1, c2 = O.rsync_signatures(basis, blength, s2length, csum_type, seed)
    assert list(map(int, c1)) == s1 and [bytes(x) for x in c2] == s2, name
    m = R.match(src, s1, s2, blength, remainder, s2length, csum_type, seed)
    cm, _ = O.rsync_match(src, c1, c2, blength, remainder, csum_type, seed)
    assert m == cm, name
    doc = {
        "name": name, "note": note, "input": spec,
        "params": {"csum_type": csum_type, "seed": seed, "block_size": bs},
        "sizes": {"blength": blength, "s2length": s2length, "count": count,
                  "remainder": remainder, "source_len": int(len(src))},
        "generator": "tests/golden/make_golden_rsync.py (oracle/rsync_ref.py, checked vs rsync_ref.c)",
        "sum1": [int(x) for x in s1], "sum2": [x.hex() for x in s2],
        "matches": [[int(o), int(i)] for o, i in m],
    }
    with open(os.path.join(OUT, f"rsync_{name}.json"), "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(name, "blocks", count, "blength", blength, "s2", s2length, "matches", len(m), flush=True)


def main():
    c4 = {"kind": "mutate", "seed": 4, "edit_seed": 5, "frac": 0.10}
    case("c4_4m_xxh128", dict(c4, basis_len=4 << 20), note="C4 shape scaled: 10% blocks edited")
    case("c4_4m_md5", dict(c4, basis_len=4 << 20), csum_type=R.CSUM_MD5)
    case("c4_3m_xxh64", dict(c4, basis_len=3 << 20, frac=0.2), csum_type=R.CSUM_XXH64)
    case("c4_3m_xxh3", dict(c4, basis_len=3 << 20, frac=0.2), csum_type=R.CSUM_XXH3_64)
    case("bs4096_shift", dict(c4, basis_len=6 << 20, block_size=4096, shift=777),
         note="--block-size override, whole source shifted by an insertion")
    case("heavy_edit", dict(c4, basis_len=2 << 20, frac=0.6, edit_seed=8))
    case("tail_partial", dict(c4, basis_len=(1 << 20) + 12345, frac=0.05),
         note="last block shorter than blength")
    case("identical", {"kind": "identical", "seed": 6, "basis_len": 3 << 20})
    case("disjoint", {"kind": "disjoint", "seed": 7, "basis_len": 1 << 20, "src_len": 1 << 20})
    case("dup_blocks", {"kind": "dup_blocks", "seed": 9, "period": 700, "basis_len": 70000,
                        "edit_seed": 3, "frac": 0.2}, note="identical blocks: chains + want_i")
    case("dup_blocks_md5_seed0", {"kind": "dup_blocks", "seed": 9, "period": 1400,
                                  "basis_len": 140000, "edit_seed": 4, "frac": 0.3,
                                  "block_size": 700}, csum_type=R.CSUM_MD5, seed=0)
    case("tiny", {"kind": "mutate", "seed": 10, "edit_seed": 1, "frac": 0.0, "basis_len": 100})
    case("src_shorter_than_block", {"kind": "prefix", "seed": 11, "basis_len": 5000,
                                    "src_len": 300})
    case("empty_source", {"kind": "prefix", "seed": 12, "basis_len": 5000, "src_len": 0})
    case("empty_basis", {"kind": "disjoint", "seed": 13, "basis_len": 0, "src_len": 3000})


if __name__ == "__main__":
    main()
