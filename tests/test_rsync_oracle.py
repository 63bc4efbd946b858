"""rsync delta-matcher oracle (R1-R6) against the committed golden fixtures (CPU only).

Both restatements -- oracle/rsync_ref.c (rolling hash_search loop) and
oracle/rsync_ref.py (closed-form weak sums + jump walk) -- must reproduce every
fixture; the strong sums are pinned by the xxhash package and hashlib.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import golden_util as G
from tests import oracle_lib as O

FIX = G.fixtures("rsync_*.json")


def fixture_case(path):
    doc = G.load(path)
    basis, src = G.rsync_pair(doc["input"])
    p, z = doc["params"], doc["sizes"]
    sum1 = np.array(doc["sum1"], np.uint32)
    sum2 = [bytes.fromhex(h) for h in doc["sum2"]]
    return doc, basis, src, p, z, sum1, sum2


def test_fixture_set_present():
    names = {os.path.basename(p) for p in FIX}
    assert len(FIX) >= 15
    assert {"rsync_c4_4m_xxh128.json", "rsync_dup_blocks.json", "rsync_empty_basis.json"} <= names


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_c_oracle_vs_golden(path):
    doc, basis, src, p, z, sum1, sum2 = fixture_case(path)
    assert len(src) == z["source_len"]
    assert O.rsync_sizes(len(basis), p["block_size"]) == (z["blength"], z["s2length"], z["count"],
                                                          z["remainder"])
    c1, c2 = O.rsync_signatures(basis, z["blength"], z["s2length"], p["csum_type"], p["seed"])
    assert (c1 == sum1).all() and [bytes(x) for x in c2] == sum2
    s2 = np.frombuffer(b"".join(sum2), np.uint8).reshape(len(sum2), z["s2length"]) if sum2 else \
        np.zeros((0, z["s2length"]), np.uint8)
    m, _ = O.rsync_match(src, sum1, s2, z["blength"], z["remainder"], p["csum_type"], p["seed"])
    assert m == [tuple(x) for x in doc["matches"]]


@pytest.mark.parametrize("path", [p for p in FIX if "c4_" not in p and "shift" not in p],
                         ids=os.path.basename)
def test_python_oracle_vs_golden(path):
    doc, basis, src, p, z, sum1, sum2 = fixture_case(path)
    s1, s2 = R.signatures(basis, z["blength"], z["s2length"], p["csum_type"], p["seed"])
    assert s1 == list(map(int, sum1)) and s2 == sum2
    m = R.match(src, s1, s2, z["blength"], z["remainder"], z["s2length"], p["csum_type"], p["seed"])
    assert m == [tuple(x) for x in doc["matches"]]


def test_matches_are_consistent():
    """Every golden match is a real copy: source bytes == basis block, and
    matches never overlap (the greedy walk jumps a whole block)."""
    for path in FIX:
        doc, basis, src, p, z, *_ = fixture_case(path)
        bl, count, rem = z["blength"], z["count"], z["remainder"]
        prev_end = 0
        for o, i in doc["matches"]:
            n = rem if (i == count - 1 and rem) else bl
            assert o >= prev_end
            assert (src[o:o + n] == basis[i * bl:i * bl + n]).all(), (path, o, i)
            prev_end = o + n


def test_checksum2_forms():
    import xxhash
    buf = O.synth(3, 0, 5000).tobytes()
    for n in (0, 1, 3, 4, 8, 9, 16, 17, 128, 129, 240, 241, 700, 1024, 1025, 5000):
        b = buf[:n]
        assert R.checksum2(b, R.CSUM_XXH3_128, 77) == \
            xxhash.xxh3_128_intdigest(b, seed=77).to_bytes(16, "little")
        assert R.checksum2(b, R.CSUM_MD5, 0) == hashlib.md5(b).digest()
        assert R.checksum2(b, R.CSUM_MD5, 5) == hashlib.md5(b"\x05\0\0\0" + b).digest()


def test_sum_sizes_table():
    """sum_sizes_sqroot at the sizes SURVEY 8(c) lists (C and Python agree)."""
    for n, bs in [(0, 0), (1, 0), (700 * 700, 0), (700 * 700 + 1, 0), (1 << 20, 0), (1 << 30, 0),
                  (1 << 38, 0), (1 << 40, 0), (12345, 4096), (10, 1 << 17)]:
        assert O.rsync_sizes(n, bs) == R.sum_sizes(n, bs), n
    assert R.sum_sizes(1 << 38) == (131072, 5, 2097152, 0)
