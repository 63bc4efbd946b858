"""tests/golden/full_configs.json (tests/golden/make_golden_full.py): the
full-size chunk / match list digests the bench lines check themselves against.
CPU: their internal consistency, and the smallest C2 prefix recomputed by the C
oracle here."""
import json
import os

import numpy as np
import pytest

from tests import oracle_lib as O
from tests.golden import make_golden_full as G

GiB = 1 << 30


@pytest.fixture(scope="module")
def gold():
    return json.load(open(G.OUT))


def test_c3_rank_splits_partition_the_stream(gold):
    """Per-rank C3 entries (bench.py --share R/8 in CDC mode): the ranks' chunk
    counts add up to the stream's, rank 0 enters at 0, every true entry lies
    within MaxSize of the rank's own_lo, and the split is volsync_amd.shard's."""
    from volsync_amd.shard import ShardSpec
    c3 = gold["cdc"]["3"]
    for total, ent in c3.items():
        total = int(total)
        ranks = ent.get("ranks")
        if not ranks:
            assert total == 128 * GiB
            continue
        W = total // (128 * GiB)
        assert len(ranks) == W
        assert sum(r["chunks"] for r in ranks) == ent["chunks"]
        assert ranks[0]["entry"] == 0
        for r in ranks:
            sp = ShardSpec.for_rank(total, W, r["rank"], G.MX)
            assert (sp.own_lo, sp.own_hi) == (r["own_lo"], r["own_hi"])
            assert sp.own_lo <= r["entry"] < sp.own_lo + G.MX
    # the non-final ranks of every split are the same chunks (rank r owns
    # [r, r+1) x 128 GiB whatever the world; the final rank ends in an EOF chunk)
    r8 = c3[str(1024 * GiB)]["ranks"]
    r4 = c3[str(512 * GiB)]["ranks"]
    for a, b in zip(r4[:3], r8[:3]):
        assert (a["entry"], a["chunks"], a["digest"]) == (b["entry"], b["chunks"], b["digest"])


def test_c2_prefix_counts_grow(gold):
    c2 = gold["cdc"]["2"]
    lens = sorted(int(k) for k in c2)
    counts = [c2[str(L)]["chunks"] for L in lens]
    assert lens[-1] == 64 * GiB and counts == sorted(counts)
    assert c2[str(64 * GiB)]["chunks"] == 43708


def test_c2_first_gib_recomputed(gold):
    """The 1 GiB C2 prefix's chunk list recomputed by the C oracle (cdc_ref.c,
    multi-threaded) matches the committed digest."""
    want = gold["cdc"]["2"][str(GiB)]
    s, ln, c, ids = O.cdc_synth_mt(2, GiB, G.POL, G.MN, G.MX, G.AVG, os.cpu_count() or 4)
    ends = s + ln
    k = int(np.searchsorted(ends, GiB, side="right"))
    rec = G.chunk_records(s[:k], ln[:k], c[:k], ids[:k])
    if k < len(s) and int(s[k]) < GiB:
        e = G.eof_chunk(2, int(s[k]), GiB)
        rec = np.concatenate([rec, G.chunk_records([e[0]], [e[1]], [e[2]],
                                                   np.frombuffer(e[3], np.uint8))])
    assert (len(rec), G.digest(rec)) == (want["chunks"], want["digest"])


def test_rsync_entries_consistent(gold):
    """C4 match-list goldens: the 8-rank split of 256 GiB adds up to the whole."""
    rs = gold["rsync"]
    ent = rs[str(256 * GiB)]
    per = ent["ranks"]["8"]
    assert sum(r["matches"] for r in per) == ent["matches"]
    assert sum(r["false_alarms"] for r in per) == ent["false_alarms"]
    assert per[0]["entry"] == [0, 0]
    for g in (8, 16, 64, 128, 256):
        e = rs[str(g * GiB)]
        assert e["dlen"] == g * GiB and len(e["digest"]) == 64 and len(e["file_sum"]) == 32


def test_c5_entry_matches_layout(gold):
    """The C5 golden (bench.py --mode smallfiles checks its line against it):
    its byte count and distinct-ID count follow from bench.c5_layout -- one
    distinct blob per distinct payload -- so the layout the digest was made
    from is the one the bench runs."""
    import bench
    g = gold["c5"]["1000000"]
    sizes, pick, psize, npay = bench.c5_layout(1_000_000, 0)
    assert g["bytes"] == int(sizes.sum()) and g["payloads"] == npay
    assert g["unique_ids"] == len(np.unique(pick))
    assert len(g["id_digest"]) == 64
