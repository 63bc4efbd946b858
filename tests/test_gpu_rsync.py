"""GPU parity tests of rsync delta matching (R1-R6) through the C ABI.

Bar: bit-exact sum1/sum2 signatures and match lists (offset, block index)
against the committed golden fixtures and the C restatement of hash_search
(oracle/rsync_ref.c) on seeded inputs; at larger sizes, properties (every
match is a byte-exact copy, matches tile without overlap, the unedited blocks
are found).
"""
import os

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import golden_util as G
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

FIX = G.fixtures("rsync_*.json")


def to_dev(arr: np.ndarray):
    import torch
    t = torch.empty(max(len(arr), 16), dtype=torch.uint8, device="cuda")
    if len(arr):
        t[: len(arr)].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t


def load_fixture(path):
    doc = G.load(path)
    basis, src = G.rsync_pair(doc["input"])
    return doc, basis, src


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_signatures_vs_golden(gpu, path):
    from volsync_amd import generate_sums
    doc, basis, _ = load_fixture(path)
    p, z = doc["params"], doc["sizes"]
    s = generate_sums(basis, p["csum_type"], p["seed"], p["block_size"])
    assert (s.blength, s.s2length, s.count, s.remainder) == \
        (z["blength"], z["s2length"], z["count"], z["remainder"])
    assert [int(x) for x in s.sum1] == doc["sum1"]
    assert [bytes(r).hex() for r in s.sum2] == doc["sum2"]


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_match_vs_golden(gpu, path):
    from volsync_amd import SumStruct, match_sums
    doc, _, src = load_fixture(path)
    p, z = doc["params"], doc["sizes"]
    s = SumStruct(flength=0, count=z["count"], blength=z["blength"], s2length=z["s2length"],
                  remainder=z["remainder"], sum1=np.array(doc["sum1"], np.uint32),
                  sum2=np.array([list(bytes.fromhex(h)) for h in doc["sum2"]], np.uint8).reshape(
                      z["count"], z["s2length"]))
    got = match_sums(src, s, p["csum_type"], p["seed"])
    assert got == [tuple(m) for m in doc["matches"]]


@pytest.mark.parametrize("csum_type,seed,n,frac,block_size", [
    (R.CSUM_XXH3_128, 0x5EED5EED, 48 << 20, 0.10, 0),
    (R.CSUM_MD5, 0x5EED5EED, 24 << 20, 0.10, 0),
    (R.CSUM_XXH3_64, 7, 16 << 20, 0.30, 0),
    (R.CSUM_XXH64, 0, 16 << 20, 0.05, 0),
    (R.CSUM_XXH3_128, 1, 8 << 20, 0.20, 1000),        # odd block size: unaligned blocks
    (R.CSUM_XXH3_128, 2, (5 << 20) + 777, 0.10, 0),   # short last block
])
def test_device_path_vs_c_oracle(gpu, csum_type, seed, n, frac, block_size):
    """Signatures on the device (vs_rsync_signatures_device), table loaded from
    device arrays, match on a device-resident source: == the C hash_search."""
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot
    basis = O.synth(100 + n % 97, 0, n)
    hdr = sum_sizes_sqroot(n, block_size)
    src = R.mutate(basis, hdr.blength, seed=n % 1000, frac=frac)
    db, ds = to_dev(basis), to_dev(src)
    s1 = torch.zeros(max(hdr.count, 1), dtype=torch.int32, device="cuda")
    s2 = torch.zeros(max(hdr.count, 1) * hdr.s2length, dtype=torch.uint8, device="cuda")
    m = Matcher()
    m.signatures_device(db.data_ptr(), n, hdr.blength, hdr.s2length, csum_type, seed,
                        s1.data_ptr(), s2.data_ptr())
    m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder, s1.data_ptr(),
                       s2.data_ptr(), csum_type, seed)
    got = m.match_sums(ds.data_ptr(), len(src))
    st = m.stats()
    m.close()
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, csum_type, seed)
    assert (s1.cpu().numpy().view(np.uint32)[: hdr.count] == c1).all()
    assert (s2.cpu().numpy()[: hdr.count * hdr.s2length].reshape(-1, hdr.s2length) == c2).all()
    want, fa = O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, csum_type, seed)
    assert got == want
    assert st["false_alarms"] == fa


def test_weak_collisions_and_false_alarms(gpu):
    """Tiny strong sums (s2length 2, the minimum) over a small-block table make
    false alarms and strong collisions likely: the walk must follow rsync
    exactly through them (want_i, chain order, false-alarm continue)."""
    from volsync_amd import SumStruct, match_sums
    rng = np.random.default_rng(11)
    # low-entropy data: weak sums collide often
    basis = rng.integers(0, 3, 300_000, dtype=np.uint8)
    src = np.concatenate([basis[1000:150_000], rng.integers(0, 3, 20_000, dtype=np.uint8),
                          basis[:100_000]])
    for csum_type, seed in [(R.CSUM_XXH3_128, 3), (R.CSUM_MD5, 0), (R.CSUM_XXH64, 9)]:
        bl, s2l, cnt, rem = O.rsync_sizes(len(basis), 700)
        c1, c2 = O.rsync_signatures(basis, bl, s2l, csum_type, seed)
        want, fa = O.rsync_match(src, c1, c2, bl, rem, csum_type, seed)
        s = SumStruct(0, cnt, bl, s2l, rem, c1, c2)
        assert match_sums(src, s, csum_type, seed) == want
        # device-resident source through a Matcher: the false-alarm count too
        # (the no-replay branch completes it from the round-1 needs' compares)
        import torch
        from volsync_amd import Matcher
        ds = torch.from_numpy(src.copy()).to("cuda")
        m = Matcher()
        m.load_sums(s, csum_type, seed)
        assert m.match_sums(ds.data_ptr(), len(src)) == want
        st = m.stats()
        m.close()
        assert st["false_alarms"] == fa


@pytest.mark.parametrize("bbits", [2, 10])
def test_membership_bucket_overflow_fallback(gpu, bbits):
    """The walk's membership buckets (one 32-byte load per probe: a count and
    7 sums) with so few buckets (VS_OPT_BUCKET_BITS) that most overflow: the
    probe falls back to the directory and the match list and false alarms
    stay hash_search's."""
    from volsync_amd import Matcher, SumStruct
    from volsync_amd._lib import VS_OPT_BUCKET_BITS
    n, csum, seed = 24 << 20, R.CSUM_XXH3_128, 0x5EED5EED
    basis = O.synth(31, 0, n)
    bl, s2l, cnt, rem = O.rsync_sizes(n, 2048)
    src = R.mutate(basis, bl, seed=3, frac=0.2)
    c1, c2 = O.rsync_signatures(basis, bl, s2l, csum, seed)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, csum, seed)
    ds = to_dev(src)
    m = Matcher()
    m.set_option(VS_OPT_BUCKET_BITS, bbits)
    m.load_sums(SumStruct(0, cnt, bl, s2l, rem, c1, c2), csum, seed)
    got = m.match_sums(ds.data_ptr(), len(src))
    st = m.stats()
    m.close()
    assert cnt > 10000   # 2^10 buckets: ~12 sums each, most of them overflowing
    assert got == want and st["false_alarms"] == fa


def test_repeated_blocks_prefer_adjacent(gpu):
    """Identical blocks: rsync's chain offers the highest index first and the
    want_i rule then prefers the block after the previous match."""
    from volsync_amd import generate_sums, match_sums
    unit = O.synth(5, 0, 700)
    basis = np.tile(unit, 64)
    src = np.concatenate([basis[:7000], O.synth(6, 0, 333), basis[:14000]])
    s = generate_sums(basis, R.CSUM_XXH3_128, 77)
    want, _ = O.rsync_match(src, s.sum1, s.sum2, s.blength, s.remainder, R.CSUM_XXH3_128, 77)
    assert match_sums(src, s, R.CSUM_XXH3_128, 77) == want


def test_empty_inputs(gpu):
    from volsync_amd import generate_sums, match_sums
    s = generate_sums(np.zeros(0, np.uint8))
    assert s.count == 0
    assert match_sums(O.synth(1, 0, 5000), s) == []
    s = generate_sums(O.synth(1, 0, 5000))
    assert match_sums(np.zeros(0, np.uint8), s) == []


def test_c4_shape_properties(gpu):
    """C4 shape at 4 GiB on one device (blength 65536): every match is a
    byte-exact copy of its block, matches never overlap, >= 85% of the blocks
    are found, and the list equals the C oracle on a 256 MiB window pair."""
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device
    n = 4 << 30
    hdr = sum_sizes_sqroot(n)
    db = torch.empty(n, dtype=torch.uint8, device="cuda")
    synth_fill_device(db.data_ptr(), 4, 0, n)
    # source: basis with edits at 10% of the blocks, assembled on the device
    rng = np.random.default_rng(5)
    edits = np.sort(rng.choice(hdr.count, hdr.count // 10, replace=False))
    pieces, pos = [], 0
    for b in edits.tolist():
        at = b * hdr.blength + int(rng.integers(0, hdr.blength - 4096))
        pieces.append(db[pos:at])
        kind = int(rng.integers(0, 3))
        if kind == 0:
            pieces.append(torch.randint(0, 256, (4096,), dtype=torch.uint8, device="cuda"))
            pos = at + 4096
        elif kind == 1:
            pieces.append(torch.randint(0, 256, (int(rng.integers(1, 65)),), dtype=torch.uint8,
                                        device="cuda"))
            pos = at
        else:
            pos = at + int(rng.integers(1, 65))
    pieces.append(db[pos:])
    ds = torch.cat(pieces)
    del pieces
    s1 = torch.zeros(hdr.count, dtype=torch.int32, device="cuda")
    s2 = torch.zeros(hdr.count * hdr.s2length, dtype=torch.uint8, device="cuda")
    m = Matcher()
    m.signatures_device(db.data_ptr(), n, hdr.blength, hdr.s2length, R.CSUM_XXH3_128,
                        0x5EED5EED, s1.data_ptr(), s2.data_ptr())
    m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder, s1.data_ptr(),
                       s2.data_ptr(), R.CSUM_XXH3_128, 0x5EED5EED)
    got = m.match_sums(ds.data_ptr(), ds.numel())
    m.close()
    assert len(got) >= 0.85 * hdr.count
    prev = 0
    rng2 = np.random.default_rng(1)
    picks = set(rng2.integers(0, len(got), 200).tolist())
    for j, (o, i) in enumerate(got):
        assert o >= prev
        prev = o + hdr.blength
        if j in picks:
            assert torch.equal(ds[o:o + hdr.blength], db[i * hdr.blength:(i + 1) * hdr.blength])
    # exact list on a window pair that fits the CPU oracle
    w = 256 << 20
    bw = db[:w].cpu().numpy()
    sw = ds[:w].cpu().numpy()
    del db, ds
    torch.cuda.empty_cache()
    hw = sum_sizes_sqroot(w)
    c1, c2 = O.rsync_signatures(bw, hw.blength, hw.s2length, R.CSUM_XXH3_128, 0x5EED5EED)
    want, _ = O.rsync_match(sw, c1, c2, hw.blength, hw.remainder, R.CSUM_XXH3_128, 0x5EED5EED)
    from volsync_amd import SumStruct, match_sums
    s = SumStruct(0, hw.count, hw.blength, hw.s2length, hw.remainder, c1, c2)
    assert match_sums(sw, s, R.CSUM_XXH3_128, 0x5EED5EED) == want


@pytest.mark.parametrize("world,n,block_size", [
    (2, (5 << 20) + 777, 0),      # short last block on the last shard
    (3, 8 << 20, 1000),           # odd block size: shard byte ranges unaligned
    (8, 3 << 20, 0),
])
def test_block_sharded_signatures_on_device(gpu, world, n, block_size):
    """The device side of the sharded signature pass: each "rank" runs
    vs_rsync_signatures_device over ONLY its block range's bytes (a separate
    device buffer), gather_sums assembles the pieces (identity all-gather on
    one device), and the table and the match list equal the whole-file ones."""
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot
    from volsync_amd.rsync_shard import BlockShard, gather_sums
    csum, seed = R.CSUM_XXH3_128, 0x5EED5EED
    basis = O.synth(300 + world, 0, n)
    hdr = sum_sizes_sqroot(n, block_size)
    m = Matcher()
    pieces = []
    for sh in BlockShard.split(n, hdr.blength, world):
        db = to_dev(basis[sh.byte_lo:sh.byte_hi])
        s1 = torch.zeros(max(sh.blocks, 1), dtype=torch.int32, device="cuda")
        s2 = torch.zeros(max(sh.blocks, 1) * hdr.s2length, dtype=torch.uint8, device="cuda")
        m.signatures_device(db.data_ptr(), sh.byte_hi - sh.byte_lo, hdr.blength, hdr.s2length,
                            csum, seed, s1.data_ptr(), s2.data_ptr())
        # db stays referenced until the synchronize below: the kernel runs on
        # the matcher's stream, which torch's allocator does not track
        pieces.append((sh, s1, s2, db))
    torch.cuda.synchronize()
    contrib = {}
    for sh, s1, s2, _ in pieces:
        def fake_gather(out, t, sh=sh):
            # stands in for dist.all_gather: every rank's padded contribution
            # (one packed record per rank); the last rank sees them all
            contrib[sh.rank] = t.clone()
            if len(contrib) == world:
                for r in range(world):
                    out[r].copy_(contrib[r])
        f1, f2 = gather_sums(s1, s2, sh, hdr.s2length, fake_gather)
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, csum, seed)
    assert (f1.cpu().numpy().view(np.uint32) == c1).all()
    assert (f2.cpu().numpy().reshape(-1, hdr.s2length) == c2).all()
    src = R.mutate(basis, hdr.blength, seed=11)
    ds = to_dev(src)
    m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder, f1.data_ptr(),
                       f2.data_ptr(), csum, seed)
    got = m.match_sums(ds.data_ptr(), len(src))
    m.close()
    assert got == O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, csum, seed)[0]


def _sharded_device_match(src, hdr_or_sums, world, csum, seed, dev_sums=None, seg_blocks=0):
    """One Matcher per "rank", each holding ONLY its source window (own range
    + blength - 1 bytes of right halo) in its own device buffer; the walk
    stitch runs in one process (run_walk_shards_local, the same Jacobi rounds
    as the distributed protocol).  Returns (matches, false-alarm total)."""
    from volsync_amd import Matcher, SumStruct
    from volsync_amd.rsync_shard import SourceShard, run_walk_shards_local
    s = hdr_or_sums
    specs = SourceShard.split(len(src), s.blength, world)
    hs, bufs = [], []
    from volsync_amd._lib import VS_OPT_WALK_SEGMENT_BLOCKS
    for sp in specs:
        m = Matcher()
        m.set_option(VS_OPT_WALK_SEGMENT_BLOCKS, seg_blocks)
        m.load_sums(s, csum, seed)
        bufs.append(to_dev(src[sp.data_lo:sp.data_hi]))
        hs.append(m)
    got = run_walk_shards_local(hs, specs, [b.data_ptr() for b in bufs])
    fa = sum(m.stats()["false_alarms"] for m in hs)
    for m in hs:
        m.close()
    return got, fa


@pytest.mark.parametrize("world,n,block_size,csum,seed,frac", [
    (2, (5 << 20) + 777, 0, R.CSUM_XXH3_128, 0x5EED5EED, 0.10),   # short last block
    (3, 8 << 20, 1000, R.CSUM_XXH3_128, 1, 0.20),                 # unaligned blocks
    (5, 6 << 20, 0, R.CSUM_MD5, 0x5EED5EED, 0.10),
    (8, 3 << 20, 0, R.CSUM_XXH64, 0, 0.30),
    (7, 2 << 20, 65536, R.CSUM_XXH3_64, 9, 0.05),                 # ranges of ~4.5 blocks
])
def test_sharded_walk_on_device(gpu, world, n, block_size, csum, seed, frac):
    """Byte-range sharded hash_search on the device: matches and false alarms
    of the concatenated ranges == ONE hash_search over the file (C oracle)."""
    from volsync_amd import SumStruct
    basis = O.synth(500 + world, 0, n)
    bl, s2l, cnt, rem = O.rsync_sizes(n, block_size)
    c1, c2 = O.rsync_signatures(basis, bl, s2l, csum, seed)
    src = R.mutate(basis, bl, seed=world, frac=frac)
    s = SumStruct(n, cnt, bl, s2l, rem, c1, c2)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, csum, seed)
    got, gfa = _sharded_device_match(src, s, world, csum, seed)
    assert got == want
    assert gfa == fa


def test_sharded_walk_boundaries_in_edits_and_duplicates(gpu):
    """Shard boundaries placed ON edited regions and inside runs of identical
    blocks (want_i decides), for every boundary offset within one block."""
    from volsync_amd import SumStruct
    from volsync_amd import Matcher
    from volsync_amd.rsync_shard import SourceShard, run_walk_shards_local
    unit = O.synth(5, 0, 700)
    basis = np.concatenate([np.tile(unit, 40), O.synth(7, 0, 30_000)])
    bl, s2l, cnt, rem = O.rsync_sizes(len(basis))
    c1, c2 = O.rsync_signatures(basis, bl, s2l, R.CSUM_XXH3_128, 77)
    src = np.concatenate([basis[:7000], O.synth(6, 0, 333), basis[:14000], basis[350:40_000]])
    want, fa = O.rsync_match(src, c1, c2, bl, rem, R.CSUM_XXH3_128, 77)
    s = SumStruct(len(basis), cnt, bl, s2l, rem, c1, c2)
    d = to_dev(src)
    for cut in list(range(6900, 7400, 37)) + [7000, 7333, 7334, 21_333, 21_334, 22_000]:
        specs = [SourceShard(0, 2, len(src), bl, 0, cut, 0, min(cut + bl - 1, len(src))),
                 SourceShard(1, 2, len(src), bl, cut, len(src), cut & ~15, len(src))]
        hs = []
        for _ in specs:
            m = Matcher()
            m.load_sums(s, R.CSUM_XXH3_128, 77)
            hs.append(m)
        got = run_walk_shards_local(hs, specs, [d.data_ptr() + sp.data_lo for sp in specs])
        gfa = sum(m.stats()["false_alarms"] for m in hs)
        for m in hs:
            m.close()
        assert got == want, cut
        assert gfa == fa, cut


def test_c4_params_exact_1g(gpu):
    """C4's own matcher parameters -- blength 131072, s2length 5, xxh128,
    checksum_seed 0x5EED5EED -- on a 1 GiB basis with C4 edits (10 % of the
    blocks: 4 KiB overwrites, 1-64 B inserts/deletes): the device match list
    and false-alarm count equal the C hash_search exactly, on one device and
    byte-range sharded 4 ways."""
    import torch
    from volsync_amd import Matcher, SumStruct
    n, bl, s2l, csum, seed = 1 << 30, 131072, 5, R.CSUM_XXH3_128, 0x5EED5EED
    basis = O.synth(4, 0, n)
    src = R.mutate(basis, bl, seed=5, frac=0.10)
    db = to_dev(basis)
    cnt, rem = n // bl, 0
    s1 = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    s2 = torch.zeros(cnt * s2l, dtype=torch.uint8, device="cuda")
    m = Matcher()
    m.signatures_device(db.data_ptr(), n, bl, s2l, csum, seed, s1.data_ptr(), s2.data_ptr())
    torch.cuda.synchronize()
    del db
    c1, c2 = O.rsync_signatures(basis, bl, s2l, csum, seed)
    assert (s1.cpu().numpy().view(np.uint32) == c1).all()
    assert (s2.cpu().numpy().reshape(-1, s2l) == c2).all()
    want, fa = O.rsync_match(src, c1, c2, bl, rem, csum, seed)
    m.load_sums_device(cnt, bl, s2l, rem, s1.data_ptr(), s2.data_ptr(), csum, seed)
    ds = to_dev(src)
    got = m.match_sums(ds.data_ptr(), len(src))
    st = m.stats()
    m.close()
    assert got == want
    assert st["false_alarms"] == fa
    del ds
    s = SumStruct(n, cnt, bl, s2l, rem, c1, c2)
    got4, fa4 = _sharded_device_match(src, s, 4, csum, seed)
    assert got4 == want and fa4 == fa


def _plan_host(plan, lo, hi):
    out = np.zeros(hi - lo, np.uint8)
    for d, seed, off, n in plan.segments(lo, hi):
        out[d:d + n] = O.synth(seed, off, n)
    return out


def test_c4plan_source_sharded_exact(gpu):
    """bench.py's C4 workload generator at 256 MiB (blength 16384): every
    rank's device-generated source range equals the host-generated one, and
    the sharded walk over them (3 ranks, the bench's run_walk_shard protocol)
    equals ONE hash_search over the whole source (C oracle)."""
    import bench
    import torch
    from volsync_amd import Matcher, SumStruct, sum_sizes_sqroot
    from volsync_amd.rsync_shard import SourceShard, run_walk_shards_local
    dlen = 256 << 20
    hdr = sum_sizes_sqroot(dlen)
    plan = bench.C4Plan(dlen, hdr.blength)
    src = _plan_host(plan, 0, plan.total)
    basis = O.synth(bench.C4Plan.D_SEED, 0, dlen)
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, R.CSUM_XXH3_128, 0x5EED5EED)
    want, fa = O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, R.CSUM_XXH3_128, 0x5EED5EED)
    s = SumStruct(dlen, hdr.count, hdr.blength, hdr.s2length, hdr.remainder, c1, c2)
    specs = SourceShard.split(plan.total, hdr.blength, 3)
    hs, bufs = [], []
    for sp in specs:
        b = torch.empty(sp.data_hi - sp.data_lo + 16, dtype=torch.uint8, device="cuda")
        plan.fill_device(b.data_ptr(), sp.data_lo, sp.data_hi)
        torch.cuda.synchronize()
        assert np.array_equal(b[: sp.data_hi - sp.data_lo].cpu().numpy(), src[sp.data_lo:sp.data_hi])
        m = Matcher()
        m.load_sums(s, R.CSUM_XXH3_128, 0x5EED5EED)
        hs.append(m)
        bufs.append(b)
    got = run_walk_shards_local(hs, specs, [b.data_ptr() for b in bufs])
    gfa = sum(m.stats()["false_alarms"] for m in hs)
    for m in hs:
        m.close()
    assert got == want and gfa == fa


def _file_sum_want(data: bytes, csum: int) -> bytes:
    """rsync 3.2.3 sum_end over sum_update(whole file), pinned by libxxhash
    (the xxhash package) and hashlib: no seed for these types."""
    import hashlib
    import xxhash
    if csum == 8:
        return xxhash.xxh3_128_intdigest(data).to_bytes(16, "little")
    if csum == 7:
        return xxhash.xxh3_64_intdigest(data).to_bytes(8, "little")
    if csum == 6:
        return xxhash.xxh64_intdigest(data, seed=0).to_bytes(8, "little")
    return hashlib.md5(data).digest()


@pytest.mark.parametrize("csum", [8, 7])
def test_file_sum_xxh3_lengths(gpu, csum):
    """Whole-file checksum (R7) across the XXH3 length classes: short paths,
    exactly one block, partial stripes, the last-stripe overlap, and a 64 MiB
    file (65 536-step scramble chain), against libxxhash."""
    from volsync_amd import Matcher
    m = Matcher()
    base = O.synth(61, 0, (64 << 20) + 4099)
    for n in [0, 1, 16, 17, 128, 129, 240, 241, 1023, 1024, 1025, 1087, 1088, 2048, 4095,
              65536 + 63, (1 << 20) + 777, 64 << 20]:
        data = base[:n]
        t = to_dev(data)
        assert m.file_sum(t.data_ptr(), n, csum) == _file_sum_want(data.tobytes(), csum), n
    m.close()


def test_file_sum_multi_pass_and_other_types(gpu):
    """The XXH3 chain and the host MD5 / XXH64 carried across many read-back
    pieces (VS_OPT_FILE_SUM_PIECE forced small: 1000 blocks = 62.5 KiB of
    bytes per serial piece), and every type on C4-fixture sources."""
    from volsync_amd import Matcher
    from volsync_amd._lib import VS_OPT_FILE_SUM_PIECE
    m = Matcher()
    data = O.synth(62, 0, (9 << 20) + 321)
    t = to_dev(data)
    # a nonzero piece forces the bounded device ring (XXH3's multi-piece
    # contribution ring; the path files over 128 GiB and hosts without the
    # DMA agents take); 0 = rows first (every row, then one SDMA read-back)
    m.set_option(VS_OPT_FILE_SUM_PIECE, 1000)
    for csum in (8, 7, 6, 5):
        assert m.file_sum(t.data_ptr(), len(data), csum) == _file_sum_want(data.tobytes(), csum)
    m.set_option(VS_OPT_FILE_SUM_PIECE, 0)
    for csum in (8, 7):
        assert m.file_sum(t.data_ptr(), len(data), csum) == _file_sum_want(data.tobytes(), csum)
    for path in FIX[:6]:
        _, _, src = load_fixture(path)
        ts = to_dev(src)
        for csum in (8, 7, 6, 5):
            n = len(src)
            got = m.file_sum(ts.data_ptr(), n, csum)
            assert got == _file_sum_want(src[:n].tobytes(), csum), (path, csum)
    m.close()


@pytest.mark.parametrize("path", FIX[:8], ids=os.path.basename)
def test_receiver_reconstruct(gpu, path):
    """receiver.c receive_data: the new file rebuilt on the device
    from the basis, the match list and the gaps' literal bytes equals the
    source, and its whole-file checksum equals the sender's."""
    from volsync_amd import Matcher
    doc, basis, src = load_fixture(path)
    p = doc["params"] if "params" in doc else {}
    m = Matcher()
    db, ds = to_dev(basis), to_dev(src)
    hdr = O.rsync_sizes(len(basis), p.get("block_size", 0))
    bl = hdr[0]
    csum, seed = 8, 0x5EED5EED
    n1 = max(hdr[2], 1)
    import torch
    s1 = torch.zeros(n1, dtype=torch.int32, device="cuda")
    s2 = torch.zeros(n1 * hdr[1], dtype=torch.uint8, device="cuda")
    m.signatures_device(db.data_ptr(), len(basis), bl, hdr[1], csum, seed, s1.data_ptr(),
                        s2.data_ptr())
    m.load_sums_device(hdr[2], bl, hdr[1], hdr[3], s1.data_ptr(), s2.data_ptr(), csum, seed)
    matches = m.match_sums(ds.data_ptr(), len(src))
    lit, pos = [], 0
    for o, i in matches:
        lit.append(src[pos:o])
        pos = o + min(bl, len(basis) - i * bl)
    lit.append(src[pos:])
    lits = np.concatenate(lit) if lit else np.zeros(0, np.uint8)
    dl = to_dev(lits)
    out = torch.zeros(max(len(src), 16), dtype=torch.uint8, device="cuda")
    m.reconstruct(out.data_ptr(), len(src), db.data_ptr(), len(basis), bl, matches, dl.data_ptr(),
                  len(lits))
    assert (out[: len(src)].cpu().numpy() == src).all()
    assert m.file_sum(out.data_ptr(), len(src), 8) == _file_sum_want(src.tobytes(), 8)
    m.close()


def test_c4_real_density_window_exact(gpu):
    """C4 at its real table density: the 2,097,152-block table of the 256 GiB
    destination (blength 131072, s2length 5, xxh128, checksum_seed
    0x5EED5EED) from the device signature pass -- D generated on the device
    32 GiB at a time -- equals a 16-thread C signature pass over the same
    stream; then a 2 GiB window of rank 3's (of 8) source range, entered at the
    walk's true state there, gives exactly the C hash_search's match list,
    false-alarm count and exit state.  This is the density at which one rank
    meets ~1.7 M false alarms; the 1 GiB test above is 256x
    sparser.

    Entry: the C walk from 64 MiB before the window (want_i = count, "no
    preference") gives the state at the window start; every walk that makes a
    match continues identically from there (the exit-stitch argument of
    DESIGN.md 6), and random data leaves no duplicate blocks for want_i to
    choose among, so this is the state the walk from offset 0 reaches."""
    import bench
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device
    from volsync_amd.rsync_shard import SourceShard
    dlen, csum, seed = 256 << 30, R.CSUM_XXH3_128, 0x5EED5EED
    hdr = sum_sizes_sqroot(dlen)
    bl, s2l, cnt, rem = hdr.blength, hdr.s2length, hdr.count, hdr.remainder
    assert (bl, s2l, cnt, rem) == (131072, 5, 2097152, 0)
    # 1. signatures on the device, 32 GiB of D at a time
    s1 = torch.zeros(cnt, dtype=torch.int32, device="cuda")
    s2 = torch.zeros(cnt * s2l, dtype=torch.uint8, device="cuda")
    piece = 32 << 30
    buf = torch.empty(piece, dtype=torch.uint8, device="cuda")
    m = Matcher()
    for p0 in range(0, dlen, piece):
        synth_fill_device(buf.data_ptr(), bench.C4Plan.D_SEED, p0, piece)
        b0 = p0 // bl
        m.signatures_device(buf.data_ptr(), piece, bl, s2l, csum, seed, s1.data_ptr() + 4 * b0,
                            s2.data_ptr() + s2l * b0)
    torch.cuda.synchronize()
    del buf
    torch.cuda.empty_cache()
    c1, c2 = O.rsync_signatures_synth_mt(bench.C4Plan.D_SEED, dlen, bl, s2l, csum, seed, 16)
    assert (s1.cpu().numpy().view(np.uint32) == c1).all()
    assert (s2.cpu().numpy().reshape(-1, s2l) == c2).all()
    # 2. the window: rank 3's range start + 2 GiB of the C4Plan source
    plan = bench.C4Plan(dlen, bl)
    sh = SourceShard.for_rank(plan.total, bl, 8, 3)
    lo, hi = sh.own_lo, sh.own_lo + (2 << 30)
    pre = lo - (64 << 20)
    win_lo = pre & ~15
    host = _plan_host(plan, win_lo, min(hi + bl - 1, plan.total))
    _, _, e, w = O.rsync_walk(host, win_lo, plan.total, lo, pre, cnt, c1, c2, bl, rem, csum, seed)
    assert lo <= e < lo + bl
    want, fa, wexit, wwant = O.rsync_walk(host, win_lo, plan.total, hi, e, w, c1, c2, bl, rem,
                                          csum, seed)
    # 3. the device: the rank's scan + speculative walk of [lo, hi), then the
    # stitch from the true entry (run_walk_shard's protocol)
    data_lo = lo & ~15
    n = min(hi + bl - 1, plan.total) - data_lo
    ds = torch.empty(n, dtype=torch.uint8, device="cuda")
    plan.fill_device(ds.data_ptr(), data_lo, data_lo + n)
    torch.cuda.synchronize()
    assert (ds[:4096].cpu().numpy() == host[data_lo - win_lo:data_lo - win_lo + 4096]).all()
    m.load_sums_device(cnt, bl, s2l, rem, s1.data_ptr(), s2.data_ptr(), csum, seed)
    assert len(want) > 14000 and fa > 50000   # the density this test is for
    # the rank's speculative walk + the stitch from the true entry.  (The
    # streamed form's walk from a piece's true entry -- match_scan's has_entry
    # path -- is covered at the 64 GiB table density by
    # tests/test_gpu_rsync_stream.py's 3 GiB C4-plan files; no public entry
    # point starts a streamed walk in mid-file, as this window would need.)
    m.match_scan(ds.data_ptr(), n, data_lo, plan.total, lo, hi)
    gexit = m.match_stitch(e, w)
    nm = m.match_finish()
    got = m.matches(0, nm)
    st = m.stats()
    assert got == want
    assert st["false_alarms"] == fa
    assert gexit == (wexit, wwant)
    m.close()


def test_file_sum_async_overlaps_match(gpu):
    """vs_rsync_file_sum_start / _wait (R7 beside the walk, as the C4 step runs
    it): the digest equals libxxhash while a match run proceeds on the same
    handle, and the timing split is reported."""
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot
    n = (96 << 20) + 333
    basis = O.synth(63, 0, n)
    src = R.mutate(basis, 4096, seed=3, frac=0.1)
    hdr = sum_sizes_sqroot(n, 4096)
    db, ds = to_dev(basis), to_dev(src)
    s1 = torch.zeros(hdr.count, dtype=torch.int32, device="cuda")
    s2 = torch.zeros(hdr.count * hdr.s2length, dtype=torch.uint8, device="cuda")
    m = Matcher()
    m.signatures_device(db.data_ptr(), n, hdr.blength, hdr.s2length, 8, 5, s1.data_ptr(),
                        s2.data_ptr())
    m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder, s1.data_ptr(),
                       s2.data_ptr(), 8, 5)
    for csum in (8, 7):
        m.file_sum_start(ds.data_ptr(), len(src), csum)
        got_m = m.match_sums(ds.data_ptr(), len(src))
        assert m.file_sum_wait() == _file_sum_want(src.tobytes(), csum)
        assert len(got_m) > 0.8 * hdr.count
        t = m.file_sum_timing()
        assert t["device_ms"] > 0 and t["host_chain_ms"] > 0
    m.close()


def test_file_sum_relay_across_ranges(gpu):
    """A file split across ranks: each range's whole 1 KiB blocks chained from
    the previous range's accumulators (vs_rsync_file_sum_blocks_*), the last
    owner finishing with the file's last bytes == one whole-file XXH3."""
    import volsync_amd as V
    from volsync_amd import Matcher
    n = (40 << 20) + 4321
    data = O.synth(64, 0, n)
    t = to_dev(data)
    nb = (n - 1) // 1024
    cuts = [0, 7 * 1024 + 0, (13 << 20) // 1024, nb]   # block indices: ranges of 7, ~13 K, rest
    m = Matcher()
    acc = V.file_sum_init()
    for lo, hi in zip(cuts, cuts[1:]):
        m.file_sum_blocks_start(t.data_ptr() + lo * 1024, hi - lo, acc)
        acc = m.file_sum_blocks_wait()
    keep = min(n, 1088)
    for csum in (8, 7):
        got = V.file_sum_finish(acc, data[n - keep:].tobytes(), n, csum)
        assert got == _file_sum_want(data.tobytes(), csum)
    # an empty range passes the state through unchanged
    m.file_sum_blocks_start(t.data_ptr(), 0, acc)
    assert (m.file_sum_blocks_wait() == acc).all()
    m.close()


def test_file_sum_64g_exact(gpu):
    """R7 at C2 / C4 scale: the whole-file XXH3-128 of 64 GiB of the synthetic
    stream (device-generated) equals libxxhash's streaming digest of the same
    stream (oracle/rsync_ref.c ref_xxh3_synth, 16 generator threads)."""
    import torch
    from volsync_amd import Matcher, synth_fill_device
    n = (64 << 30) + 777
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    synth_fill_device(t.data_ptr(), 5, 0, n)
    torch.cuda.synchronize()
    m = Matcher()
    got = m.file_sum(t.data_ptr(), n, 8)
    tm = m.file_sum_timing()
    m.close()
    del t
    torch.cuda.empty_cache()
    assert got == O.xxh3_synth(5, n, 8, 16)
    print(f"64 GiB file sum: device {tm['device_ms']:.1f} ms, host chain {tm['host_chain_ms']:.1f} ms")


def test_file_sum_serial_types_large(gpu):
    """MD5 / XXH64 whole-file sums at C4-mode scale (MD5 as the
    second mode): a 4 GiB + 333 B file's bytes read back through the pinned
    ring and hashed on the library's host thread == hashlib / libxxhash."""
    import hashlib
    import torch
    import xxhash
    from volsync_amd import Matcher, synth_fill_device
    n = (4 << 30) + 333
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    synth_fill_device(t.data_ptr(), 65, 0, n)
    torch.cuda.synchronize()
    host = O.synth(65, 0, n)
    m = Matcher()
    got5 = m.file_sum(t.data_ptr(), n, 5)
    got6 = m.file_sum(t.data_ptr(), n, 6)
    tm = m.file_sum_timing()
    m.close()
    assert got5 == hashlib.md5(host).digest()
    assert got6 == xxhash.xxh64_intdigest(host, seed=0).to_bytes(8, "little")
    print(f"4 GiB XXH64 file sum: host {tm['host_chain_ms']:.0f} ms")


def test_file_sum_jobs_fifo(gpu):
    """Several whole-file checksums in flight on one handle (the C4 bench keeps
    two: file k's chain overlaps file k+1's walk): digests come back in start
    order; a fifth job is refused until one is waited for."""
    from volsync_amd import Matcher, VsError
    files = [O.synth(70 + k, 0, (k + 1) * (3 << 20) + 17 * k + 241) for k in range(4)]
    devs = [to_dev(f) for f in files]
    m = Matcher()
    for csum in (8, 7, 5):
        for f, t in zip(files, devs):
            m.file_sum_start(t.data_ptr(), len(f), csum)
        with pytest.raises(VsError):
            m.file_sum_start(devs[0].data_ptr(), len(files[0]), csum)
        for f in files:
            assert m.file_sum_wait() == _file_sum_want(f.tobytes(), csum)
    with pytest.raises(VsError):
        m.file_sum_wait()
    # the blocking form beside jobs in flight: it returns its own
    # file's digest and the pending jobs keep their order
    m.file_sum_start(devs[0].data_ptr(), len(files[0]), 8)
    m.file_sum_start(devs[1].data_ptr(), len(files[1]), 8)
    assert m.file_sum(devs[2].data_ptr(), len(files[2]), 6) == _file_sum_want(files[2].tobytes(), 6)
    m.file_sum_start(devs[3].data_ptr(), len(files[3]), 8)
    for k in (0, 1, 3):
        assert m.file_sum_wait() == _file_sum_want(files[k].tobytes(), 8), k
    with pytest.raises(VsError):
        m.file_sum_wait()
    # the blocking form has a job of its own, so with three jobs
    # in flight it can be called again and again (it used to take the 4th
    # FIFO slot until the older jobs were waited for)
    for k in range(3):
        m.file_sum_start(devs[k].data_ptr(), len(files[k]), 8)
    for csum in (6, 5, 8, 7):
        assert m.file_sum(devs[3].data_ptr(), len(files[3]), csum) == \
            _file_sum_want(files[3].tobytes(), csum)
    m.file_sum_start(devs[3].data_ptr(), len(files[3]), 8)   # the 4th slot is still free
    for k in range(4):
        assert m.file_sum_wait() == _file_sum_want(files[k].tobytes(), 8), k
    m.close()


@pytest.mark.parametrize("seg,prefilter,flushq,span,predict,tail,margin", [
    (8, 1, 16, 0, 1, 0, -1), (16, 1, 4, 0, 1, 0, -1), (64, 1, 16, 8192, 1, 0, 777),
    (0, 0, 16, 0, 1, 0, -1), (0, 1, 16, 40000, 0, 0, -1), (0, 1, 4, 3000, 0, 0, 0),
    (0, 1, 16, 0, 1, 30, -1), (32, 1, 16, 0, 1, 90, -1), (0, 1, 16, 0, 1, -1, 0),
    (8, 1, 16, 0, 1, -1, 131071), (0, 1, 16, 0, 1, -1, 1)])
def test_walk_segment_lengths_exact(gpu, seg, prefilter, flushq, span, predict, tail, margin):
    """The device walk with other segment lengths (VS_OPT_WALK_SEGMENT_BLOCKS;
    the default 0 is 48 blocks, shorter for small ranges), without the LDS
    prefilter (VS_OPT_WALK_PREFILTER 0), with four-window flushes in place of
    the wide address-lockstep ones (VS_OPT_WALK_FLUSH_WINDOWS) and with flushes
    bounded by a span (VS_OPT_WALK_FLUSH_SPAN), with and without the early
    flush at a likely resync (VS_OPT_WALK_FLUSH_PREDICT), with quarter-length
    tail segments (VS_OPT_WALK_TAIL_PCT), with segment starts at other margins
    before a block boundary (VS_OPT_WALK_SEG_MARGIN): more or fewer speculative
    segments, stitches and flushes, the same hash_search -- seeded shifted /
    overwritten sources (false alarms, runs, short last blocks), the C4
    parameters on a 1 GiB basis, and the 4-way sharded walk."""
    from volsync_amd import Matcher, SumStruct
    from volsync_amd._lib import (VS_OPT_WALK_FLUSH_PREDICT, VS_OPT_WALK_FLUSH_SPAN,
                                  VS_OPT_WALK_FLUSH_WINDOWS, VS_OPT_WALK_PREFILTER,
                                  VS_OPT_WALK_SEG_MARGIN, VS_OPT_WALK_SEGMENT_BLOCKS,
                                  VS_OPT_WALK_TAIL_PCT)

    def opts(m):
        m.set_option(VS_OPT_WALK_SEGMENT_BLOCKS, seg)
        m.set_option(VS_OPT_WALK_PREFILTER, prefilter)
        m.set_option(VS_OPT_WALK_FLUSH_WINDOWS, flushq)
        m.set_option(VS_OPT_WALK_FLUSH_SPAN, span)
        m.set_option(VS_OPT_WALK_FLUSH_PREDICT, predict)
        m.set_option(VS_OPT_WALK_TAIL_PCT, tail)
        m.set_option(VS_OPT_WALK_SEG_MARGIN, margin)
    for csum_type, seed, n, frac, bs in [(R.CSUM_XXH3_128, 0x5EED5EED, 40 << 20, 0.10, 0),
                                         (R.CSUM_XXH3_64, 7, 12 << 20, 0.30, 0),
                                         (R.CSUM_XXH3_128, 1, 6 << 20, 0.20, 1000),
                                         (R.CSUM_XXH3_128, 2, (5 << 20) + 777, 0.10, 0)]:
        basis = O.synth(200 + n % 97, 0, n)
        bl, s2l, cnt, rem = O.rsync_sizes(n, bs)
        src = R.mutate(basis, bl, seed=n % 1000, frac=frac)
        c1, c2 = O.rsync_signatures(basis, bl, s2l, csum_type, seed)
        want, fa = O.rsync_match(src, c1, c2, bl, rem, csum_type, seed)
        ds = to_dev(src)
        m = Matcher()
        opts(m)
        m.load_sums(SumStruct(0, cnt, bl, s2l, rem, c1, c2), csum_type, seed)
        got = m.match_sums(ds.data_ptr(), len(src))
        st = m.stats()
        m.close()
        assert got == want and st["false_alarms"] == fa, (csum_type, n)
    # C4 parameters, 1 GiB: the density of false alarms the coop flushes share
    n, bl, s2l, csum, seed = 1 << 30, 131072, 5, R.CSUM_XXH3_128, 0x5EED5EED
    basis = O.synth(4, 0, n)
    src = R.mutate(basis, bl, seed=5, frac=0.10)
    c1, c2 = O.rsync_signatures(basis, bl, s2l, csum, seed)
    want, fa = O.rsync_match(src, c1, c2, bl, 0, csum, seed)
    ds = to_dev(src)
    m = Matcher()
    opts(m)
    m.load_sums(SumStruct(n, n // bl, bl, s2l, 0, c1, c2), csum, seed)
    got = m.match_sums(ds.data_ptr(), len(src))
    st = m.stats()
    m.close()
    assert got == want and st["false_alarms"] == fa
    s = SumStruct(n, n // bl, bl, s2l, 0, c1, c2)
    got4, fa4 = _sharded_device_match(src, s, 4, csum, seed, seg_blocks=seg)
    assert got4 == want and fa4 == fa


def _dup_pair():
    """A basis of 2048 identical 1 KiB blocks then 6 MiB of random bytes; the
    source interleaves shifted runs of both with small edits, so segment
    boundaries (1 MiB segments at blength 1024) fall inside runs of equal
    blocks, where want_i decides the block and stitches enter the
    speculative walks with another want_i."""
    unit = O.synth(41, 0, 1024)
    basis = np.concatenate([np.tile(unit, 2048), O.synth(42, 0, 6 << 20)])
    rnd = basis[2 << 20:]
    src = np.concatenate([O.synth(43, 0, 333), basis[: (1 << 20) + 517], rnd[:(3 << 20) + 11],
                          O.synth(44, 0, 70_000), basis[5000:(2 << 20) - 3], rnd[1 << 20:]])
    return basis, src


@pytest.mark.parametrize("facap", [-1, 3, 0])
@pytest.mark.parametrize("data", ["edits", "duplicates"])
def test_stitch_merge_at_visited_entry(gpu, facap, data):
    """Stitch re-walks whose entry the speculative walk visited merge there
    (same want_i) or at its next match (another want_i), with false alarms
    from the speculative walk's recorded windows; VS_OPT_FA_RECORD shrinks
    that record so segments with more false-alarm windows fall back to the
    re-walk.  Every mix: hash_search's match list and false alarms."""
    from volsync_amd import Matcher, SumStruct
    from volsync_amd._lib import VS_OPT_FA_RECORD
    csum, seed = R.CSUM_XXH3_128, 0x5EED5EED
    if data == "edits":
        n = 24 << 20
        basis = O.synth(51, 0, n)
        bl, s2l, cnt, rem = O.rsync_sizes(n, 2048)
        src = R.mutate(basis, bl, seed=8, frac=0.25)
    else:
        basis, src = _dup_pair()
        bl, s2l, cnt, rem = O.rsync_sizes(len(basis), 1024)
    c1, c2 = O.rsync_signatures(basis, bl, s2l, csum, seed)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, csum, seed)
    ds = to_dev(src)
    m = Matcher()
    m.set_option(VS_OPT_FA_RECORD, facap)
    m.load_sums(SumStruct(len(basis), cnt, bl, s2l, rem, c1, c2), csum, seed)
    got = m.match_sums(ds.data_ptr(), len(src))
    st = m.stats()
    m.close()
    assert len(want) > 1000
    assert got == want and st["false_alarms"] == fa
