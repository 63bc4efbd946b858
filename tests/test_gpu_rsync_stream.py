"""GPU parity tests of the streamed rsync forms (vs_rsync_match_* /
vs_rsync_sig_*): a file fed from host memory in order, as rsync's sender and
generator read it through map_ptr (fileio.c, an int32 sliding window), with
only a ring of pieces on the device.

Bar: the match list and false-alarm count equal the C hash_search
(oracle/rsync_ref.c) over the whole file, and the streamed signatures equal
the C generate_and_send_sums, bit for bit; at a C4-plan source of >= 3 GiB
fed in 256 MiB pieces through the C ABI (tests/native/abi_client.c and
ctypes) with a device window <= 1 GiB.
"""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED5EED
BIG = 3 << 30          # the streamed C4-plan test's destination (and ~source) size


def _plan_host(plan, lo, hi):
    out = np.empty(hi - lo, np.uint8)
    for d, seed, off, n in plan.segments(lo, hi):
        O.lib().ref_synth_fill(seed, off, n, out[d:].ctypes.data)
    return out


@pytest.fixture(scope="module")
def c4plan_3g():
    """bench.py's C4 workload at a 3 GiB destination: the plan, its source on
    the host, the C signatures of D and the C hash_search over the source."""
    import bench
    bl, s2l, cnt, rem = O.rsync_sizes(BIG)
    plan = bench.C4Plan(BIG, bl)
    src = _plan_host(plan, 0, plan.total)
    c1, c2 = O.rsync_signatures_synth_mt(bench.C4Plan.D_SEED, BIG, bl, s2l, R.CSUM_XXH3_128,
                                         SEED, 16)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, R.CSUM_XXH3_128, SEED)
    assert len(want) > 20000 and plan.total > BIG - (1 << 20)
    return {"plan": plan, "src": src, "hdr": (bl, s2l, cnt, rem), "c1": c1, "c2": c2,
            "want": want, "fa": fa}


def _file_sum_want(data, csum: int) -> bytes:
    """checksum.c sum_end of the whole file (no seed), by libxxhash / hashlib."""
    import hashlib
    import xxhash
    b = data if isinstance(data, (bytes, memoryview)) else np.ascontiguousarray(data)
    if csum == 8:
        return xxhash.xxh3_128_intdigest(b).to_bytes(16, "little")
    if csum == 7:
        return xxhash.xxh3_64_intdigest(b).to_bytes(8, "little")
    if csum == 6:
        return xxhash.xxh64_intdigest(b, seed=0).to_bytes(8, "little")
    return hashlib.md5(b).digest()


def _stream_match(m, data, feeds, piece, ring, file_csum=0):
    """feed `data` in the given feed sizes, draining matches after each feed
    (as matched() would be called); returns (matches, false alarms[, file
    checksum])."""
    m.match_begin(len(data), piece, ring, file_csum)
    got, pos = [], 0
    base = data.ctypes.data if isinstance(data, np.ndarray) else data.data_ptr()
    for n in feeds:
        m.match_feed(base + pos, n)
        pos += n
        while True:
            r = m.match_next()
            if not r:
                break
            got.extend(r)
    assert pos == len(data)
    while True:
        r = m.match_next()
        if r is None:
            break
        got.extend(r)
    r = m.match_end()
    assert r[0] == len(got)
    return (got,) + tuple(r[1:])


def _stream_sigs(m, data, feeds, hdr, csum, seed, piece=0, ring=0):
    bl, s2l, cnt, rem = hdr
    m.sig_begin(len(data), bl, s2l, csum, seed, piece, ring)
    s1, s2, pos = [], [], 0
    for n in feeds:
        m.sig_feed(data.ctypes.data + pos, n)
        pos += n
        r = m.sig_next()
        if r and len(r[0]):
            s1.append(r[0].copy())
            s2.append(r[1].copy())
    while True:
        r = m.sig_next()
        if r is None:
            break
        s1.append(r[0].copy())
        s2.append(r[1].copy())
    s1 = np.concatenate(s1) if s1 else np.zeros(0, np.uint32)
    s2 = np.concatenate(s2) if s2 else np.zeros((0, s2l), np.uint8)
    return s1, s2


def test_stream_c4plan_3g_pageable_exact(gpu, c4plan_3g):
    """The 3 GiB C4-plan source from pageable host memory in 256 MiB feeds,
    256 MiB pieces x 3 on the device: exactly the C hash_search, false alarms
    included; the library's device memory for the stream stays <= 1 GiB plus
    the table and walk scratch."""
    import torch
    from volsync_amd import Matcher, SumStruct
    c = c4plan_3g
    bl, s2l, cnt, rem = c["hdr"]
    m = Matcher()
    m.load_sums(SumStruct(BIG, cnt, bl, s2l, rem, c["c1"], c["c2"]), R.CSUM_XXH3_128, SEED)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    src = c["src"]
    piece = 256 << 20
    feeds = [min(piece, len(src) - o) for o in range(0, len(src), piece)]
    got, fa, fsum = _stream_match(m, src, feeds, piece, 3, file_csum=8)
    used = free0 - torch.cuda.mem_get_info()[0]
    st = m.match_stream_stats()
    m.close()
    assert got == c["want"]
    assert fa == c["fa"]
    assert fsum == _file_sum_want(src, 8)   # R7 as the file passed
    assert st["piece_bytes"] * st["ring"] <= 1 << 30 and st["staged_bytes"] == len(src)
    # ring slots (3 x (256 MiB + halo)) + walk scratch; never the file
    assert used < (1 << 30) + (256 << 20), used


def test_stream_c4plan_3g_c_client(gpu, c4plan_3g):
    """The same file through the C ABI from C (abi_client rsync-plan): the
    basis streamed through vs_rsync_sig_* and the source through
    vs_rsync_match_*, both generated 256 MiB at a time into one host buffer
    (no file bigger than a read is ever in memory), 256 MiB pieces x 3."""
    import bench
    c = c4plan_3g
    plan = c["plan"]
    bl, s2l, cnt, rem = c["hdr"]
    seeds = np.where(plan.kind == 1, bench.C4Plan.LIT_SEED, bench.C4Plan.D_SEED).astype(np.uint64)
    rec = np.zeros(len(plan.length), dtype=[("l", "<i8"), ("s", "<u8"), ("o", "<i8")])
    rec["l"], rec["s"], rec["o"] = plan.length, seeds, plan.srcoff
    client = os.path.join(ROOT, "tests", "native", "build", "abi_client")
    if not os.path.exists(client):
        import __graft_entry__
        __graft_entry__.build_native_client()
    with tempfile.NamedTemporaryFile(suffix=".plan", delete=False) as f:
        f.write(struct.pack("<qiIiIq", BIG, R.CSUM_XXH3_128, SEED, 0, bench.C4Plan.D_SEED, len(rec)))
        f.write(rec.tobytes())
        path = f.name
    try:
        r = subprocess.run([client, "rsync-plan", path, str(256 << 20), str(256 << 20), "3"],
                           capture_output=True, text=True, timeout=600)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.split("\n") if ln]
    assert lines[0].split()[1:] == [str(bl), str(s2l), str(cnt), str(rem)]
    assert lines[-1].startswith("false_alarms ") and lines[-2].startswith("file_sum ")
    got = [tuple(int(x) for x in ln.split()) for ln in lines[1:-2]]
    assert got == c["want"]
    assert int(lines[-1].split()[1]) == c["fa"]
    assert lines[-2].split()[1] == _file_sum_want(c["src"], 8).hex()


def test_stream_signatures_3g(gpu, c4plan_3g):
    """generate_and_send_sums streamed: the 3 GiB destination fed in 100 MiB
    reads (not block-aligned) from pinned host memory: every sum1 / sum2 equals
    the C signature pass."""
    import bench
    import torch
    from volsync_amd import Matcher
    c = c4plan_3g
    bl, s2l, cnt, rem = c["hdr"]
    d = torch.empty(BIG, dtype=torch.uint8, pin_memory=True)
    O.lib().ref_synth_fill(bench.C4Plan.D_SEED, 0, BIG, d.data_ptr())
    m = Matcher()
    step = 100 << 20
    feeds = [min(step, BIG - o) for o in range(0, BIG, step)]
    m.sig_begin(BIG, bl, s2l, R.CSUM_XXH3_128, SEED)
    s1, s2, pos = [], [], 0
    for n in feeds:
        m.sig_feed(d.data_ptr() + pos, n)
        pos += n
        while True:
            r = m.sig_next()
            if not r or not len(r[0]):
                break
            s1.append(r[0].copy())
            s2.append(r[1].copy())
    while (r := m.sig_next()) is not None:
        s1.append(r[0].copy())
        s2.append(r[1].copy())
    m.close()
    assert np.array_equal(np.concatenate(s1), c["c1"])
    assert np.array_equal(np.concatenate(s2), c["c2"])


@pytest.mark.parametrize("csum,seed", [(R.CSUM_XXH3_128, SEED), (R.CSUM_MD5, 0x1234),
                                       (R.CSUM_XXH64, 0)])
def test_stream_ragged_feeds(gpu, csum, seed):
    """Feeds of every size (1 byte to several pieces), 1 MiB pieces x 2: the
    halo of a piece arrives over several feeds and a feed spans pieces.  The
    device walk (XXH3) and the host walk with device verification (MD5,
    XXH64) both equal the C hash_search; streamed signatures equal the C
    pass."""
    from volsync_amd import Matcher, SumStruct, sum_sizes_sqroot
    n = (24 << 20) + 4321
    basis = O.synth(71, 0, n)
    hdr = sum_sizes_sqroot(n, 8192)
    src = R.mutate(basis, hdr.blength, seed=9, frac=0.15)
    rng = np.random.default_rng(3)
    feeds, pos = [], 0
    while pos < len(src):
        k = int(rng.choice([1, 7, 4096, 8191, 65536, 700_000, 3 << 20]))
        k = min(k, len(src) - pos)
        feeds.append(k)
        pos += k
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, csum, seed)
    want, fa = O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, csum, seed)
    m = Matcher()
    bfeeds, pos = [], 0
    while pos < n:
        k = min(int(rng.integers(1, 3 << 20)), n - pos)
        bfeeds.append(k)
        pos += k
    g1, g2 = _stream_sigs(m, basis, bfeeds, (hdr.blength, hdr.s2length, hdr.count, hdr.remainder),
                          csum, seed, piece=1 << 20, ring=2)
    assert np.array_equal(g1, c1) and np.array_equal(g2, c2)
    m.load_sums(SumStruct(n, hdr.count, hdr.blength, hdr.s2length, hdr.remainder, c1, c2), csum,
                seed)
    got, gfa, fsum = _stream_match(m, src, feeds, 1 << 20, 2, file_csum=csum)
    # the other XXH3 width through the device-contribution path too
    got2, _, fsum2 = _stream_match(m, src, feeds[::-1], 1 << 20, 3, file_csum=7)
    m.close()
    assert got == want and got2 == want
    assert gfa == fa
    assert fsum == _file_sum_want(src, csum) and fsum2 == _file_sum_want(src, 7)


@pytest.mark.parametrize("slen", [0, 1, 5000, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (2 << 20) + 77])
def test_stream_edge_lengths(gpu, slen):
    """Empty file, a file shorter than one block, exactly one piece, one byte
    past it (a second piece holding only halo bytes' owner), fed in one
    pinned buffer: the streamed walk equals the C hash_search; the one-shot
    vs_rsync_match (which now streams) agrees too."""
    import torch
    from volsync_amd import Matcher, SumStruct, match_sums, sum_sizes_sqroot
    n = (3 << 20) + 99
    basis = O.synth(72, 0, n)
    hdr = sum_sizes_sqroot(n, 16384)
    src0 = np.concatenate([basis[5000:], basis[:5000]])
    src = src0[:slen]
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, R.CSUM_XXH3_128, SEED)
    want, fa = O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, R.CSUM_XXH3_128, SEED)
    s = SumStruct(n, hdr.count, hdr.blength, hdr.s2length, hdr.remainder, c1, c2)
    pin = torch.empty(max(slen, 1), dtype=torch.uint8, pin_memory=True)
    if slen:
        pin[:slen].copy_(torch.from_numpy(src))
    m = Matcher()
    m.load_sums(s, R.CSUM_XXH3_128, SEED)
    m.match_begin(slen, 1 << 20, 2, 8)
    if slen:
        m.match_feed(pin.data_ptr(), slen)
    got = []
    while (r := m.match_next()) is not None:
        got.extend(r)
    nm, gfa, fsum = m.match_end()
    st = m.match_stream_stats()
    m.close()
    assert got == want and nm == len(want) and gfa == fa
    assert fsum == _file_sum_want(src, 8)   # 0, <= 240 and long files
    assert st["pinned_bytes"] == slen
    assert match_sums(src, s, R.CSUM_XXH3_128, SEED) == want


def test_stream_errors(gpu):
    """Out-of-sequence and over-length calls fail cleanly (VS_ERR_STATE /
    VS_ERR_ARG) and leave the handle usable."""
    from volsync_amd import Matcher, SumStruct, VsError, sum_sizes_sqroot
    m = Matcher()
    with pytest.raises(VsError):
        m.match_begin(100)          # no table loaded
    n = 1 << 20
    basis = O.synth(73, 0, n)
    hdr = sum_sizes_sqroot(n)
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, R.CSUM_XXH3_128, SEED)
    m.load_sums(SumStruct(n, hdr.count, hdr.blength, hdr.s2length, hdr.remainder, c1, c2),
                R.CSUM_XXH3_128, SEED)
    m.match_begin(1000)
    with pytest.raises(VsError):
        m.match_feed(np.zeros(1001, np.uint8))   # past the length given to begin
    m.match_feed(basis[:600])
    with pytest.raises(VsError):
        m.match_end()                            # 400 bytes still to come
    m.match_feed(basis[600:1000])
    assert m.match_end()[0] == len(O.rsync_match(basis[:1000], c1, c2, hdr.blength,
                                                 hdr.remainder, R.CSUM_XXH3_128, SEED)[0])
    m.match_begin(n)                              # a new stream on the same handle
    m.match_feed(basis)
    got = []
    while (r := m.match_next()) is not None:
        got.extend(r)
    m.close()
    assert got == [(i * hdr.blength, i) for i in range(hdr.count)]
