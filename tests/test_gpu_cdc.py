"""GPU parity tests: the HIP path (through the C ABI) against the oracle and fixtures.

Bar: bit-exact chunk boundaries (Start, Length), Cut values and SHA-256 blob IDs.
"""
import hashlib
import io
import os

import numpy as np
import pytest

from oracle import cdc_ref as P
from tests import golden_util as G
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

MIN, MAX = P.MIN_SIZE, P.MAX_SIZE


def to_dev(arr: np.ndarray):
    import torch
    t = torch.empty(max(len(arr), 16), dtype=torch.uint8, device="cuda")
    if len(arr):
        t[: len(arr)].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t


def dev_chunks(data: np.ndarray, pol, mn, mx, ab, dc=None):
    from volsync_amd import DeviceChunker
    own = dc is None
    dc = dc or DeviceChunker(pol, mn, mx, ab)
    t = to_dev(data)
    n, consumed = dc.process(t.data_ptr(), len(data), 0, True)
    assert consumed == len(data)
    ch = dc.chunks(0, n)
    if own:
        dc.close()
    return [(c.Start, c.Length, c.Cut, c.ID.hex()) for c in ch]


@pytest.mark.parametrize("path", G.fixtures(), ids=lambda p: os.path.basename(p))
def test_device_vs_golden(gpu, path):
    doc = G.load(path)
    data = G.make_input(doc["input"]) if "1g" not in path else O.synth(1, 0, 1 << 30)
    pol, mn, mx, ab = G.params(doc)
    assert dev_chunks(data, pol, mn, mx, ab) == G.expected(doc)


@pytest.mark.parametrize("path", [p for p in G.fixtures() if "1g" not in p and "eof_" not in p],
                         ids=lambda p: os.path.basename(p))
def test_stream_chunker_vs_golden(gpu, path):
    """The Chunker mirror (New/Next) with small reads and batches: multi-batch carry-over."""
    from volsync_amd import EOF, NewWithBoundaries
    doc = G.load(path)
    data = G.make_input(doc["input"])
    pol, mn, mx, ab = G.params(doc)
    ck = NewWithBoundaries(io.BytesIO(data.tobytes()), pol, mn, mx, read_size=3 << 20,
                           batch_bytes=5 << 20)
    ck.SetAverageBits(ab)
    got = []
    buf = bytearray()
    while True:
        try:
            c = ck.Next(buf)
        except EOF:
            break
        assert bytes(c.Data) == data[c.Start:c.Start + c.Length].tobytes()
        assert hashlib.sha256(c.Data).digest() == c.ID
        got.append((c.Start, c.Length, c.Cut, c.ID.hex()))
    ck.close()
    assert got == G.expected(doc)


def test_stream_chunker_bounded_hold(gpu):
    """A Chunker with a bound on held stream bytes (vs_cdc_next_wait, ADVICE r02:
    the Go binding's per-Chunker memory): same chunks as the oracle, and the
    bytes held never pass max(bound, 2 batches + 2 MaxSize) + one read."""
    from volsync_amd import EOF, New
    n = 160 << 20
    data = O.synth(7, 0, n)
    read, batch, bound = 4 << 20, 16 << 20, 20 << 20
    ck = New(io.BytesIO(data.tobytes()), P.TEST_POL, read_size=read, batch_bytes=batch,
             max_pending=bound)
    got = []
    while True:
        try:
            c = ck.Next()
        except EOF:
            break
        got.append((c.Start, c.Length, c.Cut, c.ID.hex()))
    held = ck.max_held
    ck.close()
    assert got == O.cdc_hash(data, P.TEST_POL, MIN, MAX, 20)
    assert held <= max(bound, 2 * batch + 2 * MAX + (1 << 20)) + read, held


def test_stream_pol_zero_error(gpu):
    import volsync_amd
    ck = volsync_amd.New(io.BytesIO(b"abc"), 0)
    with pytest.raises(volsync_amd.VsError, match="not initialized"):
        ck.Next()


def test_reader_error_propagates(gpu):
    import volsync_amd

    class Bad(io.RawIOBase):
        def read(self, n=-1):
            raise IOError("disk on fire")

    ck = volsync_amd.New(Bad(), P.TEST_POL)
    with pytest.raises(IOError, match="disk on fire"):
        ck.Next()


@pytest.mark.parametrize("seed,n,mn,mx,ab", [
    (31, 3 << 20, 1024, 4096, 10),
    (32, (7 << 20) + 13, 4096, 16384, 12),
    (33, 20 << 20, 64, 64, 5),              # min == max == window: every chunk forced
    (34, 5 << 20, 2048, 1 << 20, 16),
    (35, 33 << 20, 65536, 1 << 20, 14),     # many segments
    (36, 9 << 20, 1024, 2048, 30),          # rare candidates -> all forced
    (37, 6 << 20, 4096, 8192, 33),          # 64-bit splitmask path
])
def test_device_vs_oracle_random(gpu, seed, n, mn, mx, ab):
    data = O.synth(seed, 0, n)
    assert dev_chunks(data, P.TEST_POL, mn, mx, ab) == O.cdc_hash(data, P.TEST_POL, mn, mx, ab)


def test_dense_zero_volume_overflows_pool(gpu):
    """An all-zero 96 MiB volume: every position is a candidate; exercises the
    dense-strip bitmask pool and its regrow path."""
    data = np.zeros(96 << 20, np.uint8)
    data[50 << 20:(50 << 20) + 1000] = 7
    assert dev_chunks(data, P.TEST_POL, MIN, MAX, 20) == O.cdc_hash(data, P.TEST_POL, MIN, MAX, 20)


def test_periodic_data_small_min(gpu):
    base = O.synth(40, 0, 777)
    data = np.tile(base, (4 << 20) // 777 + 1)[: 4 << 20].copy()
    assert dev_chunks(data, P.TEST_POL, 1024, 8192, 6) == O.cdc_hash(data, P.TEST_POL, 1024, 8192, 6)


def test_handle_reuse_across_sizes(gpu):
    from volsync_amd import DeviceChunker
    dc = DeviceChunker(P.TEST_POL, 4096, 16384, 12)
    for seed, n in [(50, 8 << 20), (51, 100), (52, 1 << 20), (53, 0), (54, 12 << 20)]:
        data = O.synth(seed, 0, n)
        assert dev_chunks(data, P.TEST_POL, 4096, 16384, 12, dc=dc) == \
            O.cdc_hash(data, P.TEST_POL, 4096, 16384, 12)
    dc.close()


def test_sharded_equals_single(gpu):
    """Byte-range shards with halos + exit exchange == one-device result (the
    multi-GPU protocol of volsync_amd.shard, run in one process)."""
    from volsync_amd import DeviceChunker
    from volsync_amd.shard import ShardSpec, run_shards_local
    n = 40 << 20
    mn, mx, ab = 16384, 1 << 20, 14
    data = O.synth(60, 0, n)
    want = O.cdc_hash(data, P.TEST_POL, mn, mx, ab)
    for world in (2, 3, 5):
        specs = ShardSpec.split(n, world, mx)
        handles = [DeviceChunker(P.TEST_POL, mn, mx, ab) for _ in range(world)]
        bufs = [to_dev(data[s.data_lo:s.data_hi]) for s in specs]
        got = run_shards_local(handles, specs, [b.data_ptr() for b in bufs])
        for h in handles:
            h.close()
        assert [(c.Start, c.Length, c.Cut, c.ID.hex()) for c in got] == want


def test_sha256_batch_vs_hashlib(gpu):
    from volsync_amd import sha256_batch
    rng = np.random.default_rng(3)
    buf = O.synth(70, 0, 3 << 20).tobytes()
    offs, lens = [], []
    for n in list(range(0, 130)) + [4096, 65536, 65537, 100000, 1 << 20]:
        o = int(rng.integers(0, len(buf) - n))
        offs.append(o)
        lens.append(n)
    got = sha256_batch(buf, offs, lens)
    for o, n, g in zip(offs, lens, got):
        assert g == hashlib.sha256(buf[o:o + n]).digest()


@pytest.mark.parametrize("iso", [1, 0])
@pytest.mark.parametrize("pct", [0, 1, 50, 100, -1])
def test_sha256_drain_modes_vs_hashlib(gpu, pct, iso):
    """The final drain's latency (quad, 4 lanes per chain) and split tiles:
    VS_OPT_SHA_QUAD_PCT 0 is split only, 1 puts nearly every chain in quad
    tiles, 50 / 100 mix the two, -1 the automatic rule; VS_OPT_SHA_ISOLATE 1
    runs the quad tiles as their own launch, a CU each, beside the split
    launch, 0 as one launch; every length class from 0 to 1 MiB."""
    import torch
    from volsync_amd import DeviceSha256
    from volsync_amd._lib import VS_OPT_SHA_ISOLATE, VS_OPT_SHA_QUAD_PCT
    rng = np.random.default_rng(pct + 11)
    host = O.synth(71, 0, 4 << 20)
    buf = host.tobytes()
    lens = [int(x) for x in rng.integers(0, 200, 300)] + [55, 56, 63, 64, 65, 119, 120] + \
        [int(x) for x in rng.integers(1 << 19, 1 << 20, 40)]
    offs = [int(rng.integers(0, len(buf) - n)) for n in lens]
    d = torch.from_numpy(host).cuda()
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
    sh = DeviceSha256(0)
    sh.set_option(VS_OPT_SHA_QUAD_PCT, pct)
    sh.set_option(VS_OPT_SHA_ISOLATE, iso)
    sh.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), len(lens), out.data_ptr(), None)
    torch.cuda.synchronize()
    sh.close()
    got = out.cpu().numpy().reshape(-1, 32)
    for o, n, g in zip(offs, lens, got):
        assert g.tobytes() == hashlib.sha256(buf[o:o + n]).digest(), n


def test_sha256_drain_shared_tail_vs_hashlib(gpu):
    """A tail-bound drain with more long chains than the isolated tiles take
    (16 per two CUs): the first cap chains run in sha_iso_kernel, a CU per
    tile, and the rest as latency tiles of the split launch beside the split
    tiles (ShaSliceArgs.quad_lo; the C3 rank's drain, profiles/r06_iso32).
    vs_sha256_drain_stats shows both parts ran; every digest = hashlib's."""
    import torch
    from volsync_amd import DeviceSha256
    from volsync_amd._lib import VS_OPT_SHA_ISOLATE, VS_OPT_SHA_QUAD_PCT
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    cap = cus // 2 * 16
    n_long = cap + cap // 2
    rng = np.random.default_rng(29)
    host = O.synth(73, 0, 16 << 20)
    buf = host.tobytes()
    lens = [int(x) for x in rng.integers(192 << 10, 320 << 10, n_long)] + \
        [int(x) for x in rng.integers(0, 4096, 500)]
    offs = [int(rng.integers(0, len(buf) - n)) for n in lens]
    d = torch.from_numpy(host).cuda()
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
    sh = DeviceSha256(0)
    sh.set_option(VS_OPT_SHA_QUAD_PCT, -1)
    sh.set_option(VS_OPT_SHA_ISOLATE, 1)
    sh.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), len(lens), out.data_ptr(), None)
    torch.cuda.synchronize()
    latency, isolated = sh.drain_stats()
    sh.close()
    assert isolated == cap, (latency, isolated, cap)
    assert cap < latency <= n_long, (latency, isolated, n_long)
    got = out.cpu().numpy().reshape(-1, 32)
    for o, n, g in zip(offs, lens, got):
        assert g.tobytes() == hashlib.sha256(buf[o:o + n]).digest(), n


def test_fence_distinct_volumes(gpu):
    """bench.py --distinct: volumes of three seeds in rotation, step k fenced
    on step k - 3 (vs_cdc_fence) with a short slice budget, so the fences
    drain chains still queued; every batch's chunk list (Start, Length, Cut,
    blob ID) equals the oracle's for its volume."""
    import torch
    from volsync_amd import DeviceChunker, TestPol
    n = 48 << 20
    seeds = (2, 7, 8)
    host = [O.synth(sd, 0, n) for sd in seeds]
    dev = [torch.from_numpy(h).cuda() for h in host]
    want = [O.cdc_hash(h, TestPol, 512 << 10, 8 << 20, 20) for h in host]
    torch.cuda.synchronize()
    dc = DeviceChunker(TestPol, 512 << 10, 8 << 20, 20, device=0)
    dc.set_hash_slice(64)
    first, _ = dc.batches()
    got_n = []
    for j in range(9):
        if j >= 3:
            dc.fence(first + j - 3)
        nch, _ = dc.process(dev[j % 3].data_ptr(), n, 0, True)
        got_n.append(nch)
    for j in range(6, 9):
        got = [(c.Start, c.Length, c.Cut, c.ID.hex()) for c in dc.batch_chunks(first + j, 0, got_n[j])]
        assert got == want[j % 3], (j, len(got), len(want[j % 3]))
    with pytest.raises(Exception):
        dc.fence(first + 9)      # not finished yet
    dc.close()


def test_small_files_device_sha(gpu):
    """C5 shape (scaled): many 4-64 KiB files packed in one device buffer, ~50%
    duplicate payloads; one blob ID per file from the work-queue kernel."""
    import torch
    from volsync_amd import DeviceSha256
    rng = np.random.default_rng(6)
    nfiles = 20000
    sizes = rng.integers(4096, 65537, nfiles)
    sizes[::97] = rng.integers(0, 200, len(sizes[::97]))   # some tiny / empty files
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    total = int(sizes.sum())
    pool = O.synth(8, 0, 4 << 20)
    buf = np.empty(total, np.uint8)
    for i, (o, n) in enumerate(zip(offs.tolist(), sizes.tolist())):
        src = int(rng.integers(0, 2000)) * 1024      # dedup-heavy: few distinct payloads
        buf[o:o + n] = pool[src:src + n]
    d = to_dev(buf)
    do = torch.from_numpy(offs.astype(np.int64)).cuda()
    dl = torch.from_numpy(sizes.astype(np.int32)).cuda()
    out = torch.zeros((nfiles, 32), dtype=torch.uint8, device="cuda")
    sh = DeviceSha256()
    sh.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), nfiles, out.data_ptr())
    torch.cuda.synchronize()
    sh.close()
    got = out.cpu().numpy()
    for i in range(0, nfiles, 7):
        o, n = int(offs[i]), int(sizes[i])
        assert bytes(got[i]) == hashlib.sha256(buf[o:o + n].tobytes()).digest(), i


def test_synth_device_matches_oracle(gpu):
    import torch
    from volsync_amd import synth_fill_device
    for seed, off, n in [(1, 0, 1 << 20), (9, 13, 100001), (2, (1 << 36) - 5, 4099)]:
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        synth_fill_device(t.data_ptr(), seed, off, n)
        torch.cuda.synchronize()
        assert (t.cpu().numpy() == O.synth(seed, off, n)).all()


@pytest.mark.timeout(900)
def test_full_size_c2_properties(gpu):
    """Config C2 size (64 GiB, seed 2, default parameters) through properties
    and then exactly:
    chunks tile the volume, lengths obey min/max, Cut & mask == 0 unless forced,
    and sampled chunks match the oracle (cut rule from the chunk start) and
    hashlib (blob ID)."""
    import torch
    from volsync_amd import DeviceChunker, synth_fill_device
    n = 64 << 30
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    synth_fill_device(t.data_ptr(), 2, 0, n)
    dc = DeviceChunker(P.TEST_POL, MIN, MAX, 20)
    nch, consumed = dc.process(t.data_ptr(), n, 0, True)
    assert consumed == n
    ch = dc.chunks(0, nch)
    dc.close()
    assert 40000 < nch < 48000
    pos = 0
    for i, c in enumerate(ch):
        assert c.Start == pos
        pos += c.Length
        if i < nch - 1:
            assert MIN <= c.Length <= MAX
            if c.Length < MAX:
                assert c.Cut & ((1 << 20) - 1) == 0
    assert pos == n
    rng = np.random.default_rng(0)
    picks = sorted(set([0, nch - 1] + [int(x) for x in rng.integers(0, nch, 12)]))
    for i in picks:
        c = ch[i]
        hi = min(n, c.Start + MAX + 64)
        host = t[c.Start:hi].cpu().numpy()
        final = hi == n
        ref = O.cdc_hash(host, P.TEST_POL, MIN, MAX, 20)[0]
        if not final and ref[1] >= len(host):
            continue
        assert (c.Start + ref[0], ref[1], ref[2], ref[3]) == (c.Start, c.Length, c.Cut, c.ID.hex())
    del t
    torch.cuda.empty_cache()
    # the whole 43.7 K-row list, exactly: (Start, Length, Cut, blob ID) of
    # every chunk against the multi-threaded oracle over the same stream
    # (candidates found in parallel byte ranges, sequential min/max selection,
    # parallel SHA-256; oracle/cdc_ref.c ref_cdc_synth_mt, pinned against the
    # sequential Chunker.Next restatement by tests/test_oracle.py)
    threads = max(1, min(16, os.cpu_count() or 1))
    s, ln, cu, ids = O.cdc_synth_mt(2, n, P.TEST_POL, MIN, MAX, 20, threads)
    assert nch == len(s)
    assert [c.Start for c in ch] == s.tolist()
    assert [c.Length for c in ch] == ln.tolist()
    assert [c.Cut for c in ch] == cu.tolist()
    assert [c.ID for c in ch] == [bytes(r) for r in ids]


@pytest.mark.parametrize("budget", [1, 2, 3, 7, 100, 0])
def test_hash_slice_budgets(gpu, budget):
    """Time-sliced SHA-256 engine: chains carry their midstate across slices
    of `budget` blocks (1 block per batch = the most slices); the blob IDs
    must not depend on the slicing."""
    from volsync_amd import DeviceChunker
    mn, mx, ab = 4096, 65536, 13
    dc = DeviceChunker(P.TEST_POL, mn, mx, ab)
    dc.set_hash_slice(budget)
    for seed, n in [(80, (3 << 20) + 5), (81, 70000), (82, 1 << 20)]:
        data = O.synth(seed, 0, n)
        assert dev_chunks(data, P.TEST_POL, mn, mx, ab, dc=dc) == O.cdc_hash(data, P.TEST_POL, mn, mx, ab)
    dc.close()


@pytest.mark.parametrize("budget", [5, 8192])
def test_pipelined_batches(gpu, budget):
    """Batches finished back to back on one handle without waiting (the bench
    pattern): each batch's chunk list and blob IDs equal the oracle's, read
    back after the engine drained."""
    from volsync_amd import DeviceChunker
    mn, mx, ab = 16384, 1 << 18, 15
    dc = DeviceChunker(P.TEST_POL, mn, mx, ab)
    dc.set_hash_slice(budget)
    datas, bufs, counts = [], [], []
    first, ring = dc.batches()
    for i in range(6):
        data = O.synth(90 + i, 0, (4 << 20) + 977 * i)
        t = to_dev(data)
        n, consumed = dc.process(t.data_ptr(), len(data), 0, True)
        assert consumed == len(data)
        datas.append(data)
        bufs.append(t)      # device data must outlive its batch's hashing
        counts.append(n)
    done, ring = dc.batches()
    assert done == first + 6
    for i in range(max(0, 6 - ring), 6):
        got = [(c.Start, c.Length, c.Cut, c.ID.hex())
               for c in dc.batch_chunks(first + i, 0, counts[i])]
        assert got == O.cdc_hash(datas[i], P.TEST_POL, mn, mx, ab)
    dc.close()


@pytest.mark.parametrize("min_chains,drain", [(1, 3), (1, 0), (40, 2)])
def test_wide_mode_pipelined(gpu, min_chains, drain):
    """Throughput mode of the SHA-256 engine (whole-SHA wavefronts): forced on
    from `min_chains` active chunks, with drains of `drain` blocks per launch
    and a split-mode finish below the threshold; pipelined batches under
    budgeted slices of 5 blocks.  Blob IDs must equal the oracle's."""
    from volsync_amd import DeviceChunker
    mn, mx, ab = 16384, 1 << 18, 15
    dc = DeviceChunker(P.TEST_POL, mn, mx, ab)
    dc.set_hash_slice(5)
    dc.set_hash_wide(min_chains, drain)
    datas, bufs, counts = [], [], []
    first, ring = dc.batches()
    for i in range(5):
        data = O.synth(190 + i, 0, (3 << 20) + 1213 * i)
        t = to_dev(data)
        n, consumed = dc.process(t.data_ptr(), len(data), 0, True)
        datas.append(data)
        bufs.append(t)
        counts.append(n)
    dc.wait()
    done, ring = dc.batches()
    for i in range(max(0, 5 - ring), 5):
        got = [(c.Start, c.Length, c.Cut, c.ID.hex())
               for c in dc.batch_chunks(first + i, 0, counts[i])]
        assert got == O.cdc_hash(datas[i], P.TEST_POL, mn, mx, ab)
    dc.close()


@pytest.mark.parametrize("drain", [1, 2, 4096])
def test_wide_mode_blobs_vs_hashlib(gpu, drain):
    """Throughput mode over blobs of every length 0..200 at every alignment
    (padding in one or two blocks, misaligned starts) plus 4-64 KiB files."""
    import torch
    from volsync_amd import DeviceSha256
    rng = np.random.default_rng(11)
    buf = O.synth(71, 0, 2 << 20)
    lens = list(range(0, 201)) + [int(x) for x in rng.integers(4096, 65537, 300)]
    offs = [int(rng.integers(0, len(buf) - n)) for n in lens]
    d = to_dev(buf)
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = torch.zeros((len(lens), 32), dtype=torch.uint8, device="cuda")
    sh = DeviceSha256()
    sh.set_wide(1, drain)
    sh.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), len(lens), out.data_ptr())
    torch.cuda.synchronize()
    sh.close()
    got = out.cpu().numpy()
    raw = buf.tobytes()
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert bytes(got[i]) == hashlib.sha256(raw[o:o + n]).digest(), (i, o, n)


def test_reset_drains_queued_chains(gpu):
    """vs_cdc_reset to a different max_size changes the ring length;
    chains that an earlier batch left queued in the time-sliced engine (budget
    3 blocks, no wait) must be hashed to the end before the slots are released,
    else their next slice writes blob IDs into freed memory.  The batch after
    the reset must equal the oracle."""
    from volsync_amd import DeviceChunker
    mn, ab = 8192, 13
    dc = DeviceChunker(P.TEST_POL, mn, 1 << 17, ab)
    dc.set_hash_slice(3)
    a = O.synth(401, 0, (6 << 20) + 31)
    ta = to_dev(a)
    dc.process(ta.data_ptr(), len(a), 0, True)     # no wait: chains stay queued
    dc.reset(P.TEST_POL, mn, 1 << 19, ab)          # ring length changes with max_size
    b = O.synth(402, 0, (5 << 20) + 77)
    assert dev_chunks(b, P.TEST_POL, mn, 1 << 19, ab, dc=dc) == \
        O.cdc_hash(b, P.TEST_POL, mn, 1 << 19, ab)
    dc.close()
    del ta


def _stream_pinned(data: np.ndarray, pol, mn, mx, ab, read, batch=None, reuse=None):
    """Feed `data` from pinned host memory through vs_cdc_feed / vs_cdc_next
    (the streaming drop-in path, as gpuchunker's Next drives it)."""
    import ctypes
    import torch
    from volsync_amd._lib import VS_EOF, VsChunk, check, lib
    host = torch.empty(max(len(data), 1), dtype=torch.uint8, pin_memory=True)
    host[: len(data)].copy_(torch.from_numpy(np.ascontiguousarray(data)))
    h = reuse or ctypes.c_void_p()
    if reuse is None:
        check(lib.vs_cdc_open(0, pol, mn, mx, ab, ctypes.byref(h)))
    else:
        check(lib.vs_cdc_reset(h, pol, mn, mx, ab))
    if batch:
        check(lib.vs_cdc_set_batch_bytes(h, batch))
    out = (VsChunk * 64)()
    got = ctypes.c_size_t(0)
    res = []

    def take():
        while True:
            rc = lib.vs_cdc_next(h, out, 64, ctypes.byref(got))
            if rc == VS_EOF:
                return True
            check(rc)
            if not got.value:
                return False
            res.extend((int(c.start), int(c.length), int(c.cut), bytes(c.id).hex())
                       for c in out[: got.value])

    for off in range(0, len(data), read):
        check(lib.vs_cdc_feed(h, ctypes.c_void_p(host.data_ptr() + off),
                              min(read, len(data) - off), 0))
        take()
    check(lib.vs_cdc_feed(h, None, 0, 1))
    assert take()
    st = (ctypes.c_double * 8)()
    check(lib.vs_cdc_stream_stats(h, st))
    return res, h, list(st)


def test_stream_1g_golden_pageable(gpu):
    """C1 (1 GiB, seed 1, default parameters) through the Chunker mirror with
    64 MiB reads from pageable memory (staged through the pinned buffers) and
    the default 512 MiB batches: the committed golden chunk list exactly."""
    from volsync_amd import EOF, NewWithBoundaries
    doc = G.load(os.path.join(G.GOLDEN, "cdc_synth1_1g.json"))
    data = G.make_input(doc["input"])
    pol, mn, mx, ab = G.params(doc)
    ck = NewWithBoundaries(io.BytesIO(data.tobytes()), pol, mn, mx, read_size=64 << 20,
                           batch_bytes=512 << 20)
    ck.SetAverageBits(ab)
    got = []
    while True:
        try:
            c = ck.Next()
        except EOF:
            break
        got.append((c.Start, c.Length, c.Cut, c.ID.hex()))
    ck.close()
    assert got == G.expected(doc)


def test_stream_1g_golden_pinned(gpu):
    """The same 1 GiB fixture fed from pinned host memory (direct DMA) in
    64 MiB reads with 128 MiB batches."""
    import ctypes
    from volsync_amd._lib import lib
    doc = G.load(os.path.join(G.GOLDEN, "cdc_synth1_1g.json"))
    data = G.make_input(doc["input"])
    pol, mn, mx, ab = G.params(doc)
    got, h, st = _stream_pinned(data, pol, mn, mx, ab, 64 << 20, batch=128 << 20)
    lib.vs_cdc_close(h)
    assert got == G.expected(doc)
    assert st[0] == len(data) and st[1] == 0 and st[3] >= 8


def test_stream_ring_wraps_and_reuse(gpu):
    """Small batches (2*MaxSize + 1 MiB) so the 24-slot ring wraps many times
    (backpressure: a batch's slot is reused only after its chunks were
    collected); then the handle is reset and reused for a second stream."""
    import ctypes
    from volsync_amd._lib import lib
    mn, mx, ab = 4096, 1 << 20, 16
    data = O.synth(41, 0, (100 << 20) + 12345)
    want = O.cdc_hash(data, P.TEST_POL, mn, mx, ab)
    got, h, st = _stream_pinned(data, P.TEST_POL, mn, mx, ab, 5 << 20, batch=1)
    assert got == want and st[3] > 30
    data2 = O.synth(42, 0, 7 << 20)
    got2, h, _ = _stream_pinned(data2, P.TEST_POL, mn, mx, ab, 1 << 20, batch=1, reuse=h)
    lib.vs_cdc_close(h)
    assert got2 == O.cdc_hash(data2, P.TEST_POL, mn, mx, ab)


def test_stream_empty_and_tiny(gpu):
    import ctypes
    from volsync_amd._lib import lib
    for n in (0, 1, 63, 100):
        data = O.synth(43, 0, n)
        got, h, _ = _stream_pinned(data, P.TEST_POL, MIN, MAX, 20, 1 << 20)
        lib.vs_cdc_close(h)
        assert got == O.cdc_hash(data, P.TEST_POL, MIN, MAX, 20)


def test_blob_dedup_vs_hashlib(gpu):
    """SaveBlob's dedup seam (vs_blob_dedup) on the 20 K-file C5-shape batch:
    the distinct-ID count and every blob's first occurrence, against hashlib
    IDs deduplicated on the host; plus identical, empty and single inputs."""
    import torch
    from volsync_amd import DeviceSha256
    rng = np.random.default_rng(7)
    nfiles = 20000
    sizes = rng.integers(4096, 65537, nfiles)
    sizes[::97] = rng.integers(0, 3, len(sizes[::97]))      # empty / 1-2 byte files
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    pool = O.synth(8, 0, 4 << 20)
    buf = np.empty(int(sizes.sum()), np.uint8)
    for o, n in zip(offs.tolist(), sizes.tolist()):
        src = int(rng.integers(0, 3000)) * 1024
        buf[o:o + n] = pool[src:src + n]
    want_ids = [hashlib.sha256(buf[o:o + n].tobytes()).digest()
                for o, n in zip(offs.tolist(), sizes.tolist())]
    seen, want_first = {}, []
    for i, d in enumerate(want_ids):
        want_first.append(seen.setdefault(d, i))
    d = to_dev(buf)
    do = torch.from_numpy(offs.astype(np.int64)).cuda()
    dl = torch.from_numpy(sizes.astype(np.int32)).cuda()
    ids = torch.zeros((nfiles, 32), dtype=torch.uint8, device="cuda")
    first = torch.zeros(nfiles, dtype=torch.int32, device="cuda")
    sh = DeviceSha256()
    sh.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), nfiles, ids.data_ptr())
    nu = sh.dedup(ids.data_ptr(), nfiles, first.data_ptr())
    assert [bytes(r) for r in ids.cpu().numpy()] == want_ids
    assert nu == len(seen)
    assert first.cpu().numpy().tolist() == want_first
    # one ID repeated 50 000 times, a single blob, no blobs
    same = torch.tensor(list(want_ids[5]) * 50000, dtype=torch.uint8, device="cuda").view(-1, 32)
    f2 = torch.full((50000,), -1, dtype=torch.int32, device="cuda")
    assert sh.dedup(same.data_ptr(), 50000, f2.data_ptr()) == 1
    assert int(f2.max()) == 0 and int(f2.min()) == 0
    assert sh.dedup(ids.data_ptr(), 1, first.data_ptr()) == 1
    assert sh.dedup(ids.data_ptr(), 0, first.data_ptr()) == 0
    sh.close()


@pytest.mark.parametrize("n", [1_000_000, 999_983])
def test_blob_dedup_c5_size(gpu, n):
    """vs_blob_dedup at C5's own batch size (1 M blob IDs drawn from n/2 distinct
    ones, as the C5 bench makes them) and at an odd size: first occurrences and
    the distinct count against numpy's first-index unique.  Some IDs share
    their first 8 bytes (the sort key) but differ later."""
    import torch
    from volsync_amd import DeviceSha256
    rng = np.random.default_rng(11)
    distinct = rng.integers(0, 256, (n // 2, 32), dtype=np.uint8)
    distinct[1::1000, :8] = distinct[0:-1:1000, :8][: len(distinct[1::1000])]
    ids_h = distinct[rng.integers(0, len(distinct), n)]
    _, first_idx, inv = np.unique(ids_h.view(np.dtype((np.void, 32))).ravel(),
                                  return_index=True, return_inverse=True)
    want_first = first_idx[inv.ravel()]
    ids = torch.from_numpy(ids_h).cuda()
    first = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    sh = DeviceSha256()
    for _ in range(2):    # the second call reuses the scratch
        assert sh.dedup(ids.data_ptr(), n, first.data_ptr()) == len(first_idx)
        assert np.array_equal(first.cpu().numpy(), want_first)
    sh.close()


@pytest.mark.parametrize("n,known_frac", [(1_000_000, 0.5), (77_777, 0.0), (50_000, 1.0)])
def test_blob_dedup_known_index(gpu, n, known_frac):
    """SaveBlob against the repository's index (vs_blob_index_sort +
    vs_blob_dedup_known; restic v0.13.1 Repository.SaveBlob skips a blob the
    master index holds, /root/reference/mover-restic/entry.sh:43-65 re-runs
    backups into an initialised repository): 1 M blob IDs from 500 K distinct
    ones, half of the distinct IDs in a 'known' index padded with IDs the
    batch never uses (some sharing a batch ID's first 8 bytes, the sort key);
    every blob's mark (known, or its first occurrence) and the count of new
    distinct IDs against a host set."""
    import torch
    from volsync_amd import DeviceSha256
    from volsync_amd._lib import VS_DEDUP_KNOWN
    rng = np.random.default_rng(13 + n)
    distinct = rng.integers(0, 256, (n // 2, 32), dtype=np.uint8)
    ids_h = distinct[rng.integers(0, len(distinct), n)]
    nk = int(len(distinct) * known_frac)
    extra = rng.integers(0, 256, (max(nk // 4, 1), 32), dtype=np.uint8)
    extra[::3, :8] = distinct[: len(extra[::3]), :8]          # same prefix, other ID
    known_h = np.concatenate([distinct[rng.permutation(len(distinct))[:nk]], extra])
    known_h = known_h[rng.permutation(len(known_h))]
    kset = {bytes(r) for r in known_h}
    first_seen, want, new = {}, np.empty(n, np.int64), 0
    for i, r in enumerate(ids_h):
        b = bytes(r)
        if b in kset:
            want[i] = VS_DEDUP_KNOWN
        else:
            f = first_seen.setdefault(b, i)
            want[i] = f
            new += f == i
    ids = torch.from_numpy(ids_h).cuda()
    known = torch.from_numpy(known_h).cuda()
    first = torch.zeros(n, dtype=torch.int32, device="cuda")
    sh = DeviceSha256()
    sh.index_sort(known.data_ptr(), len(known_h))
    ks = known.cpu().numpy()
    keys = ks[:, :8].copy().view(">u8").ravel()
    assert (np.diff(keys.astype(np.uint64)) >= 0).all()            # sorted by prefix
    assert {bytes(r) for r in ks} == kset and len(ks) == len(known_h)   # a permutation
    for _ in range(2):
        assert sh.dedup_known(ids.data_ptr(), n, known.data_ptr(), len(known_h),
                              first.data_ptr()) == new
        assert np.array_equal(first.cpu().numpy().view(np.uint32).astype(np.int64), want)
    # an empty index is vs_blob_dedup
    assert sh.dedup_known(ids.data_ptr(), n, 0, 0, first.data_ptr()) == len(first_seen) + \
        len({bytes(r) for r in ids_h} & kset)
    sh.close()


def test_sha256_blocks_syncthing(gpu):
    """syncthing's scanner blocks: SHA-256 of every block of a
    device buffer, for the block size lib/protocol picks and a larger one,
    against hashlib; a short last block and an empty buffer included."""
    import torch
    from volsync_amd import DeviceSha256, syncthing_block_size
    data = O.synth(71, 0, (5 << 20) + 333)
    d = to_dev(data)
    sh = DeviceSha256()
    for bs in (syncthing_block_size(len(data)), 1 << 20, 4096):
        n = (len(data) + bs - 1) // bs
        out = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
        assert sh.blocks(d.data_ptr(), len(data), bs, out.data_ptr()) == n
        torch.cuda.synchronize()
        got = [bytes(r) for r in out.cpu().numpy()]
        want = [hashlib.sha256(data[i * bs:(i + 1) * bs].tobytes()).digest() for i in range(n)]
        assert got == want, bs
    assert sh.blocks(d.data_ptr(), 0, 1 << 17, d.data_ptr()) == 0
    sh.close()


def test_blob_verify_restore(gpu):
    """Repository.LoadBlob's ID check on restore: blobs whose
    SHA-256 differs from the expected ID are flagged and counted."""
    import torch
    from volsync_amd import DeviceSha256
    rng = np.random.default_rng(9)
    sizes = rng.integers(0, 70000, 3000)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    data = O.synth(72, 0, int(sizes.sum()) + 16)
    want = np.stack([np.frombuffer(hashlib.sha256(data[o:o + n].tobytes()).digest(), np.uint8)
                     for o, n in zip(offs.tolist(), sizes.tolist())])
    corrupt = sorted(set(rng.integers(0, 3000, 9).tolist()))
    for i in corrupt:
        want[i, i % 32] ^= 0x5A
    d = to_dev(data)
    do = torch.from_numpy(offs).cuda()
    dl = torch.from_numpy(sizes.astype(np.int32)).cuda()
    dw = torch.from_numpy(want).cuda()
    bad = torch.zeros(3000, dtype=torch.int32, device="cuda")
    sh = DeviceSha256()
    assert sh.verify(d.data_ptr(), do.data_ptr(), dl.data_ptr(), 3000, dw.data_ptr(),
                     bad.data_ptr()) == len(corrupt)
    assert np.nonzero(bad.cpu().numpy())[0].tolist() == corrupt
    sh.close()
