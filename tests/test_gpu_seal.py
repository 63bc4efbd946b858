"""restic Key.Seal on the device vs oracle/seal_ref.py.

vs_seal_run_device encrypts every blob with AES-256-CTR under its own nonce
and computes its Poly1305-AES tag; the oracle is libcrypto AES + the RFC 8439
Poly1305 restatement, pinned by the standards' vectors in
test_seal_oracle.py.  Bit-exact comparisons on ciphertext and tags.
"""
import numpy as np
import pytest

from oracle import seal_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["fused", "separate"])
def seal_variant(request, monkeypatch):
    """Every test runs on both launch paths: the MAC fused into the CTR pass
    (default: per-lane Horner sums lifted by r^e and added per blob) and the
    separate CTR + one-wave-per-blob MAC kernels (VS_OPT_SEAL_FUSED = 0 on
    every Sealer the test opens)."""
    import volsync_amd.chunker as C
    from volsync_amd._lib import VS_OPT_SEAL_FUSED
    orig = C.Sealer.__init__
    fused = 1 if request.param == "fused" else 0

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.set_option(VS_OPT_SEAL_FUSED, fused)
    monkeypatch.setattr(C.Sealer, "__init__", init)
    return request.param


def _keys(seed):
    rng = np.random.default_rng(seed)
    return tuple(rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (32, 16, 16))


def _run(keys, data: np.ndarray, offs, lens, nonces: np.ndarray, in_place=False):
    import torch
    from volsync_amd import Sealer
    d = torch.from_numpy(data.copy()).cuda()
    out = d if in_place else torch.zeros_like(d)
    do = torch.from_numpy(np.asarray(offs, np.uint64).view(np.int64)).cuda()
    dl = torch.from_numpy(np.asarray(lens, np.uint32).view(np.int32)).cuda()
    dn = torch.from_numpy(nonces.reshape(-1).copy()).cuda()
    n = len(lens)
    macs = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device="cuda")
    s = Sealer(*keys)
    s.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), n, dn.data_ptr(), out.data_ptr(),
          macs.data_ptr())
    torch.cuda.synchronize()
    s.close()
    return out.cpu().numpy(), macs.cpu().numpy()[:16 * n].reshape(n, 16)


def _check(keys, data, offs, lens, nonces, ct, macs, which=None):
    for i in (range(len(lens)) if which is None else which):
        o, n = int(offs[i]), int(lens[i])
        want_ct, want_mac = S.seal(*keys, nonces[i].tobytes(), data[o:o + n].tobytes())
        assert ct[o:o + n].tobytes() == want_ct, (i, n)
        assert macs[i].tobytes() == want_mac, (i, n)


def test_seal_edge_lengths_and_counter_carries(gpu):
    keys = _keys(1)
    lens = [0, 1, 15, 16, 17, 31, 32, 33, 1000, 1023, 1024, 1025, 1039, 1040, 1041, 4096,
            (1 << 20) + 7, 1 << 20, 5]
    rng = np.random.default_rng(2)
    # odd gaps between blobs: unaligned blob offsets
    offs, pos = [], 3
    for n in lens:
        offs.append(pos)
        pos += n + int(rng.integers(0, 40))
    data = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    nonces[16] = np.frombuffer(b"\xff" * 15 + b"\xf0", np.uint8)             # 128-bit wrap
    nonces[17] = np.frombuffer(bytes(4) + b"\x00\x00\x00\x07" + b"\xff" * 8, np.uint8)  # 64-bit carry
    nonces[12] = np.frombuffer(b"\x12" * 8 + b"\x00\x00\x00\x00\xff\xff\xff\xfa", np.uint8)  # 32-bit carry
    ct, macs = _run(keys, data, offs, lens, nonces)
    _check(keys, data, offs, lens, nonces, ct, macs)
    # bytes outside the blobs are untouched (zero in the separate output)
    mask = np.ones(len(data), bool)
    for o, n in zip(offs, lens):
        mask[o:o + n] = False
    assert not ct[mask].any()


def test_seal_many_blobs_in_place(gpu):
    keys = _keys(3)
    rng = np.random.default_rng(4)
    lens = rng.integers(0, 9000, 4000)
    lens[::97] = 0
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ct, macs = _run(keys, data, offs, lens, nonces, in_place=True)
    _check(keys, data, offs, lens, nonces, ct, macs)


def test_seal_restic_sized_blobs(gpu):
    """restic chunker sizes (512 KiB .. 8 MiB): many waves per blob's CTR
    stream, one wave per blob's tag; a sample of blobs checked in full."""
    keys = _keys(5)
    rng = np.random.default_rng(6)
    lens = rng.integers(512 << 10, 8 << 20, 48)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ct, macs = _run(keys, data, offs, lens, nonces)
    _check(keys, data, offs, lens, nonces, ct, macs, which=[0, 1, 23, 46, 47])
    # every blob's ciphertext: CTR is AES(counter) XOR data, so XORing the
    # plaintext back out must give libcrypto's keystream for the nonce
    for i in range(0, 48, 7):
        o, n = int(offs[i]), int(lens[i])
        ks = S.aes256_ctr(keys[0], nonces[i].tobytes(), bytes(n))
        assert (np.frombuffer(ks, np.uint8) ^ data[o:o + n] == ct[o:o + n]).all(), i


def test_seal_key_clamping(gpu):
    """MACKey.R with every bit set: the clamp (RFC 8439; restic's mask) must
    be applied by the handle, not assumed of the caller."""
    keys = (bytes(range(32)), bytes(range(16, 32)), b"\xff" * 16)
    rng = np.random.default_rng(7)
    lens = [0, 16, 100, 70000]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = np.full(int(sum(lens)) + 16, 0xFF, np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ct, macs = _run(keys, data, offs, lens, nonces)
    _check(keys, data, offs, lens, nonces, ct, macs)


def test_seal_many_tiny_blobs_multi_tile_prefix(gpu):
    """More blobs than one prefix tile (16 K): the block prefix carries across
    tiles and the per-lane blob search spans many tiny blobs per wave."""
    keys = _keys(8)
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 70, 40000)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ct, macs = _run(keys, data, offs, lens, nonces)
    _check(keys, data, offs, lens, nonces, ct, macs)


def test_seal_rejects_misaligned_nonces(gpu):
    import torch
    from volsync_amd import Sealer
    from volsync_amd._lib import VsError
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    do = torch.zeros(1, dtype=torch.int64, device="cuda")
    dl = torch.full((1,), 16, dtype=torch.int32, device="cuda")
    dn = torch.zeros(48, dtype=torch.uint8, device="cuda")
    s = Sealer(*_keys(10))
    with pytest.raises(VsError, match="aligned"):
        s.run(d.data_ptr(), do.data_ptr(), dl.data_ptr(), 1, dn.data_ptr() + 4, d.data_ptr(),
              d.data_ptr() + 32)
    s.close()


# ---- (f)1 pack stage: pack files, pack IDs; restore: Key.Open -----------------
def _blobs(seed, sizes, tree_every=0):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, int(sum(sizes)), dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    types = np.array([(1 if tree_every and i % tree_every == tree_every - 1 else 0)
                      for i in range(len(sizes))], np.uint8)
    ids = rng.integers(0, 256, (len(sizes), 32), dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(sizes), 16), dtype=np.uint8)
    hnon = rng.integers(0, 256, (len(sizes), 16), dtype=np.uint8)
    return data, offs, types, ids, nonces, hnon


def _pack(keys, data, offs, sizes, types, ids, nonces, hnon, min_pack):
    import torch
    from volsync_amd import DeviceSha256, Sealer
    d = torch.from_numpy(data.copy()).cuda()
    s, sha = Sealer(*keys), DeviceSha256()
    out, packs, pids = s.pack(sha, d.data_ptr(), offs, sizes, types, ids, nonces, hnon, min_pack)
    torch.cuda.synchronize()
    s.close()
    sha.close()
    return out.cpu().numpy(), packs, pids


def test_restic_pack_files_vs_oracle(gpu):
    """vs_restic_pack: pack bytes (records, sealed header, trailer) and pack IDs
    equal the restatement of v0.13.1's Packer / packer managers, with data and
    tree blobs interleaved, edge blob sizes and packs closed by size."""
    keys = _keys(11)
    sizes = [1, 15, 16, 17, 1000, 70_000, 33, 200_000, 5, 150_000, 64, 100_000, 3000, 90_000,
             120_000, 7, 16 * 1024, 250_000, 1, 99_999]
    data, offs, types, ids, nonces, hnon = _blobs(12, sizes, tree_every=4)
    got, packs, pids = _pack(keys, data, offs, sizes, types, ids, nonces, hnon, 200 * 1024)
    blobs = [(int(types[i]), data[int(offs[i]):int(offs[i]) + sizes[i]].tobytes(), ids[i].tobytes(),
              nonces[i].tobytes()) for i in range(len(sizes))]
    want = S.pack_files(keys, blobs, [hnon[k].tobytes() for k in range(len(sizes))], 200 * 1024)
    assert len(packs) == len(want) > 3
    order = []
    for (o, ln, first, nb), pid, (wb, wid, wblobs) in zip(packs, pids, want):
        assert got[o:o + ln].tobytes() == wb
        assert pid == wid
        order += wblobs
        assert nb == len(wblobs)
    assert packs[-1][0] + packs[-1][1] == sum(len(w[0]) for w in want)


def test_restic_index_vs_oracle(gpu):
    """vs_restic_index ((f)3, restic's index file), checked as a decode
    round trip -- what a restore's LoadIndex + LoadBlob does with it -- not
    byte for byte: restic v0.13.1's Index.Encode walks its indexMap buckets,
    whose order is seeded per process (Go maphash), so two restic processes
    write the same index with different bytes and no byte layout is "the"
    reference.  Checked: the stored file is nonce || sealed JSON || tag and
    Key.Open (libcrypto) accepts it; the file ID is its SHA-256 (hashlib); the
    JSON decodes to exactly the packs vs_restic_pack built -- pack IDs in
    order, per pack the set of (blob ID, type, record offset, stored length)
    that the Index.Encode restatement lists -- and every entry points at its
    blob's sealed record in the pack bytes, which opens to the blob."""
    import json
    import torch
    from volsync_amd import DeviceSha256, Sealer
    keys = _keys(16)
    sizes = [1, 15, 16, 17, 1000, 70_000, 33, 200_000, 5, 150_000, 64, 100_000, 3000, 90_000,
             120_000, 7, 16 * 1024, 250_000, 1, 99_999]
    data, offs, types, ids, nonces, hnon = _blobs(17, sizes, tree_every=3)
    got, packs, pids = _pack(keys, data, offs, sizes, types, ids, nonces, hnon, 200 * 1024)
    nonce = bytes(range(16, 32))
    s, sha = Sealer(*keys), DeviceSha256()
    js, f, fid = s.index(sha, sizes, types, ids, pids, nonce, 200 * 1024)
    torch.cuda.synchronize()
    s.close()
    sha.close()
    blobs = [(int(types[i]), data[int(offs[i]):int(offs[i]) + sizes[i]].tobytes(), ids[i].tobytes(),
              nonces[i].tobytes()) for i in range(len(sizes))]
    want_packs = S.pack_files(keys, blobs, [hnon[k].tobytes() for k in range(len(sizes))],
                              200 * 1024)
    import hashlib
    wjs, _, _ = S.index_file(keys, blobs, want_packs, nonce)
    assert f[:16] == nonce and len(f) == 16 + len(js) + 16
    assert fid == hashlib.sha256(f).digest()
    plain, ok = S.open_blob(keys, f)
    assert ok and plain == js
    doc = json.loads(plain)
    assert [p["id"] for p in doc["packs"]] == [p.hex() for p in pids]

    def entries(d):   # order-independent content of an index document
        return {(p["id"], b["id"], b["type"], b["offset"], b["length"])
                for p in d["packs"] for b in p["blobs"]}
    assert entries(doc) == entries(json.loads(wjs))
    assert sum(len(p["blobs"]) for p in doc["packs"]) == len(sizes)
    seen = set()
    for (po, pl, _, _), pk in zip(packs, doc["packs"]):
        for b in pk["blobs"]:
            i = next(k for k in range(len(sizes)) if ids[k].tobytes().hex() == b["id"])
            rec = got[po + b["offset"]:po + b["offset"] + b["length"]].tobytes()
            pt, ok = S.open_blob(keys, rec)
            assert ok and pt == blobs[i][1] and b["type"] == ("tree" if types[i] else "data")
            seen.add(i)
    assert seen == set(range(len(sizes)))


def test_restic_pack_c2_chunks(gpu):
    """The pack stage on CDC output: a 256 MiB synthetic volume chunked and
    hashed on the device (blob IDs), its chunks sealed into 4 MiB packs; every
    pack and pack ID equals the oracle (libcrypto AES + Poly1305)."""
    import torch
    from tests import oracle_lib as O
    from volsync_amd import DeviceChunker, TestPol
    n = 256 << 20
    vol = O.synth(21, 0, n)
    t = torch.from_numpy(vol).cuda()
    dc = DeviceChunker(TestPol)
    nch, _ = dc.process(t.data_ptr(), n, 0, True)
    ch = dc.chunks(0, nch)
    dc.close()
    sizes = [c.Length for c in ch]
    offs = np.array([c.Start for c in ch], np.uint64)
    ids = np.stack([np.frombuffer(c.ID, np.uint8) for c in ch])
    rng = np.random.default_rng(5)
    nonces = rng.integers(0, 256, (nch, 16), dtype=np.uint8)
    hnon = rng.integers(0, 256, (nch, 16), dtype=np.uint8)
    types = np.zeros(nch, np.uint8)
    keys = _keys(13)
    got, packs, pids = _pack(keys, vol, offs, sizes, types, ids, nonces, hnon, 4 << 20)
    blobs = [(0, vol[int(offs[i]):int(offs[i]) + sizes[i]].tobytes(), ids[i].tobytes(),
              nonces[i].tobytes()) for i in range(nch)]
    want = S.pack_files(keys, blobs, [hnon[k].tobytes() for k in range(nch)], 4 << 20, fast=True)
    assert [p[3] for p in packs] == [len(w[2]) for w in want]
    for (o, ln, _, _), pid, (wb, wid, _) in zip(packs, pids, want):
        assert pid == wid and got[o:o + ln].tobytes() == wb


def test_open_verifies_and_decrypts(gpu):
    """Key.Open on the device over stored records (a pack's blob records):
    plaintext equals the original, and exactly the tampered records (one bit of
    ciphertext, of the tag, of the nonce) are flagged -- as Open's
    ErrUnauthenticated."""
    import torch
    from volsync_amd import Sealer
    keys = _keys(14)
    sizes = [1, 16, 17, 1000, 65_536, 333_333, 48, 12_345, 2, 70_000]
    data, offs, types, ids, nonces, hnon = _blobs(15, sizes)
    got, packs, _ = _pack(keys, data, offs, sizes, types, ids, nonces, hnon, 1 << 30)
    assert len(packs) == 1
    rec_off, o = [], 0
    for ln in sizes:
        rec_off.append(o)
        o += ln + 32
    stored = got.copy()
    tamper = {2: rec_off[2] + 16 + 5, 5: rec_off[5] + 16 + sizes[5] + 3, 8: rec_off[8] + 7}
    for b, pos in tamper.items():
        stored[pos] ^= 0x10
    for k, (b, pos) in enumerate(tamper.items()):
        want_pt, ok = S.open_blob(keys, stored[rec_off[b]:rec_off[b] + sizes[b] + 32].tobytes())
        assert not ok
    d = torch.from_numpy(stored).cuda()
    out = torch.zeros_like(d)
    ro = torch.tensor(np.array(rec_off, np.uint64).view(np.int64), device="cuda")
    ln = torch.tensor(np.array(sizes, np.uint32).view(np.int32), device="cuda")
    bad = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    s = Sealer(*keys)
    nbad = s.open(d.data_ptr(), ro.data_ptr(), ln.data_ptr(), len(sizes), out.data_ptr(), 0,
                  bad.data_ptr())
    # in place, as a restorer decrypting a downloaded pack buffer would
    s.open(d.data_ptr(), ro.data_ptr(), ln.data_ptr(), len(sizes), d.data_ptr(), 0, bad.data_ptr())
    torch.cuda.synchronize()
    s.close()
    assert nbad == len(tamper)
    assert sorted(np.nonzero(bad.cpu().numpy())[0].tolist()) == sorted(tamper)
    res, inplace = out.cpu().numpy(), d.cpu().numpy()
    for b, ln_ in enumerate(sizes):
        pt = res[rec_off[b] + 16:rec_off[b] + 16 + ln_].tobytes()
        assert inplace[rec_off[b] + 16:rec_off[b] + 16 + ln_].tobytes() == pt
        want_pt, ok = S.open_blob(keys, stored[rec_off[b]:rec_off[b] + ln_ + 32].tobytes())
        assert pt == want_pt and ok == (b not in tamper)
        if b not in tamper:
            assert pt == data[int(offs[b]):int(offs[b]) + ln_].tobytes()
