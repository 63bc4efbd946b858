"""Wire formats through the C ABI, on the CPU (host code).

The expected bytes come from restatements of rsync 3.2.3 io.c write_sum_head
+ generate_and_send_sums, token.c simple_send_token as match.c matched()
drives it, and restic v0.13.1's pack header entry, written here in Python
from the published formats; the committed rsync fixtures supply the sums and
match lists.  No rsync or restic binary exists in the image: the byte layouts
are pinned by the formats' definitions, round trips and the fixtures.
"""
import ctypes
import os
import struct

import numpy as np
import pytest

from tests import golden_util as G
from volsync_amd._lib import VsError, VsMatch, check, lib

FIX = G.fixtures("rsync_*.json")


def py_sums(count, blength, s2length, remainder, sum1, sum2):
    out = struct.pack("<iiii", count, blength, s2length, remainder)
    for i in range(count):
        out += struct.pack("<I", sum1[i] & 0xFFFFFFFF) + bytes(sum2[i * s2length:(i + 1) * s2length])
    return out


def py_tokens(matches, src: bytes, blength, basis_len):
    out, last = b"", 0

    def literal(a, b):
        nonlocal out
        for o in range(a, b, 32768):
            k = min(32768, b - o)
            out += struct.pack("<i", k) + src[o:o + k]

    for o, i in matches:
        literal(last, o)
        out += struct.pack("<i", -(i + 1))
        last = o + min(blength, basis_len - i * blength)
    literal(last, len(src))
    return out + struct.pack("<i", 0)


def c_write_sums(count, blength, s2, rem, sum1, sum2):
    a1 = (ctypes.c_uint32 * max(count, 1))(*[x & 0xFFFFFFFF for x in sum1])
    a2 = (ctypes.c_uint8 * max(count * s2, 1))(*sum2)
    n = ctypes.c_size_t()
    check(lib.vs_rsync_write_sums(count, blength, s2, rem, a1, a2, None, 0, ctypes.byref(n)))
    out = (ctypes.c_uint8 * n.value)()
    check(lib.vs_rsync_write_sums(count, blength, s2, rem, a1, a2, out, n.value, ctypes.byref(n)))
    return bytes(out)


def c_tokens(matches, src: bytes, blength, basis_len):
    arr = (VsMatch * max(len(matches), 1))()
    for k, (o, i) in enumerate(matches):
        arr[k].offset, arr[k].block_index = o, i
    buf = ctypes.create_string_buffer(src, max(len(src), 1))
    n = ctypes.c_size_t()
    check(lib.vs_rsync_write_tokens(arr, len(matches), len(src), blength, basis_len, buf, None, 0,
                                    ctypes.byref(n)))
    out = (ctypes.c_uint8 * n.value)()
    check(lib.vs_rsync_write_tokens(arr, len(matches), len(src), blength, basis_len, buf, out,
                                    n.value, ctypes.byref(n)))
    return bytes(out)


def c_read_tokens(stream: bytes, blength, basis_len):
    nm, nl, fl = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_int64()
    check(lib.vs_rsync_read_tokens(stream, len(stream), blength, basis_len, None, 0,
                                   ctypes.byref(nm), None, 0, ctypes.byref(nl), ctypes.byref(fl)))
    m = (VsMatch * max(nm.value, 1))()
    lits = (ctypes.c_uint8 * max(nl.value, 1))()
    check(lib.vs_rsync_read_tokens(stream, len(stream), blength, basis_len, m, nm.value,
                                   ctypes.byref(nm), lits, nl.value, ctypes.byref(nl),
                                   ctypes.byref(fl)))
    return ([(int(x.offset), int(x.block_index)) for x in m[:nm.value]],
            bytes(lits[:nl.value]), fl.value)


@pytest.mark.parametrize("path", FIX, ids=os.path.basename)
def test_sum_table_and_tokens_vs_restatement(path):
    doc = G.load(path)
    basis, src = G.rsync_pair(doc["input"])
    bl, s2, count, rem = doc["sizes"]["blength"], doc["sizes"]["s2length"], \
        doc["sizes"]["count"], doc["sizes"]["remainder"]
    sum1 = [int(x) for x in doc["sum1"]]
    sum2 = list(bytes.fromhex("".join(doc["sum2"])))
    wire = c_write_sums(count, bl, s2, rem, sum1, sum2)
    assert wire == py_sums(count, bl, s2, rem, sum1, sum2)
    # read back
    c, b, s, r = (ctypes.c_int32() for _ in range(4))
    r1 = (ctypes.c_uint32 * max(count, 1))()
    r2 = (ctypes.c_uint8 * max(count * s2, 1))()
    check(lib.vs_rsync_read_sums(wire, len(wire), ctypes.byref(c), ctypes.byref(b), ctypes.byref(s),
                                 ctypes.byref(r), r1, r2, max(count, 1)))
    assert (c.value, b.value, s.value, r.value) == (count, bl, s2, rem)
    assert list(r1[:count]) == [x & 0xFFFFFFFF for x in sum1] and list(r2[:count * s2]) == sum2
    matches = [tuple(m) for m in doc["matches"]]
    sb = src.tobytes()
    tok = c_tokens(matches, sb, bl, len(basis))
    assert tok == py_tokens(matches, sb, bl, len(basis))
    got_m, got_lit, flen = c_read_tokens(tok, bl, len(basis))
    assert got_m == matches and flen == len(sb)
    # the literals are exactly the source bytes between the matches
    pos, want = 0, b""
    for o, i in matches:
        want += sb[pos:o]
        pos = o + min(bl, len(basis) - i * bl)
    assert got_lit == want + sb[pos:]


def test_token_edge_cases():
    blen, basis_len = 700, 700 * 3 + 5
    src = bytes(range(256)) * 300       # 76 800 bytes: literal runs split at 32 KiB
    assert py_tokens([], src, blen, basis_len) == c_tokens([], src, blen, basis_len)
    assert c_tokens([], b"", blen, basis_len) == struct.pack("<i", 0)
    m = [(0, 3), (5, 0), (40000, 1)]   # short last block (5 bytes) first
    assert c_tokens(m, src, blen, basis_len) == py_tokens(m, src, blen, basis_len)
    with pytest.raises(VsError, match="out of order|out of range"):
        c_tokens([(100, 0), (50, 1)], src, blen, basis_len)
    with pytest.raises(VsError, match="past the end"):
        c_tokens([(len(src) - 10, 0)], src, blen, basis_len)
    with pytest.raises(VsError, match="truncated"):
        c_read_tokens(struct.pack("<i", 100) + b"x" * 10, blen, basis_len)


def test_restic_pack_header_entries():
    rng = np.random.default_rng(3)
    n = 5
    types = (ctypes.c_uint8 * n)(0, 1, 0, 0, 1)
    lens = (ctypes.c_uint32 * n)(*[int(x) for x in rng.integers(32, 1 << 24, n)])
    ids = (ctypes.c_uint8 * (32 * n))(*rng.integers(0, 256, 32 * n).tolist())
    sz = ctypes.c_size_t()
    check(lib.vs_restic_pack_header(types, lens, ids, n, None, 0, ctypes.byref(sz)))
    assert sz.value == 37 * n
    out = (ctypes.c_uint8 * sz.value)()
    check(lib.vs_restic_pack_header(types, lens, ids, n, out, sz.value, ctypes.byref(sz)))
    want = b"".join(struct.pack("<BI", types[i], lens[i]) + bytes(ids[32 * i:32 * i + 32])
                    for i in range(n))
    assert bytes(out) == want
    bad = (ctypes.c_uint8 * 1)(2)
    with pytest.raises(VsError, match="blob type"):
        check(lib.vs_restic_pack_header(bad, lens, ids, 1, out, sz.value, ctypes.byref(sz)))


# ---- rsync -z: the zstd token stream (token.c send_zstd_token / recv_zstd_token)
class _ZIn(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


class _ZOut(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


class PyZstdReceiver:
    """An independent restatement of recv_zstd_token's framing in Python (flag
    bytes, relative runs, DEFLATED_DATA pieces), decompressing through
    libzstd directly: test infrastructure for the library's writer."""

    def __init__(self):
        self.z = ctypes.CDLL("libzstd.so.1")
        self.z.ZSTD_createDCtx.restype = ctypes.c_void_p
        self.z.ZSTD_decompressStream.restype = ctypes.c_size_t
        self.z.ZSTD_decompressStream.argtypes = [ctypes.c_void_p, ctypes.POINTER(_ZOut),
                                                 ctypes.POINTER(_ZIn)]
        self.z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        self.d = self.z.ZSTD_createDCtx()

    def inflate(self, data: bytes) -> bytes:
        src = ctypes.create_string_buffer(data, len(data))
        zin = _ZIn(ctypes.addressof(src), len(data), 0)
        out = b""
        while True:
            dst = ctypes.create_string_buffer(1 << 18)
            zo = _ZOut(ctypes.addressof(dst), len(dst), 0)
            r = self.z.ZSTD_decompressStream(self.d, ctypes.byref(zo), ctypes.byref(zin))
            assert not self.z.ZSTD_isError(r)
            out += dst.raw[: zo.pos]
            if zin.pos == zin.size and zo.pos < zo.size:
                return out

    def file(self, s: bytes, blength: int, basis_len: int):
        r, tok, pos, matches, lit = 0, 0, 0, [], b""

        def token(t):
            nonlocal pos
            matches.append((pos, t))
            pos += min(blength, basis_len - t * blength)

        while True:
            flag = s[r]
            r += 1
            if flag & 0xC0 == 0x40:
                n = ((flag & 0x3F) << 8) + s[r]
                data = self.inflate(s[r + 1:r + 1 + n])
                r += 1 + n
                lit += data
                pos += len(data)
                continue
            if flag == 0:
                return matches, lit, pos, r
            if flag & 0x80:
                tok += flag & 0x3F
                flag >>= 6
            else:
                tok = struct.unpack_from("<i", s, r)[0]
                r += 4
            token(tok)
            if flag & 1:
                run = s[r] | (s[r + 1] << 8)
                r += 2
                for _ in range(run):
                    tok += 1
                    token(tok)


def _fixture_file(path):
    doc = G.load(path)
    _, src = G.rsync_pair(doc["input"])
    z = doc["sizes"]
    last = z["remainder"] or z["blength"]
    basis_len = (z["count"] - 1) * z["blength"] + last if z["count"] else 0
    return [tuple(m) for m in doc["matches"]], src.tobytes(), z["blength"], basis_len, last


def _gaps(matches, src, blength, basis_len):
    out, last = b"", 0
    for o, i in matches:
        out += src[last:o]
        last = o + min(blength, basis_len - i * blength)
    return out + src[last:]


def test_zstd_tokens_round_trip_every_fixture():
    """Every rsync fixture's match list through the -z token stream: the
    library's reader and an independent Python receiver both recover the
    matches, the literal bytes and the file length."""
    from volsync_amd import ZstdTokens
    for path in FIX:
        matches, src, bl, blen, last = _fixture_file(path)
        tx, rx = ZstdTokens(), ZstdTokens()
        s = tx.write(matches, src, bl, blen, last)
        got = rx.read(s, bl, blen, len(matches) + 8, len(src) + 8)
        assert got[0] == matches and got[1] == _gaps(matches, src, bl, blen), path
        assert got[2] == len(src) and got[3] == len(s), path
        py = PyZstdReceiver().file(s, bl, blen)
        assert py == got, path


def test_zstd_tokens_one_transfer_many_files():
    """rsync keeps one zstd stream per transfer: the fixtures sent as the
    files of ONE transfer decode in order on one receiver, and the second
    file's stream does not decode on a fresh receiver (it continues the
    first's zstd stream only when the first was read)."""
    from volsync_amd import ZstdTokens
    files = [_fixture_file(p) for p in FIX]
    tx, rx = ZstdTokens(), ZstdTokens()
    streams = [tx.write(m, src, bl, blen, last) for m, src, bl, blen, last in files]
    for (m, src, bl, blen, last), s in zip(files, streams):
        got = rx.read(s, bl, blen, len(m) + 8, len(src) + 8)
        assert got[0] == m and got[1] == _gaps(m, src, bl, blen) and got[2] == len(src)


def test_zstd_tokens_runs_and_long_tokens():
    """Token runs (consecutive blocks: TOKENRUN_REL with a 16-bit count, split
    at 65536), far jumps (TOKEN_LONG / TOKENRUN_LONG) and literal runs long
    enough for hash_search's early flushes (> blength + 32 KiB)."""
    from volsync_amd import ZstdTokens
    bl, nblk = 64, 70000
    basis_len = bl * nblk
    rng = np.random.default_rng(9)
    lit = rng.integers(0, 4, 200_000, dtype=np.uint8).tobytes()
    # blocks 0..66999 in order (a run past 65536), then a jump back to 5,
    # a 150 KB literal, blocks 69990..69999
    matches, src, pos = [], b"", 0
    for i in list(range(67000)) + [5]:
        matches.append((pos, i))
        pos += bl
    src = bytes(pos) + lit[:150_000]
    pos += 150_000
    for i in range(69990, 70000):
        matches.append((pos, i))
        pos += bl
    src += bytes(pos - len(src))
    tx, rx = ZstdTokens(), ZstdTokens()
    s = tx.write(matches, src, bl, basis_len, bl)
    got = rx.read(s, bl, basis_len, len(matches) + 8, len(src))
    assert got[0] == matches and got[2] == len(src)
    assert got[1] == lit[:150_000]
    assert PyZstdReceiver().file(s, bl, basis_len) == got
    assert len(s) < len(src) // 4   # zero runs and 2-bit literals compress


# ---- malformed input from a peer --------------------------
# Every parser below reads bytes a network peer sent.  Each malformed form must
# come back as VS_ERR_ARG with a message, never as a read past the input or an
# output array; tools/asan_build.sh runs these under ASan + UBSan.
def c_read_sums(wire: bytes, cap: int = 64):
    c, b, s, r = (ctypes.c_int32() for _ in range(4))
    # arrays of at most 64 blocks: a larger `cap` claims more than they hold,
    # which is safe only when the parser refuses before writing (tests below)
    r1 = (ctypes.c_uint32 * max(min(cap, 64), 1))()
    r2 = (ctypes.c_uint8 * max(min(cap, 64) * 16, 1))()
    check(lib.vs_rsync_read_sums(wire, len(wire), ctypes.byref(c), ctypes.byref(b),
                                 ctypes.byref(s), ctypes.byref(r), r1, r2, cap))
    return c.value, b.value, s.value, r.value


def test_read_sums_malformed():
    good = py_sums(3, 700, 5, 12, [1, 2, 3], list(range(15)))
    assert c_read_sums(good) == (3, 700, 5, 12)
    for k in range(16):          # every truncation of the 16-byte head
        with pytest.raises(VsError, match="truncated sum head"):
            c_read_sums(good[:k])
    for k in range(16, len(good)):   # head whole, sums cut anywhere
        with pytest.raises(VsError, match="truncated sums"):
            c_read_sums(good[:k])
    bad_heads = [(-1, 700, 5, 12), (3, -700, 5, 12), (3, (1 << 17) + 8, 5, 12), (3, 700, 17, 12),
                 (3, 700, -1, 12), (3, 700, 5, -1), (3, 700, 5, 701), (3, 0, 5, 0),
                 (-(1 << 31), 700, 2, 0)]
    for h in bad_heads:
        with pytest.raises(VsError, match="invalid sum head"):
            c_read_sums(struct.pack("<iiii", *h) + bytes(64))
    # a head that claims 2^31 - 1 blocks: refused by size, nothing read past the input
    huge = struct.pack("<iiii", (1 << 31) - 1, 700, 2, 0) + bytes(64)
    with pytest.raises(VsError, match="too small"):
        c_read_sums(huge, cap=64)
    with pytest.raises(VsError, match="truncated sums"):
        # a caller that sized its arrays by the claim: the body is checked
        # against n before anything is written (the arrays here are small)
        c_read_sums(huge, cap=(1 << 31))
    # the last-block rule: remainder == blength and count 0 are legal heads
    assert c_read_sums(struct.pack("<iiii", 0, 0, 2, 0)) == (0, 0, 2, 0)
    assert c_read_sums(struct.pack("<iiii", 1, 700, 2, 700) + bytes(6)) == (1, 700, 2, 700)


def test_read_tokens_malformed():
    blen, basis_len = 700, 700 * 3 + 5   # 4 blocks, the last 5 bytes long
    src = bytes(range(256)) * 40
    m = [(0, 3), (5, 0), (2000, 1)]
    good = c_tokens(m, src, blen, basis_len)
    assert c_read_tokens(good, blen, basis_len)[0] == m
    for k in range(len(good)):                  # every truncation
        with pytest.raises(VsError, match="truncated"):
            c_read_tokens(good[:k], blen, basis_len)
    end = struct.pack("<i", 0)
    with pytest.raises(VsError, match="past the basis"):
        c_read_tokens(struct.pack("<i", -5) + end, blen, basis_len)          # block 4 of 4
    with pytest.raises(VsError, match="past the basis"):
        c_read_tokens(struct.pack("<i", -(1 << 31)) + end, blen, basis_len)  # INT32_MIN
    with pytest.raises(VsError, match="past the basis"):
        c_read_tokens(struct.pack("<i", -1) + end, blen, 0)                  # empty basis
    with pytest.raises(VsError, match="truncated literal"):
        c_read_tokens(struct.pack("<i", (1 << 31) - 1) + b"x" * 64 + end, blen, basis_len)
    # output arrays too small for what the stream holds
    nm, nl, fl = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_int64()
    one = (VsMatch * 1)()
    with pytest.raises(VsError, match="match buffer too small"):
        check(lib.vs_rsync_read_tokens(good, len(good), blen, basis_len, one, 1, ctypes.byref(nm),
                                       None, 0, ctypes.byref(nl), ctypes.byref(fl)))
    lit = (ctypes.c_uint8 * 3)()
    with pytest.raises(VsError, match="literal buffer too small"):
        check(lib.vs_rsync_read_tokens(good, len(good), blen, basis_len, None, 0, ctypes.byref(nm),
                                       lit, 3, ctypes.byref(nl), ctypes.byref(fl)))


def test_read_tokens_zstd_malformed():
    from volsync_amd import ZstdTokens
    blen, nblk = 64, 100
    basis_len = blen * nblk
    rng = np.random.default_rng(5)
    lit = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    m, pos = [], 0
    for i in list(range(20)) + [50, 7]:
        m.append((pos, i))
        pos += blen
    src = bytes(pos) + lit
    good = ZstdTokens().write(m, src, blen, basis_len, blen)
    assert ZstdTokens().read(good, blen, basis_len, 64, len(src))[0] == m

    def rd(stream, basis=basis_len):
        return ZstdTokens().read(stream, blen, basis, 64, len(src) + 64)

    # every truncation of a real stream (cut inside a flag, a TOKEN_LONG, a run
    # count, a DEFLATED_DATA header or its compressed bytes -- a zstd frame cut
    # mid-block): an error or, where the cut falls between whole tokens, a
    # shorter file; never a read past the input
    for k in range(len(good)):
        try:
            got = rd(good[:k])
        except VsError as e:
            assert "truncated" in str(e) or "ZSTD" in str(e), e
        else:
            assert got[3] <= k
    with pytest.raises(VsError, match="truncated"):
        rd(b"")
    with pytest.raises(VsError, match="past the basis"):
        rd(bytes([0x80 | 63, 0x80 | 63, 0]), basis=blen * 100)     # relative tokens 63, 126
    with pytest.raises(VsError, match="past the basis"):
        rd(bytes([0x20]) + struct.pack("<i", -7) + b"\x00")          # TOKEN_LONG, negative
    with pytest.raises(VsError, match="past the basis"):
        rd(bytes([0x20]) + struct.pack("<i", nblk) + b"\x00")        # TOKEN_LONG, one past
    with pytest.raises(VsError, match="past the basis"):
        rd(bytes([0x21]) + struct.pack("<i", 95) + bytes([10, 0, 0]))  # TOKENRUN_LONG 95..105
    # a DEFLATED_DATA piece of garbage: zstd refuses it
    with pytest.raises(VsError, match="ZSTD"):
        rd(bytes([0x40, 16]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes() + b"\x00")


def test_wire_parsers_random_bytes():
    """Seeded random byte strings (and random mutations of real streams) into
    all three peer-facing parsers: each returns OK or VS_ERR_ARG, nothing else
    (under tools/asan_build.sh: no memory error either)."""
    from volsync_amd import ZstdTokens
    rng = np.random.default_rng(2026)
    blen, basis_len = 512, 512 * 40
    src = rng.integers(0, 4, 30_000, dtype=np.uint8).tobytes()
    m = [(0, 1), (512, 2), (4000, 39), (9000, 0)]
    plain = c_tokens(m, src, blen, basis_len)
    zst = ZstdTokens().write(m, src, blen, basis_len, blen)
    sums = py_sums(40, blen, 4, 0, list(range(40)), list(range(160)))
    for it in range(1500):
        kind = it % 3
        base = (plain, zst, sums)[kind]
        if it % 2:
            s = rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()
        else:
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            s = bytes(b[:int(rng.integers(0, len(b) + 1))])
        try:
            if kind == 0:
                c_read_tokens(s, blen, basis_len)
            elif kind == 1:
                ZstdTokens().read(s, blen, basis_len, 4096, 1 << 20)
            else:
                c_read_sums(s, cap=64)
        except VsError as e:
            assert e.code == -1, e
