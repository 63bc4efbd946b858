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
