"""CPU tests: the C oracle against the golden fixtures and independent implementations.

Pins: SHA-256 against FIPS 180-4 vectors + hashlib + OpenSSL; chunk boundaries
against the upstream zero-data known answer and the independent Python
restatement's fixtures (tests/golden/make_golden.py)."""
import hashlib
import os

import numpy as np
import pytest

from oracle import cdc_ref as P
from tests import golden_util as G
from tests import oracle_lib as O

FIPS = [
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


@pytest.mark.parametrize("msg,hexd", FIPS)
def test_sha256_fips(msg, hexd):
    assert O.sha256(msg).hex() == hexd


def test_sha256_lengths_vs_hashlib():
    rng = np.random.default_rng(1)
    d = rng.integers(0, 256, 5000, dtype=np.uint8)
    for n in list(range(0, 200)) + [511, 512, 513, 4095, 4096, 4097]:
        assert O.sha256(d[:n]) == hashlib.sha256(d[:n].tobytes()).digest()


def test_openssl_matches_portable():
    lib = O.lib()
    if not lib.ref_have_openssl():
        pytest.skip("libcrypto not loadable")
    d = O.synth(5, 0, 100003)
    a = np.zeros(32, np.uint8)
    b = np.zeros(32, np.uint8)
    lib.ref_sha256_fast(d.ctypes.data, len(d), a.ctypes.data)
    lib.ref_sha256(d.ctypes.data, len(d), b.ctypes.data)
    assert bytes(a) == bytes(b)


def test_synth_c_equals_numpy():
    for seed, off, n in [(1, 0, 4096), (7, 13, 1001), (3, 1 << 33, 77)]:
        assert (O.synth(seed, off, n) == P.synth(seed, off, n)).all()


def test_test_pol_irreducible_deg53():
    assert P.pol_deg(P.TEST_POL) == 53
    assert P.pol_irreducible(P.TEST_POL)
    assert not P.pol_irreducible(P.TEST_POL ^ 2)  # x^53... + x: divisible by x? reducible
    assert O.lib().ref_pol_deg(P.TEST_POL) == 53


def test_tables_match_python():
    out = np.zeros(256, np.uint64)
    mod = np.zeros(256, np.uint64)
    O.lib().ref_tables(P.TEST_POL, out.ctypes.data, mod.ctypes.data)
    t = P.offset_tables(P.TEST_POL)
    # out[b] = b * x^(8*63) mod P = T[0][b]
    assert (out == t[0]).all()
    k = 53
    for b in [0, 1, 2, 255]:
        assert int(mod[b]) == P.pol_mod(b << k, P.TEST_POL) | (b << k)


def test_rolling_equals_windowed_fingerprint():
    d = O.synth(9, 0, 4096)
    fp = P.window_fp_all(d, P.TEST_POL)
    for p in [63, 64, 100, 1000, 4095]:
        assert O.lib().ref_window_fp(d.ctypes.data, p, P.TEST_POL) == int(fp[p - 63])


def test_upstream_zero_known_answer():
    """chunker_test.go: 4*MinSize zero bytes -> 4 chunks of MinSize, Cut 0."""
    z = np.zeros(4 * P.MIN_SIZE, np.uint8)
    got = O.cdc_hash(z, P.TEST_POL, P.MIN_SIZE, P.MAX_SIZE, 20)
    want_id = "07854d2fef297a06ba81685e660c332de36d5d18d546927d30daad6d7fda1541"
    assert got == [(i * P.MIN_SIZE, P.MIN_SIZE, 0, want_id) for i in range(4)]


@pytest.mark.parametrize("path", [p for p in G.fixtures() if "1g" not in p],
                         ids=lambda p: os.path.basename(p))
def test_oracle_vs_golden(path):
    doc = G.load(path)
    data = G.make_input(doc["input"])
    pol, mn, mx, ab = G.params(doc)
    got = O.cdc_hash(data, pol, mn, mx, ab)
    assert got == G.expected(doc)


def test_oracle_vs_golden_1g_c1():
    """Config C1: 1 GiB synthetic stream, default parameters (677 chunks)."""
    path = os.path.join(G.GOLDEN, "cdc_synth1_1g.json")
    doc = G.load(path)
    data = O.synth(1, 0, doc["input"]["len"])
    pol, mn, mx, ab = G.params(doc)
    got = O.cdc_hash(data, pol, mn, mx, ab, n_hash=4)
    assert got == G.expected(doc)


def test_chunk_properties_small_params():
    d = O.synth(21, 0, 2 << 20)
    ch = O.chunk_all(d, P.TEST_POL, 2048, 8192, 11)
    pos = 0
    for i, (s, l, c) in enumerate(ch):
        assert s == pos
        pos += l
        if i < len(ch) - 1:
            assert 2048 <= l <= 8192
            if l < 8192:
                assert c & ((1 << 11) - 1) == 0
    assert pos == len(d)


def test_rsync_weak_sum_forms():
    """get_checksum1: unrolled C == closed form over signed bytes."""
    d = O.synth(4, 0, 5000)
    s = d.astype(np.int8).astype(np.int64)
    for n in [0, 1, 3, 4, 5, 700, 4999]:
        x = s[:n]
        s1 = int(x.sum()) & 0xFFFFFFFF
        s2 = int(((n - np.arange(n)) * x).sum()) & 0xFFFFFFFF
        want = ((s1 & 0xFFFF) + (s2 << 16)) & 0xFFFFFFFF
        assert O.lib().ref_rsync_checksum1(d.ctypes.data, n) == want


def test_rsync_sum_sizes_c4():
    import ctypes
    vals = [ctypes.c_int32() for _ in range(4)]
    assert O.lib().ref_rsync_sum_sizes(1 << 38, 0, *[ctypes.byref(v) for v in vals]) == 0
    assert [v.value for v in vals] == [131072, 5, 2097152, 0]
    assert O.lib().ref_rsync_sum_sizes(1000, 0, *[ctypes.byref(v) for v in vals]) == 0
    assert [v.value for v in vals] == [700, 2, 2, 300]


@pytest.mark.parametrize("seed,n,mn,mx,ab", [
    (1, 1 << 30, 512 << 10, 8 << 20, 20),   # C1
    (5, 40 << 20, 64 << 10, 1 << 20, 16),
    (9, 3 << 20, 4096, 65536, 13),          # forced cuts
    (11, 700 << 10, 512 << 10, 8 << 20, 20),  # one EOF chunk > MinSize
    (12, 100, 512 << 10, 8 << 20, 20),      # one tiny EOF chunk
])
def test_multithreaded_synth_oracle_equals_sequential(seed, n, mn, mx, ab):
    """The multi-threaded full-size checker (ref_cdc_synth_mt: parallel
    candidate ranges + sequential selection + parallel SHA-256) equals the
    sequential Chunker.Next restatement, Cut values and IDs included."""
    s, ln, cu, ids = O.cdc_synth_mt(seed, n, P.TEST_POL, mn, mx, ab, 7)
    got = [(int(a), int(b), int(c), bytes(i).hex()) for a, b, c, i in zip(s, ln, cu, ids)]
    assert got == O.cdc_hash(O.synth(seed, 0, n), P.TEST_POL, mn, mx, ab, n_hash=4)
