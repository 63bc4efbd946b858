"""Pins oracle/seal_ref.py (restic Key.Seal restatement) against the
standards' known answers: FIPS-197 appendix C (AES-128 / AES-256), RFC 8439
2.5.2 (Poly1305), and NIST SP 800-38A F.5.5 (AES-256-CTR)."""
from oracle import seal_ref as S


def test_fips197_aes():
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    k128 = bytes(range(16))
    k256 = bytes(range(32))
    assert S.aes128_block(k128, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert S.aes256_block(k256, pt).hex() == "8ea2b7ca516745bfeafc49904b496089"


def test_sp800_38a_ctr():
    key = bytes.fromhex("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4")
    iv = bytes.fromhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff")
    pt = bytes.fromhex("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
                       "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710")
    ct = ("601ec313775789a5b7a7f504bbf3d228f443e3ca4d62b59aca84e990cacaf5c5"
          "2b0930daa23de94ce87017ba2d84988ddfc9c58db67aada613c2dd08457941a6")
    assert S.aes256_ctr(key, iv, pt).hex() == ct


def test_rfc8439_poly1305():
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    msg = b"Cryptographic Forum Research Group"
    assert S.poly1305(msg, key).hex() == "a8061dc1305136c6c22b8baf0c0127a9"


def test_ctr_counter_carries_across_the_block():
    # Go's CTR increments the whole 16-byte block big-endian: the counter
    # ff..ff wraps to 00..00, as OpenSSL's 128-bit counter does
    key = bytes(range(32))
    iv = b"\xff" * 16
    a = S.aes256_ctr(key, iv, bytes(32))
    assert a[:16] == S.aes256_block(key, iv)
    assert a[16:] == S.aes256_block(key, bytes(16))


def test_libcrypto_poly1305_equals_restatement():
    import os
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    assert S.poly1305_evp(b"Cryptographic Forum Research Group", key).hex() == \
        "a8061dc1305136c6c22b8baf0c0127a9"
    rnd = os.urandom(5000)
    for n in (0, 1, 15, 16, 17, 1000, 5000):
        k = rnd[:32]
        assert S.poly1305_evp(rnd[:n], k) == S.poly1305(rnd[:n], k), n


def test_seal_into_equals_seal():
    import ctypes
    import os
    keys = (os.urandom(32), os.urandom(16), os.urandom(16))
    nonce, pt = os.urandom(16), os.urandom(3001)
    src = ctypes.create_string_buffer(pt, len(pt))
    dst = ctypes.create_string_buffer(len(pt))
    mac = S.seal_into(*keys, nonce, ctypes.addressof(src), len(pt), ctypes.addressof(dst))
    assert (dst.raw, mac) == S.seal(*keys, nonce, pt)


def test_index_file_restatement_format():
    """The index restatement writes what v0.13.1's json.Encoder writes for
    jsonIndex / packJSON / blobJSON: fields in struct order, no spaces,
    "supersedes" omitted when empty, IDs as hex, BlobType as "data" / "tree",
    Offset / Length of the record in the pack (plaintext + 32), a trailing
    newline -- and the stored file opens back to it."""
    keys = (bytes(range(32)), bytes(range(16)), bytes(range(16, 32)))
    blobs = [(0, b"a" * 10, bytes([1] * 32), bytes(16)), (1, b"b" * 5, bytes([2] * 32), bytes(16)),
             (0, b"c" * 7, bytes([3] * 32), bytes(16))]
    packs = S.pack_files(keys, blobs, [bytes(16)] * 3, 1 << 20)
    js, f, fid = S.index_file(keys, blobs, packs, bytes(range(16)))
    p0, p1 = packs[0][1].hex(), packs[1][1].hex()
    want = ('{"packs":[{"id":"%s","blobs":[{"id":"%s","type":"data","offset":0,"length":42},'
            '{"id":"%s","type":"data","offset":42,"length":39}]},{"id":"%s","blobs":[{"id":"%s",'
            '"type":"tree","offset":0,"length":37}]}]}\n') % (p0, "01" * 32, "03" * 32, p1, "02" * 32)
    assert js.decode() == want
    assert len(f) == len(js) + 32 and S.open_blob(keys, f) == (js, True)
