"""CPU restatement of restic's blob encryption -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product path never does.

restic v0.13.1 internal/crypto/crypto.go (fetched at image build time by
mover-restic/Dockerfile; not present under /root/reference):

  Key.Seal(dst, nonce, plaintext, nil):
    ciphertext = AES-256-CTR(EncryptionKey, IV = nonce)(plaintext)
      (Go cipher.NewCTR: the 16-byte IV is the initial counter block and the
      whole block is incremented as a 128-bit big-endian integer)
    mac = poly1305MAC(ciphertext, nonce, MACKey)
        = Poly1305(ciphertext, key = MACKey.R || AES-128(MACKey.K, nonce))
    returns ciphertext || mac
  The repository stores nonce || ciphertext || mac per blob
  (internal/repository saveAndEncrypt).

AES comes from the system OpenSSL libcrypto (EVP aes-256-ctr / aes-128-ecb,
loaded with ctypes); Poly1305 is restated here with Python integers from RFC
8439 section 2.5.  Both are pinned by their standards' vectors in
tests/test_seal_oracle.py (FIPS-197 C.1/C.3, RFC 8439 2.5.2).
"""
from __future__ import annotations

import ctypes

_lib = None


def _crypto():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL("libcrypto.so.3")
        for f in ("EVP_CIPHER_CTX_new", "EVP_aes_256_ctr", "EVP_aes_128_ecb", "EVP_aes_256_ecb"):
            getattr(_lib, f).restype = ctypes.c_void_p
        _lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        _lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_char_p, ctypes.c_char_p]
        _lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                           ctypes.c_int]
        _lib.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
    return _lib


def _evp(cipher: str, key: bytes, iv, data: bytes) -> bytes:
    c = _crypto()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        ok = c.EVP_EncryptInit_ex(ctx, getattr(c, cipher)(), None, key, iv)
        assert ok == 1
        c.EVP_CIPHER_CTX_set_padding(ctx, 0)
        out = ctypes.create_string_buffer(len(data) + 32)
        n = ctypes.c_int(0)
        total = 0
        # EVP_EncryptUpdate takes an int length: feed in pieces
        for o in range(0, len(data), 1 << 30):
            piece = data[o:o + (1 << 30)]
            ok = c.EVP_EncryptUpdate(ctx, ctypes.addressof(out) + total, ctypes.byref(n), piece,
                                     len(piece))
            assert ok == 1
            total += n.value
        return out.raw[:total]
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


def aes256_ctr(key: bytes, iv: bytes, data: bytes) -> bytes:
    return _evp("EVP_aes_256_ctr", key, iv, data)


def aes128_block(key: bytes, block: bytes) -> bytes:
    return _evp("EVP_aes_128_ecb", key, None, block)


def aes256_block(key: bytes, block: bytes) -> bytes:
    return _evp("EVP_aes_256_ecb", key, None, block)


P1305 = (1 << 130) - 5


def poly1305(msg: bytes, key: bytes) -> bytes:
    """RFC 8439 2.5.1: r = clamp(key[0:16]), s = key[16:32]."""
    r = int.from_bytes(key[:16], "little") & 0x0ffffffc0ffffffc0ffffffc0fffffff
    s = int.from_bytes(key[16:32], "little")
    acc = 0
    for i in range(0, len(msg), 16):
        blk = msg[i:i + 16] + b"\x01"
        acc = (acc + int.from_bytes(blk, "little")) * r % P1305
    return ((acc + s) % (1 << 128)).to_bytes(16, "little")


def poly1305_evp(msg, key: bytes) -> bytes:
    """libcrypto's Poly1305 (EVP_MAC "POLY1305"): the CPU-baseline speed path,
    checked equal to poly1305() in tests/test_seal_oracle.py.  msg: bytes or
    an address (int) with msg_len given as a (addr, len) tuple."""
    c = _crypto()
    if not hasattr(c, "_vs_mac"):
        c.EVP_MAC_fetch.restype = ctypes.c_void_p
        c.EVP_MAC_fetch.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
        c.EVP_MAC_CTX_new.restype = ctypes.c_void_p
        c.EVP_MAC_CTX_new.argtypes = [ctypes.c_void_p]
        c.EVP_MAC_CTX_free.argtypes = [ctypes.c_void_p]
        c.EVP_MAC_init.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        c.EVP_MAC_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        c.EVP_MAC_final.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t]
        c._vs_mac = c.EVP_MAC_fetch(None, b"POLY1305", None)
        assert c._vs_mac, "libcrypto has no POLY1305 EVP_MAC"
    ctx = c.EVP_MAC_CTX_new(c._vs_mac)
    try:
        assert c.EVP_MAC_init(ctx, key, 32, None) == 1
        if isinstance(msg, tuple):
            addr, n = msg
        else:
            buf = ctypes.create_string_buffer(msg, max(len(msg), 1))
            addr, n = ctypes.addressof(buf), len(msg)
        if n:
            assert c.EVP_MAC_update(ctx, addr, n) == 1
        out = ctypes.create_string_buffer(16)
        ol = ctypes.c_size_t(0)
        assert c.EVP_MAC_final(ctx, out, ctypes.byref(ol), 16) == 1
        return out.raw[:16]
    finally:
        c.EVP_MAC_CTX_free(ctx)


def seal(enc_key: bytes, mac_k: bytes, mac_r: bytes, nonce: bytes, plaintext: bytes):
    """(ciphertext, mac) of restic's Key.Seal."""
    ct = aes256_ctr(enc_key, nonce, plaintext)
    mac = poly1305(ct, mac_r + aes128_block(mac_k, nonce))
    return ct, mac


def seal_into(enc_key: bytes, mac_k: bytes, mac_r: bytes, nonce: bytes, src_addr: int, n: int,
              dst_addr: int) -> bytes:
    """seal() over raw addresses (libcrypto AES-256-CTR + Poly1305, no copies):
    the CPU-baseline leg of bench.py --mode seal.  Returns the mac."""
    c = _crypto()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, c.EVP_aes_256_ctr(), None, enc_key, nonce) == 1
        ol = ctypes.c_int(0)
        for o in range(0, n, 1 << 30):
            k = min(1 << 30, n - o)
            assert c.EVP_EncryptUpdate(ctx, dst_addr + o, ctypes.byref(ol),
                                       ctypes.c_char_p(src_addr + o), k) == 1
    finally:
        c.EVP_CIPHER_CTX_free(ctx)
    return poly1305_evp((dst_addr, n), mac_r + aes128_block(mac_k, nonce))


# ---- restic v0.13.1 pack files (internal/pack, internal/repository) ----------
MIN_PACK_SIZE = 4 * 1024 * 1024   # repository packer_manager.go minPackSize


def seal_fast(enc_key: bytes, mac_k: bytes, mac_r: bytes, nonce: bytes, plaintext: bytes):
    """seal() with libcrypto's Poly1305 (equal to the restatement, checked in
    tests/test_seal_oracle.py): for the large pack cases."""
    ct = aes256_ctr(enc_key, nonce, plaintext)
    return ct, poly1305_evp(ct, mac_r + aes128_block(mac_k, nonce))


def pack_files(keys, blobs, hdr_nonces, min_pack_size: int = MIN_PACK_SIZE, fast: bool = False):
    """Packer.Add / Finalize as repository.SaveBlob drives them with one
    packer per blob type: blobs = [(type, plaintext, id32, nonce16)] in save
    order.  A blob's record is nonce || Seal(plaintext) (ciphertext || tag);
    a pack is finalised once its records reach min_pack_size bytes (and at
    Flush: the data pack, then the tree pack); Finalize appends the header
    (per blob: type byte, uint32 LE record length, ID) sealed with the pack's
    nonce (nonce || ciphertext || tag) and the sealed header's length (uint32
    LE).  The pack ID is the SHA-256 of the pack file.  Returns
    [(pack bytes, pack id, [blob indices])] in the order packs are written."""
    import hashlib
    enc, mk, mr = keys
    sl = seal_fast if fast else seal
    out, cur, size = [], {0: [], 1: []}, {0: 0, 1: 0}
    recs = {}

    def close(t):
        if not cur[t]:
            return
        body = b"".join(recs[i] for i in cur[t])
        hdr = b""
        for i in cur[t]:
            typ, _, bid, _ = blobs[i]
            hdr += bytes([typ]) + len(recs[i]).to_bytes(4, "little") + bid
        hn = hdr_nonces[len(out)]
        ct, tag = sl(enc, mk, mr, hn, hdr)
        sealed = hn + ct + tag
        pack = body + sealed + len(sealed).to_bytes(4, "little")
        out.append((pack, hashlib.sha256(pack).digest(), list(cur[t])))
        cur[t], size[t] = [], 0

    for i, (typ, plain, _, nonce) in enumerate(blobs):
        ct, tag = sl(enc, mk, mr, nonce, plain)
        recs[i] = nonce + ct + tag
        t = 1 if typ else 0
        cur[t].append(i)
        size[t] += len(recs[i])
        if size[t] >= min_pack_size:
            close(t)
    close(0)
    close(1)
    return out


def open_blob(keys, record: bytes):
    """Key.Open of one stored blob: (plaintext, ok).  The tag is checked
    before decryption; ok False means Open would return ErrUnauthenticated."""
    enc, mk, mr = keys
    nonce, ct, tag = record[:16], record[16:-16], record[-16:]
    ok = poly1305(ct, mr + aes128_block(mk, nonce)) == tag
    return aes256_ctr(enc, nonce, ct), ok


def index_file(keys, blobs, packs, nonce: bytes, fast: bool = False):
    """restic v0.13.1 internal/index Index.Encode + repository.SaveUnpacked
    for the packs pack_files() made: the JSON document
      {"packs":[{"id":<pack id hex>,"blobs":[{"id":<hex>,"type":"data"|"tree",
       "offset":<record offset in the pack>,"length":<record length>}]}]}
    as Go's json.Encoder writes it (struct field order, no spaces,
    "supersedes" omitted when empty, a trailing newline), packs in write
    order and blobs in pack order; the stored file = nonce || Seal(JSON); its
    ID = SHA-256 of the file.  Returns (json bytes, file bytes, file id)."""
    import hashlib
    import json
    doc = {"packs": []}
    for _, pid, members in packs:
        off, bl = 0, []
        for i in members:
            typ, plain, bid, _ = blobs[i]
            rl = len(plain) + 32        # nonce + ciphertext + tag
            bl.append({"id": bid.hex(), "type": "tree" if typ else "data", "offset": off,
                       "length": rl})
            off += rl
        doc["packs"].append({"id": pid.hex(), "blobs": bl})
    js = (json.dumps(doc, separators=(",", ":")) + "\n").encode()
    enc, mk, mr = keys
    ct, tag = (seal_fast if fast else seal)(enc, mk, mr, nonce, js)
    f = nonce + ct + tag
    return js, f, hashlib.sha256(f).digest()
