"""Independent Python restatement of rsync 3.2.3's delta matcher.

TEST INFRASTRUCTURE ONLY (fixture generation and cross-checks; see
oracle/cdc_ref.c header for the rule).  Reference behaviour (rsync 3.2.3 as
installed by /root/reference/mover-rsync/Dockerfile:5-13, run from
mover-rsync/source.sh:54; source not vendored), SURVEY.md 8(a) rows R1-R6:

  checksum.c get_checksum1 / get_checksum2, generator.c sum_sizes_sqroot /
  generate_and_send_sums, match.c build_hash_table / hash_search.

Algorithm differs from the C oracle (oracle/rsync_ref.c), which restates the
rolling loop: here the weak sum at every offset is computed in closed form
from prefix sums, and the greedy walk jumps between offsets whose weak sum
occurs in the signature table.
"""
from __future__ import annotations

import hashlib

import numpy as np

CSUM_MD5, CSUM_XXH64, CSUM_XXH3_64, CSUM_XXH3_128 = 5, 6, 7, 8
BLOCK_SIZE, MAX_BLOCK_SIZE, BLOCKSUM_BIAS, SUM_LENGTH, SHORT_SUM_LENGTH = 700, 1 << 17, 10, 16, 2


def sum_sizes(length: int, block_size: int = 0):
    """generator.c sum_sizes_sqroot (protocol >= 30): blength, s2length, count, remainder."""
    if block_size:
        blength = block_size
    elif length <= BLOCK_SIZE * BLOCK_SIZE:
        blength = BLOCK_SIZE
    else:
        c, l = 1, length
        while True:
            l >>= 2
            if not l:
                break
            c <<= 1
        if c >= MAX_BLOCK_SIZE:
            blength = MAX_BLOCK_SIZE
        else:
            blength = 0
            while True:
                blength |= c
                if length < blength * blength:
                    blength &= ~c
                c >>= 1
                if c < 8:
                    break
            blength = max(blength, BLOCK_SIZE)
    b = BLOCKSUM_BIAS
    l = length
    while True:
        l >>= 1
        if not l:
            break
        b += 2
    c = blength
    while True:
        c >>= 1
        if not c or not b:
            break
        b -= 1
    s2length = int((b + 1 - 32 + 7) / 8)   # C division truncates toward zero
    s2length = min(max(s2length, SHORT_SUM_LENGTH), SUM_LENGTH)
    remainder = length % blength
    count = length // blength + (remainder != 0)
    return blength, s2length, count, remainder


def checksum1(buf: np.ndarray) -> int:
    x = buf.astype(np.int8).astype(np.int64)
    n = len(x)
    s1 = int(x.sum()) & 0xFFFFFFFF
    s2 = int(((n - np.arange(n)) * x).sum()) & 0xFFFFFFFF
    return ((s1 & 0xFFFF) + (s2 << 16)) & 0xFFFFFFFF


def checksum2(buf: bytes, csum_type: int, seed: int) -> bytes:
    import xxhash
    if csum_type == CSUM_XXH3_128:
        d = xxhash.xxh3_128_intdigest(buf, seed=seed)
        return d.to_bytes(16, "little")   # low64 LE, then high64 LE
    if csum_type == CSUM_XXH3_64:
        return xxhash.xxh3_64_intdigest(buf, seed=seed).to_bytes(8, "little") + bytes(8)
    if csum_type == CSUM_XXH64:
        return xxhash.xxh64_intdigest(buf, seed=seed).to_bytes(8, "little") + bytes(8)
    if csum_type == CSUM_MD5:
        m = hashlib.md5()
        if seed:
            m.update((seed & 0xFFFFFFFF).to_bytes(4, "little"))
        m.update(buf)
        return m.digest()
    raise ValueError(csum_type)


def signatures(basis: np.ndarray, blength: int, s2length: int, csum_type: int, seed: int):
    n = len(basis)
    count = (n + blength - 1) // blength
    s1, s2 = [], []
    for i in range(count):
        blk = basis[i * blength:(i + 1) * blength]
        s1.append(checksum1(blk))
        s2.append(checksum2(blk.tobytes(), csum_type, seed)[:s2length])
    return s1, s2


def weak_all(src: np.ndarray, blength: int) -> np.ndarray:
    """sum(o) for every offset: weak checksum of [o, min(o+blength, len))."""
    x = src.astype(np.int8).astype(np.int64)
    n = len(x)
    p0 = np.concatenate([[0], np.cumsum(x)])
    p1 = np.concatenate([[0], np.cumsum(np.arange(n, dtype=np.int64) * x)])
    o = np.arange(n, dtype=np.int64)
    e = np.minimum(o + blength, n)
    k = e - o
    s1 = p0[e] - p0[o]
    s2 = k * s1 - (p1[e] - p1[o] - o * s1)
    return ((s1 & 0xFFFF) | ((s2 & 0xFFFF) << 16)).astype(np.uint64)


def match(src: np.ndarray, sum1, sum2, blength: int, remainder: int, s2length: int,
          csum_type: int, seed: int):
    """match.c hash_search: ordered [(source offset, block index)]."""
    n = len(src)
    count = len(sum1)
    if n == 0 or count == 0:
        return []
    blen = lambda i: remainder if (i == count - 1 and remainder) else blength  # noqa: E731
    sums = weak_all(src, blength)
    by_sum = {}
    for i in range(count - 1, -1, -1):          # chains: highest index first
        by_sum.setdefault(int(sum1[i]), []).append(i)
    present = np.isin(sums, np.array(list(by_sum.keys()), dtype=np.uint64))
    cand = np.nonzero(present)[0]
    end = n + 1 - blen(count - 1)
    out = []
    want_i = 0
    offset = 0
    strong_cache = {}
    first = True
    while first or offset < end:
        first = False
        # next offset the walk evaluates that has a table hit (do-while: 0 always)
        j = int(np.searchsorted(cand, offset))
        if j >= len(cand):
            break
        o = int(cand[j])
        if o != offset and o >= end:
            break
        offset = o
        s = int(sums[offset])
        l = min(blength, n - offset)
        hit = None
        for i in by_sum.get(s, []):
            if l != blen(i):
                continue
            if offset not in strong_cache:
                strong_cache[offset] = checksum2(src[offset:offset + l].tobytes(), csum_type, seed)[:s2length]
            st = strong_cache[offset]
            if st != sum2[i]:
                continue
            if i != want_i and want_i < count and s == sum1[want_i] and st == sum2[want_i]:
                i = want_i
            hit = i
            break
        if hit is not None:
            want_i = hit + 1
            out.append((offset, hit))
            offset += blen(hit)
        else:
            offset += 1
    return out


def mutate(basis: np.ndarray, blength: int, seed: int, frac: float = 0.10, run: int = 4096):
    """C4-style source: `frac` of the blocks edited -- half overwrite a run of
    min(run, blength//2) bytes inside the block, half insert or delete 1-64 bytes."""
    rng = np.random.default_rng(seed)
    count = (len(basis) + blength - 1) // blength
    nedit = int(round(count * frac))
    blocks = np.sort(rng.choice(count, size=min(nedit, count), replace=False))
    parts = []
    pos = 0
    for b in blocks:
        a = int(b) * blength
        kind = rng.integers(0, 3)
        span = min(blength, len(basis) - a)
        if kind == 0:        # overwrite
            r = max(1, min(run, blength // 2, span))
            at = a + int(rng.integers(0, span - r + 1))
            parts.append(basis[pos:at])
            parts.append(rng.integers(0, 256, r, dtype=np.uint8))
            pos = at + r
        elif kind == 1:      # insert
            at = a + int(rng.integers(0, span))
            parts.append(basis[pos:at])
            parts.append(rng.integers(0, 256, int(rng.integers(1, 65)), dtype=np.uint8))
            pos = at
        else:                # delete
            d = int(rng.integers(1, 65))
            at = a + int(rng.integers(0, max(1, span - d)))
            parts.append(basis[pos:at])
            pos = min(len(basis), at + d)
    parts.append(basis[pos:])
    return np.concatenate(parts) if parts else basis.copy()


# ---- whole-file XXH3 as a relay of accumulator states (R7 across ranks) ----
# The public XXH3 long-input algorithm (xxhash 0.8 XXH3_hashLong, default
# secret, no seed -- rsync 3.2.3's sum_init seeds no xxhash file sum): eight
# 64-bit accumulators; each 64-byte stripe n of a 1 KiB block adds its words
# (acc[i ^ 1] += d_i) and the 32x32 products of (d_i ^ secret word n + i);
# after the block's 16 stripes every accumulator is scrambled.  A file split
# by byte range hands the accumulators from range to range; the ranks
# together chain the file's (len - 1) // 1024 whole blocks (the block holding
# the last byte is the finish's partial block even when len % 1024 == 0).
XXH3_SECRET64 = np.array([
    0xbe4ba423396cfeb8, 0x1cad21f72c81017c, 0xdb979083e96dd4de, 0x1f67b3b7a4a44072,
    0x78e5c0cc4ee679cb, 0x2172ffcc7dd05a82, 0x8e2443f7744608b8, 0x4c263a81e69035e0,
    0xcb00c391bb52283c, 0xa32e531b8b65d088, 0x4ef90da297486471, 0xd8acdea946ef1938,
    0x3f349ce33f76faa8, 0x1d4f0bc7c7bbdcf9, 0x3159b4cd4be0518a, 0x647378d9c97e9fc8,
    0xc3ebd33483acc5ea, 0xeb6313faffa081c5, 0x49daf0b751dd0d17, 0x9e68d429265516d3,
    0xfca1477d58be162b, 0xce31d07ad1b8f88f, 0x280416958f3acb45, 0x7e404bbbcafbd7af],
    dtype=np.uint64)
_P32_1, _P32_2, _P32_3 = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D
_P64 = [0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9, 0x85EBCA77C2B2AE63,
        0x27D4EB2F165667C5]


def xxh3_acc_init() -> np.ndarray:
    """XXH3_INIT_ACC."""
    return np.array([_P32_3, _P64[0], _P64[1], _P64[2], _P64[3], _P32_2, _P64[4], _P32_1],
                    dtype=np.uint64)


def xxh3_acc_blocks(data, acc) -> np.ndarray:
    """The accumulators after the whole 1 KiB blocks of `data` (a multiple of
    1024 bytes), chained from `acc`."""
    d = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    assert len(d) % 1024 == 0
    a = np.array(acc, dtype=np.uint64)
    if not len(d):
        return a
    w = np.ascontiguousarray(d).view("<u8").reshape(-1, 16, 8)          # block, stripe, lane
    key = XXH3_SECRET64[np.arange(16)[:, None] + np.arange(8)[None, :]]  # stripe n lane i
    dk = w ^ key
    with np.errstate(over="ignore"):
        prod = (dk & np.uint64(0xFFFFFFFF)) * (dk >> np.uint64(32))
        c = prod.sum(axis=1, dtype=np.uint64)                            # [block, lane]
        c[:, [1, 0, 3, 2, 5, 4, 7, 6]] += w.sum(axis=1, dtype=np.uint64)  # acc[i ^ 1] += d_i
        sec = XXH3_SECRET64[16:24]
        p = np.uint64(_P32_1)
        for b in range(len(c)):
            u = a + c[b]
            a = (u ^ (u >> np.uint64(47)) ^ sec) * p
    return a
