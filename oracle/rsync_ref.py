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
