"""Independent Python restatement of restic's chunker + SHA-256 blob IDs.

TEST INFRASTRUCTURE ONLY -- used by tests/golden/make_golden.py to produce the
committed golden fixtures and by tests/ as a second opinion.  The product path
never imports this module.

It deliberately uses a *different* algorithm from the C oracle
(oracle/cdc_ref.c, which restates chunker.go's rolling loop byte by byte):

* the fingerprint at every offset is computed in closed form,
  FP(p) = (sum_i B[p-63+i] * x^(8*(63-i))) mod P, as an XOR of 64 per-offset
  256-entry tables (vectorised with numpy);
* cut selection is then the min/max rule of chunker.go Next()
   applied to the candidate set.

Reference behaviour restated (upstream module pinned by restic v0.13.1, which
/root/reference/mover-restic/Dockerfile:8-11 clones; not vendored):
  github.com/restic/chunker@v0.4.0 polynomials.go (Pol.Deg, Pol.Mod),
  chunker.go (fillTables, reset, Next); restic internal/restic/id.go Hash
  = crypto/sha256.Sum256 (patched in by mover-restic/patch-sources.sh:16-27).
"""
from __future__ import annotations

import hashlib

import numpy as np

TEST_POL = 0x3DA3358B4DC173          # chunker_test.go testPol (degree 53, irreducible)
MIN_SIZE = 512 * 1024                 # chunker.go MinSize
MAX_SIZE = 8 * 1024 * 1024            # chunker.go MaxSize
AVG_BITS = 20                         # splitmask = 2^20 - 1
WINDOW = 64

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def pol_deg(p: int) -> int:
    return p.bit_length() - 1


def pol_mod(x: int, d: int) -> int:
    dd = pol_deg(d)
    while x and pol_deg(x) >= dd:
        x ^= d << (pol_deg(x) - dd)
    return x


def pol_mulmod(a: int, b: int, p: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        b >>= 1
    return pol_mod(r, p)


def pol_irreducible(p: int) -> bool:
    """Ben-Or test: p irreducible iff gcd(x^(2^i) - x, p) == 1 for i <= deg/2."""
    def gcd(a, b):
        while b:
            a, b = b, pol_mod(a, b)
        return a
    d = pol_deg(p)
    xp = 2  # x
    for _ in range(d // 2):
        xp = pol_mulmod(xp, xp, p)
        if gcd(p, xp ^ 2) != 1:
            return False
    return True


def offset_tables(pol: int) -> np.ndarray:
    """T[i][b] = b * x^(8*(63-i)) mod pol, i = 0..63 (i = 63 is the newest byte)."""
    t = np.zeros((WINDOW, 256), dtype=np.uint64)
    for i in range(WINDOW):
        e = pol_mod(1, pol)                  # x^(8*(63-i)) mod pol
        for _ in range(63 - i):
            e = pol_mod(e << 8, pol)
        for b in range(256):
            t[i, b] = pol_mulmod(b, e, pol)
    return t


def window_fp_all(data: np.ndarray, pol: int, tables: np.ndarray | None = None) -> np.ndarray:
    """FP(p) for p in [63, len): returns array of length len-63 (index p-63)."""
    if tables is None:
        tables = offset_tables(pol)
    n = data.shape[0]
    if n < WINDOW:
        return np.zeros(0, dtype=np.uint64)
    m = n - 63
    fp = np.zeros(m, dtype=np.uint64)
    for i in range(WINDOW):
        fp ^= tables[i][data[i:i + m]]
    return fp


def candidates(data: np.ndarray, pol: int, avg_bits: int, block: int = 1 << 24):
    """Sorted candidate positions p (p >= 63) with FP(p) & mask == 0, plus their FP."""
    mask = np.uint64((1 << avg_bits) - 1)
    tables = offset_tables(pol)
    n = data.shape[0]
    pos_l, fp_l = [], []
    lo = 63
    while lo < n:
        hi = min(n, lo + block)
        fp = window_fp_all(data[lo - 63:hi], pol, tables)
        hit = np.nonzero((fp & mask) == 0)[0]
        pos_l.append(hit.astype(np.int64) + lo)
        fp_l.append(fp[hit])
        lo = hi
    if not pos_l:
        return np.zeros(0, np.int64), np.zeros(0, np.uint64)
    return np.concatenate(pos_l), np.concatenate(fp_l)


def fp_at(data: np.ndarray, p: int, pol: int) -> int:
    h = 0
    for i in range(WINDOW):
        h = pol_mod((h << 8) | int(data[p - 63 + i]), pol)
    return h


def eof_cut(data: np.ndarray, s: int, n: int, pol: int, min_size: int) -> int:
    """Chunk.Cut of the final (EOF) chunk [s, n): the live digest after reset().

    reset() slides a 1 into a zeroed window (digest 1) and skips MinSize-64
    bytes; h = bytes actually hashed.  For h >= 64 the 1 has left the window.
    """
    length = n - s
    h = length - (min_size - WINDOW) if length > min_size - WINDOW else 0
    if h >= WINDOW:
        return fp_at(data, n - 1, pol)
    d = 1
    for j in range(n - h, n):
        d = pol_mod((d << 8) | int(data[j]), pol)
    return d


def chunk(data: np.ndarray, pol: int = TEST_POL, min_size: int = MIN_SIZE,
          max_size: int = MAX_SIZE, avg_bits: int = AVG_BITS, with_ids: bool = True):
    """List of (start, length, cut, sha256-hex) for the whole buffer."""
    n = int(data.shape[0])
    cpos, cfp = candidates(data, pol, avg_bits)
    out = []
    s = 0
    while s < n:
        q = s + min_size - 1
        lim = s + max_size - 1
        k = int(np.searchsorted(cpos, q, side="left"))
        if k < len(cpos) and cpos[k] <= lim:
            c, cut = int(cpos[k]), int(cfp[k])
        elif lim <= n - 1:
            c, cut = lim, fp_at(data, lim, pol)
        else:
            c, cut = n - 1, eof_cut(data, s, n, pol, min_size)
        length = c - s + 1
        ident = hashlib.sha256(data[s:c + 1].tobytes()).hexdigest() if with_ids else ""
        out.append((s, length, cut, ident))
        s = c + 1
    return out


def synth(seed: int, off: int, n: int) -> np.ndarray:
    """Bytes [off, off+n) of the splitmix64 word stream."""
    w0 = off >> 3
    w1 = (off + n + 7) >> 3
    i = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    a = off - (w0 << 3)
    return b[a:a + n].copy()
