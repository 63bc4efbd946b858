"""Full-configuration goldens: the chunk lists and match
lists of BASELINE.json's configs at their real sizes, computed in this
container by the C oracle (oracle/cdc_ref.c, oracle/rsync_ref.c) with many
threads, and stored as (count, SHA-256 digest) so a bench line can check its
own output without holding the list.

Digests (the record layouts are the ABI structs, so a bench line hashes the
arrays it read back as they are):
  * chunk list: SHA-256 over 56-byte records -- start, length, cut (u64 LE)
    and the 32-byte blob ID -- in stream order (vs_chunk);
  * match list: SHA-256 over 16-byte records -- offset (i64 LE), block index
    (i32 LE), 0 (i32) -- in file order (vs_match), plus the false-alarm count
    (rsync's stats, part of hash_search's output).

CDC: C2 (64 GiB, seed 2) and the C3 stream (seed 3) at the bench's per-GPU
share: the N-rank bench runs N x 128 GiB of it as one final stream, and a
prefix's chunk list is the full list's chunks that end inside it plus one EOF
chunk, so one 1 TiB pass gives N = 1, 2, 4, 8.

rsync (C4, bench.py C4Plan): destinations of 8, 16, 64, 128 and 256 GiB (seed 4,
xxh128, checksum_seed 0x5EED5EED), each against its 10 %-edited source.  The
source is walked in 1 GiB ranges in parallel from speculative entries, then
stitched in order: the walk from each range's true entry runs to the first
speculative match at or after it and merges there (same state from then on;
the false alarms before the merge are the speculative record's `fab`), else
the range is re-walked whole.  256 GiB also gets the 8-rank split of the real
C4 (SourceShard), per rank: its own matches, false alarms and true entry.

C5 (bench.py --mode smallfiles): the digest of all 1 M blob IDs in file order,
the distinct-ID count and the bytes.

usage: python tests/golden/make_golden_full.py [cdc|c3|distinct|rsync|filesum|c5|all] [--threads T]
       [--rsync-gib G ...] [--skip-c3]
writes tests/golden/full_configs.json (merged with what is there).
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from tests import oracle_lib as O  # noqa: E402

OUT = os.path.join(HERE, "full_configs.json")
POL, MN, MX, AVG = 0x3DA3358B4DC173, 512 << 10, 8 << 20, 20
GiB = 1 << 30
CSUM_XXH3_128, SEED = 8, 0x5EED5EED
DISTINCT_SEEDS = (2, 7, 8)   # bench.py --distinct: volume k of the run is seed [k % B]


def chunk_records(starts, lens, cuts, ids) -> np.ndarray:
    rec = np.zeros((len(starts), 56), np.uint8)
    rec[:, 0:8] = np.asarray(starts, np.uint64).reshape(-1, 1).view(np.uint8)
    rec[:, 8:16] = np.asarray(lens, np.uint64).reshape(-1, 1).view(np.uint8)
    rec[:, 16:24] = np.asarray(cuts, np.uint64).reshape(-1, 1).view(np.uint8)
    rec[:, 24:56] = np.asarray(ids, np.uint8).reshape(-1, 32)
    return rec


def match_records(offs, idxs) -> np.ndarray:
    rec = np.zeros((len(offs), 16), np.uint8)
    rec[:, 0:8] = np.asarray(offs, np.int64).reshape(-1, 1).view(np.uint8)
    rec[:, 8:12] = np.asarray(idxs, np.int32).reshape(-1, 1).view(np.uint8)
    return rec


def digest(rec: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(rec).tobytes()).hexdigest()


def eof_chunk(seed: int, s: int, end: int):
    """The final chunk [s, end) of a stream that ends at `end`: Next()'s Cut
    from its start (the EOF digest rules) and its blob ID."""
    tail = O.synth(seed, s, end - s)
    ch = O.cdc_hash(tail, POL, MN, MX, AVG)
    assert len(ch) == 1 and ch[0][1] == end - s, ch[:2]
    return s, end - s, ch[0][2], bytes.fromhex(ch[0][3])


def cdc_golden(seed: int, length: int, prefixes, threads: int, per_rank: int = 0) -> dict:
    t0 = time.time()
    s, ln, c, ids = O.cdc_synth_mt(seed, length, POL, MN, MX, AVG, threads)
    print(f"cdc seed {seed}: {length >> 30} GiB, {len(s)} chunks in {time.time() - t0:.0f} s",
          flush=True)
    ends = s + ln
    out = {}
    for L in prefixes:
        k = int(np.searchsorted(ends, L, side="right"))   # chunks ending at or before L
        rec = chunk_records(s[:k], ln[:k], c[:k], ids[:k])
        if k < len(s) and int(s[k]) < L:
            e = eof_chunk(seed, int(s[k]), L)
            rec = np.concatenate([rec, chunk_records([e[0]], [e[1]], [e[2]],
                                                     np.frombuffer(e[3], np.uint8))])
        out[str(L)] = {"seed": seed, "bytes": L, "chunks": int(len(rec)), "digest": digest(rec),
                       "first": [int(rec[0, :8].view(np.uint64)[0]), int(rec[0, 8:16].view(np.uint64)[0])],
                       "pol": hex(POL), "min": MN, "max": MX, "avg_bits": AVG}
        if per_rank and L % per_rank == 0 and L > per_rank:
            # the W-rank byte-range split of this prefix (volsync_amd/shard.py
            # ShardSpec): rank r's chunks are those starting in [own_lo, own_hi),
            # its true entry the first chunk start at or after own_lo
            W = L // per_rank
            st = rec[:, 0:8].copy().view(np.uint64).ravel()
            ranks = []
            for r in range(W):
                lo, hi = L * r // W, L * (r + 1) // W
                a = int(np.searchsorted(st, lo, side="left"))
                b = int(np.searchsorted(st, hi, side="left"))
                ranks.append({"rank": r, "own_lo": lo, "own_hi": hi,
                              "entry": int(st[a]) if a < len(st) else L,
                              "chunks": b - a, "digest": digest(rec[a:b])})
            out[str(L)]["ranks"] = ranks
    return out


# ---- rsync ----------------------------------------------------------------
_L = None


def walk_lib():
    global _L
    if _L is None:
        L = O._rs()
        i64, i32, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.ref_rsync_walk_fab.restype = i64
        L.ref_rsync_walk_fab.argtypes = [vp, i64, i64, i64, i64, i32, i32, i32, i32, i32, vp, vp,
                                         ctypes.c_int, ctypes.c_uint32, vp, vp, vp, i64,
                                         ctypes.POINTER(i64), ctypes.POINTER(i64),
                                         ctypes.POINTER(i32)]
        _L = L
    return _L


def fill_source(plan, lo: int, hi: int) -> np.ndarray:
    buf = np.empty(max(hi - lo, 1), np.uint8)
    for d, seed, off, n in plan.segments(lo, hi):
        O.lib().ref_synth_fill(seed, off, n, buf[d:].ctypes.data)
    return buf[: hi - lo]


def walk(plan, tab, lo: int, hi: int, entry: int, want: int):
    """ref_rsync_walk_fab over [entry, hi) of the plan's source: (offs, idxs,
    fab, fa, exit_off, exit_want)."""
    s1, s2, blength, rem = tab
    win_hi = min(hi + blength - 1, plan.total)
    win = fill_source(plan, entry, win_hi)
    cap = max(0, hi - entry) // blength + 8
    mo, mi, mf = np.zeros(cap, np.int64), np.zeros(cap, np.int32), np.zeros(cap, np.int64)
    fa, eo, ew = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
    n = walk_lib().ref_rsync_walk_fab(win.ctypes.data, entry, plan.total, hi, entry, want, len(s1),
                                      blength, rem, s2.shape[1], s1.ctypes.data, s2.ctypes.data,
                                      CSUM_XXH3_128, SEED, mo.ctypes.data, mi.ctypes.data,
                                      mf.ctypes.data, cap, ctypes.byref(fa), ctypes.byref(eo),
                                      ctypes.byref(ew))
    assert 0 <= n <= cap, n
    return mo[:n], mi[:n], mf[:n], int(fa.value), int(eo.value), int(ew.value)


def rsync_golden(dlen: int, threads: int, ranks: int = 0, piece: int = GiB) -> dict:
    from bench import C4Plan
    t0 = time.time()
    bl, s2l, count, rem = O.rsync_sizes(dlen)
    s1, s2 = O.rsync_signatures_synth_mt(C4Plan.D_SEED, dlen, bl, s2l, CSUM_XXH3_128, SEED,
                                         threads)
    keys = s1.astype(np.uint64) << np.uint64(32)
    dup = len(np.unique(np.concatenate([s1.reshape(-1, 1).view(np.uint8).reshape(-1, 4), s2],
                                       axis=1), axis=0)) != count
    plan = C4Plan(dlen, bl)
    print(f"rsync {dlen >> 30} GiB: table of {count} blocks in {time.time() - t0:.0f} s "
          f"(duplicate blocks: {dup}); source {plan.total} bytes, {plan.edits} edits", flush=True)
    del keys
    tab = (s1, s2, bl, rem)
    # ranges: each rank's own range (the real C4 split when ranks > 0) cut into pieces
    cuts = {0, plan.total}
    if ranks:
        cuts |= {plan.total * r // ranks for r in range(ranks)}
    bounds = sorted(cuts)
    ranges = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        k = max(1, -(-(b - a) // piece))
        ranges += [(a + (b - a) * j // k, a + (b - a) * (j + 1) // k) for j in range(k)]
    t1 = time.time()

    def spec(r):
        lo, hi = r
        return walk(plan, tab, lo, hi, lo, 0 if lo == 0 else count)
    with ThreadPoolExecutor(threads) as ex:
        specs = list(ex.map(spec, ranges))
    print(f"  speculative walks of {len(ranges)} ranges in {time.time() - t1:.0f} s", flush=True)
    t2 = time.time()
    e, w = 0, 0
    res = []   # per range: offs, idxs, fa, entry
    rewalks = 0
    for (lo, hi), sp in zip(ranges, specs):
        so, si, sf, sfa, sx, sw = sp
        ent = (e, w)
        if e >= hi:
            res.append((so[:0], si[:0], 0, ent))
            continue
        if (e, w) == (lo, 0 if lo == 0 else count):
            res.append((so, si, sfa, ent))
            e, w = sx, sw
            continue
        j = int(np.searchsorted(so, e, side="left"))
        merged = False
        if j < len(so) and not dup:
            ho, hi_, _, hfa, hx, hw = walk(plan, tab, lo, int(so[j]), e, w)
            if hx == int(so[j]):
                res.append((np.concatenate([ho, so[j:]]), np.concatenate([hi_, si[j:]]),
                            hfa + sfa - int(sf[j]), ent))
                e, w = sx, sw
                merged = True
        if not merged:
            rewalks += 1
            ro, ri, _, rfa, rx, rw = walk(plan, tab, lo, hi, e, w)
            res.append((ro, ri, rfa, ent))
            e, w = rx, rw
    print(f"  stitched in {time.time() - t2:.0f} s ({rewalks} whole-range re-walks)", flush=True)
    offs = np.concatenate([r[0] for r in res])
    idxs = np.concatenate([r[1] for r in res])
    fa = sum(r[2] for r in res)
    assert np.all(np.diff(offs) > 0)
    out = {"dlen": dlen, "source_bytes": plan.total, "edits": plan.edits, "blength": bl,
           "s2length": s2l, "count": count, "csum": "xxh128", "checksum_seed": hex(SEED),
           "matches": int(len(offs)), "false_alarms": int(fa),
           "digest": digest(match_records(offs, idxs)),
           "duplicate_blocks": bool(dup)}
    if ranks:
        per = []
        for r in range(ranks):
            lo, hi = plan.total * r // ranks, plan.total * (r + 1) // ranks
            sel = [k for k, rg in enumerate(ranges) if lo <= rg[0] < hi]
            o = np.concatenate([res[k][0] for k in sel])
            i = np.concatenate([res[k][1] for k in sel])
            per.append({"rank": r, "own_lo": lo, "own_hi": hi,
                        "entry": [int(res[sel[0]][3][0]), int(res[sel[0]][3][1])],
                        "matches": int(len(o)), "false_alarms": int(sum(res[k][2] for k in sel)),
                        "digest": digest(match_records(o, i))})
        out["ranks"] = {str(ranks): per}
    print(f"  {out['matches']} matches, {fa} false alarms, total {time.time() - t0:.0f} s",
          flush=True)
    return out


def file_sum_golden(dlen: int, threads: int) -> str:
    """checksum.c's whole-file xxh128 (unseeded) of the C4 source S for a
    destination of dlen bytes: libxxhash streaming over S generated in 256 MiB
    pieces by `threads` threads, in order."""
    import xxhash
    from bench import C4Plan
    bl = O.rsync_sizes(dlen)[0]
    plan = C4Plan(dlen, bl)
    h = xxhash.xxh3_128()
    step = 256 << 20
    offs = list(range(0, plan.total, step))
    with ThreadPoolExecutor(threads) as ex:
        for k in range(0, len(offs), threads):
            for buf in ex.map(lambda o: fill_source(plan, o, min(o + step, plan.total)),
                              offs[k:k + threads]):
                h.update(buf)
    return h.intdigest().to_bytes(16, "little").hex()


def c5_golden(files: int, threads: int) -> dict:
    """C5 (bench.py --mode smallfiles, c5_layout): SHA-256 over the 32-byte
    blob IDs of all files in file order, the number of distinct IDs and the
    file bytes.  A file's content is its payload, so each distinct payload is
    hashed once (hashlib / OpenSSL, `threads` threads) from the C oracle's
    synthetic stream."""
    import bench
    sizes, pick, psize, npay = bench.c5_layout(files, 0)
    used = np.unique(pick)
    ids = np.zeros((npay, 32), np.uint8)

    def one(j):
        ids[j] = np.frombuffer(hashlib.sha256(O.synth(6, int(j) << 16, int(psize[j])).tobytes())
                               .digest(), np.uint8)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, used.tolist()))
    d = digest(ids[pick])
    return {"files": files, "bytes": int(sizes.sum()), "unique_ids": int(len(used)),
            "id_digest": d, "payloads": npay}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all",
                    choices=["cdc", "c3", "distinct", "rsync", "filesum", "c5", "all"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--rsync-gib", type=int, nargs="*", default=[8, 16, 64, 128, 256])
    ap.add_argument("--skip-c3", action="store_true", help="cdc: keep the 1 TiB entries")
    a = ap.parse_args()
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data["_about"] = ("tests/golden/make_golden_full.py: full-size chunk / match list digests "
                      "(vs_chunk / vs_match records, SHA-256) from the C oracle")
    if a.what in ("cdc", "all"):
        # data["cdc"][seed][length]: the chunk list of the stream's first
        # `length` bytes as one final stream (C2 = seed 2 at 64 GiB and its
        # power-of-two prefixes, for the shared-GPU rehearsals; C3 = seed 3
        # at N x 128 GiB)
        cdc = data.setdefault("cdc", {})
        cdc.setdefault("2", {}).update(
            cdc_golden(2, 64 * GiB, [(1 << k) * GiB for k in range(7)], a.threads))
        json.dump(data, open(OUT, "w"), indent=1)
    if a.what in ("cdc", "c3", "all"):
        cdc = data.setdefault("cdc", {})
        if not a.skip_c3:
            cdc.setdefault("3", {}).update(
                cdc_golden(3, 1024 * GiB, [128 * GiB, 256 * GiB, 512 * GiB, 1024 * GiB], a.threads,
                           per_rank=128 * GiB))
        json.dump(data, open(OUT, "w"), indent=1)
    if a.what in ("distinct", "all"):
        # bench.py --distinct B: the C2 shape over distinct volumes, seeds 2, 7, 8
        cdc = data.setdefault("cdc", {})
        for sd in DISTINCT_SEEDS[1:]:
            cdc.setdefault(str(sd), {}).update(cdc_golden(sd, 64 * GiB, [64 * GiB], a.threads))
            json.dump(data, open(OUT, "w"), indent=1)
    if a.what in ("rsync", "all"):
        data.setdefault("rsync", {})
        for g in a.rsync_gib:
            data["rsync"][str(g * GiB)] = rsync_golden(g * GiB, a.threads,
                                                        ranks=8 if g == 256 else 0)
            json.dump(data, open(OUT, "w"), indent=1)
    if a.what in ("filesum", "all"):
        for g in a.rsync_gib:
            t0 = time.time()
            ent = data.setdefault("rsync", {}).setdefault(str(g * GiB), {})
            ent["file_sum"] = file_sum_golden(g * GiB, a.threads)
            print(f"file sum of the {g} GiB C4 source in {time.time() - t0:.0f} s", flush=True)
            json.dump(data, open(OUT, "w"), indent=1)
    if a.what in ("c5", "all"):
        t0 = time.time()
        data.setdefault("c5", {})["1000000"] = c5_golden(1_000_000, a.threads)
        print(f"C5 IDs in {time.time() - t0:.0f} s", flush=True)
    json.dump(data, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
