"""Host-side mirror of rsync 3.2.3's sender-side delta interface over the C ABI.

rsync (installed by /root/reference/mover-rsync/Dockerfile:11-12, run from
mover-rsync/source.sh:54) is C; its delta stage is a handful of functions over
`struct sum_struct`.  Names and argument meaning follow them:

  sum_sizes_sqroot(len)            generator.c  -> SumStruct header
  generate_sums(basis, ...)        generator.c generate_and_send_sums
                                   (get_checksum1 + get_checksum2 per block)
  Matcher.load_sums(sums)          match.c build_hash_table
  Matcher.match_sums(src)          match.c match_sums -> hash_search
                                   -> [(offset, block_index)] = matched() calls

All compute runs in volsync_amd/lib/libvsgpu.so on a gfx950 device; there is
no CPU fallback (a missing library raises ImportError, a missing device
VsError(VS_ERR_NO_DEVICE)).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from ._lib import VsMatch, VsSigTable, check, lib

CSUM_MD5, CSUM_XXH64, CSUM_XXH3_64, CSUM_XXH3_128 = 5, 6, 7, 8


@dataclass
class SumStruct:
    """match.c / rsync.h `struct sum_struct`: header plus per-block sums."""
    flength: int
    count: int
    blength: int
    s2length: int
    remainder: int
    sum1: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    sum2: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.uint8))

    def block_len(self, i: int) -> int:
        return self.remainder if (i == self.count - 1 and self.remainder) else self.blength


def sum_sizes_sqroot(length: int, block_size: int = 0) -> SumStruct:
    v = [ctypes.c_int32() for _ in range(4)]
    check(lib.vs_rsync_sizes(int(length), int(block_size), *[ctypes.byref(x) for x in v]))
    bl, s2, cnt, rem = (x.value for x in v)
    return SumStruct(flength=int(length), count=cnt, blength=bl, s2length=s2, remainder=rem)


def _host_bytes(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def generate_sums(basis, csum_type: int = CSUM_XXH3_128, seed: int = 0, block_size: int = 0,
                  device: int = 0) -> SumStruct:
    """Signatures of a host buffer (copied to the device)."""
    b = _host_bytes(basis)
    s = sum_sizes_sqroot(len(b), block_size)
    s.sum1 = np.zeros(max(s.count, 1), np.uint32)
    s.sum2 = np.zeros((max(s.count, 1), s.s2length), np.uint8)
    check(lib.vs_rsync_signatures(device, b.ctypes.data if len(b) else None, len(b), s.blength,
                                  s.s2length, csum_type, seed & 0xFFFFFFFF, s.sum1.ctypes.data,
                                  s.sum2.ctypes.data))
    s.sum1, s.sum2 = s.sum1[: s.count], s.sum2[: s.count]
    return s


class Matcher:
    """A vs_rsync handle: device signatures, table and match runs."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        check(lib.vs_rsync_open(device, ctypes.byref(self._h)))

    def close(self) -> None:
        if self._h:
            lib.vs_rsync_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream: int) -> None:
        check(lib.vs_rsync_set_stream(self._h, ctypes.c_void_p(hip_stream or None)))

    def signatures_device(self, dev_basis: int, length: int, blength: int, s2length: int,
                          csum_type: int, seed: int, dev_sum1: int, dev_sum2: int) -> None:
        check(lib.vs_rsync_signatures_device(self._h, ctypes.c_void_p(dev_basis or None), length,
                                             blength, s2length, csum_type, seed & 0xFFFFFFFF,
                                             ctypes.c_void_p(dev_sum1 or None),
                                             ctypes.c_void_p(dev_sum2 or None)))

    def load_sums(self, s: SumStruct, csum_type: int = CSUM_XXH3_128, seed: int = 0) -> None:
        s1 = np.ascontiguousarray(s.sum1, np.uint32)
        s2 = np.ascontiguousarray(s.sum2, np.uint8)
        check(lib.vs_rsync_load_sums(self._h, s.count, s.blength, s.s2length, s.remainder,
                                     s1.ctypes.data if s.count else None,
                                     s2.ctypes.data if s.count else None, csum_type,
                                     seed & 0xFFFFFFFF))

    def load_sums_device(self, count: int, blength: int, s2length: int, remainder: int,
                         dev_sum1: int, dev_sum2: int, csum_type: int, seed: int) -> None:
        check(lib.vs_rsync_load_sums_device(self._h, count, blength, s2length, remainder,
                                            ctypes.c_void_p(dev_sum1 or None),
                                            ctypes.c_void_p(dev_sum2 or None), csum_type,
                                            seed & 0xFFFFFFFF))

    def match_device(self, dev_src: int, length: int) -> int:
        n = ctypes.c_int64(0)
        check(lib.vs_rsync_match_device(self._h, ctypes.c_void_p(dev_src or None), length,
                                        ctypes.byref(n)))
        self._last_n = n.value
        return n.value

    # ---- sharded hash_search (volsync_amd/rsync_shard.py run_walk_shard) ----
    def match_scan(self, dev_src: int, length: int, origin: int, file_len: int, own_lo: int,
                   own_hi: int) -> Tuple[int, int]:
        """Candidates + speculative walk of file offsets [own_lo, own_hi);
        returns the speculative exit state (offset, want_i)."""
        eo, ew = ctypes.c_int64(0), ctypes.c_int32(0)
        check(lib.vs_rsync_match_scan(self._h, ctypes.c_void_p(dev_src or None), length, origin,
                                      file_len, own_lo, own_hi, ctypes.byref(eo), ctypes.byref(ew)))
        return int(eo.value), int(ew.value)

    def match_stitch(self, entry: int, want_i: int) -> Tuple[int, int]:
        """Re-walk from the true entry state; returns the new exit state."""
        eo, ew = ctypes.c_int64(0), ctypes.c_int32(0)
        check(lib.vs_rsync_match_stitch(self._h, entry, want_i, ctypes.byref(eo),
                                        ctypes.byref(ew)))
        return int(eo.value), int(ew.value)

    def match_finish(self) -> int:
        n = ctypes.c_int64(0)
        check(lib.vs_rsync_match_finish(self._h, ctypes.byref(n)))
        self._last_n = n.value
        return n.value

    def matches(self, first: int = 0, n: Optional[int] = None) -> List[Tuple[int, int]]:
        if n is None:
            n = self.stats()["matches"] - first
        arr = (VsMatch * max(n, 1))()
        check(lib.vs_rsync_get_matches(self._h, first, n, arr))
        return [(arr[i].offset, arr[i].block_index) for i in range(n)]

    def stats(self) -> dict:
        c, fa, sh = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        r = ctypes.c_int32()
        check(lib.vs_rsync_stats(self._h, ctypes.byref(c), ctypes.byref(fa), ctypes.byref(sh),
                                 ctypes.byref(r)))
        return {"candidates": c.value, "false_alarms": fa.value, "strong_hashed": sh.value,
                "rounds": r.value, "matches": self._last_n}

    def timing(self) -> dict:
        ms = (ctypes.c_double * 5)()
        check(lib.vs_rsync_timing(self._h, ms))
        return dict(zip(["signatures", "table", "scan", "verify", "walk"], list(ms)))

    KERNELS = ("scan", "verify", "signatures", "stitch", "file_sum")

    def kernel_time(self, reset: bool = False) -> dict:
        """{kernel: (ms summed over launches, launches)} from HIP events."""
        out = {}
        for w, name in enumerate(self.KERNELS):
            ms, n = ctypes.c_double(0), ctypes.c_int64(0)
            check(lib.vs_rsync_kernel_time(self._h, w, 1 if reset else 0, ctypes.byref(ms),
                                           ctypes.byref(n)))
            out[name] = (ms.value, n.value)
        return out

    def file_sum(self, dev_src: int, length: int, csum_type: int = 8) -> bytes:
        """checksum.c sum_init/sum_update/sum_end over the whole device file
        (vs_rsync_file_sum): 16 bytes for xxh128 / md5, 8 for xxh3 / xxh64."""
        out = ctypes.create_string_buffer(16)
        check(lib.vs_rsync_file_sum(self._h, ctypes.c_void_p(dev_src), length, csum_type, out))
        return out.raw[: 16 if csum_type in (CSUM_MD5, CSUM_XXH3_128) else 8]

    def file_sum_start(self, dev_src: int, length: int, csum_type: int = 8) -> None:
        """vs_rsync_file_sum_start: the device part queued, the host chain on a
        library thread; dev_src must stay valid until file_sum_wait."""
        check(lib.vs_rsync_file_sum_start(self._h, ctypes.c_void_p(dev_src or None), length,
                                          csum_type))
        self._fs_csum = csum_type

    def file_sum_wait(self) -> bytes:
        out = ctypes.create_string_buffer(16)
        check(lib.vs_rsync_file_sum_wait(self._h, out))
        return out.raw[: 16 if self._fs_csum in (CSUM_MD5, CSUM_XXH3_128) else 8]

    def file_sum_blocks_start(self, dev_blocks: int, nblocks: int, acc_in=None) -> None:
        """One byte range of a file split across ranks: chain its whole 1 KiB
        blocks from acc_in (None: the initial state)."""
        a = None if acc_in is None else np.ascontiguousarray(acc_in, np.uint64)
        self._acc_in = a
        check(lib.vs_rsync_file_sum_blocks_start(self._h, ctypes.c_void_p(dev_blocks or None),
                                                 nblocks, None if a is None else a.ctypes.data))

    def file_sum_blocks_wait(self) -> np.ndarray:
        acc = np.zeros(8, np.uint64)
        check(lib.vs_rsync_file_sum_blocks_wait(self._h, acc.ctypes.data))
        return acc

    def file_sum_timing(self) -> dict:
        d, hm = ctypes.c_double(0), ctypes.c_double(0)
        check(lib.vs_rsync_file_sum_timing(self._h, ctypes.byref(d), ctypes.byref(hm)))
        return {"device_ms": d.value, "host_chain_ms": hm.value}

    _fs_csum = 8

    def reconstruct(self, dev_out: int, out_len: int, dev_basis: int, basis_len: int,
                    blength: int, matches: List[Tuple[int, int]], dev_literals: int,
                    literal_len: int) -> None:
        """receiver.c receive_data (vs_rsync_reconstruct): rebuild the file from
        the basis, the match list and the gaps' literal bytes."""
        arr = (VsMatch * max(len(matches), 1))()
        for k, (o, i) in enumerate(matches):
            arr[k].offset, arr[k].block_index = o, i
        check(lib.vs_rsync_reconstruct(self._h, ctypes.c_void_p(dev_out), out_len,
                                       ctypes.c_void_p(dev_basis), basis_len, blength, arr,
                                       len(matches), ctypes.c_void_p(dev_literals), literal_len))

    def match_sums(self, dev_src: int, length: int) -> List[Tuple[int, int]]:
        return self.matches(0, self.match_device(dev_src, length))

    # ---- streamed forms: a file fed from host memory (vs_rsync_match_* / sig_*) ----
    def match_begin(self, file_len: int, piece: int = 0, ring: int = 0, file_csum: int = 0) -> None:
        """match_sums over a file of file_len bytes that arrives by feed();
        the device holds at most `ring` pieces of `piece` bytes; file_csum:
        also the whole-file checksum of that type (match_end returns it)."""
        check(lib.vs_rsync_match_begin(self._h, file_len, file_csum, piece, ring))
        self._ms_csum = file_csum

    def match_feed(self, buf, n: Optional[int] = None) -> None:
        """Next bytes of the file: a host address with n, or a buffer."""
        if n is None:
            b = _host_bytes(buf)
            check(lib.vs_rsync_match_feed(self._h, b.ctypes.data if len(b) else None, len(b)))
        else:
            check(lib.vs_rsync_match_feed(self._h, ctypes.c_void_p(buf or None), n))

    def match_next(self, cap: int = 65536) -> Optional[List[Tuple[int, int]]]:
        """Matches found so far, in order; None at the end of the list."""
        arr = (VsMatch * max(cap, 1))()
        n = ctypes.c_size_t(0)
        rc = check(lib.vs_rsync_match_next(self._h, arr, cap, ctypes.byref(n)))
        if rc == 1 and n.value == 0:
            return None
        return [(arr[i].offset, arr[i].block_index) for i in range(n.value)]

    def match_end(self):
        """Waits for the walk: (matches, false alarms) of the whole file, plus
        the whole-file checksum when the stream was begun with file_csum."""
        nm, fa = ctypes.c_int64(0), ctypes.c_int64(0)
        fs = ctypes.create_string_buffer(16) if self._ms_csum else None
        check(lib.vs_rsync_match_end(self._h, ctypes.byref(nm), ctypes.byref(fa), fs))
        self._last_n = nm.value
        if fs is None:
            return nm.value, fa.value
        return nm.value, fa.value, fs.raw[: 16 if self._ms_csum in (CSUM_MD5, CSUM_XXH3_128) else 8]

    _ms_csum = 0

    def match_stream_stats(self) -> dict:
        st = (ctypes.c_double * 10)()
        check(lib.vs_rsync_match_stream_stats(self._h, st))
        return {"pinned_bytes": st[0], "staged_bytes": st[1], "feed_wait_ms": st[2],
                "walk_ms": st[3], "walk_idle_ms": st[4], "pieces": int(st[5]),
                "piece_bytes": int(st[6]), "ring": int(st[7]), "file_sum_ms": st[8],
                "file_csum": int(st[9])}

    def sig_begin(self, length: int, blength: int, s2length: int, csum_type: int, seed: int,
                  piece: int = 0, ring: int = 0) -> None:
        check(lib.vs_rsync_sig_begin(self._h, length, blength, s2length, csum_type,
                                     seed & 0xFFFFFFFF, piece, ring))
        self._sig_s2 = s2length

    def sig_feed(self, buf, n: Optional[int] = None) -> None:
        if n is None:
            b = _host_bytes(buf)
            check(lib.vs_rsync_sig_feed(self._h, b.ctypes.data if len(b) else None, len(b)))
        else:
            check(lib.vs_rsync_sig_feed(self._h, ctypes.c_void_p(buf or None), n))

    def sig_next(self, cap: int = 1 << 16):
        """(sum1 [n] u32, sum2 [n, s2length]) of the next finished blocks, or
        None after the last."""
        s1 = np.zeros(max(cap, 1), np.uint32)
        s2 = np.zeros((max(cap, 1), self._sig_s2), np.uint8)
        n = ctypes.c_size_t(0)
        rc = check(lib.vs_rsync_sig_next(self._h, s1.ctypes.data, s2.ctypes.data, cap,
                                         ctypes.byref(n)))
        if rc == 1 and n.value == 0:
            return None
        return s1[: n.value], s2[: n.value]

    def set_option(self, option: int, value: int) -> None:
        """vs_rsync_set_option (volsync_amd._lib VS_OPT_*)."""
        check(lib.vs_rsync_set_option(self._h, option, value))

    _sig_s2 = 2

    _last_n = 0


class ZstdTokens:
    """One rsync -z transfer's token-stream state (token.c send_zstd_token /
    recv_zstd_token, vs_ztok): write() the files of a transfer in order on the
    sender's object, read() them in order on the receiver's."""

    def __init__(self, level: int = 3):
        self._z = ctypes.c_void_p()
        check(lib.vs_ztok_open(level, ctypes.byref(self._z)))

    def close(self) -> None:
        if self._z:
            lib.vs_ztok_close(self._z)
            self._z = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def write(self, matches, src, blength: int, basis_len: int, last_block_len: int) -> bytes:
        arr = (VsMatch * max(len(matches), 1))()
        for k, (o, i) in enumerate(matches):
            arr[k].offset, arr[k].block_index = o, i
        b = _host_bytes(src)
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        check(lib.vs_rsync_write_tokens_zstd(self._z, arr, len(matches), len(b), blength, basis_len,
                                             last_block_len, b.ctypes.data if len(b) else None,
                                             ctypes.byref(out), ctypes.byref(n)))
        return ctypes.string_at(out, n.value) if n.value else b""

    def read(self, stream: bytes, blength: int, basis_len: int, max_matches: int,
             max_literal: int):
        """-> (matches, literal bytes, file length, bytes consumed)"""
        buf = np.frombuffer(stream, np.uint8) if len(stream) else np.zeros(1, np.uint8)
        arr = (VsMatch * max(max_matches, 1))()
        lit = np.zeros(max(max_literal, 1), np.uint8)
        nm, nl, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        flen = ctypes.c_int64()
        check(lib.vs_rsync_read_tokens_zstd(self._z, buf.ctypes.data, len(stream), blength,
                                            basis_len, arr, max_matches, ctypes.byref(nm),
                                            lit.ctypes.data, len(lit), ctypes.byref(nl),
                                            ctypes.byref(flen), ctypes.byref(used)))
        return ([(arr[k].offset, arr[k].block_index) for k in range(nm.value)],
                lit[: nl.value].tobytes(), flen.value, used.value)


def file_sum_init() -> np.ndarray:
    """The XXH3 accumulators of an empty file (the relay's first acc_in)."""
    acc = np.zeros(8, np.uint64)
    check(lib.vs_rsync_file_sum_init(acc.ctypes.data))
    return acc


def file_sum_finish(acc, last: bytes, length: int, csum_type: int = CSUM_XXH3_128) -> bytes:
    """sum_end for a file split across ranks: the accumulators after the
    file's whole 1 KiB blocks ((length - 1) // 1024 of them) and its last
    min(length, 1088) bytes."""
    a = np.ascontiguousarray(acc, np.uint64)
    b = np.frombuffer(bytes(last), np.uint8)
    out = ctypes.create_string_buffer(16)
    check(lib.vs_rsync_file_sum_finish(a.ctypes.data, b.ctypes.data, length, csum_type, out))
    return out.raw[: 16 if csum_type == CSUM_XXH3_128 else 8]


def match_sums(src, s: SumStruct, csum_type: int = CSUM_XXH3_128, seed: int = 0,
               device: int = 0) -> List[Tuple[int, int]]:
    """One-shot host form: the greedy match list of `src` against `s`."""
    b = _host_bytes(src)
    s1 = np.ascontiguousarray(s.sum1, np.uint32)
    s2 = np.ascontiguousarray(s.sum2, np.uint8)
    t = VsSigTable(s.count, s.blength, s.s2length, s.remainder,
                   s1.ctypes.data if s.count else None, s2.ctypes.data if s.count else None)
    cap = len(b) // max(1, min(s.blength, s.remainder or s.blength)) + 8
    out = (VsMatch * cap)()
    n = ctypes.c_size_t(0)
    check(lib.vs_rsync_match(device, b.ctypes.data if len(b) else None, len(b), ctypes.byref(t),
                             csum_type, seed & 0xFFFFFFFF, out, cap, ctypes.byref(n)))
    return [(out[i].offset, out[i].block_index) for i in range(n.value)]
