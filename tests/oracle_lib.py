"""ctypes loader for the C oracle (oracle/build/liboracle.so) -- test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# VSGPU_ORACLE_LIB: the sanitizer build of the oracle (tools/asan_build.sh)
ORACLE_SO = os.environ.get("VSGPU_ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "liboracle.so")

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = ctypes.CDLL(ORACLE_SO)
        u64, vp, ci = ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
        L.ref_chunk_all.restype = ctypes.c_int64
        L.ref_chunk_all.argtypes = [vp, u64, u64, u64, u64, ci, vp, vp, vp, u64]
        L.ref_cdc_hash.restype = ctypes.c_int64
        L.ref_cdc_hash.argtypes = [vp, u64, u64, u64, u64, ci, ci, vp, vp, vp, vp, u64]
        L.ref_synth_fill.argtypes = [u64, u64, u64, vp]
        L.ref_sha256.argtypes = [vp, u64, vp]
        L.ref_sha256_fast.argtypes = [vp, u64, vp]
        L.ref_sha256_list.restype = ci
        L.ref_sha256_list.argtypes = [vp, vp, vp, ctypes.c_int64, vp, ci]
        L.ref_have_openssl.restype = ci
        L.ref_pol_deg.argtypes = [u64]
        L.ref_pol_mod.restype = u64
        L.ref_pol_mod.argtypes = [u64, u64]
        L.ref_tables.argtypes = [u64, vp, vp]
        L.ref_window_fp.restype = u64
        L.ref_window_fp.argtypes = [vp, u64, u64]
        L.ref_rsync_checksum1.restype = ctypes.c_uint32
        L.ref_rsync_checksum1.argtypes = [vp, ctypes.c_int32]
        L.ref_rsync_sum_sizes.argtypes = [ctypes.c_int64, ctypes.c_int32] + [ctypes.POINTER(ctypes.c_int32)] * 4
        _lib = L
    return _lib


def chunk_all(data: np.ndarray, pol: int, mn: int, mx: int, avg_bits: int):
    d = np.ascontiguousarray(data, dtype=np.uint8)
    cap = len(d) // max(1, mn) + 8
    s = np.zeros(cap, np.uint64)
    ln = np.zeros(cap, np.uint64)
    c = np.zeros(cap, np.uint64)
    n = lib().ref_chunk_all(d.ctypes.data if len(d) else None, len(d), pol, mn, mx, avg_bits,
                            s.ctypes.data, ln.ctypes.data, c.ctypes.data, cap)
    if n < 0:
        raise ValueError("oracle rejected the chunker parameters")
    return [(int(s[i]), int(ln[i]), int(c[i])) for i in range(n)]


def cdc_hash(data: np.ndarray, pol: int, mn: int, mx: int, avg_bits: int, n_hash: int = 0):
    d = np.ascontiguousarray(data, dtype=np.uint8)
    cap = len(d) // max(1, mn) + 8
    s = np.zeros(cap, np.uint64)
    ln = np.zeros(cap, np.uint64)
    c = np.zeros(cap, np.uint64)
    ids = np.zeros((cap, 32), np.uint8)
    n = lib().ref_cdc_hash(d.ctypes.data if len(d) else None, len(d), pol, mn, mx, avg_bits,
                           n_hash, s.ctypes.data, ln.ctypes.data, c.ctypes.data, ids.ctypes.data,
                           cap)
    if n < 0:
        raise ValueError("oracle failed")
    return [(int(s[i]), int(ln[i]), int(c[i]), bytes(ids[i]).hex()) for i in range(n)]


def sha256_list(src: np.ndarray, off: np.ndarray, ln: np.ndarray, threads: int):
    """SHA-256 of src[off[i] : off[i] + ln[i]] on `threads` threads
    (ref_sha256_list): ((n, 32) uint8 IDs, threads that ran)."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint64)
    ids = np.zeros((max(len(off), 1), 32), np.uint8)
    ran = lib().ref_sha256_list(src.ctypes.data, off.ctypes.data, ln.ctypes.data, len(off),
                                ids.ctypes.data, threads)
    if ran < 0:
        raise MemoryError("ref_sha256_list")
    return ids[:len(off)], ran


def synth(seed: int, off: int, n: int) -> np.ndarray:
    out = np.zeros(max(n, 1), np.uint8)
    lib().ref_synth_fill(seed, off, n, out.ctypes.data)
    return out[:n]


def sha256(data) -> bytes:
    d = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    out = np.zeros(32, np.uint8)
    lib().ref_sha256(d.ctypes.data if len(d) else None, len(d), out.ctypes.data)
    return bytes(out)


# ---- rsync restatement (oracle/rsync_ref.c) ---------------------------------
def _rs():
    L = lib()
    if not getattr(L, "_rs_ready", False):
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.ref_rsync_checksum2.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int,
                                          ctypes.c_uint32, ctypes.c_void_p]
        L.ref_have_xxhash.restype = ctypes.c_int
        L.ref_rsync_signatures.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.ref_rsync_match.restype = ctypes.c_int64
        L.ref_rsync_match.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        L._rs_ready = True
    return L


def rsync_sizes(length: int, block_size: int = 0):
    v = [ctypes.c_int32() for _ in range(4)]
    rc = lib().ref_rsync_sum_sizes(length, block_size, *[ctypes.byref(x) for x in v])
    if rc < 0:
        raise ValueError("sum_sizes overflow")
    return tuple(x.value for x in v)   # blength, s2length, count, remainder


def rsync_signatures(basis: np.ndarray, blength: int, s2length: int, csum_type: int, seed: int):
    n = len(basis)
    count = (n + blength - 1) // blength
    s1 = np.zeros(max(count, 1), np.uint32)
    s2 = np.zeros(max(count, 1) * s2length, np.uint8)
    rc = _rs().ref_rsync_signatures(basis.ctypes.data if n else None, n, blength, s2length,
                                    csum_type, seed, s1.ctypes.data, s2.ctypes.data)
    if rc < 0:
        raise RuntimeError("signature restatement failed")
    return s1[:count], s2[:count * s2length].reshape(count, s2length)


def rsync_signatures_synth_mt(dseed: int, length: int, blength: int, s2length: int,
                              csum_type: int, seed: int, threads: int = 16):
    """generate_and_send_sums over the synthetic stream `dseed` of `length`
    bytes on `threads` threads (oracle/rsync_ref.c ref_rsync_signatures_synth_mt)."""
    L = _rs()
    if not getattr(L, "_sigmt_ready", False):
        L.ref_rsync_signatures_synth_mt.argtypes = [
            ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
            ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L._sigmt_ready = True
    count = (length + blength - 1) // blength
    s1 = np.zeros(max(count, 1), np.uint32)
    s2 = np.zeros(max(count, 1) * s2length, np.uint8)
    if L.ref_rsync_signatures_synth_mt(dseed, length, blength, s2length, csum_type, seed, threads,
                                       s1.ctypes.data, s2.ctypes.data) < 0:
        raise RuntimeError("multi-threaded signature restatement failed")
    return s1[:count], s2[:count * s2length].reshape(count, s2length)


def xxh3_synth(dseed: int, length: int, csum_type: int, threads: int = 16) -> bytes:
    """sum_end's 16 bytes of the whole-file XXH3 (xxh128 / xxh3) of the
    synthetic stream's first `length` bytes (oracle/rsync_ref.c ref_xxh3_synth,
    libxxhash streaming)."""
    L = _rs()
    if not getattr(L, "_xs_ready", False):
        L.ref_xxh3_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p]
        L._xs_ready = True
    out = np.zeros(16, np.uint8)
    if L.ref_xxh3_synth(dseed, length, csum_type, threads, out.ctypes.data) < 0:
        raise RuntimeError("streaming XXH3 oracle failed (libxxhash streaming API missing?)")
    return bytes(out[: 16 if csum_type == 8 else 8])


def rsync_match(src: np.ndarray, sum1: np.ndarray, sum2: np.ndarray, blength: int,
                remainder: int, csum_type: int, seed: int):
    count = len(sum1)
    s2length = sum2.shape[1] if count else 2
    cap = len(src) // max(1, blength) + 8
    mo = np.zeros(cap, np.int64)
    mi = np.zeros(cap, np.int32)
    fa = ctypes.c_int64(0)
    s1 = np.ascontiguousarray(sum1, np.uint32)
    s2 = np.ascontiguousarray(sum2, np.uint8)
    n = _rs().ref_rsync_match(src.ctypes.data if len(src) else None, len(src), count, blength,
                              remainder, s2length, s1.ctypes.data if count else None,
                              s2.ctypes.data if count else None, csum_type, seed,
                              mo.ctypes.data, mi.ctypes.data, cap, ctypes.byref(fa))
    if n < 0:
        raise RuntimeError("match restatement failed")
    return [(int(mo[i]), int(mi[i])) for i in range(n)], int(fa.value)


def rsync_walk(win: np.ndarray, win_lo: int, length: int, hi: int, entry: int, want: int,
               sum1: np.ndarray, sum2: np.ndarray, blength: int, remainder: int, csum_type: int,
               seed: int):
    """hash_search over the shard [entry, hi) of a source of `length` bytes
    (oracle/rsync_ref.c ref_rsync_walk): (matches, false_alarms, exit_off,
    exit_want).  win holds file bytes from win_lo."""
    L = _rs()
    if not getattr(L, "_walk_ready", False):
        i64, i32, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.ref_rsync_walk.restype = i64
        L.ref_rsync_walk.argtypes = [vp, i64, i64, i64, i64, i32, i32, i32, i32, i32, vp, vp,
                                     ctypes.c_int, ctypes.c_uint32, vp, vp, i64,
                                     ctypes.POINTER(i64), ctypes.POINTER(i64),
                                     ctypes.POINTER(i32)]
        L._walk_ready = True
    count = len(sum1)
    s2length = sum2.shape[1] if count else 2
    cap = max(0, hi - entry) // max(1, min(blength, remainder or blength)) + 8
    mo = np.zeros(cap, np.int64)
    mi = np.zeros(cap, np.int32)
    fa, eo, ew = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
    w = np.ascontiguousarray(win, np.uint8)
    s1 = np.ascontiguousarray(sum1, np.uint32)
    s2 = np.ascontiguousarray(sum2, np.uint8)
    n = L.ref_rsync_walk(w.ctypes.data if len(w) else None, win_lo, length, hi, entry, want,
                         count, blength, remainder, s2length, s1.ctypes.data if count else None,
                         s2.ctypes.data if count else None, csum_type, seed, mo.ctypes.data,
                         mi.ctypes.data, cap, ctypes.byref(fa), ctypes.byref(eo),
                         ctypes.byref(ew))
    if n < 0:
        raise RuntimeError("walk restatement failed")
    return [(int(mo[i]), int(mi[i])) for i in range(n)], int(fa.value), int(eo.value), int(ew.value)


def cdc_synth_mt(seed: int, length: int, pol: int, mn: int, mx: int, avg_bits: int,
                 threads: int):
    """Chunk list + blob IDs of the synthetic stream's first `length` bytes,
    multi-threaded (oracle/cdc_ref.c ref_cdc_synth_mt): [(start, len, cut, id)]."""
    L = lib()
    if not getattr(L, "_mt_ready", False):
        u64, vp, ci = ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
        L.ref_cdc_synth_mt.restype = ctypes.c_int64
        L.ref_cdc_synth_mt.argtypes = [u64, u64, u64, u64, u64, ci, ci, vp, vp, vp, vp, u64]
        L._mt_ready = True
    cap = length // max(1, mn) + 8
    s = np.zeros(cap, np.uint64)
    ln = np.zeros(cap, np.uint64)
    c = np.zeros(cap, np.uint64)
    ids = np.zeros((cap, 32), np.uint8)
    n = L.ref_cdc_synth_mt(seed, length, pol, mn, mx, avg_bits, threads, s.ctypes.data,
                           ln.ctypes.data, c.ctypes.data, ids.ctypes.data, cap)
    if n < 0:
        raise RuntimeError(f"multi-threaded oracle failed ({n})")
    return s[:n], ln[:n], c[:n], ids[:n]
