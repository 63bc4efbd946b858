"""ctypes binding of the product library volsync_amd/lib/libvsgpu.so (C ABI: include/vsgpu.h).

There is no CPU fallback: importing works without a GPU (so the ABI can be
inspected), but every compute call fails with VsError(VS_ERR_NO_DEVICE) unless
a gfx950 device is present, and a missing library raises ImportError.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VSGPU_LIB: an alternative build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("VSGPU_LIB") or os.path.join(_HERE, "lib", "libvsgpu.so")

VS_OK = 0
VS_EOF = 1
VS_ERR_ARG = -1
VS_ERR_POLY = -2
VS_ERR_NO_DEVICE = -3
VS_ERR_NOMEM = -4
VS_ERR_STATE = -5
VS_ERR_HIP = -6

# handle options (vsgpu.h "options"): tests and measurement only
VS_OPT_WALK_SEGMENT_BLOCKS = 1
VS_OPT_FILE_SUM_PIECE = 2
VS_OPT_BUCKET_BITS = 3
VS_OPT_FA_RECORD = 4
VS_OPT_HOST_WALK = 5
VS_OPT_WALK_PREFILTER = 6
VS_OPT_WALK_FLUSH_WINDOWS = 7
VS_OPT_WALK_FLUSH_SPAN = 8
VS_OPT_WALK_FLUSH_PREDICT = 9
VS_OPT_WALK_TAIL_PCT = 10
VS_OPT_WALK_SEG_MARGIN = 11
VS_OPT_SHA_QUAD_PCT = 16
VS_OPT_SHA_ISOLATE = 19
VS_OPT_FP_GENERIC = 17
VS_OPT_SHA_GRID_PER_CU = 18
VS_DEDUP_KNOWN = 0xFFFFFFFF
VS_OPT_SEAL_FUSED = 32

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_int = ctypes.c_int
c_size = ctypes.c_size_t
i32 = ctypes.c_int32
i64 = ctypes.c_int64
i32p = ctypes.POINTER(ctypes.c_int32)
i64p = ctypes.POINTER(ctypes.c_int64)


class VsChunk(ctypes.Structure):
    _fields_ = [("start", c_u64), ("length", c_u64), ("cut", c_u64), ("id", ctypes.c_uint8 * 32)]


class VsMatch(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("block_index", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class VsPack(ctypes.Structure):
    _fields_ = [("offset", c_u64), ("length", c_u64), ("first_blob", c_u32), ("n_blobs", c_u32)]


class VsSigTable(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int32), ("blength", ctypes.c_int32),
                ("s2length", ctypes.c_int32), ("remainder", ctypes.c_int32),
                ("sum1", vp), ("sum2", vp)]


class VsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vsgpu error {code}: {msg}")
        self.code = code


def _one_hip_runtime() -> None:
    """PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7) and
    loads it by file name.  If libvsgpu.so pulled /opt/rocm's copy in first, the
    process would hold two HIP runtimes and torch's would find no GPU.  Loading
    torch first makes libvsgpu.so bind to the already-loaded runtime (same
    SONAME), so device pointers, streams and events are shared."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load() -> ctypes.CDLL:
    _one_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is the only implementation; there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "vs_last_error": (ctypes.c_char_p, []),
        "vs_version": (ctypes.c_char_p, []),
        "vs_device_count": (c_int, []),
        "vs_pol_deg": (c_int, [c_u64]),
        "vs_pol_irreducible": (c_int, [c_u64]),
        "vs_pol_tables": (c_int, [c_u64, u64p, u64p]),
        "vs_cdc_open": (c_int, [c_int, c_u64, c_u32, c_u32, c_u32, ctypes.POINTER(vp)]),
        "vs_cdc_reset": (c_int, [vp, c_u64, c_u32, c_u32, c_u32]),
        "vs_cdc_feed": (c_int, [vp, vp, c_size, c_int]),
        "vs_cdc_next": (c_int, [vp, ctypes.POINTER(VsChunk), c_size, ctypes.POINTER(c_size)]),
        "vs_cdc_next_wait": (c_int, [vp, ctypes.POINTER(VsChunk), c_size, ctypes.POINTER(c_size)]),
        "vs_cdc_inflight": (c_int, [vp, ctypes.POINTER(c_u64)]),
        "vs_cdc_close": (None, [vp]),
        "vs_cdc_set_batch_bytes": (c_int, [vp, c_u64]),
        "vs_cdc_stream_stats": (c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "vs_blob_dedup": (c_int, [vp, vp, c_size, vp, ctypes.POINTER(c_u64), vp]),
        "vs_blob_dedup_known": (c_int, [vp, vp, c_size, vp, c_size, vp, ctypes.POINTER(c_u64), vp]),
        "vs_blob_index_sort": (c_int, [vp, vp, c_size, vp]),
        "vs_rsync_file_sum": (c_int, [vp, vp, ctypes.c_int64, c_int, ctypes.c_char_p]),
        "vs_rsync_file_sum_start": (c_int, [vp, vp, ctypes.c_int64, c_int]),
        "vs_rsync_file_sum_wait": (c_int, [vp, ctypes.c_char_p]),
        "vs_rsync_file_sum_init": (c_int, [vp]),
        "vs_rsync_file_sum_blocks_start": (c_int, [vp, vp, ctypes.c_int64, vp]),
        "vs_rsync_file_sum_blocks_wait": (c_int, [vp, vp]),
        "vs_rsync_file_sum_finish": (c_int, [vp, vp, ctypes.c_int64, c_int, ctypes.c_char_p]),
        "vs_rsync_file_sum_timing": (c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]),
        "vs_sha256_blocks": (c_int, [vp, vp, c_u64, c_u32, vp, vp]),
        "vs_syncthing_block_size": (c_int, [ctypes.c_int64]),
        "vs_blob_verify": (c_int, [vp, vp, vp, vp, c_size, vp, vp, ctypes.POINTER(c_u64), vp]),
        "vs_rsync_reconstruct": (c_int, [vp, vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.POINTER(VsMatch), ctypes.c_int64, vp, ctypes.c_int64]),
        "vs_rsync_write_sums": (c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        vp, vp, vp, c_size, ctypes.POINTER(c_size)]),
        "vs_rsync_read_sums": (c_int, [vp, c_size, i32p, i32p, i32p, i32p, vp, vp, c_size]),
        "vs_rsync_write_tokens": (c_int, [ctypes.POINTER(VsMatch), ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int32, ctypes.c_int64, vp, vp, c_size,
                                          ctypes.POINTER(c_size)]),
        "vs_rsync_read_tokens": (c_int, [vp, c_size, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.POINTER(VsMatch), c_size, ctypes.POINTER(c_size), vp,
                                         c_size, ctypes.POINTER(c_size), i64p]),
        "vs_ztok_open": (c_int, [c_int, ctypes.POINTER(vp)]),
        "vs_ztok_close": (None, [vp]),
        "vs_rsync_write_tokens_zstd": (c_int, [vp, ctypes.POINTER(VsMatch), ctypes.c_int64,
                                               ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                               ctypes.c_int32, vp, ctypes.POINTER(vp),
                                               ctypes.POINTER(c_size)]),
        "vs_rsync_read_tokens_zstd": (c_int, [vp, vp, c_size, ctypes.c_int32, ctypes.c_int64,
                                              ctypes.POINTER(VsMatch), c_size, ctypes.POINTER(c_size),
                                              vp, c_size, ctypes.POINTER(c_size),
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(c_size)]),
        "vs_restic_pack_header": (c_int, [vp, vp, vp, c_size, vp, c_size, ctypes.POINTER(c_size)]),
        "vs_seal_open": (c_int, [c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                 ctypes.POINTER(vp)]),
        "vs_seal_run_device": (c_int, [vp, vp, vp, vp, c_size, vp, vp, vp, vp]),
        "vs_seal_set_timing": (c_int, [vp, c_int]),
        "vs_seal_kernel_ms": (c_int, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int)]),
        "vs_seal_close": (None, [vp]),
        "vs_seal_records_device": (c_int, [vp, vp, vp, vp, c_size, vp, vp, vp, vp]),
        "vs_open_run_device": (c_int, [vp, vp, vp, vp, c_size, vp, vp, vp, ctypes.POINTER(c_u64),
                                       vp]),
        "vs_restic_pack": (c_int, [vp, vp, vp, vp, vp, vp, vp, c_size, vp, vp, c_u64, vp, c_u64,
                                   vp, c_size, ctypes.POINTER(c_size), ctypes.POINTER(c_u64), vp,
                                   vp]),
        "vs_restic_index": (c_int, [vp, vp, vp, vp, vp, c_size, c_u64, vp, vp, vp, c_size,
                                    ctypes.POINTER(c_size), vp, vp]),
        "vs_cdc_set_stream": (c_int, [vp, vp]),
        "vs_cdc_set_hash_stream": (c_int, [vp, vp]),
        "vs_cdc_set_hash_slice": (c_int, [vp, c_u32]),
        "vs_cdc_set_hash_wide": (c_int, [vp, c_u32, c_u32]),
        "vs_cdc_batches": (c_int, [vp, u64p, u64p]),
        "vs_cdc_get_batch_chunks": (c_int, [vp, c_u64, c_u64, c_u64, ctypes.POINTER(VsChunk)]),
        "vs_cdc_scan": (c_int, [vp, vp, c_u64, c_u64, c_u64, c_u64, c_int]),
        "vs_cdc_stitch": (c_int, [vp, c_u64, u64p, ctypes.POINTER(c_int)]),
        "vs_cdc_finish": (c_int, [vp, u64p]),
        "vs_cdc_wait": (c_int, [vp]),
        "vs_cdc_process": (c_int, [vp, vp, c_u64, c_u64, c_int, u64p, u64p]),
        "vs_cdc_get_chunks": (c_int, [vp, c_u64, c_u64, ctypes.POINTER(VsChunk)]),
        "vs_cdc_timing": (c_int, [vp, c_int, ctypes.POINTER(ctypes.c_double), u64p]),
        "vs_cdc_timing_detail": (c_int, [vp, ctypes.POINTER(ctypes.c_double), u64p]),
        "vs_cdc_fence": (c_int, [vp, ctypes.c_uint64]),
        "vs_sha256_open": (c_int, [c_int, ctypes.POINTER(vp)]),
        "vs_sha256_run_device": (c_int, [vp, vp, vp, vp, c_size, vp, vp]),
        "vs_sha256_close": (None, [vp]),
        "vs_sha256_set_wide": (c_int, [vp, c_u32, c_u32]),
        "vs_sha256_batch": (c_int, [c_int, vp, c_size, vp, vp, c_size, vp]),
        "vs_synth_fill_device": (c_int, [c_int, c_u64, c_u64, c_u64, vp, vp]),
        "vs_rsync_sizes": (c_int, [i64, i32, i32p, i32p, i32p, i32p]),
        "vs_rsync_open": (c_int, [c_int, ctypes.POINTER(vp)]),
        "vs_rsync_set_stream": (c_int, [vp, vp]),
        "vs_rsync_close": (None, [vp]),
        "vs_rsync_signatures_device": (c_int, [vp, vp, i64, i32, i32, c_int, c_u32, vp, vp]),
        "vs_rsync_load_sums": (c_int, [vp, i32, i32, i32, i32, vp, vp, c_int, c_u32]),
        "vs_rsync_load_sums_device": (c_int, [vp, i32, i32, i32, i32, vp, vp, c_int, c_u32]),
        "vs_rsync_match_device": (c_int, [vp, vp, i64, i64p]),
        "vs_rsync_match_scan": (c_int, [vp, vp, i64, i64, i64, i64, i64, i64p, i32p]),
        "vs_rsync_match_stitch": (c_int, [vp, i64, i32, i64p, i32p]),
        "vs_rsync_match_finish": (c_int, [vp, i64p]),
        "vs_rsync_get_matches": (c_int, [vp, i64, i64, ctypes.POINTER(VsMatch)]),
        "vs_rsync_stats": (c_int, [vp, i64p, i64p, i64p, i32p]),
        "vs_rsync_timing": (c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "vs_rsync_kernel_time": (c_int, [vp, c_int, c_int, ctypes.POINTER(ctypes.c_double), i64p]),
        "vs_rsync_match_begin": (c_int, [vp, i64, c_int, c_u64, c_u32]),
        "vs_rsync_match_feed": (c_int, [vp, vp, c_size]),
        "vs_rsync_match_next": (c_int, [vp, ctypes.POINTER(VsMatch), c_size, ctypes.POINTER(c_size)]),
        "vs_rsync_match_end": (c_int, [vp, i64p, i64p, vp]),
        "vs_rsync_match_stream_stats": (c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "vs_rsync_sig_begin": (c_int, [vp, i64, i32, i32, c_int, c_u32, c_u64, c_u32]),
        "vs_rsync_sig_feed": (c_int, [vp, vp, c_size]),
        "vs_rsync_sig_next": (c_int, [vp, vp, vp, c_size, ctypes.POINTER(c_size)]),
        "vs_rsync_set_option": (c_int, [vp, c_int, i64]),
        "vs_cdc_set_option": (c_int, [vp, c_int, i64]),
        "vs_sha256_set_option": (c_int, [vp, c_int, i64]),
        "vs_sha256_drain_stats": (c_int, [vp, vp]),
        "vs_seal_set_option": (c_int, [vp, c_int, i64]),
        "vs_rsync_signatures": (c_int, [c_int, vp, i64, i32, i32, c_int, c_u32, vp, vp]),
        "vs_rsync_match": (c_int, [c_int, vp, i64, ctypes.POINTER(VsSigTable), c_int, c_u32,
                                   ctypes.POINTER(VsMatch), c_size, ctypes.POINTER(c_size)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    return lib.vs_last_error().decode(errors="replace")


def check(rc: int) -> int:
    if rc < 0:
        raise VsError(rc, last_error())
    return rc


def device_count() -> int:
    return int(lib.vs_device_count())
