"""Host-side mirror of restic's chunker API over the gfx950 C ABI.

Mirrors github.com/restic/chunker@v0.4.0 (the module restic v0.13.1 uses;
fetched by /root/reference/mover-restic/Dockerfile:8-11, not vendored):

    New(rd, pol) / NewWithBoundaries(rd, pol, min, max)
    (*Chunker).Reset / ResetWithBoundaries / SetAverageBits
    (*Chunker).Next(data []byte) (Chunk, error)     -> io.EOF at the end
    type Chunk struct{ Start, Length uint; Cut uint64; Data []byte }

plus the blob ID restic computes for every chunk (internal/restic/id.go Hash =
sha256.Sum256), returned as Chunk.ID so FileSaver.saveFile can hand it to
Repository.SaveBlob(..., id, ...) pre-computed.

Names, argument meaning and error behaviour follow the Go package:
pol == 0 is accepted by New and fails in Next() with "tables for polynomial
computation not initialized"; reader errors propagate; Next() signals the end
with EOF (an EOFError, the io.EOF analogue).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Iterator, List, Optional

from . import _lib
from ._lib import VsChunk, VsError, check, lib

KiB = 1024
MiB = 1024 * KiB
MinSize = 512 * KiB
MaxSize = 8 * MiB
AverageBits = 20
TestPol = 0x3DA3358B4DC173  # chunker_test.go testPol

__all__ = ["Chunk", "Chunker", "EOF", "New", "NewWithBoundaries", "Pol", "DeviceChunker",
           "DeviceSha256",
           "MinSize", "MaxSize", "KiB", "MiB", "syncthing_block_size", "Sealer"]


class EOF(EOFError):
    """io.EOF: the stream is exhausted."""


class Pol(int):
    """chunker polynomials.go `type Pol uint64` (host-side helpers)."""

    def Deg(self) -> int:
        return int(lib.vs_pol_deg(ctypes.c_uint64(int(self))))

    def Irreducible(self) -> bool:
        return bool(lib.vs_pol_irreducible(ctypes.c_uint64(int(self))))

    def tables(self):
        out = (ctypes.c_uint64 * 256)()
        mod = (ctypes.c_uint64 * 256)()
        check(lib.vs_pol_tables(int(self), out, mod))
        return list(out), list(mod)


@dataclass
class Chunk:
    Start: int
    Length: int
    Cut: int
    Data: Optional[bytes] = None
    ID: bytes = b""  # restic blob ID (SHA-256 of Data)


def _chunk_from(c: VsChunk, data=None) -> Chunk:
    return Chunk(int(c.start), int(c.length), int(c.cut), data, bytes(c.id))


class Chunker:
    """A restic chunker whose fingerprinting, cut selection and blob hashing run
    on the GPU.  Not goroutine-/thread-safe (same contract as the Go type)."""

    def __init__(self, rd, pol: int, min_size: int = MinSize, max_size: int = MaxSize,
                 device: int = 0, read_size: int = 64 * MiB, batch_bytes: int = 256 * MiB,
                 max_pending: Optional[int] = None):
        """max_pending bounds the stream bytes held for chunks not yet returned
        (Chunk.Data): at or above it, Next waits for batches in flight instead
        of reading more (vs_cdc_next_wait).  None = 4 batches.  The bytes held
        never exceed max(max_pending, 2 * batch + 2 * MaxSize) + read_size."""
        self._h = ctypes.c_void_p()
        self._device = device
        self._read_size = read_size
        self._batch_bytes = batch_bytes
        self._max_pending = 4 * batch_bytes if max_pending is None else int(max_pending)
        self.max_held = 0          # high-water mark of the bytes held (tests)
        self._avg_bits = AverageBits
        self.ResetWithBoundaries(rd, pol, min_size, max_size)

    # ---- chunker.go API ---------------------------------------------------
    def Reset(self, rd, pol: int) -> None:
        self.ResetWithBoundaries(rd, pol, MinSize, MaxSize)

    def ResetWithBoundaries(self, rd, pol: int, min_size: int, max_size: int) -> None:
        self._rd = rd
        self.pol = Pol(pol)
        self.MinSize = int(min_size)
        self.MaxSize = int(max_size)
        self._avg_bits = AverageBits
        self._buf = bytearray()   # host copy of bytes not yet returned (for Chunk.Data)
        self._borigin = 0          # stream offset of _buf[0]
        self._eof_fed = False
        self._configured = False

    def SetAverageBits(self, average_bits: int) -> None:
        self._avg_bits = int(average_bits)
        self._configured = False

    def Next(self, data: Optional[bytearray] = None) -> Chunk:
        if self.pol == 0:
            raise VsError(_lib.VS_ERR_POLY, "tables for polynomial computation not initialized")
        self._configure()
        one = (VsChunk * 1)()
        n = ctypes.c_size_t(0)
        while True:
            # at the bound, wait for a batch in flight rather than read more;
            # with none in flight the bytes held belong to batches whose cuts
            # need more input, so the stream must be fed anyway
            nxt = lib.vs_cdc_next_wait if len(self._buf) >= self._max_pending else lib.vs_cdc_next
            rc = nxt(self._h, one, 1, ctypes.byref(n))
            if rc == _lib.VS_EOF:
                raise EOF()
            check(rc)
            if n.value:
                break
            self._pump()
        c = one[0]
        lo = int(c.start) - self._borigin
        payload = bytes(self._buf[lo:lo + int(c.length)])
        del self._buf[:lo + int(c.length)]
        self._borigin = int(c.start) + int(c.length)
        if data is not None:          # Go: Data = append(data[:0], ...)
            data[:] = payload
            payload = data
        return _chunk_from(c, payload)

    def __iter__(self) -> Iterator[Chunk]:
        while True:
            try:
                yield self.Next()
            except EOF:
                return

    def close(self) -> None:
        if self._h:
            lib.vs_cdc_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- internals ------------------------------------------------------------
    def _configure(self) -> None:
        if self._configured:
            return
        if not self._h:
            check(lib.vs_cdc_open(self._device, int(self.pol), self.MinSize, self.MaxSize,
                                  self._avg_bits, ctypes.byref(self._h)))
        else:
            check(lib.vs_cdc_reset(self._h, int(self.pol), self.MinSize, self.MaxSize,
                                   self._avg_bits))
        check(lib.vs_cdc_set_batch_bytes(self._h, self._batch_bytes))
        self._configured = True

    def _pump(self) -> None:
        if self._eof_fed:
            raise VsError(_lib.VS_ERR_STATE, "chunk stream stalled after EOF")
        block = self._rd.read(self._read_size)   # reader errors propagate
        if not block:
            check(lib.vs_cdc_feed(self._h, None, 0, 1))
            self._eof_fed = True
            return
        block = bytes(block)
        self._buf += block
        self.max_held = max(self.max_held, len(self._buf))
        buf = ctypes.create_string_buffer(block, len(block))
        check(lib.vs_cdc_feed(self._h, buf, len(block), 0))


def New(rd, pol: int, **kw) -> Chunker:
    return Chunker(rd, pol, MinSize, MaxSize, **kw)


def NewWithBoundaries(rd, pol: int, min_size: int, max_size: int, **kw) -> Chunker:
    return Chunker(rd, pol, min_size, max_size, **kw)


class DeviceChunker:
    """Chunks device-resident byte ranges (data already in HBM): the batch API
    used by bench.py and the multi-GPU path."""

    def __init__(self, pol: int = TestPol, min_size: int = MinSize, max_size: int = MaxSize,
                 avg_bits: int = AverageBits, device: int = 0):
        self.device = device
        self._h = ctypes.c_void_p()
        check(lib.vs_cdc_open(device, int(pol), int(min_size), int(max_size), int(avg_bits),
                              ctypes.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def reset(self, pol: int = TestPol, min_size: int = MinSize, max_size: int = MaxSize,
              avg_bits: int = AverageBits) -> None:
        """Chunker.ResetWithBoundaries + SetAverageBits on the same device buffers
        (finishes hashing every queued batch first)."""
        check(lib.vs_cdc_reset(self._h, int(pol), int(min_size), int(max_size), int(avg_bits)))

    def set_stream(self, hip_stream: int) -> None:
        check(lib.vs_cdc_set_stream(self._h, ctypes.c_void_p(hip_stream or None)))

    def set_hash_stream(self, hip_stream: int) -> None:
        """Run the SHA-256 stage on another stream (0 = the handle's own)."""
        check(lib.vs_cdc_set_hash_stream(self._h, ctypes.c_void_p(hip_stream or None)))

    def set_hash_slice(self, blocks: int) -> None:
        """Blocks per chunk per batch of the time-sliced SHA-256 engine (0 = unbounded)."""
        check(lib.vs_cdc_set_hash_slice(self._h, int(blocks)))

    def set_hash_wide(self, min_chains: int = 0, drain_blocks: int = 0) -> None:
        """Throughput mode of the SHA-256 engine from min_chains active chunks
        (0 = default, 0xffffffff = never); drain_blocks per drain launch."""
        check(lib.vs_cdc_set_hash_wide(self._h, int(min_chains), int(drain_blocks)))

    def set_option(self, option: int, value: int) -> None:
        """vs_cdc_set_option (volsync_amd._lib VS_OPT_*)."""
        check(lib.vs_cdc_set_option(self._h, option, value))

    def batches(self):
        """(batches finished so far, batches the ring keeps)."""
        f = ctypes.c_uint64(0)
        r = ctypes.c_uint64(0)
        check(lib.vs_cdc_batches(self._h, ctypes.byref(f), ctypes.byref(r)))
        return int(f.value), int(r.value)

    def batch_chunks(self, batch: int, first: int, n: int) -> List[Chunk]:
        """Chunks of an earlier batch (pipelined use; waits for its blob IDs)."""
        if n <= 0:
            return []
        arr = (VsChunk * n)()
        check(lib.vs_cdc_get_batch_chunks(self._h, batch, first, n, arr))
        return [_chunk_from(c) for c in arr]

    def process(self, dev_ptr: int, length: int, origin: int = 0, final: bool = True):
        n = ctypes.c_uint64(0)
        consumed = ctypes.c_uint64(0)
        check(lib.vs_cdc_process(self._h, ctypes.c_void_p(dev_ptr), length, origin,
                                 1 if final else 0, ctypes.byref(n), ctypes.byref(consumed)))
        return int(n.value), int(consumed.value)

    def scan(self, dev_ptr: int, length: int, origin: int, own_lo: int, own_hi: int,
             final: bool) -> None:
        check(lib.vs_cdc_scan(self._h, ctypes.c_void_p(dev_ptr), length, origin, own_lo, own_hi,
                              1 if final else 0))

    def stitch(self, entry: int):
        ex = ctypes.c_uint64(0)
        complete = ctypes.c_int(0)
        check(lib.vs_cdc_stitch(self._h, entry, ctypes.byref(ex), ctypes.byref(complete)))
        return int(ex.value), bool(complete.value)

    def finish(self) -> int:
        """Emit the chunk list; blob IDs stay queued (see wait())."""
        n = ctypes.c_uint64(0)
        check(lib.vs_cdc_finish(self._h, ctypes.byref(n)))
        return int(n.value)

    def wait(self) -> None:
        check(lib.vs_cdc_wait(self._h))

    def chunks(self, first: int = 0, n: Optional[int] = None, total: Optional[int] = None
               ) -> List[Chunk]:
        if n is None:
            n = (total or 0) - first
        if n <= 0:
            return []
        arr = (VsChunk * n)()
        check(lib.vs_cdc_get_chunks(self._h, first, n, arr))
        return [_chunk_from(c) for c in arr]

    def timing(self, enable: bool = True):
        ms = (ctypes.c_double * 4)()
        cnt = (ctypes.c_uint64 * 4)()
        check(lib.vs_cdc_timing(self._h, 1 if enable else 0, ms, cnt))
        return list(ms), list(cnt)

    def fence(self, batch: int) -> None:
        """Order the next scan after batch `batch`'s blob IDs are final
        (vs_cdc_fence): what a producer overwriting that batch's bytes needs."""
        check(lib.vs_cdc_fence(self._h, batch))

    def timing_detail(self):
        """The interval the last timing() call closed: SHA-256 kernel ms in
        all, outside every fingerprint window, inside one, the fingerprint
        windows' union; and the chunks the final drains hashed in latency mode."""
        d = (ctypes.c_double * 4)()
        q = ctypes.c_uint64(0)
        check(lib.vs_cdc_timing_detail(self._h, d, ctypes.byref(q)))
        return {"sha_ms": d[0], "sha_outside_fp_ms": d[1], "sha_inside_fp_ms": d[2],
                "fp_union_ms": d[3], "quad_chains": q.value}

    def close(self) -> None:
        if self._h:
            lib.vs_cdc_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sha256_batch(buf: bytes, offs, lens, device: int = 0) -> List[bytes]:
    """restic.Hash over many blobs of one host buffer, on the GPU."""
    import numpy as np
    n = len(offs)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros((max(n, 1), 32), dtype=np.uint8)
    if isinstance(buf, np.ndarray):   # the caller's bytes, no copy
        b = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    else:
        b = np.frombuffer(bytes(buf), dtype=np.uint8)
    if not len(b):
        b = np.zeros(1, np.uint8)
    check(lib.vs_sha256_batch(device, b.ctypes.data, len(buf), o.ctypes.data, ln.ctypes.data, n,
                              out.ctypes.data))
    return [bytes(out[i]) for i in range(n)]


class DeviceSha256:
    """restic.Hash over many device-resident blobs (vs_sha256_* work-queue
    kernel): the C5 small-file path, one blob ID per file."""

    def __init__(self, device: int = 0):
        self.device = device
        self._h = ctypes.c_void_p()
        check(lib.vs_sha256_open(device, ctypes.byref(self._h)))

    def run(self, dev_buf: int, dev_off: int, dev_len: int, n: int, dev_out: int,
            stream: Optional[int] = None) -> None:
        check(lib.vs_sha256_run_device(self._h, ctypes.c_void_p(dev_buf), ctypes.c_void_p(dev_off),
                                       ctypes.c_void_p(dev_len), n, ctypes.c_void_p(dev_out),
                                       ctypes.c_void_p(stream or None)))

    def drain_stats(self) -> tuple:
        """(latency-mode chains, of those isolated) of the last run's drain."""
        out = (ctypes.c_uint64 * 2)()
        check(lib.vs_sha256_drain_stats(self._h, out))
        return int(out[0]), int(out[1])

    def set_wide(self, min_chains: int = 0, drain_blocks: int = 0) -> None:
        """Throughput mode from min_chains active blobs (0 = default, 0xffffffff = never)."""
        check(lib.vs_sha256_set_wide(self._h, int(min_chains), int(drain_blocks)))

    def set_option(self, option: int, value: int) -> None:
        check(lib.vs_sha256_set_option(self._h, option, value))

    def blocks(self, dev_buf: int, length: int, block_size: int, dev_out: int,
               stream: Optional[int] = None) -> int:
        """syncthing's scanner: SHA-256 of every block_size block (vs_sha256_blocks);
        returns the number of blocks."""
        check(lib.vs_sha256_blocks(self._h, ctypes.c_void_p(dev_buf), length, block_size,
                                   ctypes.c_void_p(dev_out), ctypes.c_void_p(stream or None)))
        return (length + block_size - 1) // block_size

    def verify(self, dev_buf: int, dev_off: int, dev_len: int, n: int, dev_want: int,
               dev_bad: Optional[int] = None, stream: Optional[int] = None) -> int:
        """Repository.LoadBlob's check (vs_blob_verify): the number of blobs
        whose SHA-256 differs from the expected ID (waits)."""
        bad = ctypes.c_uint64(0)
        check(lib.vs_blob_verify(self._h, ctypes.c_void_p(dev_buf), ctypes.c_void_p(dev_off),
                                 ctypes.c_void_p(dev_len), n, ctypes.c_void_p(dev_want),
                                 ctypes.c_void_p(dev_bad or None), ctypes.byref(bad),
                                 ctypes.c_void_p(stream or None)))
        return int(bad.value)

    def dedup(self, dev_ids: int, n: int, dev_first: int, stream: Optional[int] = None,
              count: bool = True) -> Optional[int]:
        """Repository.SaveBlob's dedup over n device blob IDs (vs_blob_dedup):
        dev_first[i] = first index with the same ID; returns the distinct-ID
        count (waits) when count is set."""
        u = ctypes.c_uint64(0)
        check(lib.vs_blob_dedup(self._h, ctypes.c_void_p(dev_ids), n, ctypes.c_void_p(dev_first),
                                ctypes.byref(u) if count else None,
                                ctypes.c_void_p(stream or None)))
        return int(u.value) if count else None

    def dedup_known(self, dev_ids: int, n: int, dev_known: int, n_known: int, dev_first: int,
                    stream: Optional[int] = None, count: bool = True) -> Optional[int]:
        """SaveBlob's dedup against the repository's index too
        (vs_blob_dedup_known): dev_first[i] = VS_DEDUP_KNOWN for a known ID;
        returns the number of distinct new IDs (waits) when count is set."""
        u = ctypes.c_uint64(0)
        check(lib.vs_blob_dedup_known(self._h, ctypes.c_void_p(dev_ids), n,
                                      ctypes.c_void_p(dev_known), n_known,
                                      ctypes.c_void_p(dev_first), ctypes.byref(u) if count else None,
                                      ctypes.c_void_p(stream or None)))
        return int(u.value) if count else None

    def index_sort(self, dev_known: int, n: int, stream: Optional[int] = None) -> None:
        """vs_blob_index_sort: the known IDs into dedup_known's search order."""
        check(lib.vs_blob_index_sort(self._h, ctypes.c_void_p(dev_known), n,
                                     ctypes.c_void_p(stream or None)))

    def close(self) -> None:
        if self._h:
            lib.vs_sha256_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Sealer:
    """restic Key.Seal over many device-resident blobs (vs_seal_*): AES-256-CTR
    + Poly1305-AES with one repository key."""

    def __init__(self, enc_key: bytes, mac_k: bytes, mac_r: bytes, device: int = 0):
        if len(enc_key) != 32 or len(mac_k) != 16 or len(mac_r) != 16:
            raise ValueError("enc_key 32 bytes, mac_k and mac_r 16 bytes")
        self._h = ctypes.c_void_p()
        check(lib.vs_seal_open(device, enc_key, mac_k, mac_r, ctypes.byref(self._h)))

    def run(self, dev_in: int, dev_off: int, dev_len: int, n: int, dev_nonces: int, dev_out: int,
            dev_macs: int, stream: Optional[int] = None) -> None:
        check(lib.vs_seal_run_device(self._h, ctypes.c_void_p(dev_in), ctypes.c_void_p(dev_off),
                                     ctypes.c_void_p(dev_len), n, ctypes.c_void_p(dev_nonces),
                                     ctypes.c_void_p(dev_out), ctypes.c_void_p(dev_macs),
                                     ctypes.c_void_p(stream or None)))

    def run_records(self, dev_in: int, dev_off: int, dev_len: int, n: int, dev_nonces: int,
                    dev_out: int, dev_ct_off: int, stream: Optional[int] = None) -> None:
        """Key.Seal into the pack layout: nonce || ciphertext || tag around
        dev_out + ct_off[i] (vs_seal_records_device)."""
        check(lib.vs_seal_records_device(self._h, ctypes.c_void_p(dev_in), ctypes.c_void_p(dev_off),
                                         ctypes.c_void_p(dev_len), n, ctypes.c_void_p(dev_nonces),
                                         ctypes.c_void_p(dev_out), ctypes.c_void_p(dev_ct_off),
                                         ctypes.c_void_p(stream or None)))

    def open(self, dev_in: int, dev_rec_off: int, dev_len: int, n: int, dev_out: int,
             dev_out_off: int, dev_bad: int, stream: Optional[int] = None) -> int:
        """Key.Open over stored records (vs_open_run_device): verify each tag,
        decrypt; returns the number of blobs whose tag did not match."""
        nb = ctypes.c_uint64(0)
        check(lib.vs_open_run_device(self._h, ctypes.c_void_p(dev_in), ctypes.c_void_p(dev_rec_off),
                                     ctypes.c_void_p(dev_len), n, ctypes.c_void_p(dev_out),
                                     ctypes.c_void_p(dev_out_off or None), ctypes.c_void_p(dev_bad),
                                     ctypes.byref(nb), ctypes.c_void_p(stream or None)))
        return nb.value

    def pack(self, sha: "DeviceSha256", dev_in: int, offs, lens, types, ids, blob_nonces,
             hdr_nonces, min_pack_size: int = 4 << 20, stream: Optional[int] = None):
        """restic v0.13.1 pack files of the blobs (vs_restic_pack): returns
        (device tensor of the packs back to back, [(offset, length, first, n)],
        [pack id bytes]).  offs/lens/types: per blob; ids: n x 32 bytes;
        blob_nonces: n x 16; hdr_nonces: >= n_packs x 16 (n rows suffice)."""
        import numpy as np
        import torch
        from ._lib import VsPack
        n = len(lens)
        o = np.ascontiguousarray(offs, np.uint64)
        ln = np.ascontiguousarray(lens, np.uint32)
        ty = np.ascontiguousarray(types, np.uint8)
        idb = np.ascontiguousarray(np.frombuffer(b"".join(ids), np.uint8) if isinstance(ids, list)
                                   else ids, np.uint8)
        bn = np.ascontiguousarray(blob_nonces, np.uint8)
        hn = np.ascontiguousarray(hdr_nonces, np.uint8)
        npk, olen = ctypes.c_size_t(), ctypes.c_uint64()
        args = [self._h, sha._h, ctypes.c_void_p(dev_in), o.ctypes.data, ln.ctypes.data,
                ty.ctypes.data, idb.ctypes.data, n, bn.ctypes.data, hn.ctypes.data, min_pack_size]
        check(lib.vs_restic_pack(*args, None, 0, None, 0, ctypes.byref(npk), ctypes.byref(olen),
                                 None, ctypes.c_void_p(stream or None)))
        out = torch.zeros(max(olen.value, 16), dtype=torch.uint8, device="cuda")
        packs = (VsPack * max(npk.value, 1))()
        pid = np.zeros((max(npk.value, 1), 32), np.uint8)
        check(lib.vs_restic_pack(*args, ctypes.c_void_p(out.data_ptr()), olen.value, packs,
                                 npk.value, ctypes.byref(npk), ctypes.byref(olen), pid.ctypes.data,
                                 ctypes.c_void_p(stream or None)))
        return (out, [(p.offset, p.length, p.first_blob, p.n_blobs) for p in packs[:npk.value]],
                [bytes(pid[k]) for k in range(npk.value)])

    def index(self, sha: "DeviceSha256", lens, types, ids, pack_ids, nonce: bytes,
              min_pack_size: int = 4 << 20):
        """restic v0.13.1's index file of the packs pack() made from the same
        blobs (vs_restic_index): (index JSON bytes, stored file bytes =
        nonce || sealed JSON || tag, file ID)."""
        import numpy as np
        n = len(lens)
        ln = np.ascontiguousarray(lens, np.uint32)
        ty = np.ascontiguousarray(types, np.uint8)
        idb = np.ascontiguousarray(np.frombuffer(b"".join(ids), np.uint8) if isinstance(ids, list)
                                   else ids, np.uint8)
        pk = np.ascontiguousarray(np.frombuffer(b"".join(pack_ids), np.uint8) if pack_ids
                                  else np.zeros(32, np.uint8))
        nj = ctypes.c_size_t()
        args = [self._h, sha._h, ln.ctypes.data, ty.ctypes.data, idb.ctypes.data, n, min_pack_size,
                pk.ctypes.data, nonce]
        check(lib.vs_restic_index(*args, None, 0, ctypes.byref(nj), None, None))
        js = ctypes.create_string_buffer(max(nj.value, 1))
        fo = ctypes.create_string_buffer(nj.value + 32)
        fid = ctypes.create_string_buffer(32)
        check(lib.vs_restic_index(*args, js, nj.value, ctypes.byref(nj), fo, fid))
        return js.raw[:nj.value], fo.raw[:nj.value + 32], fid.raw

    def set_timing(self, on: bool) -> None:
        check(lib.vs_seal_set_timing(self._h, int(on)))

    def set_option(self, option: int, value: int) -> None:
        check(lib.vs_seal_set_option(self._h, option, value))

    def kernel_ms(self):
        """(ctr_ms, mac_ms, runs) summed over the timed runs since the last call."""
        ms = (ctypes.c_double * 2)()
        runs = ctypes.c_int()
        check(lib.vs_seal_kernel_ms(self._h, ms, ctypes.byref(runs)))
        return ms[0], ms[1], runs.value

    def close(self) -> None:
        if self._h:
            lib.vs_seal_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def syncthing_block_size(file_size: int) -> int:
    """syncthing lib/protocol BlockSize (vs_syncthing_block_size)."""
    return int(lib.vs_syncthing_block_size(int(file_size)))


def synth_fill_device(dev_ptr: int, seed: int, off: int, n: int, device: int = 0,
                      stream: Optional[int] = None) -> None:
    check(lib.vs_synth_fill_device(device, seed, off, n, ctypes.c_void_p(dev_ptr),
                                   ctypes.c_void_p(stream or None)))
