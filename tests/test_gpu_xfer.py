"""GPU regression test of the round-2 driver failure.

`test_match_vs_golden[rsync_tail_partial.json]` failed on a fresh box with
VsError -6 "source upload failed": the one-shot vs_rsync_match's pageable
hipMemcpy of the caller's source returned hipErrorInvalidValue.  The runtime
refuses a pageable copy whose host range overlaps a *registered* range it does
not fully lie in (probe: tools/probe/pin_overlap.py at git 2fcace1, profiles/r03_xfer), and
round 2's library registered heap storage (std::vector read-backs,
hipHostRegister) that a later numpy array could come to occupy.

A second defect hid behind it: the runtime's last error is per thread and
sticky, and the library's launch wrappers return hipGetLastError() -- so a
failed runtime call of the CALLER's made the library's next launch report
it as its own (first run of this test: "launch_rs_signatures: invalid
argument").  Every entry point now clears it first (enter_device).

This test builds that exact overlap deterministically -- a registered range
covering the first bytes of the caller's buffer -- and checks that every
entry point that takes caller host memory still works (they stage it through
the library's own pinned chunks), bit-exact against the oracle / hashlib.
"""
import ctypes
import hashlib
import mmap

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

PG = 4096


def _hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    h.hipHostUnregister.argtypes = [ctypes.c_void_p]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    return h


class Overlapped:
    """An mmap'd host buffer of n bytes at page offset 256 whose first 192
    bytes lie in a foreign registered range (the stale registration)."""

    def __init__(self, data: np.ndarray):
        self.hip = _hip()
        n = len(data)
        self.m = mmap.mmap(-1, (n + 256 + PG - 1) // PG * PG + PG)
        self.raw = (ctypes.c_char * len(self.m)).from_buffer(self.m)
        base = ctypes.addressof(self.raw)
        self.reg = base + 128
        assert self.hip.hipHostRegister(ctypes.c_void_p(self.reg), 320, 0) == 0
        self.arr = np.frombuffer(self.m, np.uint8, count=n, offset=256)
        self.arr[:] = data

    def runtime_copy_fails(self) -> bool:
        """The precondition: the runtime's own pageable copy of the buffer fails."""
        d = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(d), len(self.arr)) == 0
        e = self.hip.hipMemcpy(d, ctypes.c_void_p(self.arr.ctypes.data), len(self.arr), 1)
        self.hip.hipFree(d)
        return e != 0

    def close(self):
        self.hip.hipHostUnregister(ctypes.c_void_p(self.reg))
        del self.arr, self.raw
        try:
            self.m.close()
        except BufferError:   # a failing assert's traceback still holds a view
            pass


def test_one_shot_rsync_with_overlapping_registration(gpu):
    from volsync_amd import generate_sums, match_sums
    basis = O.synth(31, 0, 1_060_921)
    src = R.mutate(basis, 1024, seed=4, frac=0.05)
    for csum_type, seed in [(R.CSUM_XXH3_128, 0x5EED5EED), (R.CSUM_MD5, 7)]:
        bl, s2l, cnt, rem = O.rsync_sizes(len(basis), 0)
        c1, c2 = O.rsync_signatures(basis, bl, s2l, csum_type, seed)
        want, _ = O.rsync_match(src, c1, c2, bl, rem, csum_type, seed)
        ob, os_ = Overlapped(basis), Overlapped(src)
        try:
            assert ob.runtime_copy_fails() and os_.runtime_copy_fails()
            s = generate_sums(ob.arr, csum_type, seed)
            assert (s.sum1 == c1).all() and (s.sum2 == c2).all()
            assert match_sums(os_.arr, s, csum_type, seed) == want
        finally:
            ob.close()
            os_.close()


def test_sha256_batch_and_load_sums_with_overlapping_registration(gpu):
    from volsync_amd import Matcher, SumStruct, sha256_batch
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    ob = Overlapped(data)
    try:
        assert ob.runtime_copy_fails()
        offs = np.array([0, 1000, 1 << 20, (3 << 20) - 5], np.uint64)
        lens = np.array([1000, 70_000, 2 << 20, 5], np.uint32)
        got = sha256_batch(ob.arr, offs, lens)
        for k, (o, l) in enumerate(zip(offs, lens)):
            assert bytes(got[k]) == hashlib.sha256(data[int(o):int(o) + int(l)].tobytes()).digest()
    finally:
        ob.close()
    # the sum arrays of vs_rsync_load_sums: 300 K blocks (1.2 MB of sum1)
    basis = O.synth(32, 0, 300_000 * 700)
    bl, s2l, cnt, rem = O.rsync_sizes(len(basis), 700)
    c1, c2 = O.rsync_signatures(basis, bl, s2l, R.CSUM_XXH3_128, 1)
    o1 = Overlapped(c1.view(np.uint8))
    try:
        assert o1.runtime_copy_fails()
        import torch
        m = Matcher()
        m.load_sums(SumStruct(0, cnt, bl, s2l, rem, o1.arr.view(np.uint32), c2), R.CSUM_XXH3_128, 1)
        ds = torch.from_numpy(basis[: 4 << 20].copy()).to("cuda")
        got = m.match_sums(ds.data_ptr(), 4 << 20)
        m.close()
        assert got[:5] == [(i * bl, i) for i in range(5)]
    finally:
        o1.close()
