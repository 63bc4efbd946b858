"""CPU tests of the product library's C ABI surface (no compute without a GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import cdc_ref as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vsgpu.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vs_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header_symbols():
    from volsync_amd import _lib
    so = _lib.LIB_PATH
    assert os.path.exists(so)
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (vs_[a-z0-9_]+)", out))
    want = set(header_functions())
    assert want, "no declarations parsed"
    assert want <= exported, f"missing: {sorted(want - exported)}"
    # nothing product-facing is exported that the header does not declare
    assert exported <= want, f"undeclared exports: {sorted(exported - want)}"


def test_library_links_no_oracle():
    from volsync_amd import _lib
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    strings = open(_lib.LIB_PATH, "rb").read()
    assert b"liboracle" not in strings and b"ref_chunk_all" not in strings


def test_library_never_registers_host_memory():
    """Round 2's driver failure: the library page-locked its
    std::vector read-back storage with hipHostRegister; a stale registration
    over heap bytes a later caller buffer reused made the runtime's pageable
    copy of that buffer fail.  The library now pins only what it allocates
    (hipHostMalloc) and stages caller memory: it must not import the call."""
    from volsync_amd import _lib
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert "hipHostRegister" not in out and "hipHostUnregister" not in out
    assert "hipHostMalloc" in out


def test_pol_helpers_match_oracle():
    from volsync_amd import Pol
    p = Pol(P.TEST_POL)
    assert p.Deg() == 53
    assert p.Irreducible()
    assert not Pol(P.TEST_POL ^ 2).Irreducible()
    out, mod = p.tables()
    from tests import oracle_lib as O
    ro = np.zeros(256, np.uint64)
    rm = np.zeros(256, np.uint64)
    O.lib().ref_tables(P.TEST_POL, ro.ctypes.data, rm.ctypes.data)
    assert out == [int(x) for x in ro] and mod == [int(x) for x in rm]


def test_random_polynomials_irreducibility_agrees():
    from volsync_amd import Pol
    rng = np.random.default_rng(7)
    for _ in range(40):
        p = int(rng.integers(0, 1 << 53, dtype=np.uint64)) | (1 << 53) | 1
        assert Pol(p).Irreducible() == P.pol_irreducible(p)


def test_pol_zero_is_rejected_like_upstream():
    from volsync_amd import _lib
    out = (ctypes.c_uint64 * 256)()
    mod = (ctypes.c_uint64 * 256)()
    rc = _lib.lib.vs_pol_tables(0, out, mod)
    assert rc == _lib.VS_ERR_POLY
    assert "not initialized" in _lib.last_error()


def test_no_cpu_fallback_without_device():
    from volsync_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    rc = _lib.lib.vs_cdc_open(0, P.TEST_POL, P.MIN_SIZE, P.MAX_SIZE, 20, ctypes.byref(h))
    assert rc == _lib.VS_ERR_NO_DEVICE
    assert not h.value
    import volsync_amd
    with pytest.raises(volsync_amd.VsError):
        list(volsync_amd.New(__import__("io").BytesIO(b"x" * 100), P.TEST_POL))


def test_file_sum_finish_on_host_vs_xxhash():
    """The host end of the whole-file XXH3 (vs_rsync_file_sum_finish: last
    partial block, last stripe, merge) from the initial accumulators: for files
    of 241..1024 bytes there are no whole blocks before it, so the result must
    be XXH3 of the file itself (no GPU needed)."""
    import xxhash
    import volsync_amd as V
    rng = np.random.default_rng(3)
    for n in [241, 255, 256, 300, 512, 1000, 1023, 1024]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        acc = V.file_sum_init()
        assert V.file_sum_finish(acc, d, n, 8) == xxhash.xxh3_128(d).intdigest().to_bytes(16, "little")
        assert V.file_sum_finish(acc, d, n, 7) == xxhash.xxh3_64(d).intdigest().to_bytes(8, "little")


def test_library_reads_no_environment():
    """The product library takes its settings from the caller (the handle
    options of vsgpu.h), never from the environment: a mover pod's environment
    cannot change which kernels run.  No VSGPU_* name is in the
    shipped object (the one getenv left is rocPRIM's, inlined by the hipcub
    radix sorts of rsync.hip and dedup.hip)."""
    from volsync_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"VSGPU_" not in data
