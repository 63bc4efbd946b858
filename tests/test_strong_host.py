"""CPU self-test of the device strong-sum restatement (volsync_amd/csrc/strong.hpp,
compiled for the host by g++) against the xxhash package and hashlib.

Covers every XXH3 length class (0, 1-3, 4-8, 9-16, 17-128, 129-240, >240 with
1 KiB block and last-stripe edges), XXH64's 32-byte loop and tails, and MD5
with and without rsync's seed prefix.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

from oracle import rsync_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "strong_host.cpp")
OUT = os.path.join(HERE, "native", "build", "libstrong_host.so")

LENGTHS = sorted(set(list(range(0, 260)) + [511, 512, 513, 1023, 1024, 1025, 1087, 1088, 1089,
                                            2047, 2048, 2049, 4096, 5000, 65536, 131071, 131072]))
SEEDS = [0, 1, 0x5EED5EED, 0xFFFFFFFF]


@pytest.fixture(scope="module")
def strong():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", OUT, SRC], check=True)
    L = ctypes.CDLL(OUT)
    L.strong_host_checksum2.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_uint32, ctypes.c_void_p]
    return L


def run(L, buf: bytes, csum_type: int, seed: int) -> bytes:
    out = ctypes.create_string_buffer(16)
    src = ctypes.create_string_buffer(buf, max(len(buf), 1))
    L.strong_host_checksum2(src, len(buf), csum_type, seed, out)
    return out.raw


@pytest.mark.parametrize("csum_type", [R.CSUM_XXH3_128, R.CSUM_XXH3_64, R.CSUM_XXH64, R.CSUM_MD5])
def test_strong_restatement(strong, csum_type):
    data = np.random.default_rng(csum_type).integers(0, 256, 131072 + 64, dtype=np.uint8).tobytes()
    for seed in SEEDS:
        for n in LENGTHS:
            off = (n * 7 + seed) % 61           # unaligned starts too
            b = data[off:off + n]
            assert run(strong, b, csum_type, seed) == R.checksum2(b, csum_type, seed), (n, seed)
