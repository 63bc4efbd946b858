"""volsync_amd -- MI355X-native hot path behind VolSync's restic (and rsync) movers.

Product: volsync_amd/lib/libvsgpu.so (hand-written gfx950 HIP kernels behind the
C ABI in include/vsgpu.h).  This package is the host-side mirror of the
reference's interface for that path (restic chunker API + blob IDs).
"""
from ._lib import VsError, device_count, last_error  # noqa: F401
from .chunker import (Chunk, Chunker, DeviceChunker, DeviceSha256, EOF, MaxSize, MinSize, New,  # noqa: F401
                      NewWithBoundaries, Pol, TestPol, sha256_batch, synth_fill_device)

__version__ = "0.1.0"
