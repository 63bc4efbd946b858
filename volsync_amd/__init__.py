"""volsync_amd -- MI355X-native hot path behind VolSync's restic and rsync movers.

Product: volsync_amd/lib/libvsgpu.so (hand-written gfx950 HIP kernels behind the
C ABI in include/vsgpu.h).  This package is the host-side mirror of the
reference's interfaces for that path: the restic chunker API + blob IDs
(volsync_amd.chunker) and rsync's sender-side delta functions (volsync_amd.rsync).
"""
from ._lib import VsError, device_count, last_error  # noqa: F401
from .chunker import (Chunk, Chunker, DeviceChunker, DeviceSha256, EOF, MaxSize, MinSize, New,  # noqa: F401
                      NewWithBoundaries, Pol, TestPol, sha256_batch, synth_fill_device,
                      syncthing_block_size, Sealer)
from .rsync import (CSUM_MD5, CSUM_XXH3_64, CSUM_XXH3_128, CSUM_XXH64, Matcher, file_sum_finish, file_sum_init,  # noqa: F401
                    SumStruct, ZstdTokens, generate_sums, match_sums, sum_sizes_sqroot)

__version__ = "0.1.0"
