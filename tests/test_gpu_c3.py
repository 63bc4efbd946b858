"""Config C3 at full size on one GPU.

C3 is 1 TiB of the seed-3 stream byte-range sharded over 8 GPUs, 128 GiB per
rank (the backup it stands for: restic backup of one
volume, /root/reference/mover-restic/entry.sh:60-65).  The driver's 8-GPU run
is the real thing; here every rank's work runs in turn on the one GPU, exactly
as the rank would do it: its 128 GiB share plus halos generated on the device,
vs_cdc_scan over it, vs_cdc_stitch from its true entry (the previous rank's
exit, which the 8-rank run receives from the all-gather and which the golden
records), vs_cdc_finish + vs_cdc_wait, and the rank's chunk list as vs_chunk
records (Start, Length, Cut, blob ID) compared with the per-rank digest the C
oracle computed (tests/golden/make_golden_full.py -> full_configs.json).  The
exit each rank computes must equal the next rank's golden entry, which is the
exit exchange's own invariant, and the speculative pass from own_lo must
converge to the same exit.
"""
import ctypes
import hashlib
import json
import os

import pytest

from volsync_amd.shard import ShardSpec

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED, PER, WORLD = 3, 128 << 30, 8
TOTAL = PER * WORLD
MIN, MAX = 512 << 10, 8 << 20


def _golden():
    doc = json.load(open(os.path.join(ROOT, "tests", "golden", "full_configs.json")))
    return doc["cdc"][str(SEED)][str(TOTAL)]


@pytest.fixture(scope="module")
def c3_buf(gpu):
    """One device buffer large enough for any rank's share plus halos (128 GiB
    + 64 + MaxSize + 63 bytes), reused by every rank and freed afterwards."""
    import torch
    n = max(s.data_hi - s.data_lo for s in ShardSpec.split(TOTAL, WORLD, MAX))
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    yield t
    del t
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("rank", list(range(WORLD)))
def test_c3_rank_share_exact(c3_buf, rank):
    from volsync_amd import DeviceChunker, TestPol, synth_fill_device
    from volsync_amd._lib import VsChunk, check, lib
    gold = _golden()
    g = gold["ranks"][rank]
    spec = ShardSpec.for_rank(TOTAL, WORLD, rank, MAX)
    assert (g["own_lo"], g["own_hi"]) == (spec.own_lo, spec.own_hi)
    dlen = spec.data_hi - spec.data_lo
    synth_fill_device(c3_buf.data_ptr(), SEED, spec.data_lo, dlen)
    dc = DeviceChunker(TestPol, MIN, MAX, 20)
    try:
        dc.scan(c3_buf.data_ptr(), dlen, spec.data_lo, spec.own_lo, spec.own_hi, spec.final)
        # the speculative walk from own_lo (what the rank publishes first) ...
        spec_exit, spec_done = dc.stitch(spec.own_lo)
        # ... and the walk from the true entry (after the exchange)
        ex, done = dc.stitch(g["entry"])
        n = dc.finish()
        dc.wait()
        arr = (VsChunk * max(n, 1))()
        if n:
            check(lib.vs_cdc_get_chunks(dc._h, 0, n, arr))
        recs = ctypes.string_at(arr, 56 * n) if n else b""
    finally:
        dc.close()
    assert n == g["chunks"]
    assert hashlib.sha256(recs).hexdigest() == g["digest"]
    if n:
        assert arr[0].start == g["entry"]
        assert arr[n - 1].start < spec.own_hi
    if rank + 1 < WORLD:
        # the exit is the next rank's true entry; walks from different starts
        # merge at a shared chunk start, so the speculative exit agrees too
        nxt = gold["ranks"][rank + 1]["entry"]
        assert done and ex == nxt
        assert spec_done and spec_exit == nxt
    else:
        # the last rank ends the volume with its EOF chunk
        assert n and arr[n - 1].start + arr[n - 1].length == TOTAL

