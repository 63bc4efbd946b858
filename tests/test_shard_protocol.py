"""Multi-rank CPU tests (gloo) of the byte-range sharding protocol
(volsync_amd/shard.py): scan -> stitch -> all-gather exits -> re-stitch -> finish.

Each rank runs a test double of the device chunker built on the Python oracle
(test infrastructure) that sees ONLY its own byte window (own range + halos),
so the test checks both the exchange logic and that the halos suffice."""
import hashlib
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import cdc_ref as P


class OracleRank:
    """Same surface as volsync_amd.DeviceChunker for the protocol functions."""

    def __init__(self, window: np.ndarray, pol, mn, mx, ab):
        self.w = window
        self.pol, self.mn, self.mx, self.ab = pol, mn, mx, ab

    def scan(self, ptr, length, origin, own_lo, own_hi, final):
        assert length == len(self.w)
        self.origin, self.own_lo, self.own_hi, self.final = origin, own_lo, own_hi, final
        self.end = origin + length
        self.scan_end = min(own_hi + self.mx - 1, self.end)
        pos, fp = P.candidates(self.w, self.pol, self.ab)
        keep = pos + origin >= max(own_lo, origin + 63)
        self.cpos, self.cfp = pos[keep] + origin, fp[keep]

    def _cut(self, s):
        q, lim = s + self.mn - 1, s + self.mx - 1
        k = int(np.searchsorted(self.cpos, q))
        if k < len(self.cpos) and self.cpos[k] <= lim and self.cpos[k] < self.scan_end:
            return int(self.cpos[k]), "n"
        if lim < self.scan_end:
            return lim, "f"
        assert self.final and self.scan_end == self.end, "window too small for the rule"
        return self.end - 1, "e"

    def stitch(self, entry):
        self.entry = entry
        self.cuts = []
        s = entry
        while s < self.own_hi and s < self.end:
            c, t = self._cut(s)
            self.cuts.append((s, c, t))
            s = c + 1
        return s, True

    def finish(self):
        return len(self.cuts)

    def chunks(self, first, n):
        out = []
        for s, c, t in self.cuts[first:first + n]:
            seg = self.w[s - self.origin:c + 1 - self.origin]
            if t == "e":
                cut = P.eof_cut(self.w, s - self.origin, c + 1 - self.origin, self.pol, self.mn)
            else:
                cut = P.fp_at(self.w, c - self.origin, self.pol)
            out.append((s, c - s + 1, cut, hashlib.sha256(seg.tobytes()).hexdigest()))
        return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, seed, params, outdir):
    import torch.distributed as dist
    from volsync_amd.shard import ShardSpec, run_shard, torch_collectives
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pol, mn, mx, ab = params
    spec = ShardSpec.for_rank(n, world, rank, mx)
    window = P.synth(seed, spec.data_lo, spec.data_hi - spec.data_lo)
    h = OracleRank(window, pol, mn, mx, ab)
    cnt = run_shard(h, spec, 0, *torch_collectives(None))
    mine = h.chunks(0, cnt)
    allc = [None] * world
    dist.all_gather_object(allc, mine)
    if rank == 0:
        flat = [c for part in allc for c in part]
        import json
        with open(os.path.join(outdir, "result.json"), "w") as f:
            json.dump(flat, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,params", [
    (2, 6 << 20, (P.TEST_POL, 16384, 262144, 14)),
    (3, 5 << 20, (P.TEST_POL, 8192, 65536, 12)),
    (5, 700 << 10, (P.TEST_POL, 65536, 262144, 15)),   # own range < MaxSize: entries jump ranks
])
def test_sharded_protocol_gloo(world, n, params):
    import json

    import torch.multiprocessing as mp
    seed = 77
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), n, seed, params, d),
                           nprocs=world, join=True, start_method="spawn")
        got = [tuple(x) for x in json.load(open(os.path.join(d, "result.json")))]
    data = P.synth(seed, 0, n)
    want = [(s, l, c, i) for s, l, c, i in P.chunk(data, *params)]
    assert got == want
