"""Multi-rank CPU tests (gloo) of the byte-range sharded hash_search
(volsync_amd/rsync_shard.py run_walk_shard): speculative walk per rank ->
all-gather of exit states -> re-walk from the true entry -> finish.

Each rank runs a test double of the device matcher built on the C oracle
(oracle/rsync_ref.c ref_rsync_walk, test infrastructure) that sees ONLY its
own byte window (own range + blength - 1 bytes of right halo), so the test
checks the exchange logic, the want_i hand-over and that the halo suffices.
The concatenated match list and false-alarm total must equal ONE hash_search
over the whole file (ref_rsync_match)."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import oracle_lib as O


class OracleWalkRank:
    """match_scan / match_stitch / match_finish / matches, as volsync_amd.Matcher."""

    def __init__(self, window, sums, blength, remainder, csum, seed):
        self.w = window
        self.c1, self.c2 = sums
        self.bl, self.rem, self.csum, self.seed = blength, remainder, csum, seed

    def _walk(self, entry, want):
        m, fa, eo, ew = O.rsync_walk(self.w, self.origin, self.length, self.own_hi, entry, want,
                                     self.c1, self.c2, self.bl, self.rem, self.csum, self.seed)
        self.m, self.fa = m, fa
        return eo, ew

    def match_scan(self, ptr, dlen, origin, length, own_lo, own_hi):
        assert dlen == len(self.w)
        self.origin, self.length, self.own_lo, self.own_hi = origin, length, own_lo, own_hi
        # speculative entry: rank 0 starts as hash_search does; the others
        # with want_i = count ("no preference": want_i < count fails)
        return self._walk(own_lo, 0 if own_lo == 0 else len(self.c1))

    def match_stitch(self, entry, want):
        assert entry >= self.own_lo
        return self._walk(entry, want)

    def match_finish(self):
        return len(self.m)

    def matches(self, first, n):
        return self.m[first:first + n]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(n, block_size, csum, seed, frac):
    basis = O.synth(57, 0, n)
    bl, s2, cnt, rem = O.rsync_sizes(n, block_size)
    c1, c2 = O.rsync_signatures(basis, bl, s2, csum, seed)
    src = R.mutate(basis, bl, seed=9, frac=frac)
    return src, (c1, c2), bl, rem


def _worker(rank, world, port, args, outdir):
    import torch.distributed as dist
    from volsync_amd.rsync_shard import SourceShard, run_walk_shard, torch_pair_collectives
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, block_size, csum, seed, frac = args
    src, sums, bl, rem = _case(n, block_size, csum, seed, frac)
    spec = SourceShard.for_rank(len(src), bl, world, rank)
    h = OracleWalkRank(src[spec.data_lo:spec.data_hi].copy(), sums, bl, rem, csum, seed)
    st = {}
    cnt = run_walk_shard(h, spec, 0, *torch_pair_collectives(None), stats=st)
    mine = {"m": h.matches(0, cnt), "fa": h.fa, "rounds": st["exchange_rounds"]}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        with open(os.path.join(outdir, "result.json"), "w") as f:
            json.dump(allr, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,args", [
    (2, ((3 << 20) + 777, 0, R.CSUM_XXH3_128, 0x5EED5EED, 0.10)),   # short last block
    (3, (1 << 20, 4096, R.CSUM_MD5, 0x5EED5EED, 0.20)),
    (5, (700 << 10, 8192, R.CSUM_XXH64, 0, 0.10)),                   # ranks of ~17 blocks
    (4, (300_000, 100_000, R.CSUM_XXH3_128, 3, 0.30)),               # own range < blength
])
def test_sharded_walk_gloo(world, args):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), args, d), nprocs=world, join=True,
                           start_method="spawn")
        res = json.load(open(os.path.join(d, "result.json")))
    got = [tuple(x) for r in res for x in r["m"]]
    src, (c1, c2), bl, rem = _case(*args)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, args[2], args[3])
    assert got == want
    assert sum(r["fa"] for r in res) == fa


@pytest.mark.parametrize("world", [2, 3, 6, 11])
def test_sharded_walk_local_dup_blocks(world):
    """Repeated blocks (want_i decides between identical blocks) with the
    shard boundaries inside runs of duplicates: the want_i hand-over across
    ranks must reproduce hash_search's choices."""
    from volsync_amd.rsync_shard import SourceShard, run_walk_shards_local
    unit = O.synth(5, 0, 700)
    basis = np.tile(unit, 64)
    src = np.concatenate([basis[:7000], O.synth(6, 0, 333), basis[:14000], basis[350:9000]])
    bl, s2, cnt, rem = O.rsync_sizes(len(basis))
    c1, c2 = O.rsync_signatures(basis, bl, s2, R.CSUM_XXH3_128, 77)
    specs = SourceShard.split(len(src), bl, world)
    hs = [OracleWalkRank(src[s.data_lo:s.data_hi].copy(), (c1, c2), bl, rem, R.CSUM_XXH3_128, 77)
          for s in specs]
    got = run_walk_shards_local(hs, specs, [0] * world)
    want, fa = O.rsync_match(src, c1, c2, bl, rem, R.CSUM_XXH3_128, 77)
    assert got == want
    assert sum(h.fa for h in hs) == fa


class OracleChain:
    """file_sum_blocks_start / _wait, as volsync_amd.Matcher, over the rank's
    own host bytes with the numpy XXH3 restatement (oracle/rsync_ref.py)."""

    def __init__(self, window, data_lo):
        self.w, self.lo = window, data_lo

    def file_sum_blocks_start(self, addr, nblocks, acc):
        off = addr - self.lo   # the relay passes ptr + b_lo * 1024 - data_lo with ptr = data_lo
        self.acc = R.xxh3_acc_blocks(self.w[off:off + nblocks * 1024], acc)

    def file_sum_blocks_wait(self):
        return self.acc


def _relay_worker(rank, world, port, args, outdir):
    import torch.distributed as dist
    from volsync_amd.rsync_shard import FileSumRelay, SourceShard, torch_relay_p2p
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, bl, files = args
    g = dist.new_group(backend="gloo")           # the relay's own group (own thread)
    data = O.synth(58, 0, n)
    spec = SourceShard.for_rank(n, bl, world, rank)
    win = data[spec.data_lo:spec.data_hi].copy()  # only the rank's bytes
    fs = FileSumRelay(OracleChain(win, spec.data_lo), spec, spec.data_lo, spec.data_lo,
                      *torch_relay_p2p(rank, world, g),
                      last=lambda: win[len(win) - min(n, 1088):].tobytes(),
                      init=R.xxh3_acc_init)
    for _ in range(files):
        fs.submit()
        dist.barrier()                            # the main thread's collectives go on
    out = {"r": fs.results(), "nb": fs.nblocks}
    fs.close()
    allr = [None] * world
    dist.all_gather_object(allr, out)
    if rank == 0:
        with open(os.path.join(outdir, "relay.json"), "w") as f:
            json.dump(allr, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,args", [
    (2, ((3 << 20) + 777, 131072, 3)),
    (3, (3 << 20, 65536, 2)),          # len % 1024 == 0: the last whole block is the finish's
    (5, (700 << 10, 8192, 2)),
])
def test_file_sum_relay_gloo(world, args):
    """R7 across ranks (rsync_shard.FileSumRelay): each rank chains its own
    whole 1 KiB blocks from its predecessor's accumulators (point-to-point on
    a gloo group of the relay's own, beside the main thread's collectives),
    several files in flight; the last rank's digest is libxxhash's XXH3-128 of
    the whole file, and the ranks chain exactly (len - 1) // 1024 blocks."""
    import torch.multiprocessing as mp
    import xxhash
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_relay_worker, args=(world, _free_port(), args, d), nprocs=world,
                           join=True, start_method="spawn")
        res = json.load(open(os.path.join(d, "relay.json")))
    n, _, files = args
    data = O.synth(58, 0, n)
    want = xxhash.xxh3_128_intdigest(data.tobytes()).to_bytes(16, "little").hex()
    assert res[-1]["r"] == [want] * files
    assert sum(r["nb"] for r in res) == (n - 1) // 1024


def test_file_sum_relay_refuses_short_blocks():
    """with blength < 1024 a rank's last whole 1 KiB block can end
    past the bytes it holds (own_hi + blength - 1); the relay refuses such a
    split instead of reading past the rank's buffer."""
    from volsync_amd.rsync_shard import FileSumRelay, SourceShard
    n = 3 * (1024 * 100 + 1)          # own_hi of rank 0 = 1024 * 100 + 1: rounds up by 1023
    bl, _, _, _ = O.rsync_sizes(n)
    assert bl == 700
    spec = SourceShard.for_rank(n, bl, 3, 0)
    with pytest.raises(ValueError, match="beyond its data"):
        FileSumRelay(None, spec, 0, spec.data_lo, None, None, None,
                     init=R.xxh3_acc_init, finish=lambda *a: b"")
    # C4's blength (131072) and any blength >= 1024 always fit
    for world in (2, 3, 8):
        for r in range(world):
            sp = SourceShard.for_rank(n * 7, 1024, world, r)
            fs = FileSumRelay(OracleChain(np.zeros(1, np.uint8), 0), sp, 0, sp.data_lo,
                              None, None, None, init=R.xxh3_acc_init, finish=lambda *a: b"")
            fs.close()


@pytest.mark.timeout(60)
def test_file_sum_relay_poison_propagates():
    """a rank whose chain fails hands a poison state on, so every
    later rank's relay reports RelayAborted instead of waiting forever in
    recv(); the ranks before it are unaffected."""
    import queue
    from volsync_amd.rsync_shard import FileSumRelay, RelayAborted, SourceShard

    class Broken(OracleChain):
        def file_sum_blocks_start(self, addr, nblocks, acc):
            raise IOError("device lost")

    n, bl, world = 3 << 20, 65536, 3
    data = O.synth(59, 0, n)
    qs = [queue.Queue() for _ in range(world)]
    relays = []
    for r in range(world):
        sp = SourceShard.for_rank(n, bl, world, r)
        win = data[sp.data_lo:sp.data_hi].copy()
        fsm = (Broken if r == 1 else OracleChain)(win, sp.data_lo)
        relays.append(FileSumRelay(
            fsm, sp, sp.data_lo, sp.data_lo,
            send=(lambda acc, r=r: qs[r].put(acc)),
            recv=(lambda r=r: qs[r - 1].get(timeout=30)),
            last=lambda win=win: win[len(win) - 1088:].tobytes(),
            init=R.xxh3_acc_init, finish=lambda acc, last, ln, cs: b"x"))
    for fs in relays:
        fs.submit()
    assert len(relays[0].results()) == 1
    with pytest.raises(IOError, match="device lost"):
        relays[1].results()
    with pytest.raises(RelayAborted):
        relays[2].results()
    for fs in relays:
        fs.close()
