"""Block-range sharding of rsync's signature pass across GPUs (DESIGN.md 6;
SURVEY.md 8(e)).

The destination (basis) file of `count` blocks (generator.c sum_sizes_sqroot
on the WHOLE file length) is split by block range: rank r owns blocks
[count*r//W, count*(r+1)//W) and holds only their bytes.  Each rank computes
get_checksum1 / get_checksum2 for its own blocks -- generate_and_send_sums
restricted to the range; the short final block (remainder) falls on the last
rank -- and ONE all-gather of the per-rank sum arrays (RCCL over xGMI on the
GPUs, gloo in the CPU tests) leaves every rank with the full table, byte for
byte what a single generate_and_send_sums would have sent.  Each rank then
builds match.c's hash table locally (Matcher.load_sums_device) and runs
match_sums over its source.  That all-gather is the path's only collective.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Sequence, Tuple


@dataclass
class BlockShard:
    rank: int
    world: int
    length: int     # whole basis file length
    blength: int
    count: int      # blocks of the whole file
    b_lo: int
    b_hi: int

    @property
    def byte_lo(self) -> int:
        return self.b_lo * self.blength

    @property
    def byte_hi(self) -> int:
        return min(self.b_hi * self.blength, self.length)

    @property
    def blocks(self) -> int:
        return self.b_hi - self.b_lo

    @staticmethod
    def for_rank(length: int, blength: int, world: int, rank: int) -> "BlockShard":
        count = (length + blength - 1) // blength if length else 0
        return BlockShard(rank, world, length, blength, count,
                          count * rank // world, count * (rank + 1) // world)

    @staticmethod
    def split(length: int, blength: int, world: int) -> List["BlockShard"]:
        return [BlockShard.for_rank(length, blength, world, r) for r in range(world)]

    def max_blocks(self) -> int:
        return max(s.blocks for s in BlockShard.split(self.length, self.blength, self.world))


def gather_sums(sum1, sum2, shard: BlockShard, s2length: int,
                all_gather: Callable[[list, object], None]) -> Tuple[object, object]:
    """All-gather of every rank's (sum1[blocks] int32, sum2[blocks * s2length]
    uint8) torch tensors into the full table (same device as the inputs).
    Ranks own unequal block counts, so each contribution is padded to the
    largest; the padding is dropped when the pieces are concatenated."""
    import torch
    m = max(shard.max_blocks(), 1)
    dev = sum1.device
    # one packed byte record per rank -- [m x sum1 (4 B LE)] [m x s2length] --
    # so the table travels in ONE collective
    rec = torch.zeros(m * (4 + s2length), dtype=torch.uint8, device=dev)
    rec[: shard.blocks * 4] = sum1[: shard.blocks].contiguous().view(torch.uint8)
    rec[m * 4: m * 4 + shard.blocks * s2length] = sum2[: shard.blocks * s2length]
    g = [torch.empty_like(rec) for _ in range(shard.world)]
    all_gather(g, rec)
    parts = BlockShard.split(shard.length, shard.blength, shard.world)
    full1 = torch.cat([g[r][: s.blocks * 4] for r, s in enumerate(parts)]).view(sum1.dtype)
    full2 = torch.cat([g[r][m * 4: m * 4 + s.blocks * s2length] for r, s in enumerate(parts)])
    return full1, full2


# ---- sharded match_sums: byte-range walk with an exit stitch -----------------
#
# rsync's sender runs ONE hash_search over the whole source file
# (/root/reference/mover-rsync/source.sh:54); its greedy walk is sequential:
# the state at any offset is (offset, want_i).  The source is split by byte
# range: rank r owns the walk's visits to offsets [own_lo, own_hi) and holds
# the bytes [own_lo, own_hi + blength - 1) (a window starting below own_hi
# reads up to blength - 1 bytes past it).  Protocol, the rsync twin of the CDC
# exit stitch (volsync_amd/shard.py):
#   1. match_scan: every rank finds its weak-sum candidates and walks its
#      range speculatively from (own_lo, want_i = "no preference"; rank 0 from
#      (0, 0) exactly as hash_search starts) -- no communication;
#   2. all-gather the exit states (first offset >= own_hi, want_i); rank r's
#      true entry is rank r-1's exit; a rank whose entry changed re-walks from
#      it (match_stitch) until its walk reaches a match the speculative walk
#      also made -- from there the two are identical -- and reports its new
#      exit; repeat until no entry changes (sum all-reduce);
#   3. match_finish: each rank's matches with offsets in its range, in order.
# Concatenated in rank order they equal one hash_search over the whole file.
@dataclass
class SourceShard:
    rank: int
    world: int
    length: int     # whole source file length
    blength: int
    own_lo: int
    own_hi: int
    data_lo: int
    data_hi: int

    @staticmethod
    def for_rank(length: int, blength: int, world: int, rank: int) -> "SourceShard":
        lo = length * rank // world
        hi = length * (rank + 1) // world
        return SourceShard(rank, world, length, blength, lo, hi, lo & ~15,
                           min(hi + blength - 1, length))

    @staticmethod
    def split(length: int, blength: int, world: int) -> List["SourceShard"]:
        return [SourceShard.for_rank(length, blength, world, r) for r in range(world)]


def run_walk_shard(h, spec: SourceShard, ptr: int, allgather_pair, allreduce_sum,
                   stats: dict = None) -> int:
    """This rank's part of the sharded hash_search.  h: a Matcher with the
    table loaded (or a test double with the same match_scan / match_stitch /
    match_finish surface); ptr: device address of file offset spec.data_lo.
    allgather_pair((off, want)) -> every rank's pair; allreduce_sum(x) -> sum.
    Returns this rank's match count (h.matches(0, n))."""
    ex = h.match_scan(ptr, spec.data_hi - spec.data_lo, spec.data_lo, spec.length, spec.own_lo,
                      spec.own_hi)
    entry = None   # the speculative entry
    rounds = rewalks = 0
    for _ in range(spec.world + 2):
        gathered = allgather_pair(ex)
        rounds += 1
        want = (0, 0) if spec.rank == 0 else tuple(gathered[spec.rank - 1])
        moved = 0
        if spec.rank and want != entry:
            entry = want
            ex = h.match_stitch(*want)
            moved = 1
            rewalks += 1
        if allreduce_sum(moved) == 0:
            break
    if stats is not None:
        stats["exchange_rounds"] = rounds
        stats["rewalks"] = rewalks
    return h.match_finish()


def torch_pair_collectives(device=None):
    """(allgather_pair, allreduce_sum) over torch.distributed: RCCL on GPU
    tensors with the nccl backend, gloo on CPU tensors."""
    import torch
    import torch.distributed as dist

    def allgather_pair(p):
        t = torch.tensor([int(p[0]), int(p[1])], dtype=torch.int64, device=device)
        outs = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(outs, t)
        return [(int(o[0].item()), int(o[1].item())) for o in outs]

    def allreduce_sum(x: int):
        t = torch.tensor([x], dtype=torch.int64, device=device)
        dist.all_reduce(t)
        return int(t.item())

    return allgather_pair, allreduce_sum


def run_walk_shards_local(handles: Sequence, specs: Sequence[SourceShard], ptrs: Sequence[int]):
    """The same protocol with every rank in one process (Jacobi rounds, as the
    distributed version runs them): the concatenated match list."""
    world = len(specs)
    exits = [h.match_scan(p, s.data_hi - s.data_lo, s.data_lo, s.length, s.own_lo, s.own_hi)
             for h, s, p in zip(handles, specs, ptrs)]
    entry = [None] * world
    for _ in range(world + 2):
        gathered = list(exits)
        moved = 0
        for r in range(1, world):
            if gathered[r - 1] != entry[r]:
                entry[r] = gathered[r - 1]
                exits[r] = handles[r].match_stitch(*entry[r])
                moved += 1
        if moved == 0:
            break
    out = []
    for h in handles:
        out.extend(h.matches(0, h.match_finish()))
    return out


# ---- R7 across ranks: the whole-file XXH3 as a relay -------------------------
#
# match.c matched() streams every source byte into the file checksum
# (checksum.c sum_update), one serial XXH3 scramble chain per 1 KiB block.  A
# file split by byte range therefore relays the 64-byte accumulator state:
# rank r chains its whole blocks [b_lo, b_hi) from rank r-1's state
# (vs_rsync_file_sum_blocks_start / _wait: device contributions, host chain)
# and hands the result to rank r+1; the last rank finishes with the file's
# last min(len, 1088) bytes (vs_rsync_file_sum_finish).  The ranks together
# chain exactly (len - 1) // 1024 blocks.  The relay is serial per file
# (len / 1 KiB chain steps, ~2.1 ns each on the host), but files are
# independent, so a relay thread per rank runs file k's chain while its
# successor runs file k-1's: a systolic pipeline whose rate is one rank's
# chain per file, with a fill latency of world - 1 chains.
class RelayAborted(RuntimeError):
    """An earlier rank of the file-sum relay failed (it sent the poison state)."""


class FileSumRelay:
    """One rank's relay thread.  fsm: a Matcher (or a test double with
    file_sum_blocks_start / _wait); ptr: address of file offset data_lo in
    the rank's copy of its bytes; send(acc) / recv() -> acc move the 8 u64
    accumulators to the next rank / from the previous one (rank 0 starts
    from the initial state); last(): the file's last min(len, 1088) bytes
    (the last rank only).  submit() queues one file, results() waits for all
    queued files and returns the last rank's digests (others: the states
    they handed on).

    Failure: a rank whose chain raises hands send(None) on -- a poison state
    -- so every later rank's recv() returns None and its relay raises
    RelayAborted instead of blocking for a state that never comes."""

    def __init__(self, fsm, spec: SourceShard, ptr: int, data_lo: int, send, recv, last,
                 csum: int = 8, init=None, finish=None):
        import queue
        import threading
        nb_file = (spec.length - 1) // 1024 if spec.length else 0
        self.b_lo = min(-(-spec.own_lo // 1024), nb_file)
        self.b_hi = min(-(-spec.own_hi // 1024), nb_file)
        if spec.rank == spec.world - 1:
            self.b_hi = nb_file
        # the rank chains bytes [b_lo * 1024, b_hi * 1024), which must lie in
        # the bytes it holds: own_hi rounds up to a 1 KiB block by at most
        # 1023 bytes, and the halo is blength - 1 (so blength >= 1024 always
        # suffices; sum_sizes_sqroot gives 700 only for files <= 490000 bytes)
        if self.b_lo < self.b_hi and (self.b_lo * 1024 < spec.data_lo
                                      or self.b_hi * 1024 > spec.data_hi):
            raise ValueError(f"FileSumRelay: rank {spec.rank} would chain bytes "
                             f"[{self.b_lo * 1024}, {self.b_hi * 1024}) beyond its data "
                             f"[{spec.data_lo}, {spec.data_hi}) (blength {spec.blength} < 1024)")
        self.spec, self.fsm, self.csum = spec, fsm, csum
        self.addr = ptr + self.b_lo * 1024 - data_lo
        self.send, self.recv, self.last = send, recv, last
        if init is None or finish is None:
            from .rsync import file_sum_finish, file_sum_init
            init, finish = init or file_sum_init, finish or file_sum_finish
        self._init, self._finish = init, finish
        self._q = queue.Queue()
        self._out, self._err = [], []
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()

    @property
    def nblocks(self) -> int:
        return self.b_hi - self.b_lo

    def _run(self):
        while True:
            job = self._q.get()
            if job is None:
                return
            spec = self.spec
            try:
                acc = self._init() if spec.rank == 0 else self.recv()
                if acc is None:
                    raise RelayAborted(f"rank {spec.rank - 1} aborted the relay")
                self.fsm.file_sum_blocks_start(self.addr, self.nblocks, acc)
                acc = self.fsm.file_sum_blocks_wait()
                if spec.rank < spec.world - 1:
                    self.send(acc)
                    self._out.append("".join(f"{int(x):016x}" for x in acc))
                else:
                    self._out.append(self._finish(acc, self.last(), spec.length, self.csum).hex())
            except Exception as e:  # reported by results()
                self._err.append(e)
                if spec.rank < spec.world - 1:
                    try:
                        self.send(None)   # poison: the later ranks fail, not hang
                    except Exception as e2:  # the transport itself is gone
                        self._err.append(e2)
            finally:
                self._q.task_done()

    def submit(self) -> None:
        self._q.put(1)

    def results(self):
        self._q.join()
        if self._err:
            raise self._err[0]
        out, self._out = self._out, []
        return out

    def close(self) -> None:
        self._q.put(None)
        self._th.join()


def torch_relay_p2p(rank: int, world: int, group=None):
    """(send, recv) of the 8 accumulators to the next / from the previous rank
    over torch.distributed point-to-point on CPU tensors (a gloo group of its
    own: the relay thread runs beside the main thread's collectives).  A
    message is 9 int64: a flag (0 = state, 1 = poison) and the accumulators;
    send(None) sends the poison and recv() returns None for it."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def send(acc):
        t = torch.zeros(9, dtype=torch.int64)
        if acc is None:
            t[0] = 1
        else:
            t[1:] = torch.from_numpy(np.ascontiguousarray(acc, np.uint64).view(np.int64).copy())
        dist.send(t, dst=rank + 1, group=group)

    def recv():
        t = torch.zeros(9, dtype=torch.int64)
        dist.recv(t, src=rank - 1, group=group)
        if int(t[0]):
            return None
        return t[1:].numpy().view(np.uint64).copy()

    return send, recv
