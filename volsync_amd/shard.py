"""Byte-range sharding of one volume across GPUs.

Rank r owns chunk *starts* in [own_lo, own_hi) = [r*N/W, (r+1)*N/W).  It holds
the bytes [own_lo - 64, own_hi + MaxSize + 63) (clipped): a 63-byte left halo
for the fingerprint window and a MaxSize-1 right halo so that every chunk that
starts in its range can be cut and hashed locally.

Protocol (the only exchange step is an all-gather of one u64 per rank):
  1. scan: every rank fingerprints its bytes and walks its segments
     speculatively (no communication);
  2. stitch: each rank assumes its first chunk starts at own_lo and computes
     its exit (start of the first chunk at or beyond own_hi);
  3. all-gather the exits; rank r's true entry is exit[r-1]; ranks whose entry
     moved re-stitch (usually merging with their speculative path within a
     chunk or two); repeat until no entry moves (sum all-reduce);
  4. finish: each rank emits and hashes the chunks that start in its range.
Rank results concatenated in rank order equal the single-device chunk list.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence


@dataclass
class ShardSpec:
    rank: int
    world: int
    total: int
    own_lo: int
    own_hi: int
    data_lo: int
    data_hi: int

    @property
    def final(self) -> bool:
        return self.data_hi == self.total

    @staticmethod
    def for_rank(total: int, world: int, rank: int, max_size: int) -> "ShardSpec":
        lo = total * rank // world
        hi = total * (rank + 1) // world
        dlo = max(0, lo - 64) & ~15          # keep the device pointer 16-byte aligned
        dhi = min(total, hi + max_size + 63)
        return ShardSpec(rank, world, total, lo, hi, dlo, dhi)

    @staticmethod
    def split(total: int, world: int, max_size: int) -> List["ShardSpec"]:
        return [ShardSpec.for_rank(total, world, r, max_size) for r in range(world)]


class LocalComm:
    """All ranks in one process (tests): values passed as per-rank lists."""


def _scan(h, spec: ShardSpec, ptr: int) -> None:
    h.scan(ptr, spec.data_hi - spec.data_lo, spec.data_lo, spec.own_lo, spec.own_hi,
           spec.final)


def run_shards_local(handles: Sequence, specs: Sequence[ShardSpec], ptrs: Sequence[int]):
    """Run the protocol for all ranks inside one process (Jacobi rounds, exactly
    what the distributed version does), returning the concatenated chunks."""
    world = len(specs)
    for h, s, p in zip(handles, specs, ptrs):
        _scan(h, s, p)
    entry = [s.own_lo for s in specs]
    exits = [h.stitch(e)[0] for h, e in zip(handles, entry)]
    for _ in range(world + 2):
        gathered = list(exits)
        moved = 0
        for r in range(1, world):
            if gathered[r - 1] != entry[r]:
                entry[r] = gathered[r - 1]
                exits[r] = handles[r].stitch(entry[r])[0]
                moved += 1
        if moved == 0:
            break
    out = []
    for h in handles:
        n = h.finish()
        out.extend(h.chunks(0, n))
    return out


def run_shard(h, spec: ShardSpec, ptr: int, allgather_u64, allreduce_sum,
              stats: dict = None) -> int:
    """Distributed version: this rank's part.  allgather_u64(x) -> list of all
    ranks' x; allreduce_sum(x) -> sum.  Returns this rank's chunk count (read
    them with h.chunks(0, n)); stats (optional) receives the exchange rounds
    and this rank's re-stitches."""
    _scan(h, spec, ptr)
    entry = spec.own_lo
    ex = h.stitch(entry)[0]
    rounds = restitches = 0
    for _ in range(spec.world + 2):
        gathered = allgather_u64(ex)
        rounds += 1
        want = spec.own_lo if spec.rank == 0 else int(gathered[spec.rank - 1])
        moved = 0
        if want != entry:
            entry = want
            ex = h.stitch(entry)[0]
            moved = 1
            restitches += 1
        if allreduce_sum(moved) == 0:
            break
    if stats is not None:
        stats["exchange_rounds"] = rounds
        stats["restitches"] = restitches
    return h.finish()


def torch_collectives(device=None):
    """(allgather_u64, allreduce_sum) over torch.distributed (RCCL on GPU
    tensors with the nccl backend; gloo on CPU tensors)."""
    import torch
    import torch.distributed as dist

    def allgather_u64(x: int):
        t = torch.tensor([x], dtype=torch.int64, device=device)
        outs = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(outs, t)
        return [int(o.item()) & 0xFFFFFFFFFFFFFFFF for o in outs]

    def allreduce_sum(x: int):
        t = torch.tensor([x], dtype=torch.int64, device=device)
        dist.all_reduce(t)
        return int(t.item())

    return allgather_u64, allreduce_sum
