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
from typing import Callable, List, Tuple


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
