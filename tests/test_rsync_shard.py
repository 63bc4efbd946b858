"""Multi-rank CPU tests (gloo) of the block-range sharded signature pass
(volsync_amd/rsync_shard.py): each rank computes the sums of ONLY its blocks
of the destination (C restatement, test infrastructure, standing in for the
device kernel), one all-gather assembles the table, and every rank's table --
and the match list rsync's hash_search derives from it -- must equal the
single-process generate_and_send_sums result."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import rsync_ref as R
from tests import oracle_lib as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, blength, csum, outdir):
    import torch
    import torch.distributed as dist
    from volsync_amd.rsync_shard import BlockShard, gather_sums
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bl, s2, count, rem = O.rsync_sizes(n, blength)
    sh = BlockShard.for_rank(n, bl, world, rank)
    mine = O.synth(41, sh.byte_lo, sh.byte_hi - sh.byte_lo)   # only this rank's bytes
    c1, c2 = O.rsync_signatures(mine, bl, s2, csum, 0x5EED5EED)
    assert len(c1) == sh.blocks
    t1 = torch.from_numpy(c1.view(np.int32).copy())
    t2 = torch.from_numpy(c2.reshape(-1).copy())
    f1, f2 = gather_sums(t1, t2, sh, s2, dist.all_gather)
    res = {"count": count, "sum1": f1.numpy().view(np.uint32).tolist(),
           "sum2": f2.numpy().tolist()}
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,blength,csum", [
    (2, (3 << 20) + 777, 0, R.CSUM_XXH3_128),          # sum_sizes_sqroot blength, short last block
    (3, 1 << 20, 4096, R.CSUM_MD5),                    # exact multiple, 256 blocks over 3 ranks
    (4, 5000, 700, R.CSUM_XXH64),                      # fewer blocks than 2 per rank
])
def test_sharded_signatures_gloo(world, n, blength, csum):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), n, blength, csum, d),
                           nprocs=world, join=True, start_method="spawn")
        got = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(world)]
    data = O.synth(41, 0, n)
    bl, s2, count, rem = O.rsync_sizes(n, blength)
    w1, w2 = O.rsync_signatures(data, bl, s2, csum, 0x5EED5EED)
    for g in got:
        assert g["count"] == count
        assert g["sum1"] == w1.tolist()
        assert g["sum2"] == w2.reshape(-1).tolist()
    # the match list from the gathered table equals the single-process one
    src = R.mutate(data, bl, 5)
    g1 = np.array(got[-1]["sum1"], np.uint32)
    g2 = np.array(got[-1]["sum2"], np.uint8).reshape(count, s2)
    assert O.rsync_match(src, g1, g2, bl, rem, csum, 0x5EED5EED) == \
        O.rsync_match(src, w1, w2, bl, rem, csum, 0x5EED5EED)
