"""Child process of tests/test_gpu_rccl.py: the multi-GPU protocols of
volsync_amd.shard and volsync_amd.rsync_shard with their collectives on RCCL
("nccl" process group, device tensors), at world size 1 -- the one GPU a test
box has.  Every all-gather / all-reduce below is a real RCCL call on cuda:0;
at world 1 they move one rank's data, which checks the communicator set-up,
the device-tensor operands and the protocols' use of the results, not the
xGMI exchange itself (that is the driver's 8-GPU scaling run).

Results are checked against the C oracle (test infrastructure) and printed as
one JSON line; exit status 0 only when every check holds.
"""
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def to_dev(arr):
    import torch
    t = torch.empty(max(len(arr), 16), dtype=torch.uint8, device="cuda")
    if len(arr):
        t[: len(arr)].copy_(torch.from_numpy(np.ascontiguousarray(arr)))
    torch.cuda.synchronize()
    return t


def main() -> int:
    import torch
    import torch.distributed as dist
    from oracle import cdc_ref as P
    from oracle import rsync_ref as R
    from tests import oracle_lib as O

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}

    # 1. CDC byte-range shard (A3-A5 + exit exchange) over RCCL
    from volsync_amd import DeviceChunker
    from volsync_amd.shard import ShardSpec, run_shard, torch_collectives
    n, mn, mx, ab = 24 << 20, 16384, 1 << 20, 14
    data = O.synth(61, 0, n)
    spec = ShardSpec.split(n, 1, mx)[0]
    buf = to_dev(data[spec.data_lo:spec.data_hi])
    h = DeviceChunker(P.TEST_POL, mn, mx, ab)
    stats = {}
    cnt = run_shard(h, spec, buf.data_ptr(), *torch_collectives(dev), stats=stats)
    got = [(c.Start, c.Length, c.Cut, c.ID.hex()) for c in h.chunks(0, cnt)]
    h.close()
    res["cdc_chunks"] = len(got)
    res["cdc_exact"] = got == O.cdc_hash(data, P.TEST_POL, mn, mx, ab)
    res["cdc_rounds"] = stats.get("exchange_rounds")

    # 2. block-sharded signatures, assembled by an RCCL all-gather of device tensors
    from volsync_amd import Matcher, sum_sizes_sqroot
    from volsync_amd.rsync_shard import (BlockShard, SourceShard, gather_sums, run_walk_shard,
                                         torch_pair_collectives)
    csum, seed = R.CSUM_XXH3_128, 0x5EED5EED
    nb = (6 << 20) + 333
    basis = O.synth(62, 0, nb)
    hdr = sum_sizes_sqroot(nb, 0)
    sh = BlockShard.split(nb, hdr.blength, 1)[0]
    db = to_dev(basis[sh.byte_lo:sh.byte_hi])
    s1 = torch.zeros(max(sh.blocks, 1), dtype=torch.int32, device=dev)
    s2 = torch.zeros(max(sh.blocks, 1) * hdr.s2length, dtype=torch.uint8, device=dev)
    m = Matcher()
    m.signatures_device(db.data_ptr(), sh.byte_hi - sh.byte_lo, hdr.blength, hdr.s2length,
                        csum, seed, s1.data_ptr(), s2.data_ptr())
    torch.cuda.synchronize()
    f1, f2 = gather_sums(s1, s2, sh, hdr.s2length, dist.all_gather)
    c1, c2 = O.rsync_signatures(basis, hdr.blength, hdr.s2length, csum, seed)
    res["sums_exact"] = bool((f1.cpu().numpy().view(np.uint32) == c1).all()
                             and (f2.cpu().numpy().reshape(-1, hdr.s2length) == c2).all())
    m.close()

    # 3. byte-range sharded hash_search with the (offset, want_i) exchange on RCCL
    src = R.mutate(basis, hdr.blength, seed=12)
    want, want_fa = O.rsync_match(src, c1, c2, hdr.blength, hdr.remainder, csum, seed)
    from volsync_amd import SumStruct
    sums = SumStruct(nb, hdr.count, hdr.blength, hdr.s2length, hdr.remainder, c1, c2)
    sp = SourceShard.split(len(src), hdr.blength, 1)[0]
    m = Matcher()
    m.load_sums(sums, csum, seed)
    ds = to_dev(src[sp.data_lo:sp.data_hi])
    stats = {}
    cnt = run_walk_shard(m, sp, ds.data_ptr(), *torch_pair_collectives(dev), stats=stats)
    got = m.matches(0, cnt)
    fa = m.stats()["false_alarms"]
    m.close()
    res["walk_matches"] = len(got)
    res["walk_exact"] = got == want and fa == want_fa
    res["walk_rounds"] = stats.get("exchange_rounds")

    # 4. a 256 MiB device all-gather and all-reduce (the C3 sum-table size class)
    big = torch.arange(64 << 20, dtype=torch.int32, device=dev)
    outs = [torch.empty_like(big)]
    dist.all_gather(outs, big)
    red = big[:1 << 20].clone()
    dist.all_reduce(red)
    torch.cuda.synchronize()
    res["collective_exact"] = bool(torch.equal(outs[0], big) and torch.equal(red, big[:1 << 20]))

    dist.destroy_process_group()
    ok = all(res[k] for k in ("cdc_exact", "sums_exact", "walk_exact", "collective_exact"))
    res["ok"] = ok
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
