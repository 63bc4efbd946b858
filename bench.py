"""bench.py -- restic CDC + SHA-256 blob IDs on MI355X (BASELINE.json metric).

python bench.py --gpus N --steps K --warmup W
  N=1: config C2 -- one 64 GiB synthetic volume image (seed 2), device-resident,
       restic chunker (testPol, 512 KiB / 8 MiB, 20 bits) + SHA-256 blob IDs.
  N>1: launched by torch.distributed.run, one rank per GPU: one volume of
       N x 128 GiB (C3's per-GPU share; seed 3, so N=8 is C3's 1 TiB) byte-range
       sharded across the ranks (weak scaling, per-GPU work fixed); the only
       exchange is an RCCL all-gather of one u64 per rank per stitch round
       (volsync_amd/shard.py).
A step = one full pass of the hot path over the volume: fingerprint, cut
selection, Cut values, SHA-256 of every chunk.  Steps are pipelined: the
time-sliced SHA-256 engine keeps hashing step k's chunks while step k+1 is
chunked, and the timed region ends only after the engine has drained, so every
blob ID of all K volumes is final inside it.  Inputs are
generated in HBM before the timed region.  Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
# Integer VALU issue peak, measured (tools/valu/valu_peak.hip ->
# profiles/r02_valu_peak; in-kernel s_memtime / s_memrealtime stamps separate
# the clock from the issue rate): the three-source integer instructions
# SHA-256 and the fingerprint are made of (v_alignbit, v_bitop3, v_add3,
# v_perm, v_lshl_or) issue once per 4.2 shader cycles per SIMD at 8 waves,
# at the measured clock; two-source integer ops (VOP2 or _e64) and v_fma_f32
# reach ~2.35.  Priced at 2.4 GHz (above the measured 2.17-2.39 GHz, so the
# fraction is not flattered): 256 CU x 4 SIMD x 64 lanes x 2.4 GHz / 4.2.
VALU_PEAK_TOPS = 256 * 4 * 64 * 2.4e9 / 4.2 / 1e12   # 37.4 T lane-ops/s
# VALU lane-instructions per input byte, from SQ_INSTS_VALU (wave-instructions)
# x 64 / bytes in profiles/r01_final: SHA-256 ~1490 per 64-byte block, the
# fingerprint ~8.8 per byte
SHA_OPS_PER_BYTE = 1490 / 64
FP_OPS_PER_BYTE = 8.8
# Mix-weighted issue cost: the hot loops' VALU
# instructions priced by issue class (tools/isa_mix.py over the gfx950 ISA,
# profiles/r05_isa): SHA-256's split engine, consumer rounds (905 VALU,
# 3181.6 cycles per 64-chain block) + producer schedule (781, 2560.1) -> 3.41
# cycles per instruction; the fingerprint's Fast53 strip loop (2228, 6773.6
# per 256 chain-bytes) -> 3.04.  valu_frac = lane-ops/s x that cost over
# 256 CU x 4 SIMD x 64 lanes x 2.4 GHz: the fraction of the issue floor.
SHA_MIX_CYC = (3181.6 + 2560.1) / (905 + 781)
FP_MIX_CYC = 6773.6 / 2228
ISSUE_LANE_CYC = 256 * 4 * 64 * 2.4e9 / 1e12   # T lane-cycles/s


def valu_frac(gbs: float, ops_per_byte: float, cyc: float) -> float:
    """Fraction of the VALU issue floor used at gbs GB/s (mix-weighted)."""
    return round(gbs * ops_per_byte / 1e3 * cyc / ISSUE_LANE_CYC, 4)


def host_threads() -> int:
    """The logical CPUs this process may run on (its affinity mask: the GPU
    box's whole host, nproc)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def _cpu_quota():
    """The cgroup CPU quota in CPUs (cpu.max), or None when unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(sample_bytes: int, threads: int):
    """Oracle port (oracle/cdc_ref.c) timed restic-style on the host (SURVEY.md
    8(d) CPU baseline): (i) the chunker on 1 thread, (ii) SHA-256 of the chunk
    list (OpenSSL, SHA-NI when present) on 1 thread and on `threads` threads,
    (iii) restic's archiver shape -- 1 chunker thread + (threads - 1) SHA-256
    threads -- which is `value`."""
    import numpy as np
    from tests import oracle_lib as O
    data = O.synth(2, 0, sample_bytes)
    t0 = time.perf_counter()
    ch = O.cdc_hash(data, 0x3DA3358B4DC173, 512 << 10, 8 << 20, 20, n_hash=threads - 1)
    dt = time.perf_counter() - t0
    # (i) the chunker alone on one core (what restic does per file)
    t1 = time.perf_counter()
    O.chunk_all(data, 0x3DA3358B4DC173, 512 << 10, 8 << 20, 20)
    dt_chunk = time.perf_counter() - t1
    # (ii) SHA-256 over the chunk list: 1 thread, all threads
    off = np.array([c[0] for c in ch], np.uint64)
    ln = np.array([c[1] for c in ch], np.uint64)
    t2 = time.perf_counter()
    ids1, _ = O.sha256_list(data, off, ln, 1)
    dt_sha1 = time.perf_counter() - t2
    t3 = time.perf_counter()
    idsn, ran = O.sha256_list(data, off, ln, threads)
    dt_shan = time.perf_counter() - t3
    ok = bytes(ids1.ravel()) == bytes(idsn.ravel()) == b"".join(bytes.fromhex(c[3]) for c in ch)
    return {
        "value": round(sample_bytes / dt / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample_bytes >> 30} GiB of the C2 stream (seed 2), {len(ch)} chunks; "
                  f"value = 1 chunker thread + {threads - 1} SHA-256 threads (OpenSSL="
                  f"{bool(O.lib().ref_have_openssl())}), restic's archiver shape",
        "legs_GBps": {"chunker_1_thread": round(sample_bytes / dt_chunk / 1e9, 3),
                      "sha256_1_thread": round(sample_bytes / dt_sha1 / 1e9, 3),
                      f"sha256_{ran}_threads": round(sample_bytes / dt_shan / 1e9, 3),
                      "ids_agree": ok},
        "cpu": _cpu_model(),
        "nproc": os.cpu_count(),   # the host's logical CPUs
        "affinity_cpus": host_threads(),
        "cgroup_cpu_quota": _cpu_quota(),
    }


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def rsync_cpu_baseline(sample_bytes: int):
    """rsync's sender restated in C (oracle/rsync_ref.c: signatures +
    build_hash_table + hash_search with libxxhash), one thread as rsync runs,
    on a bounded C4-shaped pair of the same generator."""
    import numpy as np
    from oracle import rsync_ref as R
    from tests import oracle_lib as O
    d = O.synth(4, 0, sample_bytes)
    bl, s2, _, rem = O.rsync_sizes(sample_bytes)
    src = R.mutate(d, bl, 5)
    t0 = time.perf_counter()
    c1, c2 = O.rsync_signatures(d, bl, s2, R.CSUM_XXH3_128, 0x5EED5EED)
    t1 = time.perf_counter()
    m, _ = O.rsync_match(src, c1, c2, bl, rem, R.CSUM_XXH3_128, 0x5EED5EED)
    t2 = time.perf_counter()
    del np
    return {"value": round((len(d) + len(src)) / (t2 - t0) / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": f"{sample_bytes >> 20} MiB destination (seed 4) + C4-mutated source (seed 5), "
                      f"blength {bl}, xxh128; signatures {t1 - t0:.2f} s, match {t2 - t1:.2f} s, "
                      f"{len(m)} matches",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}



def dist_setup():
    """(world, rank, local device index, torch device) of this rank, with the
    process group up when world > 1: one GPU per rank over RCCL ("nccl").
    VSGPU_BENCH_SHARED_GPU=1 is the one-GPU rehearsal of the N-rank device
    path: every rank on cuda:0, collectives over gloo (each rank's buffers
    must then fit beside the others': use a small --per-gpu-gib)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    shared = os.environ.get("VSGPU_BENCH_SHARED_GPU") == "1"
    local = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    return world, rank, local, dev


def coll_device(dev):
    """Where collective operands live: the GPU under RCCL, the host under
    gloo (the VSGPU_BENCH_SHARED_GPU rehearsal)."""
    import torch.distributed as dist
    return dev if dist.get_backend() == "nccl" else None


def all_gather_any(outs, t):
    """dist.all_gather of a device tensor under either backend (gloo: staged
    through host memory)."""
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return dist.all_gather(outs, t)
    host = [o.cpu() for o in outs]
    dist.all_gather(host, t.cpu())
    for o, h in zip(outs, host):
        o.copy_(h)

class C4Plan:
    """The C4 source file S as a function of the destination D: D (synthetic
    stream, seed 4) with `frac` of its blocks edited (seed 5) -- a third each
    overwrite a 4 KiB run inside the block, insert 1-64 bytes, delete 1-64
    bytes (shifting everything after) -- as a list of segments of S, each a
    copy of D or literal bytes (synthetic stream seed 6, 4 KiB apart per
    edit).  Any byte range of S can be generated from it on any rank
    (fill_device), so S is ONE file, sharded by byte range, with no rank
    holding more than its own range plus halo."""

    D_SEED, LIT_SEED = 4, 6

    def __init__(self, dlen: int, blength: int, seed: int = 5, frac: float = 0.10,
                 run: int = 4096):
        import numpy as np
        rng = np.random.default_rng(seed)
        count = (dlen + blength - 1) // blength
        full = dlen // blength
        nedit = min(int(round(count * frac)), full)
        blocks = np.sort(rng.choice(full, size=nedit, replace=False)).astype(np.int64)
        kind = rng.integers(0, 3, nedit)
        at = blocks * blength + rng.integers(0, max(1, blength - run), nedit)
        ilen = rng.integers(1, 65, nedit)
        dl = rng.integers(1, 65, nedit)
        lit = np.where(kind == 0, run, np.where(kind == 1, ilen, 0)).astype(np.int64)
        skip = np.where(kind == 0, run, np.where(kind == 2, dl, 0)).astype(np.int64)
        resume = at + skip                        # D offset after edit e
        dstart = np.concatenate([[0], resume])    # D pieces: [dstart[e], at[e]) then the tail
        dend = np.concatenate([at, [dlen]])
        dlenp = np.maximum(dend - dstart, 0)
        # interleave: D piece e, literal e, ..., D tail
        n = 2 * nedit + 1
        length = np.zeros(n, np.int64)
        kindv = np.zeros(n, np.int8)               # 0 = copy of D, 1 = literal
        srcoff = np.zeros(n, np.int64)
        length[0::2] = dlenp
        srcoff[0::2] = dstart
        length[1::2] = lit
        kindv[1::2] = 1
        srcoff[1::2] = np.arange(nedit, dtype=np.int64) * run
        keep = length > 0
        self.length, self.kind, self.srcoff = length[keep], kindv[keep], srcoff[keep]
        self.start = np.concatenate([[0], np.cumsum(self.length)[:-1]]).astype(np.int64)
        self.total = int(self.length.sum())
        self.dlen, self.blength, self.edits = dlen, blength, nedit

    def segments(self, lo: int, hi: int):
        """(dest offset - lo, seed, stream offset, n) pieces covering S[lo, hi)."""
        import numpy as np
        i = max(0, int(np.searchsorted(self.start, lo, side="right")) - 1)
        out = []
        while i < len(self.start) and self.start[i] < hi:
            s0, n0 = int(self.start[i]), int(self.length[i])
            a, b = max(lo, s0), min(hi, s0 + n0)
            if b > a:
                seed = self.LIT_SEED if self.kind[i] else self.D_SEED
                out.append((a - lo, seed, int(self.srcoff[i]) + (a - s0), b - a))
            i += 1
        return out

    def fill_device(self, dev_ptr: int, lo: int, hi: int, device: int = 0, stream=None) -> None:
        from volsync_amd import synth_fill_device
        for d, seed, off, n in self.segments(lo, hi):
            synth_fill_device(dev_ptr + d, seed, off, n, device=device, stream=stream)


def rsync_main(args):
    """C4: destination D (seed 4) and source S = D with 10 % of its blocks
    edited (C4Plan), both device-resident, D and S each ONE file sharded
    across the ranks.  A step = generate_and_send_sums over D (each rank its
    block range: weak + XXH3-128 per block) + one RCCL all-gather of the sum
    table (N > 1) + build_hash_table + match_sums over S: each rank scans its
    byte range of S, walks it speculatively, and the walks are stitched by an
    all-gather of exit states (volsync_amd/rsync_shard.py run_walk_shard), so
    the concatenated match list is exactly ONE hash_search over S.
    value = (|D| + |S|) per second over all ranks."""
    import torch
    import torch.distributed as dist
    from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device
    from volsync_amd.rsync import CSUM_MD5, CSUM_XXH3_64, CSUM_XXH3_128, CSUM_XXH64
    CSUM = {"xxh128": CSUM_XXH3_128, "xxh3": CSUM_XXH3_64, "xxh64": CSUM_XXH64,
            "md5": CSUM_MD5}[args.csum]
    from volsync_amd.rsync_shard import (BlockShard, SourceShard, gather_sums, run_walk_shard,
                                         torch_pair_collectives)

    world, rank, local, dev = dist_setup()
    per = int(args.per_gpu_gib * (1 << 30))
    # --share R/N (one process, one GPU): rank R's work of the N-rank C4 --
    # its block range of D, the FULL table (every rank's sums, computed before
    # the timed region as the all-gather would deliver them) and its byte range
    # of S, re-walked once from rank R-1's speculative exit as round 1 of the
    # exit exchange does.  Only the two small collectives are absent.
    share = None
    if args.share:
        share = tuple(int(x) for x in args.share.split("/"))
        assert world == 1 and len(share) == 2 and 0 <= share[0] < share[1], args.share
    sw, sr = (share[1], share[0]) if share else (world, rank)
    dtotal = per * sw
    hdr = sum_sizes_sqroot(dtotal)
    shard = BlockShard.for_rank(dtotal, hdr.blength, sw, sr)
    n = shard.byte_hi - shard.byte_lo
    stream = torch.cuda.current_stream(dev).cuda_stream
    parts = BlockShard.split(dtotal, hdr.blength, sw)
    db = torch.empty(max(max(p.byte_hi - p.byte_lo for p in parts), 16), dtype=torch.uint8,
                     device=dev)
    plan = C4Plan(dtotal, hdr.blength)
    sspec = SourceShard.for_rank(plan.total, hdr.blength, sw, sr)
    prev = SourceShard.for_rank(plan.total, hdr.blength, sw, sr - 1) if share and sr else None
    ds = torch.empty(max(sspec.data_hi - sspec.data_lo,
                         prev.data_hi - prev.data_lo if prev else 0, 16),
                     dtype=torch.uint8, device=dev)
    s1 = torch.zeros(max(shard.blocks, 1), dtype=torch.int32, device=dev)
    s2 = torch.zeros(max(shard.blocks, 1) * hdr.s2length, dtype=torch.uint8, device=dev)
    m = Matcher(local)
    m.set_stream(stream)
    if args.walk_opt:
        # A/B: --walk-opt NAME=V[,NAME=V] (volsync_amd._lib VS_OPT_* without the prefix)
        from volsync_amd import _lib
        for kv in args.walk_opt.split(","):
            k, v = kv.split("=")
            m.set_option(getattr(_lib, "VS_OPT_" + k.upper()), int(v))
    seed = 0x5EED5EED
    full1 = full2 = None
    share_entry = None
    if share:
        # the table the all-gather would assemble: every rank's block range of
        # D generated and signed in turn (untimed)
        full1 = torch.zeros(hdr.count, dtype=torch.int32, device=dev)
        full2 = torch.zeros(hdr.count * hdr.s2length, dtype=torch.uint8, device=dev)
        for p in parts:
            synth_fill_device(db.data_ptr(), C4Plan.D_SEED, p.byte_lo, p.byte_hi - p.byte_lo,
                              device=local, stream=stream)
            m.signatures_device(db.data_ptr(), p.byte_hi - p.byte_lo, hdr.blength, hdr.s2length,
                                CSUM, seed, full1[p.b_lo:].data_ptr(),
                                full2[p.b_lo * hdr.s2length:].data_ptr())
        torch.cuda.synchronize(dev)
        if prev is not None:
            # rank R-1's speculative exit: the entry round 1 hands rank R
            plan.fill_device(ds.data_ptr(), prev.data_lo, prev.data_hi, device=local,
                             stream=stream)
            m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder,
                               full1.data_ptr(), full2.data_ptr(), CSUM, seed)
            share_entry = m.match_scan(ds.data_ptr(), prev.data_hi - prev.data_lo, prev.data_lo,
                                       prev.length, prev.own_lo, prev.own_hi)
            m.match_finish()
    synth_fill_device(db.data_ptr(), C4Plan.D_SEED, shard.byte_lo, n, device=local, stream=stream)
    plan.fill_device(ds.data_ptr(), sspec.data_lo, sspec.data_hi, device=local, stream=stream)
    torch.cuda.synchronize(dev)
    coll = torch_pair_collectives(coll_device(dev)) if world > 1 else (lambda p: [p], lambda x: x)
    xst = {}
    # R7 inside the step (checksum.c sum_update over S, xxh128 unseeded as
    # sum_init): device contributions + a host scramble chain on its own
    # handle.  The chain is one serial dependency per KiB of
    # the file, so file k's chain runs beside file k+1's step (two jobs in
    # flight -- --file-sum-jobs, each on its own host thread) and the timed region ends when the
    # last one is done.  One GPU: the whole file S.  --share: the rank's whole
    # 1 KiB blocks of S from a stand-in relay state (the value rank R-1 would
    # hand over; the chain's cost does not depend on it).
    fsm = Matcher(local)
    fsm.set_stream(stream)
    nb_file = (plan.total - 1) // 1024
    fs_blocks = None
    if share:
        b_lo = min(-(-sspec.own_lo // 1024), nb_file)
        b_hi = min(-(-sspec.own_hi // 1024), nb_file)
        fs_blocks = (ds.data_ptr() + b_lo * 1024 - sspec.data_lo, b_hi - b_lo)
    # R7 across ranks relays the XXH3 accumulators; an MD5 / XXH64 file sum
    # is one host chain over the whole file (not relayed here)
    fs_on = not args.no_file_sum and (world == 1 or share or args.csum in ("xxh128", "xxh3"))
    fs_out = []
    fs_inflight = [0]
    relay = None
    if fs_on and world > 1 and not share:
        # N ranks: the XXH3 state relayed rank to rank (rsync_shard.FileSumRelay)
        # over a gloo group of its own, one relay thread per rank; files
        # (steps) pipeline through the ranks, so the rate is one rank's chain
        # per step once the pipeline is full
        from volsync_amd.rsync_shard import FileSumRelay, torch_relay_p2p
        rg = dist.new_group(backend="gloo")
        tail_n = min(plan.total, 1088)
        relay = FileSumRelay(
            fsm, sspec, ds.data_ptr(), sspec.data_lo, *torch_relay_p2p(rank, world, rg),
            last=lambda: ds[plan.total - tail_n - sspec.data_lo:plan.total - sspec.data_lo]
            .cpu().numpy().tobytes())

    def fs_start():
        if not fs_on:
            return
        if relay is not None:
            relay.submit()
            fs_inflight[0] += 1
            return
        if fs_inflight[0] == args.file_sum_jobs:
            fs_wait()
        if fs_blocks is None:
            fsm.file_sum_start(ds.data_ptr(), plan.total, CSUM)
        else:
            fsm.file_sum_blocks_start(fs_blocks[0], fs_blocks[1], None)
        fs_inflight[0] += 1

    def fs_wait():
        if relay is not None:
            for r in relay.results():
                fs_out.append((r, fsm.file_sum_timing()))
            fs_inflight[0] = 0
            return
        r = fsm.file_sum_wait() if fs_blocks is None else fsm.file_sum_blocks_wait()
        fs_inflight[0] -= 1
        fs_out.append((r.hex() if isinstance(r, bytes) else
                       "".join(f"{int(x):016x}" for x in r), fsm.file_sum_timing()))

    def step():
        fs_start()
        m.signatures_device(db.data_ptr(), n, hdr.blength, hdr.s2length, CSUM, seed,
                            s1.data_ptr(), s2.data_ptr())
        f1, f2 = s1, s2
        if share:
            f1, f2 = full1, full2
        elif world > 1:
            f1, f2 = gather_sums(s1, s2, shard, hdr.s2length, all_gather_any)
        m.load_sums_device(hdr.count, hdr.blength, hdr.s2length, hdr.remainder, f1.data_ptr(),
                           f2.data_ptr(), CSUM, seed)
        if share:
            m.match_scan(ds.data_ptr(), sspec.data_hi - sspec.data_lo, sspec.data_lo,
                         sspec.length, sspec.own_lo, sspec.own_hi)
            if share_entry is not None:
                m.match_stitch(*share_entry)
                xst["exchange_rounds"] = 1
            return m.match_finish()
        return run_walk_shard(m, sspec, ds.data_ptr(), *coll, stats=xst)

    for _ in range(args.warmup):
        step()
    while fs_inflight[0]:
        fs_wait()
    fs_out.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    m.kernel_time(reset=True)
    t0 = time.perf_counter()
    nm = 0
    stages = dict.fromkeys(["signatures", "table", "scan", "verify", "walk"], 0.0)
    for _ in range(args.steps):
        nm = step()
        for k, v in m.timing().items():
            stages[k] += v
    t_gpu = time.perf_counter()
    while fs_inflight[0]:
        fs_wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kt = m.kernel_time()
    st = m.stats()
    # exactness evidence: the last step's match list as vs_match records
    # (SHA-256, tests/golden/make_golden_full.py), gathered in rank order
    import hashlib
    recs = _match_records(m, nm)
    mine_fa = st["false_alarms"]
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([nm, mine_fa], dtype=torch.int64, device=coll_device(dev))
        dist.all_reduce(c)
        nm, tot_fa = int(c[0].item()), int(c[1].item())
        parts = [None] * world if rank == 0 else None
        dist.gather_object(recs, parts, dst=0)
        digest = hashlib.sha256(b"".join(parts)).hexdigest() if rank == 0 else None
    else:
        tot_fa = mine_fa
        digest = hashlib.sha256(recs).hexdigest()
    exact = {"matches": nm, "false_alarms": tot_fa, "digest": digest}
    g = _golden_rsync(dtotal) if args.csum == "xxh128" else None
    if share:
        gr = (g or {}).get("ranks", {}).get(str(sw))
        exact = {"matches_rank": st["matches"], "false_alarms_rank": mine_fa,
                 "digest_rank": digest}
        if gr:
            want = gr[sr]
            exact["golden_entry"] = want["entry"]
            exact["golden_match"] = (want["matches"], want["false_alarms"], want["digest"]) == \
                (st["matches"], mine_fa, digest)
    elif g:
        exact["golden_match"] = (g["matches"], g["false_alarms"], g["digest"]) == \
            (nm, tot_fa, digest)
    own_src = sspec.own_hi - sspec.own_lo
    # a --share line counts the rank's own bytes: its D blocks and S range
    value = ((n + own_src) if share else (dtotal + plan.total)) * args.steps / dt / 1e9
    fsum = None
    if fs_on:
        # the same checksum alone, after the timed region: its latency (the
        # whole relay through every rank when N > 1)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        fs_start()
        fs_wait()
        fs_dt = time.perf_counter() - t1
        digests = {d for d, _ in fs_out}
        tm = fs_out[-1][1]
        fbytes = (plan.total if fs_blocks is None and relay is None else
                  relay.nblocks * 1024 if relay is not None else fs_blocks[1] * 1024)
        digest = sorted(digests)[0]
        if relay is not None:
            # the file's digest comes out of the last rank
            allv = [None] * world
            dist.all_gather_object(allv, (digest, len(digests), relay.nblocks))
            digest, ndig = allv[-1][0], allv[-1][1]
            digests = set([digest]) if ndig == 1 else set(range(ndig))
            chained = sum(v[2] for v in allv)
            relay.close()
        fsum = {"inside_step": True,
                "jobs_in_flight": args.file_sum_jobs if relay is None else "relay pipeline",
                "ms_alone": round(fs_dt * 1e3, 2), "GBps_alone": round(fbytes / fs_dt / 1e9, 2),
                "contrib_kernel_ms": round(tm["device_ms"], 2),
                "host_chain_ms": round(tm["host_chain_ms"], 2),
                "host_chain_ns_per_KiB": round(tm["host_chain_ms"] * 1e6 / max(fbytes / 1024, 1), 3),
                "gpu_steps_done_ms_per_step": round((t_gpu - t0) / args.steps * 1e3, 3),
                "bytes": fbytes, "csum": f"{args.csum} (unseeded, as sum_init)",
                "scope": ("whole file S" if fs_blocks is None and relay is None else
                          f"whole file S, relayed over {world} ranks ({chained} blocks chained; "
                          f"this rank's chain: {fbytes} B)" if relay is not None else
                          f"the rank's {fs_blocks[1]} whole 1 KiB blocks of S from a stand-in "
                          f"relay state: the steady state of the relay pipeline, whose predecessor "
                          f"states arrive once per step; the pipeline's fill latency (N - 1 "
                          f"chains) is not included"),
                "digest" if fs_blocks is None else "state_out": digest,
                "identical_every_step": len(digests) == 1}
        g = _golden_rsync(dtotal) if args.csum == "xxh128" else None
        if g and "file_sum" in g and fs_blocks is None:
            fsum["golden_match"] = digest == g["file_sum"]
    # the dominant kernel: rs_walk_spec_kernel, one launch per step over the
    # rank's whole source range (algorithmic bytes = those source bytes, each
    # read once by the walk: a window hash where it matches, the rolling scan
    # elsewhere); the stitch passes are reported beside it
    scan_ms, scan_n = kt["scan"]
    scan_gbs = own_src / (scan_ms / scan_n) / 1e6 if scan_n else 0.0
    sti_ms, sti_n = kt["stitch"]
    sig_ms, sig_n = kt["signatures"]
    ver_ms, ver_n = kt["verify"]
    if rank == 0:
        out = {
            "metric": "GB/s rsync delta match (|D|+|S|)",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 destination + C4 edits, device-resident)",
            "config": {"workload": f"C4-shape: {dtotal >> 30} GiB destination vs 10%-edited "
                                   f"source ({plan.edits} edits), "
                                   + (f"rank {sr} of {sw}: its {n >> 30} GiB of D, the full "
                                      f"{hdr.count}-block table, its {own_src >> 30} GiB of S "
                                      f"(one GPU; value = its own bytes per second; the sum "
                                      f"all-gather and exit exchange not included)" if share else
                                      f"D block-range and S byte-range sharded x{world} "
                                      f"({per >> 30} GiB of D per GPU; sums all-gathered, walks "
                                      f"stitched over RCCL)" if world > 1 else "1 GPU"),
                       "blength": hdr.blength, "s2length": hdr.s2length, "count": hdr.count,
                       "source_bytes": plan.total, "csum": args.csum, "checksum_seed": hex(seed),
                       "matches": nm},
            "roofline": {"bound": "hbm", "achieved": round(scan_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(scan_gbs / HBM_PEAK_GBS, 4),
                         "traffic": None,
                         "kernel": "rs_walk_spec_kernel (device hash_search, speculative pass)",
                         "avg_launch_ms": round(scan_ms / scan_n, 3) if scan_n else None,
                         "launches": scan_n},
            "kernels_ms_per_step": {"walk_spec": round(scan_ms / args.steps, 3),
                                    "walk_stitch": round(sti_ms / args.steps, 3),
                                    "stitch_launches_per_step": round(sti_n / args.steps, 2),
                                    "verify": round(ver_ms / args.steps, 3),
                                    "signatures": round(sig_ms / args.steps, 3)},
            "signatures_GBps": round(n / (sig_ms / sig_n) / 1e6, 1) if sig_n else None,
            "stages_ms_per_step": {k: round(v / args.steps, 3) for k, v in stages.items()},
            "match_stats": st,
            "rccl_world_size": dist.get_world_size() if world > 1 else 1,
            "dist_backend": dist.get_backend() if world > 1 else None,
            "exchange_rounds_last_step": xst.get("exchange_rounds", 0),
            "file_sum": fsum,
            "exact": exact,
        }
        try:
            tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
            r = tj["rs_walk_spec_share" if share else "rs_walk_spec"]
            out["roofline"]["traffic"] = round(r["bytes_per_source_byte"] * own_src)
            out["roofline"]["traffic_source"] = r["source"]
        except (OSError, ValueError, KeyError):
            pass
        if world == 1 and not args.no_cpu_baseline and not share:
            out["cpu_baseline"] = rsync_cpu_baseline(args.cpu_sample_gib << 28)
        print(json.dumps(out), flush=True)
    m.close()
    fsm.close()
    if world > 1:
        dist.destroy_process_group()


def smallfiles_cpu_baseline(sizes, sample_files: int, threads: int):
    """Go crypto/sha256 stand-in on the host: OpenSSL SHA-256 (SHA-NI) per
    file over `threads` threads (oracle ref_sha256_list, C pthreads: restic's
    NumCPU BlobSaver goroutines), over the first `sample_files` files of the
    C5 size distribution laid out back to back in a 4 GiB synthetic buffer
    (wrapping), so the hashed bytes stream from DRAM as a packed batch would."""
    import numpy as np
    from tests import oracle_lib as O
    sz = np.asarray(sizes[:sample_files], np.uint64)
    span = 4 << 30
    buf = O.synth(6, 0, span)
    off = (np.concatenate([[0], np.cumsum(sz)[:-1]]) % np.uint64(span - (1 << 17))).astype(np.uint64)
    O.sha256_list(buf, off[:1000], sz[:1000], threads)   # warm the pages and threads
    best, ran = None, threads
    for _ in range(3):
        t0 = time.perf_counter()
        _, ran = O.sha256_list(buf, off, sz, threads)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    t1 = time.perf_counter()
    O.sha256_list(buf, off[: len(sz) // 16], sz[: len(sz) // 16], 1)
    dt1 = time.perf_counter() - t1
    return {"value": round(float(sz.sum()) / best / 1e9, 3), "unit": "GB/s", "cores": ran,
            "kind": "port", "sample": f"{len(sz)} files ({float(sz.sum()) / 2**30:.2f} GiB) of the "
            f"C5 size distribution packed in a 4 GiB buffer, OpenSSL SHA-256 on {ran} threads "
            f"(best of 3)",
            "legs_GBps": {"sha256_1_thread": round(float(sz[: len(sz) // 16].sum()) / dt1 / 1e9, 3)},
            "cpu": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": host_threads(),
            "cgroup_cpu_quota": _cpu_quota()}


def c5_layout(files: int, rank: int = 0):
    """C5's file population: `files` files of 4-64 KiB drawn
    from files // 2 distinct payloads (seed 6 + rank).  Payload j is bytes
    [j * 64 KiB, j * 64 KiB + psize[j]) of the synthetic stream seed 6, and
    file i is payload pick[i] whole, so a file's content -- and blob ID --
    depends on pick[i] alone.  -> (sizes, pick, psize, npay)"""
    import numpy as np
    npay = max(1, files // 2)
    rng = np.random.default_rng(6 + rank)
    psize = rng.integers(4096, 65537, npay)
    pick = rng.integers(0, npay, files)
    return psize[pick], pick, psize, npay


def smallfiles_main(args):
    """C5: 1 M files of 4-64 KiB (seed 6) drawn from 500 K distinct payloads
    (dedup-heavy), packed contiguously in HBM with an offsets array.  Every file
    is below MinSize, so restic makes exactly one chunk per file and its blob ID
    is SHA-256 of the whole file.  A step = the blob IDs
    of all files (vs_sha256_run_device) + the SaveBlob dedup count (unique IDs).
    value = file bytes hashed per second.  Files are split evenly over ranks
    (replicas of the same shape; no collective)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from volsync_amd import DeviceSha256, synth_fill_device

    world, rank, local, dev = dist_setup()
    nf = args.files
    sizes, pick, psize, npay = c5_layout(nf, rank)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = int(sizes.sum())
    # payload j = synthetic stream (seed 6) at j * 64 KiB; files gathered into
    # one packed buffer in 1 GiB pieces
    pool = torch.empty(npay << 16, dtype=torch.uint8, device=dev)
    synth_fill_device(pool.data_ptr(), 6, 0, npay << 16, device=local)
    packed = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    src = torch.from_numpy((pick.astype(np.int64) << 16)).to(dev)
    szd = torch.from_numpy(sizes.astype(np.int64)).to(dev)
    ofd = torch.from_numpy(offs).to(dev)
    f0 = 0
    while f0 < nf:
        f1 = int(np.searchsorted(offs, offs[f0] + (1 << 30), side="left"))
        f1 = max(f1, f0 + 1)
        s_, z_, o_ = src[f0:f1], szd[f0:f1], ofd[f0:f1]
        nbytes = int(z_.sum().item())
        rel = torch.arange(nbytes, device=dev) - torch.repeat_interleave(o_ - o_[0], z_, output_size=nbytes)
        idx = torch.repeat_interleave(s_, z_, output_size=nbytes) + rel
        packed[int(offs[f0]):int(offs[f0]) + nbytes] = pool[idx]
        del rel, idx
        f0 = f1
    del pool, src, szd
    torch.cuda.empty_cache()
    lens = torch.from_numpy(sizes.astype(np.int32)).to(dev)
    ids = torch.zeros((nf, 32), dtype=torch.uint8, device=dev)
    first = torch.zeros(nf, dtype=torch.int32, device=dev)
    sh = DeviceSha256(local)
    sh.set_wide(args.hash_wide, args.wide_drain)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # the repository's index (restic SaveBlob: a blob the master index holds
    # is not stored again; a scheduled backup re-runs `restic backup` into an
    # initialised repository, /root/reference/mover-restic/entry.sh:43-65):
    # the previous backup held payloads [0, npay / 2) -- their IDs, found in
    # this batch -- and other blobs, 432 K IDs in all, sorted once per backup
    # (untimed), as LoadIndex builds the master index once
    sh.run(packed.data_ptr(), ofd.data_ptr(), lens.data_ptr(), nf, ids.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    _, rep = np.unique(pick, return_index=True)
    old_ids = ids[torch.from_numpy(rep[pick[rep] < npay // 2]).to(dev)]
    n_known = max(args.known_ids, len(old_ids))
    other = torch.from_numpy(np.random.default_rng(99).integers(
        0, 256, (n_known - len(old_ids), 32), dtype=np.uint8)).to(dev)
    known = torch.cat([old_ids, other]).contiguous()
    sh.index_sort(known.data_ptr(), n_known, stream)
    torch.cuda.synchronize(dev)

    def step():
        sh.run(packed.data_ptr(), ofd.data_ptr(), lens.data_ptr(), nf, ids.data_ptr(), stream)
        # SaveBlob's dedup on the device (vs_blob_dedup_known): per blob, known
        # to the index or its first occurrence in the batch; the count of the
        # new distinct IDs (the blobs this backup stores)
        return sh.dedup_known(ids.data_ptr(), nf, known.data_ptr(), n_known, first.data_ptr(),
                              stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # spot check against hashlib (first files of every distinct size class)
    import hashlib
    host = ids[:64].cpu().numpy()
    for i in range(64):
        o, n = int(offs[i]), int(sizes[i])
        assert bytes(host[i]) == hashlib.sha256(packed[o:o + n].cpu().numpy().tobytes()).digest()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    uniq = 0
    for _ in range(args.steps):
        uniq = step()
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # kernel time: the hash launches ran on `stream` between the two events
    # (the dedup included: an upper bound on the hash time)
    k_ms = ev0.elapsed_time(ev1) / args.steps
    gbs = total / k_ms / 1e6
    # the dedup alone (after the timed region): against the index, and the
    # batch-only form (vs_blob_dedup) with its distinct-ID count
    dd = {}
    for name, fn in (("known", lambda: sh.dedup_known(ids.data_ptr(), nf, known.data_ptr(),
                                                      n_known, first.data_ptr(), stream, False)),
                     ("batch", lambda: sh.dedup(ids.data_ptr(), nf, first.data_ptr(), stream,
                                                False))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        dd[name] = e0.elapsed_time(e1) / 5
    # one pass alone (every step hashes all its blobs to the end and carries
    # nothing to the next, so the replayed step is this pass repeated): the
    # IDs are cleared first, and the golden check below reads this pass's IDs
    ids.zero_()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    step()
    torch.cuda.synchronize(dev)
    lat = time.perf_counter() - t1
    distinct = sh.dedup(ids.data_ptr(), nf, first.data_ptr(), stream)
    # exactness: SHA-256 over all blob IDs in file order (tests/golden/
    # make_golden_full.py c5), and the distinct count
    import hashlib
    id_digest = hashlib.sha256(ids.cpu().numpy().tobytes()).hexdigest()
    if rank == 0:
        out = {
            "metric": "GB/s SHA-256 blob IDs (restic, C5 small files)",
            "value": round(total * world * args.steps / dt / 1e9, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 payloads, device-resident, packed)",
            "config": {"workload": f"C5: {nf} files of 4-64 KiB from {npay} payloads"
                                   f"{' per rank' if world > 1 else ''}",
                       "bytes": total, "unique_ids": distinct,
                       "parallelism": f"replicas x{world}"},
            "dedup": {"form": "vs_blob_dedup_known inside the step (SaveBlob against the index)",
                      "known_index_ids": n_known, "known_from_batch": len(old_ids),
                      "new_unique_ids": uniq, "batch_unique_ids": distinct,
                      "dedup_known_ms": round(dd["known"], 3),
                      "dedup_batch_only_ms": round(dd["batch"], 3)},
            "single_pass": {"ms": round(lat * 1e3, 3), "GBps_per_gpu": round(total / lat / 1e9, 2),
                            "note": "one step alone; the IDs checked below are its output"},
            "exact": {"files": nf, "unique_ids": distinct, "id_digest": id_digest},
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "valu_frac": valu_frac(gbs, SHA_OPS_PER_BYTE, SHA_MIX_CYC),
                         "valu_frac_flat42": round(gbs * SHA_OPS_PER_BYTE / 1e3 / VALU_PEAK_TOPS, 4),
                         "kernel": "sha256 (hash engine, unbounded slice)"},
            "hash_wide": args.hash_wide,
        }
        g = _goldens().get("c5", {}).get(str(nf))
        if g and world == 1:
            out["exact"]["golden_match"] = (g["unique_ids"], g["id_digest"], g["bytes"]) == \
                (distinct, id_digest, total)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = smallfiles_cpu_baseline(sizes, len(sizes), args.cpu_threads)
        print(json.dumps(out), flush=True)
    sh.close()
    if world > 1:
        dist.destroy_process_group()


def seal_cpu_baseline(sizes, keys, sample_bytes: int, threads: int):
    """restic's Key.Seal on the host: libcrypto AES-256-CTR (AES-NI) + Poly1305
    (oracle/seal_ref.seal_into, no copies) per blob over `threads` threads, on
    the first blobs of the same size distribution up to `sample_bytes`."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from oracle import seal_ref as S
    cum = np.cumsum(sizes)
    nb = max(1, int(np.searchsorted(cum, sample_bytes)))
    sz = sizes[:nb]
    src = np.random.default_rng(8).integers(0, 256, int(sz.max()), dtype=np.uint8)
    dst = [np.empty(int(sz.max()), np.uint8) for _ in range(threads)]
    nonces = np.random.default_rng(9).integers(0, 256, (nb, 16), dtype=np.uint8)

    def work(t):
        d = dst[t].ctypes.data
        for k in range(t, nb, threads):
            S.seal_into(*keys, nonces[k].tobytes(), src.ctypes.data, int(sz[k]), d)
    S.seal_into(*keys, bytes(16), src.ctypes.data, 16, dst[0].ctypes.data)   # load libcrypto
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(threads)))
    dt = time.perf_counter() - t0
    return {"value": round(float(sz.sum()) / dt / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port", "sample": f"{nb} blobs ({float(sz.sum()) / 2**30:.2f} GiB) of the same "
            f"size distribution, libcrypto AES-256-CTR + Poly1305 on {threads} threads",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def seal_main(args):
    """SURVEY.md 8(f)1, restic's pack stage: every unique blob of a backup is
    encrypted with Key.Seal (AES-256-CTR under its own random nonce +
    Poly1305-AES tag) before it is written to a pack.  The workload is one
    volume's worth of blobs (--per-gpu-gib, default 64 GiB) with restic's chunk
    size distribution (512 KiB + exponential mean 1 MiB, capped at 8 MiB),
    device-resident; a step seals all of them into a separate output buffer
    (vs_seal_run_device).  value = plaintext bytes sealed per second.  Ranks
    are replicas (independent blobs, no collective)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from volsync_amd import Sealer, synth_fill_device

    world, rank, local, dev = dist_setup()
    target = int(args.per_gpu_gib * (1 << 30))
    rng = np.random.default_rng(11 + rank)
    sizes = np.minimum((512 << 10) + rng.exponential(1 << 20, target // (1 << 20) + 16).astype(np.int64),
                       8 << 20)
    cum = np.cumsum(sizes)
    nb = int(np.searchsorted(cum, target, side="right"))
    sizes = sizes[:nb]
    offs = np.concatenate([[0], cum[:nb - 1]]).astype(np.int64)
    total = int(sizes.sum())
    data = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    synth_fill_device(data.data_ptr(), 12, 0, total + 16, device=local)
    out = torch.empty_like(data)
    ofd = torch.from_numpy(offs).to(dev)
    lens = torch.from_numpy(sizes.astype(np.int32)).to(dev)
    nonces = torch.from_numpy(rng.integers(0, 256, (nb, 16), dtype=np.uint8)).to(dev)
    macs = torch.zeros((nb, 16), dtype=torch.uint8, device=dev)
    keys = tuple(rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (32, 16, 16))
    sl = Sealer(*keys, device=local)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        sl.run(data.data_ptr(), ofd.data_ptr(), lens.data_ptr(), nb, nonces.data_ptr(),
               out.data_ptr(), macs.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # spot check: first and last blob against the oracle (libcrypto)
    from oracle import seal_ref as S
    for i in (0, nb - 1):
        o, n = int(offs[i]), int(sizes[i])
        ct, mac = S.seal(*keys, nonces[i].cpu().numpy().tobytes(), data[o:o + n].cpu().numpy().tobytes())
        assert out[o:o + n].cpu().numpy().tobytes() == ct and macs[i].cpu().numpy().tobytes() == mac
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    sl.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctr_ms, mac_ms, runs = sl.kernel_ms()
    sl.close()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ctr_ms, mac_ms = ctr_ms / max(runs, 1), mac_ms / max(runs, 1)
    # algorithmic HBM bytes: CTR reads + writes every byte (2 B/B), the MAC
    # re-reads the ciphertext (1 B/B)
    ctr_gbs, mac_gbs = 2 * total / ctr_ms / 1e6, total / mac_ms / 1e6
    dom = "ctr" if ctr_ms >= mac_ms else "mac"
    kern = {"ctr": {"kernel": "seal_ctr_kernel", "avg_launch_ms": round(ctr_ms, 3),
                    "achieved": round(ctr_gbs, 1), "bytes_per_launch": 2 * total},
            "mac": {"kernel": "seal_mac_kernel", "avg_launch_ms": round(mac_ms, 3),
                    "achieved": round(mac_gbs, 1), "bytes_per_launch": total}}
    if rank == 0:
        res = {
            "metric": "GB/s sealed (restic pack stage: AES-256-CTR + Poly1305-AES per blob)",
            "value": round(total * world * args.steps / dt / 1e9, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 plaintext, random keys and nonces, device-resident)",
            "config": {"workload": f"(f)1: {nb} blobs, {total / 2**30:.1f} GiB, restic chunk sizes"
                                   f"{' per rank' if world > 1 else ''}",
                       "bytes": total, "blobs": nb, "parallelism": f"replicas x{world}"},
            "roofline": {"bound": "hbm", "achieved": kern[dom]["achieved"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(kern[dom]["achieved"] / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": kern[dom]["kernel"],
                         "avg_launch_ms": kern[dom]["avg_launch_ms"]},
            "kernels": kern,
        }
        try:
            tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
            r = tj["seal_" + dom]
            res["roofline"]["traffic"] = round(r["bytes_per_plain_byte"] * total)
            res["roofline"]["traffic_source"] = r["source"]
        except (OSError, ValueError, KeyError):
            pass
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = seal_cpu_baseline(sizes, keys, 32 << 30,
                                                    args.cpu_threads)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """--gpus N > 1 without a torch.distributed launcher around us: start
    `torch.distributed.run --nproc-per-node N` on this same command line as a
    CHILD process (before anything here touches the GPU), wait for it and
    return its exit code.  Rank 0 of the child prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class DryChunker:
    """--dry: a stand-in for the device chunker with the same scan / stitch /
    finish surface, so the REAL multi-rank protocol (volsync_amd/shard.py) and
    its collectives run over gloo on CPU.  Candidate cut positions are a
    position-independent pseudo-random function of the byte offset (one per
    ~avg bytes, like the fingerprint's), and the min/max rule of Chunker.Next
    selects among them.  It computes no fingerprints and no hashes: it
    rehearses the launcher, the rendezvous and the exit exchange, nothing
    else (value is reported as null)."""

    def __init__(self, mn: int, mx: int, avg: int):
        self.mn, self.mx, self.avg = mn, mx, avg

    def _cands(self, lo: int, hi: int):
        import numpy as np
        blk = 1 << 20
        out = []
        for b in range(lo // blk, (hi + blk - 1) // blk):
            rng = np.random.default_rng([77, b])
            k = rng.poisson(blk / self.avg)
            pos = np.sort(rng.integers(0, blk, k)) + b * blk
            out.append(pos[(pos >= lo) & (pos < hi)])
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def scan(self, ptr, length, origin, own_lo, own_hi, final):
        self.own_lo, self.own_hi, self.end = own_lo, own_hi, origin + length
        self.final = final
        self.scan_end = min(own_hi + self.mx - 1, self.end)
        self.c = self._cands(own_lo, self.scan_end)

    def stitch(self, entry):
        import numpy as np
        self.cuts, s = [], entry
        while s < self.own_hi and s < self.end:
            k = int(np.searchsorted(self.c, s + self.mn - 1))
            if k < len(self.c) and self.c[k] <= s + self.mx - 1:
                cut = int(self.c[k])
            elif s + self.mx - 1 < self.scan_end:
                cut = s + self.mx - 1
            else:
                cut = self.end - 1
            self.cuts.append((s, cut))
            s = cut + 1
        return s, True

    def finish(self):
        return len(self.cuts)


def dry_main(args):
    """Multi-rank rehearsal on CPU (gloo): shard specs of the C3 shape at
    --per-gpu-gib per rank, the scan / exit all-gather / re-stitch protocol
    with DryChunker, and the same chunk list checked against one rank doing
    the whole volume.  Prints the bench JSON shape with value null."""
    import torch.distributed as dist
    from volsync_amd.shard import ShardSpec, run_shard, torch_collectives
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    per = int(args.per_gpu_gib * (1 << 30))
    if world > 1 and args.c3_default:
        per = 128 << 30   # the CDC mode's C3 default (main)
    total = per * world
    mn, mx = 512 << 10, 8 << 20
    spec = ShardSpec.for_rank(total, world, rank, mx)
    h = DryChunker(mn, mx, 1 << 20)
    st = {}
    t0 = time.perf_counter()
    if world > 1:
        run_shard(h, spec, 0, *torch_collectives(None), stats=st)
        parts = [None] * world
        dist.all_gather_object(parts, h.cuts)
        mine = [c for p in parts for c in p]
    else:
        h.scan(0, spec.data_hi - spec.data_lo, spec.data_lo, spec.own_lo, spec.own_hi, True)
        h.stitch(spec.own_lo)
        mine = h.cuts
    dt = time.perf_counter() - t0
    if rank == 0:
        ref = DryChunker(mn, mx, 1 << 20)
        ref.scan(0, total, 0, 0, total, True)
        ref.stitch(0)
        out = {"metric": "GB/s chunked+SHA-256 (restic CDC)", "value": None, "unit": "GB/s",
               "n_gpus": world, "steps": 0, "warmup": 0, "ms_per_step": round(dt * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
               "data": "dry run: no GPU, no fingerprints or hashes (protocol rehearsal)",
               "dry": True,
               "config": {"workload": f"C3-shape: {total >> 30} GiB volume byte-range sharded "
                                      f"over {world} ranks ({per >> 30} GiB per rank)",
                          "per_gpu_bytes": per, "parallelism": f"byte-range shards x{world}"},
               "world_size": dist.get_world_size() if world > 1 else 1,
               "backend": "gloo" if world > 1 else None,
               "exchange_rounds": st.get("exchange_rounds", 0),
               "chunks": len(mine), "protocol_matches_single_rank": mine == ref.cuts}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_main(args):
    """C2 fed from host memory through the streaming drop-in API, as
    gpuchunker's Chunker.Next does: vs_cdc_feed of 64 MiB reads taken from a
    pinned host image of the volume, vs_cdc_next for the chunks until EOF
    ("host-pinned end-to-end").  A step = one whole
    volume streamed, chunked and hashed, every chunk (with its blob ID)
    returned to the host.  value = volume bytes / wall time, H2D included;
    the H2D rate of the same pinned buffer is measured beside it."""
    import ctypes
    import torch
    from volsync_amd import MaxSize, MinSize, TestPol, synth_fill_device
    from volsync_amd._lib import VS_EOF, VsChunk, check, lib

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n = int(args.per_gpu_gib * (1 << 30))
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    piece = min(n, 4 << 30)
    tmp = torch.empty(piece, dtype=torch.uint8, device=dev)
    for off in range(0, n, piece):
        k = min(piece, n - off)
        synth_fill_device(tmp.data_ptr(), 2, off, k)
        host[off:off + k].copy_(tmp[:k])
    torch.cuda.synchronize(dev)
    # H2D reference: the same pinned buffer, one 4 GiB copy
    t = time.perf_counter()
    tmp.copy_(host[:piece], non_blocking=True)
    torch.cuda.synchronize(dev)
    h2d = piece / (time.perf_counter() - t) / 1e9
    del tmp
    torch.cuda.empty_cache()
    h = ctypes.c_void_p()
    check(lib.vs_cdc_open(0, TestPol, MinSize, MaxSize, 20, ctypes.byref(h)))
    read = 64 << 20
    cap = 4096
    out = (VsChunk * cap)()
    got = ctypes.c_size_t(0)

    def step():
        nch = 0
        last = None
        base = host.data_ptr()
        for off in range(0, n, read):
            check(lib.vs_cdc_feed(h, ctypes.c_void_p(base + off), min(read, n - off), 0))
            while True:
                check(lib.vs_cdc_next(h, out, cap, ctypes.byref(got)))
                if not got.value:
                    break
                nch += got.value
                last = out[got.value - 1]
        check(lib.vs_cdc_feed(h, None, 0, 1))
        while True:
            rc = lib.vs_cdc_next(h, out, cap, ctypes.byref(got))
            if rc == VS_EOF:
                break
            check(rc)
            nch += got.value
            if got.value:
                last = out[got.value - 1]
        assert last is not None and last.start + last.length == n, "stream not fully chunked"
        check(lib.vs_cdc_reset(h, TestPol, MinSize, MaxSize, 20))
        return nch

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    nch = 0
    for _ in range(args.steps):
        nch = step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    stats = (ctypes.c_double * 8)()
    check(lib.vs_cdc_stream_stats(h, stats))
    lib.vs_cdc_close(h)
    value = n * args.steps / dt / 1e9
    print(json.dumps({
        "metric": "GB/s chunked+SHA-256 (restic CDC), host-pinned end-to-end via vs_cdc_feed/next",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 volume image in pinned host memory, fed in 64 MiB reads)",
        "config": {"workload": f"C2 streamed: {n >> 30} GiB volume through the Chunker.Next "
                               f"drop-in path (H2D included), 1 GPU",
                   "volume_bytes": n, "read_bytes": read, "chunks": nch,
                   "pol": "0x3DA3358B4DC173", "min": MinSize, "max": MaxSize, "avg_bits": 20},
        "h2d_GBps": round(h2d, 2), "frac_of_h2d": round(value / h2d, 4),
        "stream_stats": {"pinned_bytes": stats[0], "staged_bytes": stats[1],
                         "collect_waits": stats[2], "batches": stats[3],
                         "host_ms": {"h2d_wait": round(stats[4], 1), "batches": round(stats[5], 1),
                                     "collect": round(stats[6], 1), "staging": round(stats[7], 1)}},
    }), flush=True)


def rsync_host_main(args):
    """C4 fed from host memory through the streamed drop-in path, as rsync's
    generator and sender read files (map_ptr windows): the destination D
    through vs_rsync_sig_begin/feed/next (generate_and_send_sums), the sums
    loaded (build_hash_table), the source S through vs_rsync_match_begin/
    feed/next (match_sums), in --read-mib reads from pinned host images, the
    device holding only a ring of 3 x 256 MiB pieces per stream.  A step = both
    files streamed and every sum and match returned to the host.  value =
    (|D| + |S|) / wall time, H2D included; the H2D rate
    of the same pinned buffers is measured beside it."""
    import ctypes
    import hashlib
    import numpy as np
    import torch
    from volsync_amd import Matcher, sum_sizes_sqroot, synth_fill_device
    from volsync_amd._lib import VS_EOF, VsMatch, check, lib
    from volsync_amd.rsync import CSUM_XXH3_128

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dlen = int(args.per_gpu_gib * (1 << 30))
    hdr = sum_sizes_sqroot(dlen)
    plan = C4Plan(dlen, hdr.blength)
    seed = 0x5EED5EED
    hd = torch.empty(dlen, dtype=torch.uint8, pin_memory=True)
    hs = torch.empty(plan.total, dtype=torch.uint8, pin_memory=True)
    piece = 4 << 30
    tmp = torch.empty(piece, dtype=torch.uint8, device=dev)
    for off in range(0, dlen, piece):
        k = min(piece, dlen - off)
        synth_fill_device(tmp.data_ptr(), C4Plan.D_SEED, off, k)
        hd[off:off + k].copy_(tmp[:k])
    for off in range(0, plan.total, piece):
        k = min(piece, plan.total - off)
        plan.fill_device(tmp.data_ptr(), off, off + k)
        torch.cuda.synchronize(dev)
        hs[off:off + k].copy_(tmp[:k])
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    tmp.copy_(hs[:piece], non_blocking=True)
    torch.cuda.synchronize(dev)
    h2d = piece / (time.perf_counter() - t) / 1e9
    del tmp
    torch.cuda.empty_cache()
    m = Matcher(0)
    read = args.read_mib << 20
    cnt, s2l = hdr.count, hdr.s2length
    sum1 = np.zeros(max(cnt, 1), np.uint32)
    sum2 = np.zeros(max(cnt, 1) * s2l, np.uint8)
    mcap = 1 << 16
    marr = (VsMatch * mcap)()
    got = ctypes.c_size_t(0)
    h = m._h

    def step():
        t0 = time.perf_counter()
        # generate_and_send_sums: D in `read` pieces, sums collected as they finish
        check(lib.vs_rsync_sig_begin(h, dlen, hdr.blength, s2l, CSUM_XXH3_128, seed, 0, 0))
        ns = 0
        base = hd.data_ptr()
        for off in range(0, dlen + read, read):
            if off < dlen:
                check(lib.vs_rsync_sig_feed(h, ctypes.c_void_p(base + off), min(read, dlen - off)))
            while True:
                rc = check(lib.vs_rsync_sig_next(h, sum1[ns:].ctypes.data,
                                                 sum2[ns * s2l:].ctypes.data, cnt - ns,
                                                 ctypes.byref(got)))
                ns += got.value
                if rc == VS_EOF or not got.value:
                    break
            if rc == VS_EOF:
                break
        assert ns == cnt, (ns, cnt)
        t1 = time.perf_counter()
        check(lib.vs_rsync_load_sums(h, cnt, hdr.blength, s2l, hdr.remainder, sum1.ctypes.data,
                                     sum2.ctypes.data, CSUM_XXH3_128, seed))
        t2 = time.perf_counter()
        # match_sums: S in `read` pieces, matches drained after every read
        check(lib.vs_rsync_match_begin(h, plan.total, CSUM_XXH3_128, 0, 0))
        nm = 0
        dig = hashlib.sha256()
        base = hs.data_ptr()
        off = 0
        while True:
            if off < plan.total:
                check(lib.vs_rsync_match_feed(h, ctypes.c_void_p(base + off),
                                              min(read, plan.total - off)))
                off += read
            rc = check(lib.vs_rsync_match_next(h, marr, mcap, ctypes.byref(got)))
            if got.value:
                nm += got.value
                dig.update(ctypes.string_at(marr, got.value * 16))
            if rc == VS_EOF:
                break
        nm2, fa = ctypes.c_int64(), ctypes.c_int64()
        fsum = ctypes.create_string_buffer(16)
        check(lib.vs_rsync_match_end(h, ctypes.byref(nm2), ctypes.byref(fa), fsum))
        assert nm2.value == nm
        t3 = time.perf_counter()
        return {"sig_s": t1 - t0, "load_s": t2 - t1, "match_s": t3 - t2, "matches": nm,
                "false_alarms": fa.value, "digest": dig.hexdigest(), "file_sum": fsum.raw.hex()}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    res = []
    for _ in range(args.steps):
        res.append(step())
    dt = time.perf_counter() - t0
    st = m.match_stream_stats()
    m.close()
    total = dlen + plan.total
    r = res[-1]
    golden = _golden_rsync(dlen)
    out = {
        "metric": "GB/s rsync delta match (|D|+|S|), host-pinned end-to-end via the streamed "
                  "vs_rsync_sig_* / vs_rsync_match_* path",
        "value": round(total * args.steps / dt / 1e9, 2), "unit": "GB/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic (C4 destination + 10%-edited source in pinned host memory, fed in "
                f"{args.read_mib} MiB reads)",
        "config": {"workload": f"C4-shape streamed: {dlen >> 30} GiB destination, "
                               f"{plan.total} B source, 1 GPU, device window 3 x 256 MiB per "
                               f"stream (H2D included)",
                   "blength": hdr.blength, "s2length": s2l, "count": cnt, "csum": "xxh128",
                   "checksum_seed": hex(seed), "read_bytes": read},
        "h2d_GBps": round(h2d, 2), "frac_of_h2d": round(total * args.steps / dt / 1e9 / h2d, 4),
        "stages_GBps": {"signatures_stream": round(dlen / r["sig_s"] / 1e9, 2),
                        "match_stream": round(plan.total / r["match_s"] / 1e9, 2),
                        "load_sums_ms": round(r["load_s"] * 1e3, 2)},
        "match_stream_stats": st,
        "matches": r["matches"], "false_alarms": r["false_alarms"], "digest": r["digest"],
        "file_sum": {"csum": "xxh128 (R7, computed as S streamed through)", "digest": r["file_sum"]},
        "identical_every_step": len({(x["digest"], x["file_sum"]) for x in res}) == 1,
    }
    if golden:
        out["golden_match"] = (r["digest"] == golden["digest"] and r["matches"] == golden["matches"]
                               and r["false_alarms"] == golden["false_alarms"])
        if "file_sum" in golden:
            out["file_sum"]["golden_match"] = r["file_sum"] == golden["file_sum"]
    print(json.dumps(out), flush=True)


def _chunk_records(dc, n: int, batch=None) -> bytes:
    """The last finished batch's (or batch `batch`'s) chunk list as 56-byte
    vs_chunk records (waits for their blob IDs)."""
    import ctypes
    from volsync_amd._lib import VsChunk, check, lib
    if not n:
        return b""
    arr = (VsChunk * n)()
    if batch is None:
        check(lib.vs_cdc_get_chunks(dc._h, 0, n, arr))
    else:
        check(lib.vs_cdc_get_batch_chunks(dc._h, batch, 0, n, arr))
    return ctypes.string_at(arr, 56 * n)


# bench.py --distinct B: volume k of the run is the 64 GiB stream of seed
# DISTINCT_SEEDS[k % B] (2 = C2's); goldens in full_configs.json
# (make_golden_full.py distinct)
DISTINCT_SEEDS = (2, 7, 8)


def distinct_pass(args, dc, buf0, dlen: int, local: int, dev, stream) -> dict:
    """The C2 step over B DISTINCT resident volumes in rotation, as a producer
    refilling B buffers would run it: step k reuses volume k mod B's buffer
    and therefore starts only once every blob ID of step k - B is final
    (vs_cdc_fence; the engine drains when that batch's chunks are still
    queued).  Nothing is replayed: every step chunks and hashes a volume
    whose chains were never seen before."""
    import hashlib
    import torch
    from volsync_amd import synth_fill_device
    B = args.distinct
    assert 1 <= B <= len(DISTINCT_SEEDS), B
    seeds = DISTINCT_SEEDS[:B]
    bufs = [buf0] + [torch.empty(dlen, dtype=torch.uint8, device=dev) for _ in range(B - 1)]
    for b, sd in zip(bufs[1:], seeds[1:]):
        synth_fill_device(b.data_ptr(), sd, 0, dlen, device=local, stream=stream)
    torch.cuda.synchronize(dev)
    dc.wait()
    first, ring = dc.batches()
    assert ring > B, (ring, B)
    done = []

    def dstep(j):
        if j >= B:
            dc.fence(first + j - B)
        n, _ = dc.process(bufs[j % B].data_ptr(), dlen, 0, True)
        done.append((first + j, seeds[j % B], n))

    for j in range(args.warmup):
        dstep(j)
    dc.wait()
    torch.cuda.synchronize(dev)
    dc.timing(True)
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        dstep(j)
    dc.wait()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ms, launches = dc.timing(False)
    det = dc.timing_detail()
    gold = _goldens().get("cdc", {})
    checks = []
    for bi, sd, n in done[-B:]:
        g = gold.get(str(sd), {}).get(str(dlen))
        d = hashlib.sha256(_chunk_records(dc, n, batch=bi)).hexdigest()
        checks.append({"seed": sd, "chunks": n, "digest": d,
                       "golden_match": bool(g) and (g["chunks"], g["digest"]) == (n, d)})
    del bufs[1:]
    torch.cuda.empty_cache()
    return {"volumes": B, "seeds": list(seeds),
            "GBps": round(dlen * args.steps / dt / 1e9, 2),
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "stages_ms_per_step": {"fingerprint": round(ms[0] / args.steps, 3),
                                   "sha256": round(det["sha_outside_fp_ms"] / args.steps, 3),
                                   "sha256_inside_fp": round(det["sha_inside_fp_ms"] / args.steps, 3)},
            "sha_launches": launches[2], "latency_mode_chains": det["quad_chains"],
            "rule": "step k starts after every blob ID of step k - B is final (vs_cdc_fence)",
            "exact": checks, "golden_match": all(c["golden_match"] for c in checks)}


def _match_records(m, n: int) -> bytes:
    """The handle's last match list as 16-byte vs_match records."""
    import ctypes
    from volsync_amd._lib import VsMatch, check, lib
    arr = (VsMatch * max(n, 1))()
    if n:
        check(lib.vs_rsync_get_matches(m._h, 0, n, arr))
    return ctypes.string_at(arr, n * 16) if n else b""


def _goldens() -> dict:
    """tests/golden/full_configs.json (tests/golden/make_golden_full.py): the
    full-size chunk / match list digests from the C oracle, computed in the
    build container; {} when absent."""
    try:
        return json.load(open(os.path.join(ROOT, "tests", "golden", "full_configs.json")))
    except (OSError, ValueError):
        return {}


def _golden_rsync(dlen: int):
    return _goldens().get("rsync", {}).get(str(dlen))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--per-gpu-gib", type=float, default=None,
                    help="bytes per GPU (default 64 GiB; the CDC mode at N > 1: C3's "
                         "128 GiB per GPU, i.e. 1 TiB over 8)")
    ap.add_argument("--distinct", type=int, default=None,
                    help="cdc, 1 GPU: also run the step over B distinct volumes in rotation "
                         "(step k waits for step k-B's blob IDs; default 3 for C2, 0 = off)")
    ap.add_argument("--cpu-sample-gib", type=int, default=4)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baselines' threads (0 = every CPU of the host, nproc)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--file-sum-jobs", type=int, default=3,
                    help="rsync: whole-file checksums in flight (one host chain thread each)")
    ap.add_argument("--no-file-sum", action="store_true",
                    help="rsync: leave R7 (the whole-file checksum) out of the step (A/B)")
    ap.add_argument("--hash-stream", choices=["own", "main"], default="own",
                    help="SHA-256 slices on the handle's own hash stream (overlapping the next "
                         "fingerprint pass) or serialised on the main stream")
    ap.add_argument("--hash-slice", type=int, default=512,
                    help="SHA-256 blocks per chunk per step (time-sliced engine; 0 = unbounded)")
    ap.add_argument("--hash-wide", type=lambda x: int(x, 0), default=0,
                    help="active chains from which the SHA-256 engine runs whole-SHA "
                         "wavefronts (0 = library default, 0xffffffff = never)")
    ap.add_argument("--wide-drain", type=int, default=0,
                    help="blocks per throughput-mode drain launch (0 = library default)")
    ap.add_argument("--mode", choices=["cdc", "rsync", "smallfiles", "host", "seal", "rsync-host"],
                    default="cdc",
                    help="cdc: C2/C3 chunk+hash (the BASELINE metric); rsync: C4-shape delta "
                         "match; smallfiles: C5 per-file blob IDs; host: C2 streamed from "
                         "pinned host memory through vs_cdc_feed/next; rsync-host: C4 streamed "
                         "from pinned host memory through vs_rsync_sig_*/vs_rsync_match_*")
    ap.add_argument("--csum", choices=["xxh128", "xxh3", "xxh64", "md5"], default="xxh128",
                    help="rsync: the negotiated strong / whole-file checksum (rsync 3.2.3 peers: "
                         "xxh128; md5 against peers without xxhash -- the host walk)")
    ap.add_argument("--walk-opt", default="",
                    help="rsync A/B: handle options, e.g. walk_prefilter=0,walk_segment_blocks=64")
    ap.add_argument("--read-mib", type=int, default=64,
                    help="rsync-host: bytes per feed (the reader's read size)")
    ap.add_argument("--files", type=int, default=1_000_000, help="smallfiles: files per GPU")
    ap.add_argument("--known-ids", type=int, default=432_000,
                    help="smallfiles: IDs in the repository's index the dedup checks against")
    ap.add_argument("--share", default=None, metavar="R/N",
                    help="run rank R's share of the N-rank problem on this one GPU; rsync: "
                         "the full table, its D blocks and S range (3/8 with --per-gpu-gib 32 "
                         "is one rank of C4); cdc: its 128 GiB of C3's 1 TiB, cut from its true "
                         "entry")
    ap.add_argument("--dry", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank protocol (no GPU; value null)")
    args = ap.parse_args()
    if args.cpu_threads <= 0:
        args.cpu_threads = host_threads()
    # C3: 1 TiB of the seed-3 stream over 8 GPUs, 128 GiB
    # resident per GPU; the CDC mode's N > 1 default is that per-GPU share
    args.c3_default = args.per_gpu_gib is None
    if args.distinct is None:
        args.distinct = 3 if (args.mode == "cdc" and args.gpus == 1 and not args.share
                              and args.per_gpu_gib in (None, 64.0)) else 0
    if args.per_gpu_gib is None:
        args.per_gpu_gib = 64.0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under a launcher: become one (a child process, started before
        # this process has touched the GPU)
        sys.exit(launch_ranks(args.gpus))
    if args.dry:
        return dry_main(args)
    if args.mode == "rsync":
        return rsync_main(args)
    if args.mode == "smallfiles":
        return smallfiles_main(args)
    if args.mode == "seal":
        return seal_main(args)
    if args.mode == "host":
        return host_main(args)
    if args.mode == "rsync-host":
        return rsync_host_main(args)

    import torch
    import torch.distributed as dist
    from volsync_amd import DeviceChunker, MaxSize, MinSize, TestPol, synth_fill_device
    from volsync_amd.shard import ShardSpec, run_shard, torch_collectives

    world, rank, local, dev = dist_setup()

    # --share R/N: rank R's work of the N-rank C3 on this one GPU -- its
    # byte range scanned, its chunks cut from its true entry (the exit of
    # rank R-1, from the golden) and hashed; the per-rank golden digest checks it
    share = None
    if args.share:
        share = tuple(int(x) for x in args.share.split("/"))
        assert world == 1 and len(share) == 2 and 0 <= share[0] < share[1], args.share
    sw, sr = (share[1], share[0]) if share else (world, rank)
    per = int(args.per_gpu_gib * (1 << 30))
    seed = 2                      # C2's stream
    if sw > 1 and args.c3_default:
        per, seed = 128 << 30, 3  # C3's per-GPU share of its 1 TiB stream
    total = per * sw
    spec = ShardSpec.for_rank(total, sw, sr, MaxSize)
    gold_all = _goldens().get("cdc", {}).get(str(seed), {}).get(str(total))
    gold_rank = (gold_all or {}).get("ranks", [None] * sw)[sr] if share else None
    share_entry = (gold_rank["entry"] if gold_rank else spec.own_lo) if share else None
    dlen = spec.data_hi - spec.data_lo
    buf = torch.empty(dlen, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    synth_fill_device(buf.data_ptr(), seed, spec.data_lo, dlen, device=local, stream=stream)
    torch.cuda.synchronize(dev)

    dc = DeviceChunker(TestPol, MinSize, MaxSize, 20, device=local)
    dc.set_hash_slice(args.hash_slice)
    dc.set_hash_wide(args.hash_wide, args.wide_drain)
    if args.hash_stream == "main":
        # hash slices queue behind the fingerprint pass on one stream
        one = torch.cuda.Stream(dev)
        dc.set_stream(one.cuda_stream)
        dc.set_hash_stream(one.cuda_stream)
    coll = torch_collectives(coll_device(dev)) if world > 1 else None
    xst = {}

    def step():
        # one volume pass: fingerprint + cut selection + Cut values on the main
        # stream; its chunks join the time-sliced SHA-256 engine on the hash
        # stream, which keeps hashing them while the next volume is chunked
        # (DESIGN.md 3.4).  wait() hashes everything still queued.
        if share:
            dc.scan(buf.data_ptr(), dlen, spec.data_lo, spec.own_lo, spec.own_hi, spec.final)
            dc.stitch(share_entry)
            n = dc.finish()
        elif world == 1:
            n, _ = dc.process(buf.data_ptr(), dlen, 0, True)
        else:
            n = run_shard(dc, spec, buf.data_ptr(), *coll, stats=xst)
        return n

    for _ in range(args.warmup):
        step()
    dc.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dc.timing(True)
    t0 = time.perf_counter()
    nch = 0
    for _ in range(args.steps):
        nch = step()
    dc.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ms, launches = dc.timing(False)
    detail = dc.timing_detail()
    # exactness evidence: the chunk list (this rank's chunks, gathered in rank
    # order) as vs_chunk records, SHA-256 -> golden (tests/golden/
    # make_golden_full.py); outside the timed region
    import hashlib
    recs = _chunk_records(dc, nch)
    if world > 1:
        parts = [None] * world if rank == 0 else None
        dist.gather_object(recs, parts, dst=0)
        recs = b"".join(parts) if rank == 0 else b""
    cdigest = hashlib.sha256(recs).hexdigest()
    # one pass over one volume, nothing replayed or carried (the north star's
    # workload: one restic backup of one volume, mover-restic/entry.sh:60-65):
    # scan .. drain, every blob ID final at the end
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dc.timing(True)
    t1 = time.perf_counter()
    n_single = step()
    dc.wait()
    torch.cuda.synchronize(dev)
    lat = time.perf_counter() - t1
    iso_ms, iso_launch = dc.timing(False)
    iso_detail = dc.timing_detail()
    single_ok = _chunk_records(dc, n_single) == recs if world == 1 else None
    if world > 1:
        t = torch.tensor([lat], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lat = float(t.item())
    distinct = None
    if args.distinct and world == 1 and not share:
        distinct = distinct_pass(args, dc, buf, dlen, local, dev, stream)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([nch], dtype=torch.int64, device=coll_device(dev))
        dist.all_reduce(c)
        nch = int(c.item())

    own_bytes = spec.own_hi - spec.own_lo
    stages = ["fingerprint", "select", "sha256", "other"]
    per_step = {s: ms[i] / args.steps for i, s in enumerate(stages)}
    # the SHA-256 stage is its kernels' time OUTSIDE every fingerprint window
    # (HIP events on both streams against one anchor): a slice dispatched
    # while the persistent fingerprint grid holds the CUs waits inside its
    # span without hashing; the part inside the windows is reported beside it
    sha_span_step = per_step["sha256"]
    per_step["sha256"] = detail["sha_outside_fp_ms"] / args.steps
    # kernel roofline from the timed region (HIP events on each handle's stream,
    # so overlapped volumes share the chip): algorithmic bytes per launch = the
    # volume bytes -- the fingerprint pass reads each scanned byte once (plus a
    # 64-byte warm-up per 12 KiB strip, not counted), SHA-256 reads each chunk
    # byte once; one fingerprint stage and one SHA-256 launch per volume.
    # fingerprint: one launch per volume; SHA-256: slices (one per step plus the
    # final drain) -- bytes hashed in the timed region / summed slice time
    fp_ms = ms[0] / args.steps
    sha_ms = per_step["sha256"]
    fp_gbs = own_bytes / fp_ms / 1e6 if fp_ms else 0.0
    sha_gbs = own_bytes / sha_ms / 1e6 if sha_ms else 0.0
    iso = {s: round(iso_ms[i], 3) for i, s in enumerate(stages)}
    iso["sha256_span"] = iso["sha256"]
    iso["sha256"] = round(iso_detail["sha_outside_fp_ms"], 3)
    # per-launch averages over the timed region, comparable with the
    # rocprofv3 kernel trace of the same command (profiles/r01_final)
    avg_launch = {s: round(ms[i] / launches[i], 3) if launches[i] else None
                  for i, s in enumerate(stages)}
    roof = {
        "fingerprint": {"bound": "hbm", "achieved": round(fp_gbs, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(fp_gbs / HBM_PEAK_GBS, 4),
                        "traffic": None,
                        "valu_frac": valu_frac(fp_gbs, FP_OPS_PER_BYTE, FP_MIX_CYC),
                        "valu_frac_flat42": round(fp_gbs * FP_OPS_PER_BYTE / 1e3 / VALU_PEAK_TOPS, 4)},
        "sha256": {"bound": "hbm", "achieved": round(sha_gbs, 1), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(sha_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                   "valu_frac": valu_frac(sha_gbs, SHA_OPS_PER_BYTE, SHA_MIX_CYC),
                   "valu_frac_flat42": round(sha_gbs * SHA_OPS_PER_BYTE / 1e3 / VALU_PEAK_TOPS, 4)},
    }
    # roofline.traffic: HBM bytes per step from the committed rocprofv3
    # FETCH_SIZE/WRITE_SIZE passes (profiles/traffic.json, tools/traffic.py),
    # scaled to this run's volume; null when no profile matches
    try:
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
        for k in roof:
            if k in tj:
                roof[k]["traffic"] = round(tj[k]["bytes_per_volume"] * own_bytes / tj["volume_bytes"])
                roof[k]["traffic_source"] = tj["source"]
    except (OSError, ValueError, KeyError):
        pass
    roof["fingerprint"]["avg_launch_ms"] = avg_launch["fingerprint"]
    roof["fingerprint"]["launches"] = launches[0]
    roof["sha256"]["avg_launch_ms"] = avg_launch["sha256"]   # span (rocprof-comparable)
    roof["sha256"]["launches"] = launches[2]
    roof["sha256"]["busy_ms_per_step"] = round(per_step["sha256"], 3)
    roof["sha256"]["span_ms_per_step"] = round(sha_span_step, 3)
    roof["sha256"]["inside_fp_ms_per_step"] = round(detail["sha_inside_fp_ms"] / args.steps, 3)
    dom_name = "sha256" if per_step["sha256"] >= per_step["fingerprint"] else "fingerprint"
    roofline = dict(roof[dom_name])
    roofline["kernel"] = dom_name

    # a --share line counts the rank's own bytes
    value = (own_bytes if share else total) * args.steps / dt / 1e9
    if rank == 0:
        out = {
            "metric": "GB/s chunked+SHA-256 (restic CDC)",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 volume image, device-resident)",
            "config": {"workload": (f"C3 rank {sr} of {sw}: its {own_bytes >> 30} GiB share of the "
                                    f"{total >> 30} GiB seed-{seed} volume on one GPU (scan, stitch "
                                    f"from the true entry, finish; exit exchange not included)"
                                    if share else
                                    f"C2: {total >> 30} GiB volume, restic CDC + SHA-256, 1 GPU"
                                    if world == 1 else
                                    f"{'C3' if total == 1 << 40 else 'C3-shape'}: {total >> 30} GiB "
                                    f"volume (seed {seed}) byte-range sharded over {world} GPUs "
                                    f"({per >> 30} GiB per GPU)"),
                       "seed": seed,
                       "volume_bytes": total, "per_gpu_bytes": per, "chunks": nch,
                       "pol": "0x3DA3358B4DC173", "min": MinSize, "max": MaxSize, "avg_bits": 20,
                       "parallelism": f"byte-range shards x{world}"},
            "roofline": roofline,
            "stages_ms_per_step": {k: round(v, 3) for k, v in per_step.items()},
            "kernels": roof,
            # the whole step shares one resource: VALU issue (fingerprint +
            # SHA-256 lane-ops over the step time, each priced by its mix)
            "pipeline_valu_frac": round((own_bytes if share else total) * args.steps / dt
                                        / (1 if share else world) / 1e12
                                        * (SHA_OPS_PER_BYTE * SHA_MIX_CYC + FP_OPS_PER_BYTE * FP_MIX_CYC)
                                        / ISSUE_LANE_CYC, 4),
            "hash_slice_blocks": args.hash_slice,
            "hash_stream": args.hash_stream,
            "hash_wide": args.hash_wide, "wide_drain": args.wide_drain,
            "sha_slices": launches[2],
            "rccl_world_size": dist.get_world_size() if world > 1 else 1,
            "dist_backend": dist.get_backend() if world > 1 else None,
            "exchange_rounds_last_step": xst.get("exchange_rounds", 0),
            # companion values, not the headline: one volume once (no replay,
            # nothing carried across volumes), per GPU and whole job
            "single_pass": {"ms": round(lat * 1e3, 2),
                            "GBps_per_gpu": round(own_bytes / lat / 1e9, 2),
                            "GBps": round((own_bytes if share else total) / lat / 1e9, 2),
                            "stages_ms": iso,
                            "latency_mode_chains": iso_detail["quad_chains"],
                            "same_chunk_list": single_ok},
            "exact": {"chunks": nch, "digest": cdigest},
        }
        gold = gold_all
        if share:
            out["exact"]["entry"] = share_entry
            out["exact"]["entry_source"] = "golden" if gold_rank else "speculative (no golden)"
            if gold_rank:
                out["exact"]["golden_match"] = ((gold_rank["chunks"], gold_rank["digest"])
                                                == (nch, cdigest))
        elif gold and gold.get("bytes") == total and gold.get("seed") == seed:
            out["exact"]["golden_match"] = (gold["chunks"], gold["digest"]) == (nch, cdigest)
        if distinct is not None:
            out["distinct"] = distinct
        if world == 1 and not args.no_cpu_baseline and not share:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_gib << 30, args.cpu_threads)
        print(json.dumps(out), flush=True)
    dc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
