"""The shard protocols' collectives on RCCL (backend "nccl", device tensors).

The GPU box has one GPU, so this runs the distributed code paths of
volsync_amd.shard / rsync_shard at world size 1 in a child process
(tests/rccl_world1.py): the communicator comes up on cuda:0, and the CDC exit
exchange, the signature all-gather and the walk's (offset, want_i) exchange go
through real RCCL calls on device tensors, exact against the C oracle.  The
world >= 2 exchange logic is covered over gloo on the CPU
(test_shard_protocol.py, test_rsync_shard.py, test_rsync_walk_shard.py).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_protocols_over_rccl_world1(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("MASTER_PORT", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_world1.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    res = json.loads(lines[-1])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["cdc_exact"] and res["sums_exact"] and res["walk_exact"] and res["collective_exact"]
    assert res["cdc_chunks"] > 10 and res["walk_matches"] > 10
