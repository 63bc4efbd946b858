"""bench.py's multi-rank launcher (CPU): `bench.py --gpus N` outside a
torch.distributed launcher starts one itself as a child process, and the
--dry rehearsal runs the real byte-range protocol (volsync_amd/shard.py) over
gloo with N ranks, reporting n_gpus / world_size N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launch_dry():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry",
                        "--per-gpu-gib", "1"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size"] == 2 and out["dry"] is True
    assert out["exchange_rounds"] >= 1
    assert out["protocol_matches_single_rank"] is True
    assert out["value"] is None
