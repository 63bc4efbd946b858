"""Env-knob A/B of the device walk, interleaved, two rounds:
  python tools/ab_seg.py 16,32,64 -- bench.py --mode rsync ...   (VSGPU_WALK_SEGBLOCKS)
  AB_VAR=VSGPU_WALK_TAILPCT python tools/ab_seg.py 0,15,30 -- bench.py ..."""
import os
import subprocess
import sys

var = os.environ.get("AB_VAR", "VSGPU_WALK_SEGBLOCKS")
vals = sys.argv[1].split(",")
cmd = sys.argv[3:] if sys.argv[2] == "--" else sys.argv[2:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for r in range(2):
    for v in vals:
        env = dict(os.environ, **{var: v})
        p = subprocess.run([sys.executable] + cmd, env=env, cwd=root, capture_output=True,
                           text=True, timeout=300)
        out = [l for l in (p.stdout + p.stderr).splitlines() if "amdgpu.ids" not in l]
        print(f"[{var[11:].lower()}{v} r{r}] rc={p.returncode} " + " | ".join(out[-2:]), flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)
