"""A/B driver: runs one measurement script under several builds of the
product library (VSGPU_LIB), interleaved round-robin so clock drift hits every
variant alike, and prints each variant's lines.
  python tools/ab.py --rounds 2 --libs base=volsync_amd/lib/var/fp_base/libvsgpu.so,new= \
      -- tools/fp_only.py --gib 16
(an empty path = the default in-tree library)"""
import argparse
import os
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--libs", required=True)
ap.add_argument("--timeout", type=int, default=300)
ap.add_argument("cmd", nargs=argparse.REMAINDER)
a = ap.parse_args()
cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = [kv.split("=", 1) for kv in a.libs.split(",")]
for r in range(a.rounds):
    for name, path in libs:
        env = dict(os.environ)
        if path:
            env["VSGPU_LIB"] = os.path.join(root, path)
        else:
            env.pop("VSGPU_LIB", None)
        p = subprocess.run([sys.executable] + cmd, env=env, cwd=root, capture_output=True,
                           text=True, timeout=a.timeout)
        out = [l for l in (p.stdout + p.stderr).splitlines() if "amdgpu.ids" not in l]
        print(f"[{name} r{r}] rc={p.returncode} " + " | ".join(out[-3:]), flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)
