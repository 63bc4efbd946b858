"""ISA checks of the shipped gfx950 code (CPU only: hipcc cross-compiles).

The walk's wide flush issues its LDS reads in inline asm and waits for them
with a hand-placed s_waitcnt (volsync_amd/csrc/rsync_walk.hip wide_issue /
wide_wait): the compiler cannot see those loads, so the compiled code must not
touch their destination VGPRs before the wait (a copy or a spill would read
stale data).  tools/check_lds_asm.py proves that on the device ISA of the
product build flags."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_walk_wide_flush_lds_waits(tmp_path):
    src = os.path.join(ROOT, "volsync_amd", "csrc", "rsync_walk.hip")
    out = tmp_path / "walk.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-x", "hip", src, "-o", str(out)], check=True, capture_output=True, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_lds_asm.py"), str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "0 reads of in-flight" in r.stdout
    # the check is live: a copy of a pending destination is reported
    lines = out.read_text().splitlines()
    k = next(i for i, l in enumerate(lines) if l.strip().startswith("ds_read_b64 v["))
    dst = lines[k].split()[1].split(":")[0].replace("v[", "v").rstrip(",")
    mut = tmp_path / "mut.s"
    mut.write_text("\n".join(lines[:k + 1] + [f"\tv_mov_b32 v250, {dst}"] + lines[k + 1:]) + "\n")
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_lds_asm.py"), str(mut)],
                        capture_output=True, text=True, timeout=300)
    assert r2.returncode == 1 and "1 reads of in-flight" in r2.stdout, r2.stdout[-1000:]
