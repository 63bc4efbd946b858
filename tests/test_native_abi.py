"""The C ABI driven from C (tests/native/abi_client.c), as cgo and rsync's
match.c would call it: no Python or torch between the caller and
libvsgpu.so.  The GPU cases compare its output with the golden fixtures."""
import os
import struct
import subprocess
import tempfile

import pytest

from tests import golden_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "tests", "native", "build", "abi_client")


def _client():
    if not os.path.exists(CLIENT):
        import __graft_entry__
        __graft_entry__.build_native_client()
    return CLIENT


def test_client_links_and_loads_library():
    """Runs without a GPU: the C program resolves every vs_* symbol it uses
    from libvsgpu.so at load time and reports the device count (0 here)."""
    r = subprocess.run([_client(), "version"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "gfx950" in r.stdout and "devices=" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name,read_size,batch", [
    ("cdc_synth1_8m.json", 3 << 20, 5 << 20),
    ("cdc_synth1_64m.json", 7 << 20, 24 << 20),
    ("cdc_synth1_1g.json", 64 << 20, 256 << 20),
])
def test_c_chunker_next_vs_golden(gpu, name, read_size, batch):
    doc = G.load(os.path.join(G.GOLDEN, name))
    spec = doc["input"]
    assert spec["kind"] == "synth"
    r = subprocess.run([_client(), "cdc", str(spec["seed"]), str(spec["len"]), str(read_size),
                        str(batch)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = []
    for line in r.stdout.split("\n"):
        if line:
            s, ln, cut, i = line.split()
            got.append((int(s), int(ln), int(cut, 16), i))
    assert got == G.expected(doc)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rsync_c4_4m_xxh128.json", "rsync_c4_4m_md5.json",
                                  "rsync_dup_blocks.json", "rsync_tail_partial.json",
                                  "rsync_src_shorter_than_block.json"])
def test_c_rsync_match_vs_golden(gpu, name):
    doc = G.load(os.path.join(G.GOLDEN, name))
    basis, src = G.rsync_pair(doc["input"])
    p, z = doc["params"], doc["sizes"]
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(struct.pack("<qqiIi", len(basis), len(src), p["csum_type"], p["seed"] & 0xFFFFFFFF,
                            p["block_size"]))
        f.write(basis.tobytes())
        f.write(src.tobytes())
        path = f.name
    try:
        r = subprocess.run([_client(), "rsync", path], capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.split("\n") if ln]
    assert lines[0].split()[1:] == [str(z["blength"]), str(z["s2length"]), str(z["count"]),
                                    str(z["remainder"])]
    got = [tuple(int(x) for x in ln.split()) for ln in lines[1:]]
    assert got == [tuple(m) for m in doc["matches"]]
