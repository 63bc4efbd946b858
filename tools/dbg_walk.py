"""Debug driver: one small rsync match through the device walk (VSGPU_LIB may
point at a tracing build), compared with the C oracle."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import rsync_ref as R  # noqa: E402
from tests import oracle_lib as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3 << 20
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
basis = O.synth(4, 0, n)
bl, s2l, cnt, rem = O.rsync_sizes(n, bs)
src = R.mutate(basis, bl, seed=5, frac=0.1)
c1, c2 = O.rsync_signatures(basis, bl, s2l, R.CSUM_XXH3_128, 7)
want, fa = O.rsync_match(src, c1, c2, bl, rem, R.CSUM_XXH3_128, 7)
print("oracle", len(want), fa, want[:5], "sum1[0] %08x" % c1[0], bytes(c2[0]).hex(), "w0 %08x" % O.lib().ref_rsync_checksum1(src.ctypes.data, bl), flush=True)
from volsync_amd import SumStruct, match_sums  # noqa: E402
t = time.time()
got = match_sums(src, SumStruct(n, cnt, bl, s2l, rem, c1, c2), R.CSUM_XXH3_128, 7)
print("device", len(got), time.time() - t, flush=True)
bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
print("equal", got == want, "first diff", bad[:3], [(got[i], want[i]) for i in bad[:3]], flush=True)
