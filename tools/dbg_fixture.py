"""Debug driver: one rsync golden fixture through match_sums, diff vs expected."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from tests import golden_util as G  # noqa: E402
from volsync_amd import SumStruct, match_sums  # noqa: E402

doc = G.load(os.path.join(G.GOLDEN, sys.argv[1]))
_, src = G.rsync_pair(doc["input"])
p, z = doc["params"], doc["sizes"]
s = SumStruct(0, z["count"], z["blength"], z["s2length"], z["remainder"],
              np.array(doc["sum1"], np.uint32),
              np.array([list(bytes.fromhex(h)) for h in doc["sum2"]], np.uint8).reshape(
                  z["count"], z["s2length"]))
got = match_sums(src, s, p["csum_type"], p["seed"])
want = [tuple(m) for m in doc["matches"]]
print("equal", got == want, len(got), len(want), got[-3:], want[-3:], flush=True)
