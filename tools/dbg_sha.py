import sys, hashlib, numpy as np
sys.path.insert(0, '.')
import torch
from tests import golden_util as G
from volsync_amd import DeviceChunker, sha256_batch
doc = G.load('tests/golden/cdc_small_params.json')
data = G.make_input(doc['input']); pol, mn, mx, ab = G.params(doc)
t = torch.from_numpy(data).cuda(); torch.cuda.synchronize()
dc = DeviceChunker(pol, mn, mx, ab); n, _ = dc.process(t.data_ptr(), len(data), 0, True)
ch = dc.chunks(0, n)
bad = [(i, c.Start, c.Length) for i, c in enumerate(ch) if hashlib.sha256(data[c.Start:c.Start+c.Length].tobytes()).digest() != c.ID]
print("n", n, "bad", len(bad), bad[:20])
# batch API on the same blobs
ids = sha256_batch(data.tobytes(), [c.Start for c in ch], [c.Length for c in ch])
bad2 = [i for i, c in enumerate(ch) if ids[i] != hashlib.sha256(data[c.Start:c.Start+c.Length].tobytes()).digest()]
print("batch bad", len(bad2), bad2[:20])
# single blobs
for i in [0, 1, 2]:
    c = ch[i]
    one = sha256_batch(data.tobytes(), [c.Start], [c.Length])[0]
    print(i, c.Start, c.Length, one == hashlib.sha256(data[c.Start:c.Start+c.Length].tobytes()).digest())
