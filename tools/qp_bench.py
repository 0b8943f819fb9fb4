import sys, numpy as np
sys.path.insert(0, '/root/repo')
import myscaledb_amd as mq
from oracle import oracle as O
mq.init(0)
for metric, d, mode in (("Cosine", 768, 2), ("L2", 768, 2), ("Cosine", 128, 2), ("Cosine", 768, 0)):
    seg = mq.VectorScanSegment.generate(0x5EED0001, mode, 1000, d, metric=metric)
    q = O.generate(0x5EED0001, mode, 5000, 1000, d)
    cand = np.zeros((1000, 1), np.int64)
    for _ in range(3):
        seg.rerank(q, cand, 1)
    seg.free()
print("done")
