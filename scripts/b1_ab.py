"""B = 1 drop-in A/B in one process: pageable vs pinned staging (StreamingCTCModel._pinned), alternating blocks."""
import json
import time

import numpy as np
import torch

import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tone_amd.model import StreamingCTCModel, ToneSession

sess = ToneSession(bench.replica_weights(None, None), device=0, precision="fp32", max_batch=1)
pcm = bench.synthetic_pcm(np.random.default_rng(7), 1, 8)[:, :, :, None]
res = {"pageable": [], "pinned": []}
for rep in range(6):
    for mode in ("pageable", "pinned"):
        m = StreamingCTCModel(sess)
        m._pinned = mode == "pinned"
        st = None
        for i in range(5):
            _, st = m.forward(pcm[i % 8], st)
        for i in range(100):
            t0 = time.perf_counter()
            _, st = m.forward(pcm[i % 8], st)
            res[mode].append(time.perf_counter() - t0)
print(json.dumps({k: round(float(np.median(v)) * 1e3, 4) for k, v in res.items()}))
