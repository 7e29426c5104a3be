"""Probe: bf16 / fp8 stage-by-stage against the oracle at large batch (the routes of configs 3-5), 8 sampled streams,
per (stream, frame) row the largest element error against the row's largest value, per stage -- to size the bound of
tests/test_gpu_parity.py::test_lowprec_stagewise_large_batch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch

import tone_amd.config as C
from test_gpu_parity import synthetic_pcm
from tone_amd.model import ToneSession
from tone_amd.weights import synthetic_weights
from tone_oracle import ToneOracle

w = synthetic_weights(0)
oracle = ToneOracle(w)
for prec, b in (("bf16", 4096), ("fp8", 4096), ("bf16", 2048)):
    s = ToneSession(w, precision=prec, max_batch=b)
    rng = np.random.default_rng(31)
    pick = np.sort(rng.choice(b, 8, replace=False))
    pcm0 = synthetic_pcm(rng, b, 0.0)
    pcm1 = synthetic_pcm(rng, b, 0.0)
    st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
    _, st = s.step(torch.from_numpy(pcm0).to(s.dev), st)
    st_np = st.cpu().numpy()
    trace = []
    oracle.step(pcm1[pick], st_np[pick], trace=trace)
    out = []
    for stage, ref in enumerate(trace):
        if stage == 0:
            continue
        s.debug_stop(stage)
        s.step(torch.from_numpy(pcm1).to(s.dev), st.clone())
        layer = stage - 2
        reduced = C.REDUCTION_POS <= layer < C.UPSAMPLE_POS
        t = 5 if reduced else 10
        got = s.debug_read("rB" if reduced else "rA", (b, t, C.D_MODEL))[pick]
        r = np.abs(got - ref).max(-1) / np.abs(ref).max(-1)
        out.append((stage, float(r.max()), float(np.median(r))))
    s.debug_stop(-1)
    s.close()
    print(prec, b, " ".join(f"{st_}:{mx:.3f}/{md:.3f}" for st_, mx, md in out), flush=True)
