"""Probe: bf16 / fp8 pre-encode stage (sub_conv_bf16 + Linear + out_norm) vs the oracle, per-element error stats at
B = 3 and 64 (to size a max-element bound for tests/test_gpu_parity.py::test_bf16_pre_encode_stage)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np

import tone_amd.config as C
from test_gpu_parity import gpu_step, synthetic_pcm
from tone_amd.model import ToneSession
from tone_amd.weights import synthetic_weights
from tone_oracle import ToneOracle

w = synthetic_weights(0)
oracle = ToneOracle(w)
for prec in ("bf16", "fp8"):
    for b in (3, 64):
        s = ToneSession(w, precision=prec, max_batch=b)
        rng = np.random.default_rng(23)
        _, st0 = oracle.step(synthetic_pcm(rng, b, 0.0), None)
        pcm = synthetic_pcm(rng, b, 0.0)
        trace = []
        oracle.step(pcm, st0, trace=trace)
        s.debug_stop(1)
        gpu_step(s, pcm, st0)
        got = s.debug_read("rA", (b, 10, C.D_MODEL))
        s.debug_stop(-1)
        s.close()
        ref = trace[1]
        d = np.abs(got - ref)
        rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        rowmax = (d.max(-1) / np.abs(ref).max(-1))
        print(prec, b, "relL2 %.3g" % rel, "max|d| %.3g" % d.max(), "max|ref| %.3g" % np.abs(ref).max(),
              "worst row max|d|/max|ref_row| %.3g" % rowmax.max(), "median %.3g" % np.median(rowmax), flush=True)
