"""The torch-CPU restatement timed as bench.py's cpu_baseline computes the same step as the numpy
oracle: one step from zero state to fp32 reassociation error (measured 9e-6), and the 6-chunk
staggered golden streams within 1e-3 (measured 3.1e-4: fp16 state-rounding flips accumulate, as
between the oracle and the reference itself, tests/test_oracle.py)."""

from pathlib import Path

import numpy as np
import torch

import tone_amd.config as C
from tone_amd.weights import synthetic_weights
from tone_cpu import ToneCPU
from tone_oracle import ToneOracle

GOLDEN = Path(__file__).parent / "golden"


def test_cpu_restatement_matches_oracle():
    w = synthetic_weights(0)
    orc, cpu = ToneOracle(w), ToneCPU(w)
    g = np.load(GOLDEN / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    so = np.zeros((B, C.STATE_SIZE), np.float16)
    sc = torch.zeros((B, C.STATE_SIZE), dtype=torch.float16)
    for c in range(N):
        so[np.arange(B) > c] = 0
        sc[torch.arange(B) > c] = 0
        lo, so = orc.step(pcm[:, c], so)
        lc, sc = cpu.step(torch.from_numpy(pcm[:, c]), sc)
        d = float(np.abs(lc.numpy() - lo).max())
        assert d < (5e-5 if c == 0 else 1e-3), (c, d)
        np.testing.assert_array_equal(lc.numpy().argmax(-1), lo.argmax(-1))
        assert np.mean(sc.numpy() == so) > 0.95
