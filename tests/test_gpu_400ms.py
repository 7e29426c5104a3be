"""The 400 ms chunk variant on the MI355X (3200 samples -> 13 frames, 6 in the reduced block, the
upsampling pad frame live; tone/scripts/export.py chunk_duration_ms=400, triton/ensemble/config.pbtxt).
The HIP path vs the oracle (itself pinned to forward_for_export at 400 ms, tests/test_oracle.py) on the
golden streams: stage by stage, then 5 stateful chunks with staggered restarts in every precision."""

from pathlib import Path

import numpy as np
import pytest

import tone_amd.config as C
from tone_amd.weights import synthetic_weights

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).parent / "golden"
CHUNK = 3200


@pytest.fixture(scope="module")
def oracle():
    from tone_oracle import ToneOracle
    return ToneOracle(synthetic_weights(0))


def _session(prec, b):
    from tone_amd.model import ToneSession
    return ToneSession(synthetic_weights(0), precision=prec, max_batch=b, chunk_samples=CHUNK)


def _step(s, pcm, st):
    lp, nst = s.step(torch.from_numpy(np.ascontiguousarray(pcm)).to(s.dev), torch.from_numpy(st).to(s.dev))
    return lp.cpu().numpy(), nst.cpu().numpy()


def test_400ms_stagewise(oracle):
    """Front end, pre-encode and every layer of one 400 ms step from a carried state vs the oracle trace."""
    g = np.load(GOLDEN / "golden_400ms.npz")
    pcm, st0 = g["pcm"][:, 3].astype(np.int32), g["step_state_in"]
    trace = []
    oracle.step(pcm, st0, trace=trace)
    s = _session("fp32", 4)
    assert s.frames == 13
    try:
        for stage, ref in enumerate(trace):
            s.debug_stop(stage)
            _step(s, pcm, st0)
            if stage == 0:
                got = s.debug_read("feats", (4, 40, C.N_MELS))
            else:
                t = ref.shape[1]
                got = s.debug_read("rB" if t == 6 else "rA", (4, t, C.D_MODEL))
            err = float(np.abs(got - ref).max())
            assert err < 5e-3, f"stage {stage}: {err:.3g}"   # the 300 ms stagewise bound (test_gpu_parity.py)
    finally:
        s.debug_stop(-1)
        s.close()


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-3), ("fp32-mfma", 1e-3), ("bf16", 0.08), ("fp8", 0.6)])
def test_400ms_streams_vs_oracle(oracle, prec, tol):
    """The 4 golden streams x 5 chunks (staggered restarts) stepped on the GPU and by the oracle, each on
    its own state chain: logprobs (B, 13, 35) within the precision's bound, argmax identical where clear."""
    g = np.load(GOLDEN / "golden_400ms.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    s = _session(prec, B)
    st_g = np.zeros((B, C.STATE_SIZE), np.float16)
    st_o = st_g.copy()
    try:
        for c in range(N):
            st_g[np.arange(B) > c] = 0
            st_o[np.arange(B) > c] = 0
            lp_g, st_g = _step(s, pcm[:, c], st_g)
            lp_o, st_o = oracle.step(pcm[:, c], st_o)
            assert lp_g.shape == (B, 13, 35)
            d = np.abs(lp_g - lp_o)
            assert d.max() < tol, f"{prec} chunk {c}: {d.max():.3g}"
            srt = np.sort(lp_o, -1)
            clear = (srt[..., -1] - srt[..., -2]) > 2 * tol
            np.testing.assert_array_equal(lp_g.argmax(-1)[clear], lp_o.argmax(-1)[clear])
            assert float(st_g[0, C.OFF_MHSA_LEN]) == min(13.0 * (c + 1), 30.0)
    finally:
        s.close()


@pytest.mark.parametrize("prec,b,bounds", [("fp32", 256, (1e-3, 1e-3)), ("bf16", 1024, (0.08, 0.05)),
                                           ("fp8", 1024, (0.6, 0.4))])
def test_400ms_large_batch(oracle, prec, b, bounds):
    """400 ms at the bench's batch: fp32 at B = 256 (the 400 ms leg; its FFN down at M = 3328 / 1536 takes the 3-way
    K-split route), bf16 / fp8 at B = 1024 (the large-M GEMM routes, conv2 as an implicit GEMM): sampled streams at
    the precision's bounds (fp32 1e-3; test_gpu_parity.py BF16_* / FP8_*)."""
    rng = np.random.default_rng(3)
    pick = np.arange(0, b, 64 if b >= 1024 else 16)
    s = _session(prec, b)
    st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
    st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
    try:
        for c in range(3):
            pcm = np.clip(np.round(rng.normal(0, 3000, (b, CHUNK))), -32768, 32767).astype(np.int32)
            lp, st = s.step(torch.from_numpy(pcm).to(s.dev), st)
            lp_o, st_o = oracle.step(pcm[pick], st_o)
            d = np.abs(lp.cpu().numpy()[pick] - lp_o)
            assert d.max() < bounds[0] and np.percentile(d, 99) < bounds[1], (prec, c, d.max())
    finally:
        s.close()
