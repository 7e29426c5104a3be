"""The drop-in behind the reference's own pipeline.

``tests/golden/pipeline_phrases.json`` holds the phrases that /root/reference/tone/pipeline.py itself produced
(``forward_offline``, and ``forward`` chunk by chunk + ``finalize``) with ``tone_amd.StreamingCTCModel`` bound as
its model over a CPU stand-in session (tests/golden/make_golden_pipeline.py).  The reference cannot travel to the
GPU box, so here:

* CPU: the restated splitter + greedy decoder (oracle/tone_decode_oracle.py) over the oracle's logprobs
  reproduce the reference pipeline's phrases -- the restatement is pinned to pipeline.py, not only to the
  splitter / decoder composed by hand (golden_decode.npz);
* GPU: the MI355X drop-in (``StreamingCTCModel`` over ``ToneSession``, numpy in / out, B = 1 per call exactly as
  pipeline.py:146 calls it) through that restated post-processing gives the same phrases and times.
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

import tone_amd.config as C
import tone_decode_oracle as O
from tone_amd.weights import synthetic_weights

GOLDEN = Path(__file__).parent / "golden"
FIX = json.loads((GOLDEN / "pipeline_phrases.json").read_text())


def _weights(variant: str) -> dict:
    w = synthetic_weights(0)
    if variant == "blank":
        b = w["decoder.decoder_layers.0.bias"].copy()
        b[34] += FIX["blank_shift"]
        w["decoder.decoder_layers.0.bias"] = b
    return w


def _audio(name: str) -> np.ndarray:
    return np.load(GOLDEN / f"{name}_pcm.npy").astype(np.int32)


def _chunks(pcm: np.ndarray) -> np.ndarray:
    padded = np.pad(pcm, (O.PADDING, O.PADDING))                        # pipeline.py:191
    return np.pad(padded, (0, -len(padded) % C.AUDIO_CHUNK_SAMPLES)).reshape(-1, C.AUDIO_CHUNK_SAMPLES)


def _run(step, pcm: np.ndarray) -> tuple[list, list]:
    """``step(chunk (2400,) int32) -> logprobs (10, 35)`` with the model state inside; the offline phrases
    (is_last on the final chunk) and the online ones (no is_last, then finalize's zero chunk with is_last)."""
    chunks = _chunks(pcm)
    lps = [step(ch) for ch in chunks]
    lps.append(step(np.zeros(C.AUDIO_CHUNK_SAMPLES, np.int32)))           # finalize (pipeline.py:205-217)
    off, on, so, sn = [], [], None, None
    for i, lp in enumerate(lps[:-1]):
        r, so = O.pipeline_step(lp, so, i == len(chunks) - 1)
        off += r
        r, sn = O.pipeline_step(lp, sn, False)
        on += r
    r, sn = O.pipeline_step(lps[-1], sn, True)
    on += r
    return [list(p) for p in off], [list(p) for p in on]


def _check(name: str, off: list, on: list) -> None:
    ref = FIX[name]
    for got, want in ((off, ref["forward_offline"]), (on, ref["forward_finalize"])):
        assert [p[0] for p in got] == [p[0] for p in want], name
        np.testing.assert_allclose([p[1:] for p in got], [p[1:] for p in want], atol=1e-9, err_msg=name)


@pytest.mark.parametrize("variant", ["plain", "blank"])
def test_restated_postprocessing_reproduces_reference_pipeline(variant):
    from tone_oracle import ToneOracle
    orc = ToneOracle(_weights(variant))
    st = [None]

    def step(ch):
        lp, st[0] = orc.step(ch[None], st[0])
        return lp[0]

    _check(f"{variant}/audio_short", *_run(step, _audio("audio_short")))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["plain", "blank"])
@pytest.mark.parametrize("audio", ["audio_short", "audio_long"])
def test_hip_dropin_reproduces_reference_pipeline(variant, audio):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    from tone_amd.model import StreamingCTCModel, ToneSession
    model = StreamingCTCModel(ToneSession(_weights(variant), precision="fp32", max_batch=1))
    st = [None]

    def step(ch):
        lp, st[0] = model.forward(ch[None, :, None], st[0])                # pipeline.py:146
        assert lp.dtype == np.float32 and lp.shape == (1, 10, 35)
        return lp[0]

    try:
        _check(f"{variant}/{audio}", *_run(step, _audio(audio)))
    finally:
        model.session.close()


def test_dropin_io_buffers_are_bounded():
    """StreamingCTCModel keeps device I/O buffers for at most _MAX_IO_SETS distinct batch sizes (LRU)."""
    torch = pytest.importorskip("torch")
    from tone_amd.model import StreamingCTCModel

    class Fake:
        dev, max_batch, frames = torch.device("cpu"), 64, C.CHUNK_FRAMES

        def run(self, signal, state_in, logprobs, state_out, stream=None):
            logprobs.zero_()
            state_out.copy_(state_in)

    m = StreamingCTCModel(Fake())
    for b in (1, 2, 3, 4, 5, 1, 6):
        lp, st = m.forward(np.zeros((b, C.AUDIO_CHUNK_SAMPLES, 1), np.int32))
        assert lp.shape == (b, 10, 35) and st.shape == (b, C.STATE_SIZE)
    assert list(m._buffers) == [4, 5, 1, 6]
