"""Phrases from the REFERENCE's own ``StreamingCTCPipeline`` (tone/pipeline.py) driving the drop-in model class.

Run in the build container (needs /root/reference; the fixtures travel, the reference does not):

    python tests/golden/make_golden_pipeline.py

What runs is /root/reference/tone/pipeline.py itself -- ``forward_offline`` (pipeline.py:174-203) and the
online ``forward`` + ``finalize`` loop (:111-172, :205-217) -- with the reference's own
``StreamingLogprobSplitter`` and ``GreedyCTCDecoder``.  The acoustic model is ``tone_amd.StreamingCTCModel``
(the drop-in: its input validation, zero-state creation, batch split and numpy outputs all run) bound as
``tone.pipeline.StreamingCTCModel``; only the device session under it is replaced by a CPU stand-in that
steps ``oracle/tone_oracle.py`` (no GPU here), so the phrases are the ones the MI355X path must reproduce
(tests/test_pipeline_dropin.py).

Stubs, none of them on the arithmetic path: ``tone/__init__.py`` bypassed with a bare package,
``onnxruntime`` (only ``InferenceSession`` is named, onnx_wrapper.py:77) and ``pyctcdecode`` (only the beam
decoder uses it, decoder.py:15-16) as empty modules.  Audio: audio_short.flac / audio_long.flac decoded by
``tone_amd.flac`` (STREAMINFO MD5 verified), exactly read_example_audio()'s PCM.

Fixtures: tests/golden/pipeline_phrases.json, tests/golden/audio_long_pcm.npy.  Weights: synthetic_weights(0)
("plain": random weights call every frame speech, one phrase per file) and the same with the blank logit's bias
raised by BLANK_SHIFT ("blank"), which puts the splitter's speech test (exp(lp[33]) + exp(lp[34]) <= 0.9,
logprob_splitter.py:134) near its threshold, so phrase boundaries and times depend on individual frames.
"""

from __future__ import annotations

import json
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]

import tone_amd.config as C  # noqa: E402
from tone_amd.flac import read_audio  # noqa: E402
from tone_amd.model import StreamingCTCModel  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402


def install_stubs() -> None:
    pkg = types.ModuleType("tone")
    pkg.__path__ = [str(REF / "tone")]
    sys.modules["tone"] = pkg
    ort = types.ModuleType("onnxruntime")
    ort.InferenceSession = object
    sys.modules["onnxruntime"] = ort
    pc = types.ModuleType("pyctcdecode")
    pcd = types.ModuleType("pyctcdecode.decoder")
    pcd.BeamSearchDecoderCTC = object
    pcd.build_ctcdecoder = lambda *a, **k: None
    pc.decoder = pcd
    sys.modules["pyctcdecode"] = pc
    sys.modules["pyctcdecode.decoder"] = pcd


class OracleSession:
    """CPU stand-in for tone_amd.model.ToneSession: same ``run`` contract (torch tensors in, written in place),
    the step computed by the numpy oracle."""

    def __init__(self, weights: dict):
        import torch
        from tone_oracle import ToneOracle
        self.oracle = ToneOracle(weights)
        self.dev = torch.device("cpu")
        self.max_batch = 1
        self.frames = C.CHUNK_FRAMES

    def run(self, signal, state_in, logprobs, state_out, stream=None) -> None:
        import torch
        lp, st = self.oracle.step(signal.numpy(), state_in.numpy())
        logprobs.copy_(torch.from_numpy(lp))
        state_out.copy_(torch.from_numpy(st))


BLANK_SHIFT = 7.75


def pipeline_weights(variant: str) -> dict:
    w = synthetic_weights(0)
    if variant == "blank":
        b = w["decoder.decoder_layers.0.bias"].copy()
        b[34] += BLANK_SHIFT
        w["decoder.decoder_layers.0.bias"] = b
    return w


def phrases(ps) -> list:
    return [[p.text, float(p.start_time), float(p.end_time)] for p in ps]


def main() -> None:
    install_stubs()
    import tone.pipeline as tp
    from tone.decoder import GreedyCTCDecoder
    from tone.logprob_splitter import StreamingLogprobSplitter

    tp.StreamingCTCModel = StreamingCTCModel          # the drop-in bound where the pipeline looks it up
    out = {"blank_shift": BLANK_SHIFT}
    long_pcm = read_audio(REF / "tone/demo/audio_examples/audio_long.flac")
    np.save(HERE / "audio_long_pcm.npy", long_pcm.astype(np.int16))
    for variant, name, pcm in [(v, n, x) for v in ("plain", "blank") for n, x in (
            ("audio_short", np.load(HERE / "audio_short_pcm.npy").astype(np.int32)),
            ("audio_long", long_pcm.astype(np.int32)))]:
        model = StreamingCTCModel(OracleSession(pipeline_weights(variant)))
        pipe = tp.StreamingCTCPipeline(model, StreamingLogprobSplitter(), GreedyCTCDecoder())
        off = phrases(pipe.forward_offline(pcm))
        # online: the padded signal in 2400-sample chunks through forward(), then finalize()
        padded = np.pad(pcm, (tp.StreamingCTCPipeline.PADDING, tp.StreamingCTCPipeline.PADDING))
        padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
        state, online = None, []
        for ch in padded:
            ps, state = pipe.forward(ch, state)
            online += phrases(ps)
        ps, _ = pipe.finalize(state)
        online += phrases(ps)
        out[f"{variant}/{name}"] = {"forward_offline": off, "forward_finalize": online, "chunks": int(len(padded))}
        print(variant, name, len(padded), "chunks;", len(off), "phrases offline,", len(online), "online")
    (HERE / "pipeline_phrases.json").write_text(json.dumps(out, ensure_ascii=False, indent=1) + "\n")


if __name__ == "__main__":
    main()
