"""Generate tests/golden/golden_decode.npz from the REFERENCE's own splitter and greedy decoder.

Run in the build container (needs /root/reference, which never travels to the GPU box):

    python tests/golden/make_golden_decode.py

What runs is ``tone.logprob_splitter.StreamingLogprobSplitter.forward`` and
``tone.decoder.GreedyCTCDecoder.forward`` from /root/reference, composed per chunk the way
``StreamingCTCPipeline.forward`` does (tone/pipeline.py:141-176).  ``tone/__init__.py`` is bypassed
with a bare package, and ``pyctcdecode`` (absent, only used by the beam-search decoder in the same
file) is replaced by an empty stub module so that decoder.py imports.

Inputs are seeded synthetic logprob streams (speech runs of random tokens, silences of random length
around the 20-frame separator, speech runs longer than the 2000-frame forced split, frames near the
0.9 silence threshold), fed 10 frames per call with ``is_last`` on the final call.
"""

from __future__ import annotations

import json
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent


def _install_stubs() -> None:
    pkg = types.ModuleType("tone")
    pkg.__path__ = [str(REF / "tone")]
    sys.modules["tone"] = pkg
    pc = types.ModuleType("pyctcdecode")
    pcd = types.ModuleType("pyctcdecode.decoder")
    pcd.BeamSearchDecoderCTC = object
    pcd.build_ctcdecoder = lambda *a, **k: None
    pc.decoder = pcd
    sys.modules["pyctcdecode"] = pc
    sys.modules["pyctcdecode.decoder"] = pcd


def synth_stream(rng: np.random.Generator, n_frames: int, long_speech: bool) -> np.ndarray:
    """[n_frames, 35] float32 log-softmax rows with alternating speech / silence runs."""
    lp = np.empty((n_frames, 35), np.float32)
    t = 0
    speech = bool(rng.integers(2))
    while t < n_frames:
        if speech:
            n = int(rng.integers(2100, 2600)) if (long_speech and rng.random() < 0.3) else int(rng.integers(1, 60))
        else:
            n = int(rng.choice([rng.integers(1, 19), rng.integers(19, 22), rng.integers(22, 60), rng.integers(22, 60)]))
        n = min(n, n_frames - t)
        for k in range(n):
            z = rng.normal(0.0, 1.0, 35).astype(np.float32)
            if speech:
                z[int(rng.integers(0, 34))] += 6.0 + float(rng.normal())
                if rng.random() < 0.1:
                    z[33] += 5.0          # spaces inside speech
            else:
                z[34] += 9.5 + 0.5 * float(rng.normal())
                if rng.random() < 0.03:   # borderline frames around the 0.9 threshold
                    z[int(rng.integers(0, 33))] += 4.5
            m = z.max()
            lp[t + k] = (z - m - np.log(np.exp(z - m).sum())).astype(np.float32)
        t += n
        speech = not speech
    return lp


def main() -> None:
    _install_stubs()
    from tone.decoder import GreedyCTCDecoder
    from tone.logprob_splitter import StreamingLogprobSplitter

    frame_size, time_bias, padding, sr = 0.03, 0.33, 2400, 8000     # onnx_wrapper.py:31-33, pipeline.py:40
    rng = np.random.default_rng(1234)
    streams, phrases = [], []
    for si, (n_frames, long_speech) in enumerate([(600, False), (1200, False), (5200, True), (430, False),
                                                  (3000, True), (10, False)]):
        lp = synth_stream(rng, n_frames, long_speech)
        splitter, decoder = StreamingLogprobSplitter(), GreedyCTCDecoder()
        state = None
        n_chunks = n_frames // 10
        for c in range(n_chunks):
            out, state = splitter.forward(lp[10 * c:10 * c + 10], state, is_last=(c == n_chunks - 1))
            for ph in out:
                text = decoder.forward(ph.logprobs)
                st = max(0, round(ph.start_frame * frame_size - time_bias - padding / sr, 2))
                en = max(st, round(ph.end_frame * frame_size - time_bias - padding / sr, 2))
                phrases.append({"stream": si, "chunk": c, "text": text, "start_frame": int(ph.start_frame),
                                "end_frame": int(ph.end_frame), "start_time": st, "end_time": en,
                                "n_logprob_rows": int(len(ph.logprobs))})
        streams.append(lp)
    lengths = np.array([len(s) for s in streams], np.int64)
    np.savez_compressed(HERE / "golden_decode.npz", logprobs=np.concatenate(streams), lengths=lengths,
                        phrases=np.frombuffer(json.dumps(phrases, ensure_ascii=False).encode(), np.uint8))
    print(f"{len(phrases)} phrases over {len(streams)} streams ({int(lengths.sum())} frames)")


if __name__ == "__main__":
    main()
