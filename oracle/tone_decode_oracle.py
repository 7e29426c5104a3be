"""CPU oracle for the decode side of the pipeline (TEST INFRASTRUCTURE ONLY).

Restates, on log-probabilities exactly as the reference consumes them:

  * ``GreedyCTCDecoder.forward``          tone/decoder.py:41-59   argmax per frame, collapse runs,
                                                                  drop blank (34), strip
  * ``StreamingLogprobSplitter.forward``  tone/logprob_splitter.py:90-156  speech = exp(lp[33]) +
    and ``_iterate_over_phrases``        tone/logprob_splitter.py:61-88   exp(lp[34]) <= 0.9; phrases
                                                                  between silences >= 20 frames,
                                                                  forced split at 2000, +-3 frames
  * the phrase timing of ``StreamingCTCPipeline.forward``  tone/pipeline.py:141-176

Only ``tests/`` may import it; the product's frame-based decoder (``tone_amd.pipeline``) works on
the device-computed ``frame_info`` (token | speech << 8) instead of logprobs.

Parity pin: ``tests/golden/golden_decode.npz`` holds phrases produced by the reference's own
``StreamingLogprobSplitter`` (imported from /root/reference by ``tests/golden/make_golden_decode.py``)
on seeded synthetic logprob streams; ``tests/test_decode.py`` checks this restatement against them.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

LABELS = "абвгдеёжзийклмнопрстуфхцчшщъыьэюя "   # decoder.py:24; blank = 34 = len(LABELS)
SILENCE_THRESHOLD = 0.9       # logprob_splitter.py:57
MIN_SILENCE = 20              # :58
EXPAND = 3                    # :59
MAX_PHRASE = 2000             # :60
FRAME_SIZE = 0.03             # onnx_wrapper.py:33
MEAN_TIME_BIAS = 0.33         # onnx_wrapper.py:31
PADDING = 2400                # pipeline.py:40
SAMPLE_RATE = 8000


def greedy_text(logprobs: np.ndarray) -> str:
    toks = np.argmax(logprobs, axis=-1)
    out = []
    prev = None
    for t in toks.tolist():
        if t != prev and t < len(LABELS):
            out.append(LABELS[t])
        prev = t
    return "".join(out).strip()


def speech_mask(logprobs: np.ndarray) -> np.ndarray:
    return np.exp(logprobs[..., -2:]).sum(axis=-1) <= SILENCE_THRESHOLD


def phrase_bounds(is_speech: np.ndarray, is_last: bool) -> list[tuple[int, int]]:
    """(start, end) frame pairs of finished phrases in a buffer of len(is_speech) frames."""
    n = len(is_speech)
    lead = MIN_SILENCE
    sil = np.concatenate([np.ones(lead, bool), ~is_speech.astype(bool),
                          np.ones(MIN_SILENCE if is_last else 0, bool)])
    # maximal silence runs [s, e) in buffer coordinates
    runs = []
    i = 0
    while i < len(sil):
        if sil[i]:
            j = i
            while j < len(sil) and sil[j]:
                j += 1
            runs.append((i - lead, j - lead))
            i = j
        else:
            i += 1
    seps = [r for r in runs if r[1] - r[0] >= MIN_SILENCE]
    out = []
    for k, (_, s_end) in enumerate(seps):
        start = s_end
        end = seps[k + 1][0] if k + 1 < len(seps) else n
        while end - start >= MAX_PHRASE:
            out.append((start, start + MAX_PHRASE))
            start += MAX_PHRASE
        if k + 1 < len(seps):
            out.append((start, end))
    return out


@dataclass
class SplitterState:
    past: np.ndarray = field(default_factory=lambda: np.zeros((0, 35), np.float32))
    offset: int = 0


def splitter_step(logprobs: np.ndarray, state: SplitterState | None, is_last: bool):
    """-> ([(phrase_logprobs, start_frame, end_frame)], next_state)"""
    state = state or SplitterState()
    buf = np.concatenate([state.past, logprobs], axis=0)
    speech = speech_mask(buf)
    phrases = []
    last = 0
    for s, e in phrase_bounds(speech, is_last):
        phrases.append((buf[max(0, s - EXPAND):e + EXPAND], s + state.offset, e + state.offset))
        last = e
    if not speech[last:].any():
        last = max(last, len(buf) - EXPAND)
    return phrases, SplitterState(buf[last:], state.offset + last)


def phrase_times(start_frame: int, end_frame: int) -> tuple[float, float]:
    shift = MEAN_TIME_BIAS + PADDING / SAMPLE_RATE
    st = max(0, round(start_frame * FRAME_SIZE - shift, 2))
    en = max(st, round(end_frame * FRAME_SIZE - shift, 2))
    return st, en


def pipeline_step(logprobs: np.ndarray, state: SplitterState | None, is_last: bool):
    """Splitter + greedy decoder + timing of one pipeline step -> ([(text, t0, t1)], state)."""
    phrases, state = splitter_step(logprobs, state, is_last)
    return [(greedy_text(lp), *phrase_times(s, e)) for lp, s, e in phrases], state
