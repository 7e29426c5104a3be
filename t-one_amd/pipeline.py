"""Batched streaming recognition on the device frame info.

The reference pipeline (tone/pipeline.py:141-176) moves a (10, 35) fp32 logprob block per stream and
chunk to the host, where ``StreamingLogprobSplitter`` thresholds exp(lp[33]) + exp(lp[34]) and
``GreedyCTCDecoder`` takes the argmax.  Here the head kernel already emits both per frame
(``frame_info`` = token | speech << 8, include/tonehip.h), so one step returns 10 int32 per stream
and the splitter / greedy decoder below run on (token, speech) frames with the reference's rules:

  * phrase boundaries       logprob_splitter.py:61-88   silences >= 20 frames separate phrases,
                                                       speech longer than 2000 frames is force-split,
                                                       only finished phrases are emitted
  * phrase extent           logprob_splitter.py:136-156 +-3 frames around the phrase, buffer kept
                                                       from the last phrase end (or last 3 frames)
  * greedy text             decoder.py:57-59            collapse repeats, drop blank (34), strip
  * phrase times            pipeline.py:151-168

``StreamingGreedyPipeline`` serves many concurrent streams from one ``ToneSession``: each stream owns
two rows of a device-resident state slab used in ping-pong and (resident form, the default) one conv-cache
ring updated in place, every step runs the streams that have audio as one batch through
``tone_session_run_ring`` (``tone_session_run_rows`` with ``resident=False``: read one row, write the other;
streams without audio are not touched, no state is copied), and only the frame info crosses PCIe.
``StreamScheduler`` puts an arrival queue in front of it (the role Triton's dynamic / sequence
batcher plays for the reference, configs/streaming_acoustic/config.pbtxt:35-37,
triton/model/config.pbtxt:26-69): chunks arrive per stream at any time, each step packs up to
``max_batch`` streams that have a chunk waiting (oldest waiting chunk first, one chunk per stream per
step so every stream's chunks run in order) into one device batch.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import config as C

LABELS = "абвгдеёжзийклмнопрстуфхцчшщъыьэюя "   # tone/decoder.py:24; token 34 = blank
MIN_SILENCE = 20        # logprob_splitter.py:58
SPEECH_EXPAND = 3       # logprob_splitter.py:59
MAX_PHRASE = 2000       # logprob_splitter.py:60
PADDING = 2400          # pipeline.py:40 (300 ms of left/right padding used by forward_offline)
STATE_STRIDE = 219776   # slab row stride: 219729 rounded up to 64 elements (128-byte aligned rows)


@dataclass
class TextPhrase:
    """tone/pipeline.py:16-27."""
    text: str
    start_time: float
    end_time: float


@dataclass
class FrameSplitterState:
    """Frames carried between steps (the reference keeps the logprob rows, logprob_splitter.py:36-40).
    ``tokens`` is the per-frame payload: greedy tokens (L,) int32, or the logprob rows (L, 35) float32
    when a host decoder (e.g. the reference's BeamSearchCTCDecoder + KenLM) decodes the phrases."""
    tokens: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    speech: np.ndarray = field(default_factory=lambda: np.zeros(0, bool))
    offset: int = 0


def decode_frame_info(info: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    info = np.asarray(info, np.int32)
    return (info & 0xFF).astype(np.int32), (info >> 8).astype(bool)


def greedy_text(tokens: np.ndarray) -> str:
    toks = np.asarray(tokens)
    if toks.size == 0:
        return ""
    keep = np.ones(toks.size, bool)
    keep[1:] = toks[1:] != toks[:-1]
    toks = toks[keep]
    return "".join(LABELS[t] for t in toks.tolist() if t < len(LABELS)).strip()


def _phrases(speech: np.ndarray, is_last: bool) -> list[tuple[int, int]]:
    n = speech.size
    silent = np.concatenate([np.ones(MIN_SILENCE, bool), ~speech, np.ones(MIN_SILENCE if is_last else 0, bool)])
    edges = np.diff(np.concatenate([[0], silent.astype(np.int8), [0]]))
    starts = np.flatnonzero(edges == 1) - MIN_SILENCE
    ends = np.flatnonzero(edges == -1) - MIN_SILENCE
    sep = (ends - starts) >= MIN_SILENCE
    starts, ends = starts[sep].tolist(), ends[sep].tolist()
    out = []
    for k, beg in enumerate(ends):
        stop = starts[k + 1] if k + 1 < len(starts) else n
        while stop - beg >= MAX_PHRASE:
            out.append((beg, beg + MAX_PHRASE))
            beg += MAX_PHRASE
        if k + 1 < len(starts):
            out.append((beg, stop))
    return out


def split_frames(tokens: np.ndarray, speech: np.ndarray, state: Optional[FrameSplitterState], *,
                 is_last: bool = False) -> tuple[list[tuple[np.ndarray, int, int]], FrameSplitterState]:
    """One splitter step on frames -> ([(phrase tokens, start_frame, end_frame)], next state)."""
    state = state or FrameSplitterState()
    tokens = np.asarray(tokens)
    toks = np.concatenate([state.tokens.astype(tokens.dtype, copy=False).reshape((-1,) + tokens.shape[1:]), tokens])
    sp = np.concatenate([state.speech, np.asarray(speech, bool)])
    out, last = [], 0
    for s, e in _phrases(sp, is_last):
        out.append((toks[max(0, s - SPEECH_EXPAND):e + SPEECH_EXPAND], s + state.offset, e + state.offset))
        last = e
    if not sp[last:].any():
        last = max(last, sp.size - SPEECH_EXPAND)
    return out, FrameSplitterState(toks[last:], sp[last:], state.offset + last)


def phrase_times(start_frame: int, end_frame: int) -> tuple[float, float]:
    shift = C.MEAN_TIME_BIAS + PADDING / C.SAMPLE_RATE
    st = max(0, round(start_frame * C.FRAME_SIZE - shift, 2))
    return st, max(st, round(end_frame * C.FRAME_SIZE - shift, 2))


def frames_to_phrases(tokens, speech, state, *, is_last=False, decode=greedy_text
                      ) -> tuple[list[TextPhrase], FrameSplitterState]:
    """``decode`` maps a phrase's payload to its text: greedy_text on tokens, or a host decoder's
    ``forward`` on logprob rows (tone/pipeline.py:147-150 calls ``self.decoder.forward``)."""
    found, state = split_frames(tokens, speech, state, is_last=is_last)
    return [TextPhrase(decode(t), *phrase_times(s, e)) for t, s, e in found], state


class StreamingGreedyPipeline:
    """Many concurrent streams, one device batch per step, greedy CTC decoding on device frame info.

    Drop-in counterpart of ``StreamingCTCPipeline(model, StreamingLogprobSplitter(), GreedyCTCDecoder())``
    (tone/pipeline.py) for a server: ``open_stream`` / ``close_stream`` manage slots of the device
    state slab, ``forward`` advances any subset of open streams by one 300 ms chunk each.

    Slot s owns slab rows 2s and 2s+1; ``_parity[s]`` says which one holds its current state.  A
    step reads row 2s + p and writes row 2s + 1 - p for the stepping streams only.  With ``resident`` (default)
    slot s also owns conv ring s (include/tonehip.h tone_session_run_ring: the conv caches, 84 % of the state,
    updated in place -- only the step's new frames are written); ``state_of`` then exports the flat state.

    ``decoder``: optional host decoder with the reference's ``forward(logprobs (L, 35) float32) -> str``
    (``tone.decoder.BeamSearchCTCDecoder`` -- pyctcdecode + KenLM, BASELINE config 5 -- or
    ``GreedyCTCDecoder``).  With it the step's logprobs come to the host (1.4 KB per stream-chunk),
    phrases are still cut by the device speech flags, and each finished phrase's logprob rows go to
    ``decoder.forward`` exactly as tone/pipeline.py:146-150 does.  Without it the text is the device's
    greedy tokens (10 ids + 10 bits per stream-chunk cross PCIe).
    """

    CHUNK_SIZE = C.AUDIO_CHUNK_SAMPLES   # 300 ms; a session built with chunk_samples=3200 serves 400 ms chunks

    def __init__(self, session, n_slots: int, decoder=None, resident: bool = True):
        import torch
        if n_slots <= 0:
            raise ValueError("n_slots must be positive")
        self.session = session
        self.n_slots = int(n_slots)
        self.CHUNK_SIZE = int(getattr(session, "chunk_samples", C.AUDIO_CHUNK_SAMPLES))
        self.frames = fr = int(getattr(session, "frames", C.CHUNK_FRAMES))
        dev = session.dev
        self._slab = torch.zeros((2 * self.n_slots, STATE_STRIDE), dtype=torch.float16, device=dev)
        self.resident = bool(resident)
        self._rings = torch.zeros((self.n_slots, session.ring_elems), dtype=torch.float16, device=dev) \
            if self.resident else None
        self._parity = np.zeros(self.n_slots, np.int32)
        self._open: dict[int, FrameSplitterState] = {}
        self._free = list(range(self.n_slots - 1, -1, -1))
        mb = session.max_batch
        # fixed staging buffers: the device pointers stay the same across steps (hipGraph friendly)
        self._info = torch.zeros((mb, fr), dtype=torch.int32, device=dev)
        self._logp = torch.empty((mb, fr, C.VOCAB), dtype=torch.float32, device=dev)
        self._sig = torch.zeros((mb, self.CHUNK_SIZE), dtype=torch.int32, device=dev)
        self._rows = torch.zeros((3, mb), dtype=torch.int32, device=dev)   # rows read / written, ring ids
        self._sig_h = torch.zeros((mb, self.CHUNK_SIZE), dtype=torch.int32).pin_memory()
        self._rows_h = torch.zeros((3, mb), dtype=torch.int32).pin_memory()
        self._info_h = torch.zeros((mb, fr), dtype=torch.int32).pin_memory()
        self.decoder = decoder
        self._logp_h = torch.zeros((mb, fr, C.VOCAB), dtype=torch.float32).pin_memory() \
            if decoder is not None else None
        self._last_logp: Optional[np.ndarray] = None

    def _fresh_state(self) -> FrameSplitterState:
        if self.decoder is None:
            return FrameSplitterState()
        return FrameSplitterState(tokens=np.zeros((0, C.VOCAB), np.float32))

    # --- slots -------------------------------------------------------------------------------
    def open_stream(self) -> int:
        if not self._free:
            raise RuntimeError(f"all {self.n_slots} stream slots are in use")
        slot = self._free.pop()
        self._parity[slot] = 0
        self._slab[2 * slot].zero_()          # onnx_wrapper.py:114-115: zero state at stream start
        if self.resident:
            self._rings[slot].zero_()         # (the zero row's conv section holds chunk counter 0)
        self._open[slot] = self._fresh_state()
        return slot

    def close_stream(self, slot: int) -> None:
        if slot not in self._open:
            raise KeyError(f"slot {slot} is not open")
        del self._open[slot]
        self._free.append(slot)

    @property
    def open_slots(self) -> list[int]:
        return sorted(self._open)

    def state_of(self, slot: int):
        """The current flat (219729,) fp16 state of an open stream: a view of its slab row, or with the resident
        form the row and ring exported to a new device tensor."""
        import torch
        if slot not in self._open:
            raise KeyError(f"slot {slot} is not open")
        row = 2 * slot + int(self._parity[slot])
        if not self.resident:
            return self._slab[row, : C.STATE_SIZE]
        dev = self.session.dev
        ids = torch.tensor([row, slot], dtype=torch.int32, device=dev)
        return self.session.ring_export(self._slab, ids[:1], self._rings, ids[1:])[0]

    # --- one step ----------------------------------------------------------------------------
    def step_frames(self, chunks: np.ndarray, slots: Sequence[int]) -> np.ndarray:
        """Advance ``slots`` by one chunk each on the device; returns their frame info (n, 10) int32."""
        import torch
        n = len(slots)
        mb = self.session.max_batch
        info = np.empty((n, self.frames), np.int32)
        logp = np.empty((n, self.frames, C.VOCAB), np.float32) if self.decoder is not None else None
        self.session.set_frame_info(self._info)    # frame_info is session state: claim it every step
        for b0 in range(0, n, mb):
            b1 = min(n, b0 + mb)
            nb = b1 - b0
            sl = np.asarray(slots[b0:b1], np.int64)
            par = self._parity[sl]
            self._sig_h[:nb].numpy()[:] = chunks[b0:b1]
            self._rows_h[0, :nb].numpy()[:] = 2 * sl + par
            self._rows_h[1, :nb].numpy()[:] = 2 * sl + 1 - par
            self._rows_h[2, :nb].numpy()[:] = sl
            self._sig[:nb].copy_(self._sig_h[:nb], non_blocking=True)
            self._rows[:, :nb].copy_(self._rows_h[:, :nb], non_blocking=True)
            # rows and ring ids are built here, distinct by construction
            if self.resident:
                self.session.run_ring(self._sig[:nb], self._rows[0, :nb], self._rows[1, :nb], self._slab, self._rings,
                                      self._rows[2, :nb], self._logp, check=False)
            else:
                self.session.run_rows(self._sig[:nb], self._rows[0, :nb], self._rows[1, :nb], self._slab,
                                      self._logp, check_rows=False)
            self._info_h[:nb].copy_(self._info[:nb], non_blocking=True)
            if logp is not None:
                self._logp_h[:nb].copy_(self._logp[:nb], non_blocking=True)
            torch.cuda.current_stream(self.session.dev).synchronize()
            info[b0:b1] = self._info_h[:nb].numpy()
            if logp is not None:
                logp[b0:b1] = self._logp_h[:nb].numpy()
            self._parity[sl] ^= 1
        self._last_logp = logp
        return info

    def forward(self, chunks: np.ndarray, slots: Sequence[int], is_last: Optional[Sequence[bool]] = None
                ) -> list[list[TextPhrase]]:
        """chunks int32 (n, 2400) for the open streams ``slots`` -> per stream, the finished phrases."""
        if not isinstance(chunks, np.ndarray):
            raise TypeError(f"Incorrect 'chunks' type: expected np.ndarray, but got {type(chunks)}")
        n = len(slots)
        if chunks.shape != (n, self.CHUNK_SIZE):
            raise ValueError(f"Shape of 'chunks' must be ({n}, {self.CHUNK_SIZE}), but got {chunks.shape}")
        if chunks.dtype != np.int32:
            raise ValueError(f"Incorrect dtype of 'chunks': expected np.int32, but got {chunks.dtype}")
        if n and (chunks.min() < -32768 or chunks.max() > 32767):
            raise ValueError("Audio samples must be in the int16 range [-32768, 32767]")
        if len(set(slots)) != n or any(s not in self._open for s in slots):
            raise ValueError("slots must be distinct open stream slots")
        is_last = [False] * n if is_last is None else list(is_last)
        info = self.step_frames(chunks, slots) if n else np.zeros((0, self.frames), np.int32)
        out: list[list[TextPhrase]] = []
        for i, slot in enumerate(slots):
            toks, speech = decode_frame_info(info[i])
            if self.decoder is None:
                phrases, self._open[slot] = frames_to_phrases(toks, speech, self._open[slot], is_last=is_last[i])
            else:
                phrases, self._open[slot] = frames_to_phrases(self._last_logp[i], speech, self._open[slot],
                                                              is_last=is_last[i], decode=self.decoder.forward)
            out.append(phrases)
        return out

    def forward_offline(self, audio: np.ndarray) -> list[TextPhrase]:
        """tone/pipeline.py:178-200 on one stream: pad 300 ms both sides, pad to whole chunks, decode."""
        if not isinstance(audio, np.ndarray):
            raise TypeError(f"Incorrect 'audio' type: expected np.ndarray, but got {type(audio)}")
        if audio.ndim != 1:
            raise ValueError(f"Shape of 'audio' must be (L,), but got {audio.shape}")
        audio = np.pad(audio.astype(np.int32), (PADDING, PADDING))
        audio = np.pad(audio, (0, -len(audio) % self.CHUNK_SIZE))
        chunks = audio.reshape(-1, self.CHUNK_SIZE)
        slot = self.open_stream()
        try:
            phrases: list[TextPhrase] = []
            for i, ch in enumerate(chunks):
                phrases += self.forward(ch[None], [slot], [i == len(chunks) - 1])[0]
            return phrases
        finally:
            self.close_stream(slot)


class GreedyLogprobDecoder:
    """Host restatement of ``tone.decoder.GreedyCTCDecoder.forward`` (tone/decoder.py:38-59): argmax,
    collapse repeats, drop the blank.  The stand-in host decoder for tests where pyctcdecode / KenLM
    (BeamSearchCTCDecoder) are not installed; both take (L, 35) float32 logprob rows."""

    def forward(self, logprobs: np.ndarray) -> str:
        if not isinstance(logprobs, np.ndarray):
            raise TypeError(f"Incorrect 'logprobs' type: expected np.ndarray, but got {type(logprobs)}")
        if logprobs.shape[1:] != (C.VOCAB,):
            raise ValueError(f"Shape of 'logprobs' must be (L, 35), but got {logprobs.shape}")
        if logprobs.dtype != np.float32:
            raise ValueError(f"Incorrect dtype of 'logprobs': expected np.float32, but got {logprobs.dtype}")
        return greedy_text(logprobs.argmax(axis=-1))


class StreamScheduler:
    """Arrival queue + continuous batching in front of a :class:`StreamingGreedyPipeline`.

    ``submit(stream_id, chunk, is_last)`` may be called at any time for any number of streams (a
    stream's slot is opened at its first chunk and released after its last).  ``step()`` takes the
    streams whose oldest waiting chunk arrived first, at most ``max_batch`` of them and one chunk
    each, runs them as one device batch and returns ``{stream_id: [TextPhrase, ...]}`` for the
    streams that stepped.  Streams with nothing waiting are not in the batch and their state rows
    are not touched.
    """

    def __init__(self, pipeline: StreamingGreedyPipeline, max_batch: Optional[int] = None):
        from collections import deque
        self.pipe = pipeline
        self.max_batch = int(max_batch or pipeline.session.max_batch)
        if self.max_batch <= 0:
            raise ValueError("max_batch must be positive")
        self._queues: dict = {}          # stream id -> deque[(seq, chunk, is_last)]
        self._slot: dict = {}            # stream id -> slot
        self._seq = 0
        self._deque = deque

    def submit(self, stream_id, chunk: np.ndarray, is_last: bool = False) -> None:
        chunk = np.asarray(chunk)
        size = getattr(self.pipe, "CHUNK_SIZE", C.AUDIO_CHUNK_SAMPLES)
        if chunk.shape != (size,) or chunk.dtype != np.int32:
            raise ValueError(f"chunk must be int32 ({size},), got {chunk.dtype} {chunk.shape}")
        if stream_id not in self._slot:
            self._slot[stream_id] = self.pipe.open_stream()
            self._queues[stream_id] = self._deque()
        q = self._queues[stream_id]
        if q and q[-1][2]:
            raise ValueError(f"stream {stream_id!r} already submitted its last chunk")
        q.append((self._seq, chunk, bool(is_last)))
        self._seq += 1

    @property
    def pending(self) -> int:
        return sum(len(q) for q in self._queues.values())

    @property
    def active_streams(self) -> int:
        return len(self._slot)

    def step(self) -> dict:
        ready = [(q[0][0], sid) for sid, q in self._queues.items() if q]
        if not ready:
            return {}
        ready.sort()
        pick = [sid for _, sid in ready[: self.max_batch]]
        items = [self._queues[sid].popleft() for sid in pick]
        chunks = np.stack([it[1] for it in items])
        res = self.pipe.forward(chunks, [self._slot[sid] for sid in pick], [it[2] for it in items])
        out = {}
        for sid, it, phrases in zip(pick, items, res):
            out[sid] = phrases
            if it[2]:
                self.pipe.close_stream(self._slot.pop(sid))
                del self._queues[sid]
        return out

    def drain(self) -> dict:
        """Step until nothing is waiting; phrases concatenated per stream."""
        out: dict = {}
        while self.pending:
            for sid, ph in self.step().items():
                out.setdefault(sid, []).extend(ph)
        return out
