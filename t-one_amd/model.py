"""Host side of the acoustic path: the drop-in ``StreamingCTCModel`` and the device ``ToneSession``.

``StreamingCTCModel`` mirrors ``tone.onnx_wrapper.StreamingCTCModel`` (tone/onnx_wrapper.py:17-123):
same class constants, factories, ``forward(audio_chunk, state=None)`` signature, numpy I/O, and
the same exceptions for bad inputs, so ``tone.pipeline.StreamingCTCPipeline`` (which reads the
constants from the class and calls ``model.forward``, tone/pipeline.py:49,141-147) runs unchanged
with it.  Instead of ``ort.InferenceSession.run`` it calls ``libtonehip.so``.

``ToneSession`` is the high-throughput interface: torch device tensors in and out, optional
hipGraph replay, and a slot API over a device-resident state slab.
"""

from __future__ import annotations

import ctypes
import logging
from pathlib import Path
from typing import Optional

import numpy as np
import numpy.typing as npt

from . import _lib
from . import config as C
from .weights import load_weights, synthetic_weights

log = logging.getLogger(__name__)


def _torch():
    import torch
    return torch


def _nullcontext():
    import contextlib
    return contextlib.nullcontext()


class ToneSession:
    """One libtonehip session on one GPU: folded weights + activations resident in HBM."""

    def __init__(self, weights: dict, device: int = 0, precision: str = "fp32", max_batch: int = 256,
                 graph: bool = False, chunk_samples: int = C.AUDIO_CHUNK_SAMPLES):
        """``chunk_samples``: 2400 (300 ms, the reference's StreamingCTCModel) or 3200 (400 ms, the
        Triton ensemble's chunk; 13 frames per step).  Same flat state in both."""
        torch = _torch()
        lib = _lib.load()
        if precision not in _lib.PRECISION:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISION)}, got {precision!r}")
        if not torch.cuda.is_available():
            raise RuntimeError("ToneSession needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = int(device)
        self.precision = precision
        self.max_batch = int(max_batch)
        self._lib = lib
        h = ctypes.c_void_p()
        torch.cuda.set_device(self.device)
        _lib.check(lib.tone_session_create(ctypes.byref(h), self.device, _lib.PRECISION[precision], self.max_batch),
                   "tone_session_create")
        self._h = h
        for name, arr in weights.items():
            a = np.ascontiguousarray(arr, dtype=np.float32)
            _lib.check(lib.tone_session_set_weight(h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                       f"tone_session_set_weight({name})")
        _lib.check(lib.tone_session_set_chunk(h, int(chunk_samples)), "tone_session_set_chunk")
        self.chunk_samples = int(chunk_samples)
        self.frames = int(lib.tone_session_frames_per_chunk(h))
        _lib.check(lib.tone_session_finalize(h), "tone_session_finalize")
        if graph:
            _lib.check(lib.tone_session_set_graph(h, 1), "tone_session_set_graph")
        self.dev = torch.device("cuda", self.device)

    # --- raw device-pointer step --------------------------------------------------------------
    def run(self, signal, state_in, logprobs, state_out, stream=None) -> None:
        """signal int32 (B, chunk[,1]), state_in/state_out fp16 (B, >=219729), logprobs fp32 (B, frames, 35);
        all contiguous torch tensors on this session's device."""
        torch = _torch()
        b = int(signal.shape[0])
        for t, dt in ((signal, torch.int32), (state_in, torch.float16), (state_out, torch.float16),
                      (logprobs, torch.float32)):
            if t.dtype != dt or t.device != self.dev:
                raise ValueError(f"expected {dt} tensor on {self.dev}, got {t.dtype} on {t.device}")
        if state_in.stride(1) != 1 or state_out.stride(1) != 1 or state_in.stride(0) != state_out.stride(0):
            raise ValueError("state tensors must be row-contiguous with equal row strides")
        if not signal.is_contiguous() or not logprobs.is_contiguous():
            raise ValueError("signal and logprobs must be contiguous")
        if signal.numel() != b * self.chunk_samples or logprobs.numel() < b * self.frames * C.VOCAB:
            raise ValueError(f"signal must hold (B, {self.chunk_samples}) samples and logprobs (B, {self.frames}, 35)")
        if not 0 < b <= self.max_batch:
            raise ValueError(f"batch {b} outside 1..{self.max_batch}")
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_run(self._h, signal.data_ptr(), state_in.data_ptr(), logprobs.data_ptr(),
                                              state_out.data_ptr(), b, state_in.stride(0), st),
                   "tone_session_run")

    def run_slots(self, signal, slots, slab_in, slab_out, logprobs, stream=None, check_slots: bool = True) -> None:
        """Stream i reads row slots[i] of ``slab_in`` and writes row slots[i] of ``slab_out``.

        signal int32 (B,2400), slots int32 (B,) on the device (or a host sequence, uploaded here),
        slab_in/slab_out fp16 (n_slots, >= 219729) with equal row strides, logprobs fp32 (>= B,10,35).
        Slot ids must be distinct and in [0, n_slots): with ``check_slots`` (default) a device slots
        tensor is range-checked here (one device sync), a host sequence always is."""
        torch = _torch()
        b = int(signal.shape[0])
        if not isinstance(slots, torch.Tensor):
            ids = [int(x) for x in slots]
            if len(ids) != b:
                raise ValueError(f"{len(ids)} slots for a batch of {b}")
            n = int(slab_in.shape[0])
            if any(not 0 <= x < n for x in ids) or len(set(ids)) != b:
                raise ValueError(f"slot ids must be distinct and in [0, {n})")
            slots = torch.tensor(ids, dtype=torch.int32, device=self.dev)
            check_slots = False
        for t, dt in ((signal, torch.int32), (slots, torch.int32), (slab_in, torch.float16),
                      (slab_out, torch.float16), (logprobs, torch.float32)):
            if t.dtype != dt or t.device != self.dev:
                raise ValueError(f"expected {dt} tensor on {self.dev}, got {t.dtype} on {t.device}")
        if not 0 < b <= self.max_batch:
            raise ValueError(f"batch {b} outside 1..{self.max_batch}")
        if tuple(slots.shape) != (b,) or not slots.is_contiguous():
            raise ValueError(f"slots must be a contiguous (B,) = ({b},) int32 tensor, got {tuple(slots.shape)}")
        if signal.dim() < 2 or signal.shape[1] != self.chunk_samples or not signal.is_contiguous():
            raise ValueError(f"signal must be a contiguous (B, {self.chunk_samples}) int32 tensor")
        if not logprobs.is_contiguous() or logprobs.numel() < b * self.frames * C.VOCAB:
            raise ValueError("logprobs must be contiguous with room for (B, 10, 35)")
        if slab_in.dim() != 2 or slab_out.shape != slab_in.shape or slab_in.stride(1) != 1 or slab_out.stride(1) != 1 \
                or slab_in.stride(0) != slab_out.stride(0) or slab_in.stride(0) < C.STATE_SIZE \
                or slab_in.shape[1] < C.STATE_SIZE:
            raise ValueError("slabs must be equal-shaped (n_slots, >= 219729) fp16 with unit column stride and "
                             "equal row strides")
        if slab_in.data_ptr() == slab_out.data_ptr():
            raise ValueError("slab_out must not alias slab_in")
        if check_slots and b:
            lo, hi = int(slots.min()), int(slots.max())
            if lo < 0 or hi >= slab_in.shape[0]:
                raise ValueError(f"slot ids span [{lo}, {hi}], outside [0, {slab_in.shape[0]})")
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_run_slots(self._h, signal.data_ptr(), slots.data_ptr(), slab_in.data_ptr(),
                                                    slab_out.data_ptr(), slab_in.stride(0), logprobs.data_ptr(), b, st),
                   "tone_session_run_slots")

    def run_rows(self, signal, rows_in, rows_out, slab, logprobs, stream=None, check_rows: bool = True) -> None:
        """Ping-pong step over one slab: stream i reads row rows_in[i] and writes row rows_out[i].

        rows_in/rows_out int32 (B,) device tensors; slab fp16 (n_rows, >= 219729).  No row may be both
        read and written (checked with one device sync when ``check_rows``)."""
        torch = _torch()
        b = int(signal.shape[0])
        for t, dt in ((signal, torch.int32), (rows_in, torch.int32), (rows_out, torch.int32),
                      (slab, torch.float16), (logprobs, torch.float32)):
            if t.dtype != dt or t.device != self.dev:
                raise ValueError(f"expected {dt} tensor on {self.dev}, got {t.dtype} on {t.device}")
        if not 0 < b <= self.max_batch:
            raise ValueError(f"batch {b} outside 1..{self.max_batch}")
        for r in (rows_in, rows_out):
            if tuple(r.shape) != (b,) or not r.is_contiguous():
                raise ValueError(f"rows must be contiguous (B,) = ({b},) int32 tensors, got {tuple(r.shape)}")
        if signal.dim() < 2 or signal.shape[1] != self.chunk_samples or not signal.is_contiguous():
            raise ValueError(f"signal must be a contiguous (B, {self.chunk_samples}) int32 tensor")
        if not logprobs.is_contiguous() or logprobs.numel() < b * self.frames * C.VOCAB:
            raise ValueError("logprobs must be contiguous with room for (B, 10, 35)")
        if slab.dim() != 2 or slab.stride(1) != 1 or slab.stride(0) < C.STATE_SIZE or slab.shape[1] < C.STATE_SIZE:
            raise ValueError("slab must be (n_rows, >= 219729) fp16 with unit column stride")
        if check_rows:
            both = torch.cat([rows_in, rows_out])
            lo, hi = int(both.min()), int(both.max())
            if lo < 0 or hi >= slab.shape[0]:
                raise ValueError(f"row ids span [{lo}, {hi}], outside [0, {slab.shape[0]})")
            if int(torch.unique(both).numel()) != 2 * b:
                raise ValueError("row ids must be distinct: no row both read and written, no row used twice")
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_run_rows(self._h, signal.data_ptr(), rows_in.data_ptr(), rows_out.data_ptr(),
                                                   slab.data_ptr(), slab.stride(0), logprobs.data_ptr(), b, st),
                   "tone_session_run_rows")

    # --- resident state: conv caches in per-stream rings (include/tonehip.h tone_session_run_ring) ----------------
    @property
    def ring_elems(self) -> int:
        """fp16 elements of one stream's ring ((16 conv + 2 MHSA layers) x 30 x 384)."""
        return int(self._lib.tone_session_ring_elems())

    def _check_ring_args(self, b, slab, rings, ids, *row_lists):
        torch = _torch()
        for t, dt in ((slab, torch.float16), (rings, torch.float16), (ids, torch.int32)) + tuple((r, torch.int32) for r in row_lists):
            if t.dtype != dt or t.device != self.dev:
                raise ValueError(f"expected {dt} tensor on {self.dev}, got {t.dtype} on {t.device}")
        for r in (ids,) + row_lists:
            if tuple(r.shape) != (b,) or not r.is_contiguous():
                raise ValueError(f"rows / ring ids must be contiguous (B,) = ({b},) int32 tensors, got {tuple(r.shape)}")
        if slab.dim() != 2 or slab.stride(1) != 1 or slab.stride(0) < C.STATE_SIZE or slab.shape[1] < C.STATE_SIZE:
            raise ValueError("slab must be (n_rows, >= 219729) fp16 with unit column stride")
        if rings.dim() != 2 or rings.shape[1] != self.ring_elems or not rings.is_contiguous():
            raise ValueError(f"rings must be a contiguous (n_rings, {self.ring_elems}) fp16 tensor")

    def run_ring(self, signal, rows_in, rows_out, slab, rings, ring_ids, logprobs, stream=None, check: bool = True) -> None:
        """Step on the resident state: the non-conv sections ping-pong between rows rows_in[i] / rows_out[i] of
        ``slab`` (as run_rows), stream i's conv caches live in ring ring_ids[i] of ``rings`` (n_rings, ring_elems)
        and are updated in place.  Convert with ring_import / ring_export.  With ``check`` the ids are range- and
        distinctness-checked (one device sync)."""
        torch = _torch()
        b = int(signal.shape[0])
        if signal.dtype != torch.int32 or signal.device != self.dev or logprobs.dtype != torch.float32 \
                or logprobs.device != self.dev:
            raise ValueError("signal int32 and logprobs fp32 on the session's device")
        if not 0 < b <= self.max_batch:
            raise ValueError(f"batch {b} outside 1..{self.max_batch}")
        self._check_ring_args(b, slab, rings, ring_ids, rows_in, rows_out)
        if signal.dim() < 2 or signal.shape[1] != self.chunk_samples or not signal.is_contiguous():
            raise ValueError(f"signal must be a contiguous (B, {self.chunk_samples}) int32 tensor")
        if not logprobs.is_contiguous() or logprobs.numel() < b * self.frames * C.VOCAB:
            raise ValueError("logprobs must be contiguous with room for (B, frames, 35)")
        if check:
            both = torch.cat([rows_in, rows_out])
            if int(both.min()) < 0 or int(both.max()) >= slab.shape[0] or int(torch.unique(both).numel()) != 2 * b:
                raise ValueError("row ids must be distinct and in range: no row both read and written")
            if int(ring_ids.min()) < 0 or int(ring_ids.max()) >= rings.shape[0] or int(torch.unique(ring_ids).numel()) != b:
                raise ValueError(f"ring ids must be distinct and in [0, {rings.shape[0]})")
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_run_ring(self._h, signal.data_ptr(), rows_in.data_ptr(), rows_out.data_ptr(),
                                                   slab.data_ptr(), slab.stride(0), rings.data_ptr(), ring_ids.data_ptr(),
                                                   logprobs.data_ptr(), b, st), "tone_session_run_ring")

    def ring_import(self, flat, slab, rows, rings, ring_ids, stream=None) -> None:
        """Flat states (n, >= 219729) fp16 -> slab rows ``rows`` + rings ``ring_ids`` (chunk counter 0)."""
        torch = _torch()
        n = int(flat.shape[0])
        if flat.dtype != torch.float16 or flat.device != self.dev or flat.dim() != 2 or flat.stride(1) != 1 \
                or flat.shape[1] < C.STATE_SIZE:
            raise ValueError("flat must be (n, >= 219729) fp16 on the session's device")
        self._check_ring_args(n, slab, rings, ring_ids, rows)
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_ring_import(self._h, flat.data_ptr(), flat.stride(0), slab.data_ptr(),
                                                      slab.stride(0), rows.data_ptr(), rings.data_ptr(),
                                                      ring_ids.data_ptr(), n, st), "tone_session_ring_import")

    def ring_export(self, slab, rows, rings, ring_ids, flat=None, stream=None):
        """Slab rows ``rows`` + rings ``ring_ids`` -> flat states (n, 219729) fp16 (allocated when ``flat`` is None)."""
        torch = _torch()
        n = int(rows.shape[0])
        if flat is None:
            flat = torch.empty((n, C.STATE_SIZE), dtype=torch.float16, device=self.dev)
        if flat.dtype != torch.float16 or flat.device != self.dev or flat.dim() != 2 or flat.stride(1) != 1 \
                or flat.shape[0] != n or flat.shape[1] < C.STATE_SIZE:
            raise ValueError(f"flat must be ({n}, >= 219729) fp16 on the session's device")
        self._check_ring_args(n, slab, rings, ring_ids, rows)
        st = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        _lib.check(self._lib.tone_session_ring_export(self._h, slab.data_ptr(), slab.stride(0), rows.data_ptr(),
                                                      rings.data_ptr(), ring_ids.data_ptr(), flat.data_ptr(),
                                                      flat.stride(0), n, st), "tone_session_ring_export")
        return flat

    def set_frame_info(self, frame_info=None) -> None:
        """Have later runs also write frame_info int32 (>= max_batch, 10): greedy token | speech << 8
        (include/tonehip.h); None switches it off."""
        torch = _torch()
        ptr = 0
        if frame_info is not None:
            if frame_info.dtype != torch.int32 or frame_info.device != self.dev or not frame_info.is_contiguous():
                raise ValueError(f"frame_info must be a contiguous int32 tensor on {self.dev}")
            if frame_info.numel() < self.max_batch * self.frames:
                raise ValueError(f"frame_info needs >= {self.max_batch * self.frames} elements")
            ptr = frame_info.data_ptr()
        self._frame_info = frame_info
        _lib.check(self._lib.tone_session_set_frame_info(self._h, ptr), "tone_session_set_frame_info")

    def step(self, signal, state=None):
        """Allocate-and-run convenience: returns (logprobs, next_state) device tensors."""
        torch = _torch()
        b = int(signal.shape[0])
        if state is None:
            state = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=self.dev)
        out_state = torch.empty_like(state)
        logp = torch.empty((b, self.frames, C.VOCAB), dtype=torch.float32, device=self.dev)
        self.run(signal.contiguous(), state, logp, out_state)
        return logp, out_state

    # --- timing (bench.py) --------------------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        _lib.check(self._lib.tone_session_set_timing(self._h, int(enable)), "tone_session_set_timing")

    def kernel_us(self, family: str) -> tuple[float, int]:
        n = ctypes.c_int64(0)
        us = self._lib.tone_session_kernel_us(self._h, family.encode(), ctypes.byref(n))
        return float(us), int(n.value)

    def set_graph(self, enable: bool) -> None:
        _lib.check(self._lib.tone_session_set_graph(self._h, int(enable)), "tone_session_set_graph")

    def debug_stop(self, stage: int) -> None:
        _lib.check(self._lib.tone_session_debug_stop(self._h, int(stage)), "tone_session_debug_stop")

    def debug_read(self, name: str, shape, dtype=np.float32) -> np.ndarray:
        out = np.empty(shape, dtype)
        _lib.check(self._lib.tone_session_debug_read(self._h, name.encode(), out.ctypes.data_as(ctypes.c_void_p),
                                                     out.nbytes), f"tone_session_debug_read({name})")
        return out

    @property
    def device_bytes(self) -> int:
        return int(self._lib.tone_session_device_bytes(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.tone_session_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def validate_inputs(audio_chunk, state):
    """Input checks of tone/onnx_wrapper.py:100-121 (same exception types); returns the state,
    zero-initialised when None (onnx_wrapper.py:114-115)."""
    if not isinstance(audio_chunk, np.ndarray):
        raise TypeError(f"Incorrect 'audio_chunk' type: expected np.ndarray, but got {type(audio_chunk)}")
    if audio_chunk.ndim != 3 or audio_chunk.shape[1:] != (C.AUDIO_CHUNK_SAMPLES, 1):
        raise ValueError(
            f"Shape of 'audio_chunk' must be (B, {C.AUDIO_CHUNK_SAMPLES}, 1), but got {audio_chunk.shape}",
        )
    if audio_chunk.dtype != np.int32:
        raise ValueError(f"Incorrect dtype of 'audio_chunk': expected np.int32, but got {audio_chunk.dtype}")
    if audio_chunk.size == 0:   # the reference's audio_chunk.min() raises ValueError on it (onnx_wrapper.py:108)
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    if audio_chunk.min() < -32768 or audio_chunk.max() > 32767:
        raise ValueError(
            "Samples in 'audio_chunk' must be in range [-32768; 32767], "
            f"but it is in range [{audio_chunk.min()}; {audio_chunk.max()}]",
        )
    batch_size = audio_chunk.shape[0]
    if state is None:
        state = np.zeros((batch_size, C.STATE_SIZE), dtype=np.float16)
    if not isinstance(state, np.ndarray):
        raise TypeError(f"Incorrect 'state' type: expected np.ndarray or None, but got {type(state)}")
    if state.shape != (batch_size, C.STATE_SIZE):
        raise ValueError(f"Shape of 'state' must be ({batch_size}, {C.STATE_SIZE}), but got {state.shape}")
    if state.dtype != np.float16:
        raise ValueError(f"Incorrect dtype of 'state': expected np.float16, but got {state.dtype}")
    return state


class StreamingCTCModel:
    """Drop-in for ``tone.onnx_wrapper.StreamingCTCModel`` running on an MI355X GPU.

    Class constants are identical to tone/onnx_wrapper.py:30-34 (the pipeline reads them from the
    class, tone/pipeline.py:49,141,154,161).
    """

    InputType = npt.NDArray[np.int32]
    OutputType = npt.NDArray[np.float32]
    StateType = npt.NDArray[np.float16]

    SAMPLE_RATE = C.SAMPLE_RATE
    MEAN_TIME_BIAS = C.MEAN_TIME_BIAS
    AUDIO_CHUNK_SAMPLES = C.AUDIO_CHUNK_SAMPLES
    FRAME_SIZE = C.FRAME_SIZE
    STATE_SIZE = C.STATE_SIZE

    HF_REPO = "t-tech/T-one"
    HF_MODEL = "model.onnx"          # what tone/onnx_wrapper.py:60-63 fetches
    HF_WEIGHTS = "model.safetensors"   # the torch checkpoint of the same model, used when present

    @classmethod
    def from_hugging_face(cls, **kw) -> "StreamingCTCModel":
        """tone/onnx_wrapper.py:38-50: the t-tech/T-one weights through the HF cache (see
        :meth:`download_from_hugging_face` for which file)."""
        return cls.from_local(cls.download_from_hugging_face(), **kw)

    @classmethod
    def download_from_hugging_face(cls, prefer_safetensors: bool = True) -> str:
        """tone/onnx_wrapper.py:52-63 fetches ``model.onnx``.  The torch checkpoint of the same model,
        ``model.safetensors``, carries every parameter under its own name and in fp32, so with
        ``prefer_safetensors`` it is tried first and ``model.onnx`` (read by :mod:`tone_amd.onnx_weights`, which
        attributes constant-folded initializers through the graph) is the fallback when the repository or the
        offline cache has no such file.  Any other failure (authentication, network, a corrupt cache) is raised.
        The file taken is logged."""
        from huggingface_hub import hf_hub_download
        from huggingface_hub.utils import EntryNotFoundError, LocalEntryNotFoundError
        if prefer_safetensors:
            try:
                path = hf_hub_download(cls.HF_REPO, cls.HF_WEIGHTS)
                log.info("T-one weights: %s", path)
                return path
            except (EntryNotFoundError, LocalEntryNotFoundError) as e:
                log.info("%s/%s not available (%s); using %s", cls.HF_REPO, cls.HF_WEIGHTS, type(e).__name__,
                         cls.HF_MODEL)
        path = hf_hub_download(cls.HF_REPO, cls.HF_MODEL)
        log.info("T-one weights: %s", path)
        return path

    @classmethod
    def from_local(cls, model_path: str | Path, providers: Optional[list[str]] = None, *, device: int = 0,
                   precision: str = "fp32", max_batch: int = 64, prefer_safetensors: bool = True) -> "StreamingCTCModel":
        """tone/onnx_wrapper.py:65-78.  ``model_path`` is what the reference passes -- ``model.onnx``
        (its initializers are read by :mod:`tone_amd.onnx_weights`; with ``prefer_safetensors`` a
        ``model.safetensors`` beside it, the fp32 torch checkpoint of the same model, is taken instead) -- or a
        model.safetensors / weights.npz / torch state_dict (.pt, weights_only) / a directory holding one.
        ``providers`` is accepted for signature compatibility; the MI355X device is chosen with ``device``.
        The file actually loaded is logged."""
        del providers
        p = Path(model_path)
        if prefer_safetensors and p.suffix == ".onnx" and (p.parent / cls.HF_WEIGHTS).exists():
            log.info("T-one weights: %s (found beside %s)", p.parent / cls.HF_WEIGHTS, p.name)
            p = p.parent / cls.HF_WEIGHTS
        else:
            log.info("T-one weights: %s", p)
        return cls(ToneSession(load_weights(p), device=device, precision=precision, max_batch=max_batch))

    @classmethod
    def from_synthetic(cls, seed: int = 0, **kw) -> "StreamingCTCModel":
        """Random-init weights of the T-one architecture (tests / benchmarks; no checkpoint offline)."""
        return cls(ToneSession(synthetic_weights(seed), **kw))

    def __init__(self, session: ToneSession, graph: bool = False) -> None:
        """``graph``: replay each batch size's step as one hipGraph on the model's own stream (the I/O buffers are fixed
        per batch size, so the graph key holds).  Off by default: at B = 1 the eager launches overlap their dispatch
        with the previous kernels and measured faster than the replay (0.97 vs 1.01 ms per step, profiles/r06_b1_*)."""
        self._sess = session
        self._buffers: dict = {}
        self._pinned = True
        self._stream = None          # None: the caller's current stream
        if graph and getattr(session, "dev", None) is not None and session.dev.type == "cuda":
            session.set_graph(True)
            self._stream = _torch().cuda.Stream(session.dev)   # graphs are captured on a non-default stream

    @property
    def session(self) -> ToneSession:
        return self._sess

    _MAX_IO_SETS = 4   # device I/O buffer sets kept for distinct batch sizes (least recently used evicted)

    def _io(self, b: int):
        torch = _torch()
        if b in self._buffers:
            self._buffers[b] = self._buffers.pop(b)          # most recently used last
        else:
            while len(self._buffers) >= self._MAX_IO_SETS:
                self._buffers.pop(next(iter(self._buffers)))
            dev = self._sess.dev
            fr = self._sess.frames
            cs = int(getattr(self._sess, "chunk_samples", C.AUDIO_CHUNK_SAMPLES))
            pin = dev.type == "cuda" and self._pinned
            self._buffers[b] = (
                torch.empty((b, cs), dtype=torch.int32, device=dev),
                torch.empty((b, C.STATE_SIZE), dtype=torch.float16, device=dev),
                torch.empty((b, C.STATE_SIZE), dtype=torch.float16, device=dev),
                torch.empty((b, fr, C.VOCAB), dtype=torch.float32, device=dev),
                # pinned host staging: the chunk + state go up and the logprobs + state come back as DMA copies from
                # page-locked memory (pageable copies cost ~0.1 ms per B = 1 call: 1.09 vs 0.97 ms device step, r05)
                torch.empty((b, cs), dtype=torch.int32, pin_memory=pin),
                torch.empty((b, C.STATE_SIZE), dtype=torch.float16, pin_memory=pin),
                torch.empty((b, C.STATE_SIZE), dtype=torch.float16, pin_memory=pin),
                torch.empty((b, fr, C.VOCAB), dtype=torch.float32, pin_memory=pin),
            )
        return self._buffers[b]

    def forward(self, audio_chunk: InputType, state: StateType | None = None) -> tuple[OutputType, StateType]:
        """Run the acoustic model on a batch of chunks (tone/onnx_wrapper.py:84-123).

        Returns logprobs (B, 10, 35) float32 and the next state (B, 219729) float16.
        """
        state = validate_inputs(audio_chunk, state)
        batch_size = audio_chunk.shape[0]

        torch = _torch()
        outs_l, outs_s = [], []
        for s0 in range(0, batch_size, self._sess.max_batch):
            s1 = min(batch_size, s0 + self._sess.max_batch)
            b = s1 - s0
            sig, st_in, st_out, logp, h_sig, h_in, h_out, h_logp = self._io(b)
            np.copyto(h_sig.numpy(), audio_chunk[s0:s1, :, 0])
            np.copyto(h_in.numpy(), state[s0:s1])
            gpu = self._sess.dev.type == "cuda"
            stream = (self._stream or torch.cuda.current_stream(self._sess.dev)) if gpu else None
            with (torch.cuda.stream(stream) if gpu else _nullcontext()):
                sig.copy_(h_sig, non_blocking=gpu)
                st_in.copy_(h_in, non_blocking=gpu)
                self._sess.run(sig, st_in, logp, st_out, stream=stream)
                h_logp.copy_(logp, non_blocking=gpu)
                h_out.copy_(st_out, non_blocking=gpu)
            if gpu:
                stream.synchronize()
            outs_l.append(h_logp.numpy().copy())          # fresh arrays: the staging buffers are reused
            outs_s.append(h_out.numpy().copy())
        logprobs = outs_l[0] if len(outs_l) == 1 else np.concatenate(outs_l)
        next_state = outs_s[0] if len(outs_s) == 1 else np.concatenate(outs_s)
        return logprobs, next_state
