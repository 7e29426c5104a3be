"""Flat streaming state <-> the Triton ensemble's three cache tensors.

The acoustic path carries one flat fp16 row of 219,729 values per stream (the argument order of
``Tone.forward_for_export``, reference ``tone/nn/model.py:101-113``; sections and offsets in
:mod:`tone_amd.config`).  The reference's Triton exporter carries the same numbers as three tensors
instead (reference ``tone/scripts/export.py:177-236`` builds the shapes, ``:293-333`` unpacks,
``:335-376`` packs):

``cache_last_time``     (B, 18, 384, 30) fp16
    the 2 MHSA caches transposed to (384, 30) (``export.py:306-307,350``), then the 16 conv caches
    (``:310,351``) -- mhsa (N,T,H) and conv (N,H,T) share T = 30 and H = 384 (``:187-201``).
``cache_last_channel``  (B, 32, 8, 50) fp16
    the sub2 state (32, 8, 44) in the first 44 slots of the last axis (``:314,374``), then a
    (32, 8, 6) tail holding preproc (80) | sub1 (640) | reduction (384) flattened and zero-padded
    from 1,104 to 1,536 values (``:213-230,355-373``: Tpad = ceil(1104 / 256) rounded up to even).
``cache_last_chan_len`` (B,) int64
    mhsa_len (``:409,444``).

Host logic only (numpy or torch tensors, any device); nothing here calls the HIP library.  Both
directions are exact: fp16 values are moved, never re-rounded, and mhsa_len (0, 10, 20 or 30) is an
fp16-exact integer.
"""

from __future__ import annotations

from . import config as C

__all__ = ["TIME_SHAPE", "CHANNEL_SHAPE", "TAIL_ELEMS", "TAIL_T", "flat_to_triton", "triton_to_flat"]

_SUB2 = C.STATE_SECTIONS["sub2"][1]                                     # (32, 8, 44)
_MHSA = C.STATE_SECTIONS["mhsa"][1]                                     # (2, 30, 384)
_CONV = C.STATE_SECTIONS["conv"][1]                                     # (16, 384, 30)
TIME_SHAPE = (_MHSA[0] + _CONV[0], _CONV[1], _CONV[2])                 # (18, 384, 30)
TAIL_ELEMS = C.PREPROC_STATE + C.SUB1_STATE * C.N_MELS + C.D_MODEL * C.RED_STATE   # 1104
_PER_T = _SUB2[0] * _SUB2[1]                                            # 256 values per tail slot
TAIL_T = -(-TAIL_ELEMS // _PER_T)
TAIL_T += TAIL_T % 2                                                    # export.py:222 -> 6
CHANNEL_SHAPE = (_SUB2[0], _SUB2[1], _SUB2[2] + TAIL_T)                 # (32, 8, 50)


class _Ops:
    """The handful of array operations both numpy and torch need here."""

    def __init__(self, x):
        try:
            import torch
            self.torch = torch if isinstance(x, torch.Tensor) else None
        except ImportError:  # pragma: no cover - torch is part of this image
            self.torch = None
        if self.torch is None:
            import numpy as np
            self.np = np

    def swap_last2(self, x):
        return x.transpose(-1, -2) if self.torch is not None else self.np.swapaxes(x, -1, -2)

    def cat(self, xs, axis):
        return self.torch.cat(xs, dim=axis) if self.torch is not None else self.np.concatenate(xs, axis=axis)

    def zeros(self, like, shape):
        if self.torch is not None:
            return self.torch.zeros(shape, dtype=like.dtype, device=like.device)
        return self.np.zeros(shape, dtype=like.dtype)

    def empty(self, like, shape, dtype=None):
        if self.torch is not None:
            return self.torch.empty(shape, dtype=dtype or like.dtype, device=like.device)
        return self.np.empty(shape, dtype=dtype or like.dtype)

    def contiguous(self, x):
        return x.contiguous() if self.torch is not None else self.np.ascontiguousarray(x)

    def to_int64(self, x):
        return x.to(self.torch.int64) if self.torch is not None else x.astype(self.np.int64)

    def is_fp16(self, x):
        return x.dtype == (self.torch.float16 if self.torch is not None else self.np.float16)


def _section(flat, name):
    off, shape = C.STATE_SECTIONS[name]
    n = 1
    for d in shape:
        n *= d
    return flat[:, off:off + n].reshape((flat.shape[0],) + tuple(shape))


def flat_to_triton(flat):
    """(B, 219729) fp16 -> (cache_last_time, cache_last_channel, cache_last_chan_len)."""
    ops = _Ops(flat)
    if flat.ndim != 2 or flat.shape[1] != C.STATE_SIZE or not ops.is_fp16(flat):
        raise ValueError(f"flat state must be (B, {C.STATE_SIZE}) float16, got {tuple(flat.shape)} {flat.dtype}")
    b = flat.shape[0]
    mhsa_ht = ops.swap_last2(_section(flat, "mhsa"))                     # (B, 2, 384, 30)
    time = ops.contiguous(ops.cat([mhsa_ht, _section(flat, "conv")], axis=1))
    tail = ops.cat([flat[:, C.OFF_PREPROC:C.OFF_PREPROC + C.PREPROC_STATE],
                    _section(flat, "sub1").reshape(b, -1),
                    _section(flat, "reduction").reshape(b, -1),
                    ops.zeros(flat, (b, _PER_T * TAIL_T - TAIL_ELEMS))], axis=1)
    channel = ops.contiguous(ops.cat([_section(flat, "sub2"), tail.reshape(b, _SUB2[0], _SUB2[1], TAIL_T)], axis=3))
    chan_len = ops.to_int64(flat[:, C.OFF_MHSA_LEN])
    return time, channel, chan_len


def triton_to_flat(cache_last_time, cache_last_channel, cache_last_chan_len):
    """The three Triton cache tensors -> (B, 219729) fp16 flat state."""
    ops = _Ops(cache_last_time)
    b = cache_last_time.shape[0]
    if tuple(cache_last_time.shape[1:]) != TIME_SHAPE or not ops.is_fp16(cache_last_time):
        raise ValueError(f"cache_last_time must be (B, {TIME_SHAPE}) float16, got {tuple(cache_last_time.shape)}")
    if tuple(cache_last_channel.shape) != (b,) + CHANNEL_SHAPE or not ops.is_fp16(cache_last_channel):
        raise ValueError(f"cache_last_channel must be (B, {CHANNEL_SHAPE}) float16, got {tuple(cache_last_channel.shape)}")
    chan_len = cache_last_chan_len
    if chan_len.ndim == 2 and chan_len.shape[1] == 1:                  # export.py:403-408 accepts (B,1)
        chan_len = chan_len[:, 0]
    if tuple(chan_len.shape) != (b,):
        raise ValueError(f"cache_last_chan_len must be (B,) or (B,1), got {tuple(cache_last_chan_len.shape)}")
    flat = ops.empty(cache_last_time, (b, C.STATE_SIZE))
    n_mhsa = _MHSA[0]
    mhsa = ops.swap_last2(cache_last_time[:, :n_mhsa])                 # (B, 2, 30, 384)
    flat[:, C.OFF_MHSA:C.OFF_CONV] = mhsa.reshape(b, -1)
    flat[:, C.OFF_CONV:C.OFF_MHSA_LEN] = cache_last_time[:, n_mhsa:].reshape(b, -1)
    flat[:, C.OFF_MHSA_LEN] = chan_len
    flat[:, C.OFF_SUB2:C.OFF_RED] = cache_last_channel[..., :_SUB2[2]].reshape(b, -1)
    tail = cache_last_channel[..., _SUB2[2]:].reshape(b, -1)
    n1 = C.PREPROC_STATE
    n2 = n1 + C.SUB1_STATE * C.N_MELS
    flat[:, C.OFF_PREPROC:C.OFF_PREPROC + n1] = tail[:, :n1]
    flat[:, C.OFF_SUB1:C.OFF_SUB2] = tail[:, n1:n2]
    flat[:, C.OFF_RED:C.STATE_END] = tail[:, n2:TAIL_ELEMS]
    return flat
