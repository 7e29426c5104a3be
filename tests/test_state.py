"""Flat state <-> Triton cache tensors (t-one_amd/state.py; reference tone/scripts/export.py:177-376)."""

import numpy as np
import pytest
import torch

import tone_amd.config as C
from tone_amd.state import CHANNEL_SHAPE, TAIL_ELEMS, TAIL_T, TIME_SHAPE, flat_to_triton, triton_to_flat


def random_flat(b, seed=0):
    rng = np.random.default_rng(seed)
    flat = rng.standard_normal((b, C.STATE_SIZE)).astype(np.float16)
    flat[:, C.OFF_MHSA_LEN] = rng.choice([0, 10, 20, 30], size=b)
    return flat


def test_shapes_match_the_exporter():
    # export.py:201 (n_mhsa + n_conv, H, T) and :232-236 (C1, C2, Tbase + Tpad)
    assert TIME_SHAPE == (18, 384, 30)
    assert CHANNEL_SHAPE == (32, 8, 50)
    assert TAIL_ELEMS == 80 + 640 + 384 and TAIL_T == 6


def test_round_trip_numpy_exact():
    flat = random_flat(5)
    t, c, n = flat_to_triton(flat)
    assert t.shape == (5,) + TIME_SHAPE and t.dtype == np.float16
    assert c.shape == (5,) + CHANNEL_SHAPE and c.dtype == np.float16
    assert n.dtype == np.int64 and n.shape == (5,)
    back = triton_to_flat(t, c, n)
    np.testing.assert_array_equal(back.view(np.uint16), flat.view(np.uint16))


def test_section_placement():
    flat = random_flat(3, seed=1)
    t, c, n = flat_to_triton(flat)
    mhsa = flat[:, C.OFF_MHSA:C.OFF_CONV].reshape(3, 2, 30, 384)
    conv = flat[:, C.OFF_CONV:C.OFF_MHSA_LEN].reshape(3, 16, 384, 30)
    np.testing.assert_array_equal(t[:, :2], mhsa.transpose(0, 1, 3, 2))     # export.py:350
    np.testing.assert_array_equal(t[:, 2:], conv)
    np.testing.assert_array_equal(c[..., :44], flat[:, C.OFF_SUB2:C.OFF_RED].reshape(3, 32, 8, 44))
    tail = c[..., 44:].reshape(3, -1)
    np.testing.assert_array_equal(tail[:, :80], flat[:, :80])                # preproc
    np.testing.assert_array_equal(tail[:, 80:720], flat[:, C.OFF_SUB1:C.OFF_SUB2])
    np.testing.assert_array_equal(tail[:, 720:1104], flat[:, C.OFF_RED:])
    assert not tail[:, 1104:].any()                                          # zero pad (export.py:370-371)
    np.testing.assert_array_equal(n, flat[:, C.OFF_MHSA_LEN].astype(np.int64))


def test_torch_matches_numpy_and_accepts_b1_lengths():
    flat = random_flat(4, seed=2)
    tn, cn, nn = flat_to_triton(flat)
    tt, ct, nt = flat_to_triton(torch.from_numpy(flat))
    assert isinstance(tt, torch.Tensor) and tt.dtype == torch.float16 and nt.dtype == torch.int64
    np.testing.assert_array_equal(tt.numpy(), tn)
    np.testing.assert_array_equal(ct.numpy(), cn)
    np.testing.assert_array_equal(nt.numpy(), nn)
    back = triton_to_flat(tt, ct, nt[:, None])                               # (B,1) as export.py:403
    np.testing.assert_array_equal(back.numpy().view(np.uint16), flat.view(np.uint16))


def test_zero_state_maps_to_zero_caches():
    t, c, n = flat_to_triton(np.zeros((2, C.STATE_SIZE), np.float16))
    assert not t.any() and not c.any() and not n.any()


def test_bad_shapes_and_dtypes_raise():
    with pytest.raises(ValueError):
        flat_to_triton(np.zeros((2, C.STATE_SIZE - 1), np.float16))
    with pytest.raises(ValueError):
        flat_to_triton(np.zeros((2, C.STATE_SIZE), np.float32))
    t, c, n = flat_to_triton(np.zeros((2, C.STATE_SIZE), np.float16))
    with pytest.raises(ValueError):
        triton_to_flat(t[:, :17], c, n)
    with pytest.raises(ValueError):
        triton_to_flat(t, c[..., :49], n)
    with pytest.raises(ValueError):
        triton_to_flat(t, c, n[:1])
