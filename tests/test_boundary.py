"""The drop-in boundary on CPU: the C-ABI library loads and exports every declared symbol, the
numpy front door raises the reference's exceptions, and the product path has no CPU fallback."""

import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import tone_amd
import tone_amd.config as C
from tone_amd import _lib
from tone_amd.model import StreamingCTCModel, validate_inputs
from tone_amd.weights import PARAM_SHAPES, load_weights, normalize_keys, synthetic_weights

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "tonehip.h"


def _declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(tone_[a-z_0-9]+)\s*\(", text, re.M)))


def test_header_declares_the_abi():
    syms = _declared_symbols()
    assert "tone_session_run" in syms and "tone_session_run_slots" in syms and "tone_last_error" in syms
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table and include/tonehip.h disagree"


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    for name in _declared_symbols():
        assert hasattr(lib, name), name
    assert _lib.load().tone_abi_version() == _lib.ABI_VERSION


def test_library_is_gfx950():
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "nope.so")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.load()


def test_class_constants_match_reference():
    """tone/onnx_wrapper.py:30-34; the pipeline reads them from the class (pipeline.py:49)."""
    assert StreamingCTCModel.SAMPLE_RATE == 8000
    assert StreamingCTCModel.MEAN_TIME_BIAS == 0.33
    assert StreamingCTCModel.AUDIO_CHUNK_SAMPLES == 2400
    assert StreamingCTCModel.FRAME_SIZE == 0.03
    assert StreamingCTCModel.STATE_SIZE == 219729
    for name in ("from_hugging_face", "from_local", "download_from_hugging_face", "forward"):
        assert callable(getattr(StreamingCTCModel, name))


@pytest.mark.parametrize(
    "chunk,state,exc",
    [
        ([0] * 2400, None, TypeError),                                          # not ndarray
        (np.zeros((1, 2400), np.int32), None, ValueError),                      # bad shape
        (np.zeros((1, 2399, 1), np.int32), None, ValueError),                   # bad length
        (np.zeros((1, 2400, 1), np.int16), None, ValueError),                   # bad dtype
        (np.full((1, 2400, 1), 40000, np.int32), None, ValueError),             # out of int16 range
        (np.full((1, 2400, 1), -32769, np.int32), None, ValueError),
        (np.zeros((1, 2400, 1), np.int32), [0.0], TypeError),                   # bad state type
        (np.zeros((1, 2400, 1), np.int32), np.zeros((2, 219729), np.float16), ValueError),
        (np.zeros((1, 2400, 1), np.int32), np.zeros((1, 219729), np.float32), ValueError),
        (np.zeros((0, 2400, 1), np.int32), None, ValueError),                   # B = 0: min() of empty
    ],
)
def test_input_validation_matches_onnx_wrapper(chunk, state, exc):
    """Error types of tone/onnx_wrapper.py:100-121."""
    with pytest.raises(exc):
        validate_inputs(np.asarray(chunk) if isinstance(chunk, np.ndarray) else chunk, state)


def test_validation_accepts_edges_and_zero_state():
    chunk = np.array([[-32768], [32767]] * 1200, np.int32).reshape(1, 2400, 1)
    st = validate_inputs(chunk, None)
    assert st.shape == (1, C.STATE_SIZE) and st.dtype == np.float16 and not st.any()


def test_weight_loading_roundtrip(tmp_path):
    w = synthetic_weights(3)
    np.savez(tmp_path / "weights.npz", **{"tone." + k: v for k, v in w.items()})
    back = load_weights(tmp_path)
    assert list(back) == list(PARAM_SHAPES)
    np.testing.assert_array_equal(back["encoder.layers.15.self_attn.k_ln.bias"], w["encoder.layers.15.self_attn.k_ln.bias"])
    from safetensors.numpy import save_file
    save_file(w, str(tmp_path / "model.safetensors"))
    back2 = load_weights(tmp_path / "model.safetensors")
    np.testing.assert_array_equal(back2["encoder.pre_encode.out.weight"], w["encoder.pre_encode.out.weight"])


def test_weight_loading_rejects_bad_shapes():
    w = dict(synthetic_weights(0))
    w["encoder.pre_encode.out.weight"] = np.zeros((3, 3), np.float32)
    with pytest.raises(ValueError):
        normalize_keys(w)
    w = dict(synthetic_weights(0))
    del w["decoder.decoder_layers.0.bias"]
    with pytest.raises(ValueError):
        normalize_keys(w)


def test_package_lazy_exports():
    assert tone_amd.StreamingCTCModel is StreamingCTCModel
