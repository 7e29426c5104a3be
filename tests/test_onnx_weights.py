"""model.onnx weight import (tone_amd.onnx_weights) on hand-built ONNX files (CPU only).

The reference's artifact is ``model.onnx`` (tone/onnx_wrapper.py:60-78; StreamingCTCPipeline.from_local
passes dir/model.onnx, tone/pipeline.py:90).  No onnx package exists here, so the files are written with
a ~30-line protobuf encoder following onnx.proto's field numbers; the reader is checked on every tensor
encoding it accepts (raw_data fp32/fp16/bf16, packed float_data, fp16 in int32_data, Constant nodes,
transposed MatMul weights) and on the full T-one catalogue.
"""

from __future__ import annotations

import numpy as np
import pytest

from tone_amd.onnx_weights import OnnxFormatError, load_onnx_weights, read_onnx_tensors
from tone_amd.weights import PARAM_SHAPES, load_weights, synthetic_weights


# ---- minimal protobuf writer (test infrastructure) ---------------------------------------------
def _varint(x: int) -> bytes:
    x &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        out.append(b | (0x80 if x else 0))
        if not x:
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint(field << 3 | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _vi(field: int, x: int) -> bytes:
    return _key(field, 0) + _varint(x)


def tensor_proto(name: str, arr: np.ndarray, enc: str = "raw") -> bytes:
    """TensorProto: 1 dims, 2 data_type, 4 float_data, 5 int32_data, 8 name, 9 raw_data."""
    dt = {np.float32: 1, np.float16: 10, np.int64: 7}[arr.dtype.type] if enc != "bf16" else 16
    msg = b"".join(_vi(1, d) for d in arr.shape) + _vi(2, dt) + _ld(8, name.encode())
    if enc == "raw":
        msg += _ld(9, np.ascontiguousarray(arr).astype(arr.dtype.newbyteorder("<")).tobytes())
    elif enc == "bf16":
        u = (np.ascontiguousarray(arr, np.float32).view(np.uint32) >> 16).astype("<u2")
        msg += _ld(9, u.tobytes())
    elif enc == "float_data":
        msg += _ld(4, arr.astype("<f4").tobytes())
    elif enc == "int32_data":      # fp16 bit patterns, packed varints
        msg += _ld(5, b"".join(_varint(int(v)) for v in arr.view(np.uint16).ravel()))
    return msg


def constant_node(output: str, arr: np.ndarray) -> bytes:
    attr = _ld(1, b"value") + _ld(5, tensor_proto("", arr))
    return _ld(2, output.encode()) + _ld(4, b"Constant") + _ld(5, attr)


def model_proto(initializers: list[bytes], nodes: list[bytes] = ()) -> bytes:
    graph = b"".join(_ld(1, n) for n in nodes) + _ld(2, b"tone") + b"".join(_ld(5, t) for t in initializers)
    return _vi(1, 8) + _ld(7, graph)


# ---- tests -------------------------------------------------------------------------------------
def test_tensor_encodings(tmp_path):
    rng = np.random.default_rng(0)
    a = rng.standard_normal((3, 5)).astype(np.float32)
    h = rng.standard_normal((4,)).astype(np.float16)
    inits = [tensor_proto("a_raw", a), tensor_proto("a_fd", a, "float_data"), tensor_proto("h_raw", h),
             tensor_proto("h_i32", h, "int32_data"), tensor_proto("a_bf", a, "bf16"),
             tensor_proto("i64", np.array([-3, 7], np.int64))]
    p = tmp_path / "m.onnx"
    p.write_bytes(model_proto(inits, [constant_node("c0", a[:2])]))
    t = read_onnx_tensors(p)
    np.testing.assert_array_equal(t["a_raw"], a)
    np.testing.assert_array_equal(t["a_fd"], a)
    np.testing.assert_array_equal(t["h_raw"], h)
    np.testing.assert_array_equal(t["h_i32"], h)
    assert t["h_raw"].dtype == np.float16
    bf = (a.view(np.uint32) & 0xFFFF0000).view(np.float32)
    np.testing.assert_array_equal(t["a_bf"], bf)
    np.testing.assert_array_equal(t["i64"], [-3, 7])
    np.testing.assert_array_equal(t["c0"], a[:2])


def test_rejects_non_onnx_and_external_data(tmp_path):
    p = tmp_path / "bad.onnx"
    p.write_bytes(b"\x0f\x00garbage")
    with pytest.raises(OnnxFormatError):
        read_onnx_tensors(p)
    ext = _vi(1, 2) + _vi(2, 1) + _ld(8, b"w") + _vi(14, 1)
    p.write_bytes(model_proto([ext]))
    with pytest.raises(OnnxFormatError, match="external"):
        read_onnx_tensors(p)


def test_full_catalogue_from_model_onnx(tmp_path):
    """Every T-one parameter as an fp16 initializer named like the HF checkpoint ("tone." prefix), the
    FFN linear1 weights of layer 3 in MatMul ([in, out]) form: from_local's loader gets them back
    exactly (fp16-rounded), and a directory holding only model.onnx resolves to it."""
    w = synthetic_weights(5)
    inits = []
    for k, v in w.items():
        arr = v.astype(np.float16)
        if k == "encoder.layers.3.feed_forward1.linear1.weight":
            arr = np.ascontiguousarray(arr.T)
        inits.append(tensor_proto("tone." + k, arr))
    d = tmp_path / "ckpt"
    d.mkdir()
    (d / "model.onnx").write_bytes(model_proto(inits))
    got = load_onnx_weights(d / "model.onnx")
    assert list(got) == list(PARAM_SHAPES)
    for k in ("encoder.layers.3.feed_forward1.linear1.weight", "decoder.decoder_layers.0.weight",
              "encoder.pre_encode.conv.1.0.weight"):
        np.testing.assert_array_equal(got[k], w[k].astype(np.float16).astype(np.float32))
    back = load_weights(d)
    np.testing.assert_array_equal(back["encoder.layers.15.self_attn.q_ln.bias"],
                                  got["encoder.layers.15.self_attn.q_ln.bias"])


def test_missing_parameters_are_named(tmp_path):
    w = synthetic_weights(0)
    inits = [tensor_proto(k, v.astype(np.float16)) for k, v in list(w.items())[:10]]
    inits.append(tensor_proto("onnx::MatMul_1234", np.zeros((384, 1536), np.float16)))
    p = tmp_path / "model.onnx"
    p.write_bytes(model_proto(inits))
    with pytest.raises(ValueError, match="not named initializers"):
        load_weights(p)
