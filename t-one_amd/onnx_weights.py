"""Read the weights of a T-one ``model.onnx`` without onnx / onnxruntime.

The reference loads ``model.onnx`` into an ORT session (``tone/onnx_wrapper.py:60-78``;
``StreamingCTCPipeline.from_local`` passes ``dir/model.onnx``, ``tone/pipeline.py:90``).  This path
does not execute ONNX graphs, it only needs the parameters: the graph initializers (and tensor-valued
``Constant`` nodes), which are ``TensorProto`` messages inside ``ModelProto.graph``.  Protobuf's wire
format is simple enough to walk directly, so no ``onnx`` package is needed (none is installed here).

Fields used (onnx.proto, IR version >= 3):

* ``ModelProto``:  7 graph
* ``GraphProto``:  1 node (repeated NodeProto), 5 initializer (repeated TensorProto)
* ``NodeProto``:   2 output, 4 op_type, 5 attribute (AttributeProto: 1 name, 5 t)
* ``TensorProto``: 1 dims, 2 data_type, 4 float_data, 5 int32_data, 7 int64_data, 8 name,
  9 raw_data, 10 double_data, 14 data_location (1 = EXTERNAL, not supported)

Mapping onto the reference ``state_dict`` names (:data:`tone_amd.weights.PARAM_SHAPES`): an
initializer named like a parameter (optionally prefixed ``tone.``, as the HF ``ToneForCTC`` export
does) is taken as is, or transposed when it holds the ``[in, out]`` MatMul form of a Linear weight.
Constant-folded initializers with generated names (``onnx::MatMul_123``) cannot be attributed to a
parameter from the file alone; :func:`load_onnx_weights` then names the missing parameters in its error.
"""

from __future__ import annotations

from pathlib import Path
from typing import Iterator

import numpy as np

# TensorProto.DataType -> numpy dtype (raw_data is little-endian)
_DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
           9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64, 16: "bfloat16"}


class OnnxFormatError(ValueError):
    """The file is not a readable ONNX ModelProto (or uses an unsupported feature)."""


def _varint(buf: memoryview, pos: int) -> tuple[int, int]:
    out = shift = 0
    while True:
        if pos >= len(buf):
            raise OnnxFormatError("truncated varint")
        b = buf[pos]
        pos += 1
        out |= (b & 0x7F) << shift
        if not b & 0x80:
            return out, pos
        shift += 7
        if shift > 63:
            raise OnnxFormatError("varint too long")


def _fields(buf: memoryview) -> Iterator[tuple[int, int, object]]:
    """(field number, wire type, value) of one message; length-delimited values are memoryviews."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            if pos + 8 > n:
                raise OnnxFormatError("truncated fixed64")
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            if pos + ln > n:
                raise OnnxFormatError("truncated length-delimited field")
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            if pos + 4 > n:
                raise OnnxFormatError("truncated fixed32")
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise OnnxFormatError(f"unsupported wire type {wt}")
        yield field, wt, v


def _packed_varints(v, wt) -> list[int]:
    if wt == 0:
        return [int(v)]
    out, pos = [], 0
    while pos < len(v):
        x, pos = _varint(v, pos)
        out.append(x)
    return out


def _signed64(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


def parse_tensor(buf: memoryview) -> tuple[str, np.ndarray]:
    """One TensorProto -> (name, array).  bfloat16 is widened to float32; fp16 stays fp16."""
    dims: list[int] = []
    dtype = 0
    name = ""
    raw = None
    floats: list[bytes] = []
    ints: list[int] = []
    int64s: list[int] = []
    doubles: list[bytes] = []
    for f, wt, v in _fields(buf):
        if f == 1:
            dims += [_signed64(x) for x in _packed_varints(v, wt)]
        elif f == 2:
            dtype = int(v)
        elif f == 4:
            floats.append(bytes(v))
        elif f == 5:
            ints += _packed_varints(v, wt)
        elif f == 7:
            int64s += [_signed64(x) for x in _packed_varints(v, wt)]
        elif f == 8:
            name = bytes(v).decode("utf-8", errors="replace")
        elif f == 9:
            raw = bytes(v)
        elif f == 10:
            doubles.append(bytes(v))
        elif f == 14 and int(v) == 1:
            raise OnnxFormatError(f"tensor {name or '?'} uses external data (save the model with the weights inline)")
    if dtype not in _DTYPES:
        raise OnnxFormatError(f"tensor {name}: unsupported data_type {dtype}")
    shape = tuple(dims)
    count = int(np.prod(shape)) if shape else 1
    dt = _DTYPES[dtype]
    if raw is not None:
        if dt == "bfloat16":
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        else:
            arr = np.frombuffer(raw, dtype=np.dtype(dt).newbyteorder("<")).astype(dt)
    elif floats:
        arr = np.frombuffer(b"".join(floats), dtype="<f4").astype(np.float32)
    elif doubles:
        arr = np.frombuffer(b"".join(doubles), dtype="<f8").astype(np.float64)
    elif int64s:
        arr = np.asarray(int64s, dtype=np.int64)
    elif ints or count == 0:
        if dt == np.float16:      # fp16 bit patterns carried in int32_data
            arr = np.asarray(ints, dtype=np.uint16).view(np.float16)
        elif dt == "bfloat16":
            arr = (np.asarray(ints, dtype=np.uint32) << 16).view(np.float32)
        else:
            arr = np.asarray(ints, dtype=np.int64).astype(dt)
    else:
        arr = np.zeros(0, np.float32)
    if arr.size != count:
        raise OnnxFormatError(f"tensor {name}: {arr.size} values for shape {shape}")
    return name, arr.reshape(shape)


def read_onnx_tensors(path: str | Path) -> dict[str, np.ndarray]:
    """All graph initializers plus tensor-valued Constant node outputs of an ONNX model file."""
    data = memoryview(Path(path).read_bytes())
    graph = None
    for f, wt, v in _fields(data):
        if f == 7 and wt == 2:
            graph = v
    if graph is None:
        raise OnnxFormatError(f"{path}: no ModelProto.graph (not an ONNX model?)")
    out: dict[str, np.ndarray] = {}
    for f, wt, v in _fields(graph):
        if f == 5 and wt == 2:
            name, arr = parse_tensor(v)
            out[name] = arr
        elif f == 1 and wt == 2:     # NodeProto: keep Constant(value=tensor)
            op, outs, tensor = "", [], None
            for nf, nwt, nv in _fields(v):
                if nf == 4:
                    op = bytes(nv).decode()
                elif nf == 2:
                    outs.append(bytes(nv).decode())
                elif nf == 5:
                    aname, at = "", None
                    for af, awt, av in _fields(nv):
                        if af == 1:
                            aname = bytes(av).decode()
                        elif af == 5 and awt == 2:
                            at = av
                    if aname == "value" and at is not None:
                        tensor = at
            if op == "Constant" and tensor is not None and outs:
                _, arr = parse_tensor(tensor)
                out.setdefault(outs[0], arr)
    return out


def onnx_state_dict(tensors: dict[str, np.ndarray]) -> dict[str, np.ndarray]:
    """Map ONNX tensors onto reference parameter names (PARAM_SHAPES), float32.

    Only names that match a parameter (with or without the HF ``tone.`` prefix) are used; a 2-D
    tensor whose shape is the transpose of the parameter's is the MatMul form of a Linear weight
    and is transposed back.  Missing parameters are left out (``normalize_keys`` reports them)."""
    from .weights import PARAM_SHAPES

    out: dict[str, np.ndarray] = {}
    for name, arr in tensors.items():
        key = name[len("tone."):] if name.startswith("tone.") else name
        if key not in PARAM_SHAPES or not np.issubdtype(np.asarray(arr).dtype, np.floating):
            continue
        want = PARAM_SHAPES[key]
        a = np.asarray(arr, dtype=np.float32)
        if a.shape != want and a.ndim == 2 and a.T.shape == want:
            a = a.T
        elif a.shape != want and a.size == int(np.prod(want)) and a.ndim < len(want):
            a = a.reshape(want)   # e.g. a 1x1 conv stored as its [out, in] matrix
        out[key] = np.ascontiguousarray(a)
    return out


def load_onnx_weights(path: str | Path):
    """Parameters of ``model.onnx`` by reference name (raises ValueError naming what is missing)."""
    from .weights import PARAM_SHAPES, normalize_keys

    tensors = read_onnx_tensors(path)
    sd = onnx_state_dict(tensors)
    missing = [k for k in PARAM_SHAPES if k not in sd]
    if missing:
        raise ValueError(
            f"{path}: {len(missing)} of {len(PARAM_SHAPES)} T-one parameters are not named initializers of the "
            f"ONNX graph (e.g. {missing[:3]}); constant-folded exports rename them. Export with "
            "do_constant_folding=False, or place model.safetensors from t-tech/T-one next to it.")
    return normalize_keys(sd)

