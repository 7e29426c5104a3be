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

Mapping onto the reference ``state_dict`` names (:data:`tone_amd.weights.PARAM_SHAPES`) follows the GRAPH,
because ``torch.onnx.export`` as tone/scripts/export.py:469-498 calls it (constant folding on, under fp16
autocast, the model wrapped as ``ModelToExport._model``, export.py:144) does not keep parameter names:

* an initializer still named like a parameter (prefix ``_model.`` / ``tone.`` stripped) is taken by name;
* any other float initializer (``onnx::MatMul_123``, a folded ``Cast`` output, ...) is attributed through
  the node that consumes it -- following ``Cast`` / ``Identity`` / ``Transpose`` / ``Reshape`` /
  ``Unsqueeze`` / ``Squeeze`` chains -- whose name carries the module scope
  (``/_model/encoder/layers.0/feed_forward1/linear1/MatMul`` -> ``encoder.layers.0.feed_forward1.linear1``)
  and whose operator fixes the role and the ORIENTATION: ``MatMul`` input B holds ``[in, out]`` (transposed
  back -- square q/k/v/out weights included, which a shape test cannot tell), ``Gemm`` follows ``transB``,
  a ``Transpose`` on the way applies its ``perm``; ``Conv`` inputs 1 / 2 are weight / bias; ``Add`` after
  a MatMul is the bias; ``BatchNormalization`` inputs 1-4 and ``LayerNormalization`` inputs 1-2 are the norm
  parameters; ``Mul`` is an RMSNorm gain;
* a BatchNorm the exporter fused into its convolution (eval-mode Conv+BatchNormalization peephole) leaves
  no parameters of its own: it is loaded as the identity (gain 1, shift 0, mean 0, var 1 - eps) and the conv
  carries the fused weight and bias -- only when the graph has no BatchNormalization node in that scope and the
  conv's weight and bias were both attributed through a Conv node.

The node-name convention (``/_model/<module>/<child>/.../<Op>``, nested containers as ``conv.0`` /
``conv.0.0``) is the one torch.onnx.export's TorchScript exporter writes for scoped modules; it is ASSUMED
here, not pinned: no export of the reference module is available in this environment (the ``onnx`` package
is absent, so torch.onnx.export cannot run), and the tests build graphs with the same convention.

Whatever is still unattributed is named in :func:`load_onnx_weights`'s error.
"""

from __future__ import annotations

from pathlib import Path
from typing import Iterator

import numpy as np

from . import config as C

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


def _attr_value(buf) -> tuple[str, object]:
    """AttributeProto -> (name, int | list[int] | tensor bytes): 1 name, 3 i, 5 t, 8 ints."""
    name, val, ints = "", None, []
    for f, wt, v in _fields(buf):
        if f == 1:
            name = bytes(v).decode()
        elif f == 3:
            val = _signed64(int(v))
        elif f == 5 and wt == 2:
            val = v
        elif f == 8:
            ints += [_signed64(x) for x in _packed_varints(v, wt)]
    return name, (ints if ints else val)


def read_onnx_graph(path: str | Path) -> tuple[dict[str, np.ndarray], list[dict]]:
    """Initializers plus tensor-valued Constant node outputs, and every node as
    ``{"name", "op", "inputs", "outputs", "attrs"}`` (NodeProto: 1 input, 2 output, 3 name, 4 op_type, 5 attribute)."""
    data = memoryview(Path(path).read_bytes())
    graph = None
    for f, wt, v in _fields(data):
        if f == 7 and wt == 2:
            graph = v
    if graph is None:
        raise OnnxFormatError(f"{path}: no ModelProto.graph (not an ONNX model?)")
    out: dict[str, np.ndarray] = {}
    nodes: list[dict] = []
    for f, wt, v in _fields(graph):
        if f == 5 and wt == 2:
            name, arr = parse_tensor(v)
            out[name] = arr
        elif f == 1 and wt == 2:
            node = {"name": "", "op": "", "inputs": [], "outputs": [], "attrs": {}}
            for nf, nwt, nv in _fields(v):
                if nf == 1:
                    node["inputs"].append(bytes(nv).decode())
                elif nf == 2:
                    node["outputs"].append(bytes(nv).decode())
                elif nf == 3:
                    node["name"] = bytes(nv).decode()
                elif nf == 4:
                    node["op"] = bytes(nv).decode()
                elif nf == 5:
                    an, av = _attr_value(nv)
                    node["attrs"][an] = av
            if node["op"] == "Constant" and isinstance(node["attrs"].get("value"), memoryview) and node["outputs"]:
                _, arr = parse_tensor(node["attrs"]["value"])
                out.setdefault(node["outputs"][0], arr)
            nodes.append(node)
    return out, nodes


def read_onnx_tensors(path: str | Path) -> dict[str, np.ndarray]:
    """All graph initializers plus tensor-valued Constant node outputs of an ONNX model file."""
    return read_onnx_graph(path)[0]


_PREFIXES = ("_model.", "tone.")                 # ModelToExport._model (export.py:144); HF ToneForCTC.tone
_PASS = {"Cast", "Identity", "Transpose", "Reshape", "Unsqueeze", "Squeeze", "Flatten"}


def _strip(name: str) -> str:
    for p in _PREFIXES:
        if name.startswith(p):
            return name[len(p):]
    return name


def scope_of(node_name: str) -> str:
    """Module path of a node: ``/_model/encoder/layers.0/conv/pointwise_conv1/Conv`` ->
    ``encoder.layers.0.conv.pointwise_conv1``.  A segment that repeats its parent as a prefix (the exporter's
    ``conv.0`` / ``conv.0.0`` form of nested containers) replaces the parent."""
    segs = [x for x in node_name.split("/") if x][:-1]
    path: list[str] = []
    for sg in segs:
        if path and sg.startswith(path[-1] + "."):
            path[-1] = sg
        else:
            path.append(sg)
    return _strip(".".join(path))


def _roles(node: dict, slot: int, producer_op: str) -> list[str]:
    """Parameter role(s) of input ``slot`` of ``node``."""
    op = node["op"]
    if op in ("MatMul", "Gemm", "Conv"):
        return ["weight"] if slot == 1 else (["bias"] if slot == 2 else [])
    if op == "Add":
        return ["bias"]
    if op == "BatchNormalization":
        return {1: ["weight"], 2: ["bias"], 3: ["running_mean"], 4: ["running_var"]}.get(slot, [])
    if op == "LayerNormalization":
        return {1: ["weight"], 2: ["bias"]}.get(slot, [])
    if op == "Mul":
        return ["weight"]
    return []


def _bn_conv(bn_scope: str) -> str | None:
    """The convolution a BatchNorm follows in the T-one module tree: ``pre_encode.conv.<i>.1`` after
    ``pre_encode.conv.<i>.0`` (conformer_blocks.py:631-641), ``layers.<l>.conv.batch_norm`` after
    ``layers.<l>.conv.depthwise_conv.conv`` (submodules.py:346-402)."""
    if bn_scope.endswith(".batch_norm"):
        return bn_scope[: -len("batch_norm")] + "depthwise_conv.conv"
    if bn_scope.endswith(".1"):
        return bn_scope[:-2] + ".0"
    return None


def onnx_state_dict(tensors: dict[str, np.ndarray], nodes: list[dict] | None = None) -> dict[str, np.ndarray]:
    """Map ONNX tensors onto reference parameter names (PARAM_SHAPES), float32 (see the module docstring).
    Missing parameters are left out (:func:`load_onnx_weights` reports them)."""
    from .weights import PARAM_SHAPES

    out: dict[str, np.ndarray] = {}

    def put(key: str, a: np.ndarray, transposed: bool) -> bool:
        want = PARAM_SHAPES.get(key)
        if want is None or key in out:
            return False
        a = np.asarray(a, dtype=np.float32)
        if transposed and a.ndim == 2:
            a = a.T
        if a.shape != want:
            if a.size != int(np.prod(want)) or a.ndim >= len(want):
                return False
            a = a.reshape(want)          # e.g. a 1x1 conv stored as its [out, in] matrix
        out[key] = np.ascontiguousarray(a)
        return True

    floats = {k: v for k, v in tensors.items() if np.issubdtype(np.asarray(v).dtype, np.floating)}
    # 1) by name
    for name, arr in floats.items():
        key = _strip(name)
        if key in PARAM_SHAPES:
            want = PARAM_SHAPES[key]
            put(key, arr, np.asarray(arr).shape != want and np.asarray(arr).ndim == 2 and np.asarray(arr).T.shape == want)
    if not nodes:
        return out
    # 2) through the consuming node's scope
    consumers: dict[str, list[tuple[dict, int]]] = {}
    for nd in nodes:
        for i, x in enumerate(nd["inputs"]):
            consumers.setdefault(x, []).append((nd, i))
    via_conv: set[str] = set()            # parameters attributed as a Conv node's weight / bias

    def attribute(name: str, arr: np.ndarray) -> bool:
        """Walk from one initializer through pass-through ops to the first compute node that names a
        parameter slot for it; stop at the FIRST successful put (a constant shared by several consumers is
        written under one key only)."""
        frontier = [(name, False, 0)]
        seen = set()
        while frontier:
            val, tr, depth = frontier.pop()
            if val in seen or depth > 6:
                continue
            seen.add(val)
            for nd, slot in consumers.get(val, []):
                if nd["op"] in _PASS:
                    t = tr
                    if nd["op"] == "Transpose":
                        perm = nd["attrs"].get("perm")
                        t = tr ^ (perm is None or list(perm)[-2:] == [1, 0] or list(perm) == [1, 0])
                    for o in nd["outputs"]:
                        frontier.append((o, t, depth + 1))
                    continue
                scope = scope_of(nd["name"])
                if not scope:
                    continue
                transposed = tr
                if nd["op"] == "MatMul" and slot == 1:
                    transposed = not tr                                  # B = [in, out]
                elif nd["op"] == "Gemm" and slot == 1:
                    transposed = tr ^ (not nd["attrs"].get("transB", 0))
                for role in _roles(nd, slot, ""):
                    key = f"{scope}.{role}"
                    if put(key, arr, transposed):
                        if nd["op"] == "Conv":
                            via_conv.add(key)
                        return True
        return False

    for name, arr in floats.items():
        if _strip(name) not in PARAM_SHAPES:
            attribute(name, arr)
    # 3) a BatchNorm the exporter fused into its convolution leaves no parameters: identity norm -- but only
    #    when the graph has no BatchNormalization node in that scope (an unfused BN whose inputs could not be
    #    attributed must stay missing, so load_onnx_weights raises) and the convolution it follows got both
    #    its weight and its bias from a Conv node (the fused pair)
    bn_scopes = {scope_of(nd["name"]) for nd in nodes if nd["op"] == "BatchNormalization"}
    for key in PARAM_SHAPES:
        if not key.endswith(".running_var"):
            continue
        base = key[: -len("running_var")]
        bn = [base + r for r in ("weight", "bias", "running_mean", "running_var")]
        if any(k in out for k in bn) or base[:-1] in bn_scopes:
            continue
        conv = _bn_conv(base[:-1])
        if conv is None or f"{conv}.weight" not in via_conv or f"{conv}.bias" not in via_conv:
            continue
        n = PARAM_SHAPES[key][0]
        out[bn[0]] = np.ones(n, np.float32)
        out[bn[1]] = np.zeros(n, np.float32)
        out[bn[2]] = np.zeros(n, np.float32)
        out[bn[3]] = np.full(n, 1.0 - 1e-5, np.float32)    # 1 / sqrt(var + eps) = 1
    return out


# ---- the flat state layout inside the artifact ----------------------------------------------------------
# The 2-input graph (configs/streaming_acoustic/config.pbtxt:5-33: signal (B,2400,1) int32, state (B,219729)
# fp16 -> logprobs, state_next) cuts its ``state`` input into the seven tensors of Tone.forward_for_export
# (tone/nn/model.py:101-113) with Slice / Split nodes followed by Reshape, and builds ``state_next`` with one
# Concat along axis 1.  The exporter of that artifact is not in the reference, so instead of
# assuming its order, the loader reads it from those nodes and compares it with tone_amd.config.STATE_SECTIONS.
_STATE_PASS = {"Cast", "Identity"}
_INT64_MAX = (1 << 63) - 1


def _const(tensors: dict, name: str):
    return None if name not in tensors else np.asarray(tensors[name])


def _shape_tail(tensors: dict, name: str):
    """Per-stream shape of a Reshape's constant shape input ([B or -1 or 0, ...] -> the rest), or None."""
    s = _const(tensors, name)
    if s is None or s.ndim != 1 or len(s) < 2 or np.any(s[1:] <= 0):
        return None
    return tuple(int(x) for x in s[1:])


def onnx_state_layout(tensors: dict[str, np.ndarray], nodes: list[dict], state_in: str = "state",
                      state_out: str = "state_next") -> dict | None:
    """The flat state layout a graph implements, or None when the graph has no ``state`` input consumer.

    ``input``: the segments the graph cuts from ``state``, sorted by offset: ``(offset, size, shape)`` with
    ``shape`` the per-stream shape of the Reshape that follows the cut (None when it is not a constant).
    ``output``: per input of the Concat that produces ``state_next``, in order, ``(size, shape)`` from the
    constant Reshape / Flatten in front of it (None entries where the graph computes shapes at run time);
    None when no such Concat is found."""
    consumers: dict[str, list[tuple[dict, int]]] = {}
    producer: dict[str, dict] = {}
    for nd in nodes:
        for i, x in enumerate(nd["inputs"]):
            consumers.setdefault(x, []).append((nd, i))
        for o in nd["outputs"]:
            producer[o] = nd
    if state_in not in consumers:
        return None

    def axis_ok(ax) -> bool:
        return int(ax) in (1, -1)

    segs: list[list] = []                       # [offset, size, value name]
    frontier = [(state_in, 0)]
    seen = set()
    while frontier:
        val, depth = frontier.pop()
        if val in seen or depth > 8:
            continue
        seen.add(val)
        for nd, slot in consumers.get(val, []):
            if slot != 0:
                continue
            op = nd["op"]
            if op in _STATE_PASS:
                frontier += [(o, depth + 1) for o in nd["outputs"]]
            elif op == "Slice":
                ins = nd["inputs"] + [""] * 5
                st, en = _const(tensors, ins[1]), _const(tensors, ins[2])
                ax = _const(tensors, ins[3]) if ins[3] else np.array([1])
                stp = _const(tensors, ins[4]) if ins[4] else np.array([1])
                if st is None or en is None or ax is None or stp is None or st.size != 1 or not axis_ok(ax.ravel()[0]) \
                        or int(stp.ravel()[0]) != 1:
                    raise ValueError(f"state input: Slice {nd['name'] or '?'} is not a constant unit-step cut along axis 1")
                a = int(st.ravel()[0])
                b = min(int(en.ravel()[0]), C.STATE_SIZE)
                segs.append([a, b - a, nd["outputs"][0]])
            elif op == "Split":
                ax = nd["attrs"].get("axis", 0)
                sizes = nd["attrs"].get("split")
                if sizes is None and len(nd["inputs"]) > 1 and nd["inputs"][1]:
                    sz = _const(tensors, nd["inputs"][1])
                    sizes = None if sz is None else [int(x) for x in sz.ravel()]
                if not axis_ok(ax) or not sizes:
                    raise ValueError(f"state input: Split {nd['name'] or '?'} is not a constant split along axis 1")
                off = 0
                for s, o in zip(sizes, nd["outputs"]):
                    segs.append([off, int(s), o])
                    off += int(s)
    if not segs:
        return None

    def reshape_after(val: str, depth: int = 0):
        for nd, slot in consumers.get(val, []):
            if nd["op"] in _STATE_PASS and depth < 4:
                r = reshape_after(nd["outputs"][0], depth + 1)
                if r is not None:
                    return r
            elif nd["op"] == "Reshape" and slot == 0:
                return _shape_tail(tensors, nd["inputs"][1])
        return None

    layout_in = sorted((a, s, reshape_after(v)) for a, s, v in segs)

    # state_next: Concat (axis 1) of the flattened next states
    def size_of(val: str, depth: int = 0):
        nd = producer.get(val)
        if nd is None or depth > 6:
            return None, None
        if nd["op"] in _STATE_PASS:
            return size_of(nd["inputs"][0], depth + 1)
        if nd["op"] == "Reshape":
            t = _shape_tail(tensors, nd["inputs"][1])
            if t is not None:
                if len(t) == 1:                   # [B, n]: the per-stream shape is the one before the flatten
                    inner = size_of(nd["inputs"][0], depth + 1)[1]
                    return t[0], inner
                return int(np.prod(t)), t
            inner = size_of(nd["inputs"][0], depth + 1)
            return inner
        if nd["op"] == "Flatten" and int(nd["attrs"].get("axis", 1)) == 1:
            return size_of(nd["inputs"][0], depth + 1)
        return None, None

    out_node = producer.get(state_out)
    while out_node is not None and out_node["op"] in _STATE_PASS:
        out_node = producer.get(out_node["inputs"][0])
    layout_out = None
    if out_node is not None and out_node["op"] == "Concat" and axis_ok(out_node["attrs"].get("axis", 0)):
        layout_out = [size_of(x) for x in out_node["inputs"]]
    return {"input": layout_in, "output": layout_out}


def check_state_layout(layout: dict | None, where: str = "model.onnx") -> None:
    """Compare a graph's state layout (:func:`onnx_state_layout`) with tone_amd.config.STATE_SECTIONS; raise
    ValueError naming the difference.  The seven segment sizes are distinct, so each cut is identified by its
    size; a per-stream shape is compared where the graph reshapes with a constant shape."""
    if layout is None:
        return
    want = sorted((off, int(np.prod(shp)), shp, name) for name, (off, shp) in C.STATE_SECTIONS.items())
    by_size = {w[1]: w[3] for w in want}

    def names(sizes):
        return " | ".join(by_size.get(s, f"?({s})") if s is not None else "?" for s in sizes)

    got = layout["input"]
    if [g[1] for g in got] != [w[1] for w in want] or [g[0] for g in got] != [w[0] for w in want]:
        raise ValueError(
            f"{where}: the graph cuts its state input as {names([g[1] for g in got])} "
            f"(offsets {[g[0] for g in got]}); this engine's flat state is {names([w[1] for w in want])} "
            f"(offsets {[w[0] for w in want]}, tone_amd/config.py). Convert the state (tone_amd.state) or use a "
            "matching artifact.")
    for (off, size, shp), (_, _, wshp, name) in zip(got, want):
        if shp is not None and tuple(shp) != tuple(wshp) and tuple(x for x in shp if x != 1) != tuple(x for x in wshp if x != 1):
            raise ValueError(f"{where}: state segment {name} at offset {off} is reshaped to {tuple(shp)} in the graph, "
                             f"{tuple(wshp)} in this engine (a transposed layout inside the segment)")
    out = layout["output"]
    if out is not None:
        sizes = [o[0] for o in out]
        if all(s is not None for s in sizes) and sizes != [w[1] for w in want]:
            raise ValueError(f"{where}: the graph concatenates state_next as {names(sizes)}; this engine writes "
                             f"{names([w[1] for w in want])}")
        for (size, shp), (_, _, wshp, name) in zip(out, want):
            if shp is not None and tuple(x for x in shp if x != 1) != tuple(x for x in wshp if x != 1):
                raise ValueError(f"{where}: next-state segment {name} is flattened from {tuple(shp)} in the graph, "
                                 f"{tuple(wshp)} in this engine")


def load_onnx_weights(path: str | Path):
    """Parameters of ``model.onnx`` by reference name (raises ValueError naming what is missing).  When the
    graph takes the flat ``state`` input, its state layout is checked against this engine's first
    (:func:`check_state_layout`)."""
    from .weights import PARAM_SHAPES, normalize_keys

    tensors, nodes = read_onnx_graph(path)
    check_state_layout(onnx_state_layout(tensors, nodes), str(path))
    sd = onnx_state_dict(tensors, nodes)
    missing = [k for k in PARAM_SHAPES if k not in sd]
    if missing:
        raise ValueError(
            f"{path}: {len(missing)} of {len(PARAM_SHAPES)} T-one parameters could not be attributed to ONNX "
            f"initializers by name or by their consuming node's scope (e.g. {missing[:3]}). Place model.safetensors "
            "from t-tech/T-one next to it, or export with do_constant_folding=False.")
    return normalize_keys(sd)
