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


def node_proto(name: str, op: str, inputs: list[str], outputs: list[str], ints: dict | None = None) -> bytes:
    """NodeProto: 1 input, 2 output, 3 name, 4 op_type, 5 attribute (AttributeProto 1 name, 3 i, 8 ints)."""
    msg = b"".join(_ld(1, x.encode()) for x in inputs) + b"".join(_ld(2, x.encode()) for x in outputs)
    msg += _ld(3, name.encode()) + _ld(4, op.encode())
    for k, v in (ints or {}).items():
        a = _ld(1, k.encode()) + (b"".join(_vi(8, x) for x in v) if isinstance(v, list) else _vi(3, v))
        msg += _ld(5, a)
    return msg


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
    with pytest.raises(ValueError, match="could not be attributed"):
        load_weights(p)


def _fold_bn(w: dict, conv: str, bn: str):
    """Eval Conv + BatchNormalization fused the way the exporter's peephole does: W * s, (b - mean) * s + beta."""
    s = w[bn + "weight"] / np.sqrt(w[bn + "running_var"] + 1e-5)
    wf = w[conv + "weight"] * s.reshape((-1,) + (1,) * (w[conv + "weight"].ndim - 1))
    bf = (w[conv + "bias"] - w[bn + "running_mean"]) * s + w[bn + "bias"]
    return wf.astype(np.float32), bf.astype(np.float32)


def export_like_graph(w: dict) -> bytes:
    """A graph shaped like torch.onnx.export of ModelToExport under fp16 autocast with constant folding
    (tone/scripts/export.py:144,411,469-498): Linear weights folded into anonymous ``onnx::MatMul_*`` fp16
    initializers in MatMul's [in, out] form (square q/k/v/out included), biases behind Cast nodes, 1x1 / grouped
    convolutions as anonymous ``onnx::Conv_*``, every Conv + BatchNorm pair fused (no BN parameters left), the
    pre-encode convolutions under the exporter's nested ``conv.0`` / ``conv.0.0`` scopes, one Linear through
    Gemm(transB=1) and one through an explicit Transpose, norm gains still named with the ``_model.`` prefix."""
    inits, nodes = [], []
    cnt = [0]

    def anon(kind, arr):
        cnt[0] += 1
        name = f"onnx::{kind}_{cnt[0]}"
        inits.append(tensor_proto(name, np.ascontiguousarray(arr)))
        return name

    def scope(mod):
        segs = mod.split(".")
        out, i = [], 0
        while i < len(segs):          # ModuleList children: "layers.0"; nested containers: "conv.0" / "conv.0.0"
            if i + 1 < len(segs) and segs[i + 1].isdigit():
                out.append(segs[i] + "." + segs[i + 1])
                i += 2
                while i < len(segs) and segs[i].isdigit():
                    out.append(out[-1] + "." + segs[i])
                    i += 1
            else:
                out.append(segs[i])
                i += 1
        return "/_model/" + "/".join(out)

    done = set()
    for k in PARAM_SHAPES:
        if k in done:
            continue
        mod, leaf = k.rsplit(".", 1)
        v = w[k]
        if leaf in ("running_mean", "running_var") or (leaf in ("weight", "bias") and (mod + ".running_var") in w):
            continue                                                      # BatchNorm: fused below
        if leaf == "bias" and (mod + ".weight") in w:
            continue                                                      # with its weight
        if v.ndim == 1 or "_ln." in k:                                    # norm gains / LayerNorm: named
            names = [mod + "." + r for r in ("weight", "bias") if (mod + "." + r) in w]
            for n in names:
                inits.append(tensor_proto("_model." + n, w[n].astype(np.float32)))
                done.add(n)
            op = "LayerNormalization" if "_ln." in k else "Mul"
            nodes.append(node_proto(scope(mod) + "/" + op, op, ["x"] + ["_model." + n for n in names], [mod + "_out"]))
            continue
        b = w.get(mod + ".bias")
        bn = mod.rsplit(".", 1)[0] + ".1." if mod.endswith(".0") else None
        if mod.endswith("depthwise_conv.conv"):
            bn = mod.rsplit(".", 2)[0] + ".batch_norm."
        if bn and (bn + "running_var") in w:                              # Conv + BN fused
            wf, bf = _fold_bn(w, mod + ".", bn)
            wn, bnm = anon("Conv", wf), anon("Conv", bf)
            nodes.append(node_proto(scope(mod) + "/Conv", "Conv", ["x", wn, bnm], [mod + "_out"]))
        elif v.ndim == 3:                                                  # 1x1 / grouped Conv1d
            ins = ["x", anon("Conv", v.astype(np.float16))] + ([anon("Conv", b.astype(np.float16))] if b is not None else [])
            nodes.append(node_proto(scope(mod) + "/Conv", "Conv", ins, [mod + "_out"]))
        elif k == "encoder.pre_encode.out.weight":                        # Gemm(transB=1), original orientation
            nodes.append(node_proto(scope(mod) + "/Gemm", "Gemm", ["x", anon("Gemm", v.astype(np.float16))],
                                    [mod + "_out"], {"transB": 1}))
        elif k == "encoder.layers.5.self_attn.linear_out.weight":        # explicit Transpose then MatMul
            t = anon("Transpose", v.astype(np.float16))
            nodes.append(node_proto(scope(mod) + "/Transpose", "Transpose", [t], [mod + "_wt"], {"perm": [1, 0]}))
            nodes.append(node_proto(scope(mod) + "/MatMul", "MatMul", ["x", mod + "_wt"], [mod + "_mm"]))
        else:                                                              # Linear: folded [in, out] MatMul weight
            nodes.append(node_proto(scope(mod) + "/MatMul", "MatMul", ["x", anon("MatMul", v.T.astype(np.float16))],
                                    [mod + "_mm"]))
        if b is not None and not (bn and (bn + "running_var") in w) and v.ndim == 2:
            inits.append(tensor_proto(f"onnx::Cast_{mod}", b.astype(np.float32)))
            nodes.append(node_proto(scope(mod) + "/Cast", "Cast", [f"onnx::Cast_{mod}"], [mod + "_b16"], {"to": 10}))
            nodes.append(node_proto(scope(mod) + "/Add", "Add", [mod + "_mm", mod + "_b16"], [mod + "_out"]))
    return model_proto(inits, nodes)


def test_constant_folded_export_graph(tmp_path):
    """ADVICE r2 / VERDICT r2 #5: the loader reads a model.onnx shaped like the reference's real export (see
    export_like_graph): every parameter comes back -- square Linear weights in the right orientation (decided by
    the consuming MatMul / Gemm / Transpose, not by shape), biases through Cast, fused Conv+BN as the fused conv
    with an identity BatchNorm.  The step computed from the loaded weights equals the step from the checkpoint
    (fp16-rounded, as the export stores it) up to the fusion's fp32 rounding."""
    from tone_oracle import ToneOracle
    w = {k: v.astype(np.float16).astype(np.float32) for k, v in synthetic_weights(3).items()}
    p = tmp_path / "model.onnx"
    p.write_bytes(export_like_graph(w))
    got = load_onnx_weights(p)
    assert list(got) == list(PARAM_SHAPES)
    for k in ("encoder.layers.0.self_attn.linear_q.weight", "encoder.layers.9.self_attn.linear_v.weight",
              "encoder.layers.5.self_attn.linear_out.weight", "encoder.layers.2.feed_forward2.linear2.weight",
              "encoder.pre_encode.out.weight", "encoder.layers.3.conv.pointwise_conv2.weight",
              "encoder.temportal_reduction.conv_pw.weight", "decoder.decoder_layers.0.bias",
              "encoder.layers.14.norm_self_att.weight", "encoder.layers.15.self_attn.k_ln.bias"):
        np.testing.assert_array_equal(got[k], w[k], err_msg=k)
    np.testing.assert_array_equal(got["encoder.layers.4.conv.batch_norm.weight"], np.ones(384, np.float32))
    rng = np.random.default_rng(1)
    pcm = np.clip(rng.normal(0, 3000, (2, 2400)), -32768, 32767).astype(np.int32)
    lp_ref, _ = ToneOracle(w).step(pcm)
    lp_got, _ = ToneOracle(got).step(pcm)
    assert np.abs(lp_got - lp_ref).max() < 2e-3


def test_download_prefers_safetensors_then_onnx(monkeypatch):
    """from_hugging_face asks the HF cache for model.safetensors first (every parameter by name) and falls back
    to the reference's own artifact, model.onnx (tone/onnx_wrapper.py:60-63), only when that file does not
    exist (repository or offline cache); any other failure propagates; prefer_safetensors=False goes straight
    to model.onnx."""
    import huggingface_hub
    from huggingface_hub.utils import LocalEntryNotFoundError
    from tone_amd.model import StreamingCTCModel
    asked = []

    def fake(repo, fname):
        asked.append((repo, fname))
        if fname == "model.safetensors":
            raise LocalEntryNotFoundError(fname)
        return "/cache/" + fname

    monkeypatch.setattr(huggingface_hub, "hf_hub_download", fake)
    assert StreamingCTCModel.download_from_hugging_face() == "/cache/model.onnx"
    assert asked == [("t-tech/T-one", "model.safetensors"), ("t-tech/T-one", "model.onnx")]
    asked.clear()
    assert StreamingCTCModel.download_from_hugging_face(prefer_safetensors=False) == "/cache/model.onnx"
    assert asked == [("t-tech/T-one", "model.onnx")]

    def broken(repo, fname):
        raise PermissionError("401: token rejected")

    monkeypatch.setattr(huggingface_hub, "hf_hub_download", broken)
    with pytest.raises(PermissionError):
        StreamingCTCModel.download_from_hugging_face()


# ---- the flat state layout inside the artifact -----------------------------------------
def _state_graph(order=None, shapes=None, split=False, out_order=None):
    """Nodes + initializers of the 2-input graph's state plumbing (configs/streaming_acoustic/config.pbtxt:5-33):
    ``state`` (B, 219729) fp16 cut into the seven forward_for_export tensors by Slice (or one Split) + Reshape,
    and ``state_next`` = Concat(axis 1) of the flattened next states.  ``order`` permutes the sections (a
    different artifact layout), ``shapes`` overrides a section's per-stream shape."""
    from tone_amd import config as C
    secs = [(n, int(np.prod(shp)), tuple(shp)) for n, (_, shp) in sorted(C.STATE_SECTIONS.items(), key=lambda kv: kv[1][0])]
    if order is not None:
        secs = [secs[i] for i in order]
    shapes = shapes or {}
    inits, nodes = [], []
    i64 = lambda v: np.asarray(v, np.int64)
    nodes.append(node_proto("/Cast_state", "Cast", ["state"], ["state_f32"], {"to": 1}))
    off = 0
    if split:
        inits.append(tensor_proto("split_sizes", i64([s for _, s, _ in secs])))
        nodes.append(node_proto("/Split", "Split", ["state_f32", "split_sizes"], [f"cut_{n}" for n, _, _ in secs],
                                {"axis": 1}))
    for n, size, shp in secs:
        if not split:
            for nm, v in ((f"st_{n}", [off]), (f"en_{n}", [off + size]), (f"ax_{n}", [1])):
                inits.append(tensor_proto(nm, i64(v)))
            nodes.append(node_proto(f"/Slice_{n}", "Slice", ["state_f32", f"st_{n}", f"en_{n}", f"ax_{n}"], [f"cut_{n}"]))
        shp = shapes.get(n, shp)
        inits.append(tensor_proto(f"shape_{n}", i64((-1,) + tuple(shp))))
        nodes.append(node_proto(f"/Reshape_{n}", "Reshape", [f"cut_{n}", f"shape_{n}"], [f"state_{n}"]))
        off += size
    outs = secs if out_order is None else [secs[i] for i in out_order]
    for n, size, shp in outs:
        inits.append(tensor_proto(f"flat_{n}", i64([-1, size])))
        nodes.append(node_proto(f"/Reshape_next_{n}", "Reshape", [f"next_{n}", f"flat_{n}"], [f"next_flat_{n}"]))
    nodes.append(node_proto("/Concat_next", "Concat", [f"next_flat_{n}" for n, _, _ in outs], ["state_next_f32"],
                            {"axis": 1}))
    nodes.append(node_proto("/Cast_next", "Cast", ["state_next_f32"], ["state_next"], {"to": 10}))
    return inits, nodes


@pytest.mark.parametrize("split", [False, True])
def test_state_layout_read_from_graph(split):
    """The loader recovers the seven segments' offsets and shapes from the Slice / Split + Reshape nodes that
    consume ``state`` and the Concat that makes ``state_next``, and they equal tone_amd/config.py's
    forward_for_export order (tone/nn/model.py:101-113)."""
    from tone_amd import config as C
    from tone_amd.onnx_weights import check_state_layout, onnx_state_layout, read_onnx_graph
    import tempfile, os
    inits, nodes = _state_graph(split=split)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.onnx")
        open(p, "wb").write(model_proto(inits, nodes))
        t, n = read_onnx_graph(p)
    lay = onnx_state_layout(t, n)
    want = sorted((off, int(np.prod(s)), tuple(s)) for off, s in C.STATE_SECTIONS.values())
    assert lay["input"] == want
    assert [o[0] for o in lay["output"]] == [w[1] for w in want]
    check_state_layout(lay)


@pytest.mark.parametrize("case", ["permuted", "transposed_conv", "out_permuted"])
def test_state_layout_mismatch_rejected(tmp_path, case):
    """An artifact whose flat state is ordered differently (conv before mhsa), whose conv state is stored
    (16, 30, 384) instead of (16, 384, 30), or whose state_next is concatenated in another order, is rejected
    by load_weights with an error naming the difference, instead of loading and producing garbage states."""
    kw = {"permuted": {"order": [0, 2, 1, 3, 4, 5, 6]},
          "transposed_conv": {"shapes": {"conv": (16, 30, 384)}},
          "out_permuted": {"out_order": [0, 1, 2, 3, 5, 4, 6]}}[case]
    inits, nodes = _state_graph(**kw)
    w = synthetic_weights(0)
    inits += [tensor_proto("tone." + k, v.astype(np.float16)) for k, v in w.items()]
    p = tmp_path / "model.onnx"
    p.write_bytes(model_proto(inits, nodes))
    with pytest.raises(ValueError, match="state"):
        load_weights(p)
    # the same weights with the engine's layout load
    inits, nodes = _state_graph()
    inits += [tensor_proto("tone." + k, v.astype(np.float16)) for k, v in w.items()]
    p.write_bytes(model_proto(inits, nodes))
    assert set(load_weights(p)) == set(PARAM_SHAPES)


def test_export_graph_with_state_plumbing(tmp_path):
    """export_like_graph plus the state Slice / Reshape / Concat subgraph in forward_for_export order: the
    weights load as before and the layout check passes."""
    w = {k: v.astype(np.float16).astype(np.float32) for k, v in synthetic_weights(4).items()}
    inits, nodes = _state_graph()
    # splice the state nodes / initializers into the export-like graph (both are repeated GraphProto fields)
    extra = b"".join(_ld(1, n) for n in nodes) + b"".join(_ld(5, t) for t in inits)
    p = tmp_path / "model.onnx"
    p.write_bytes(_vi(1, 8) + _ld(7, _graph_payload(export_like_graph(w)) + extra))
    got = load_onnx_weights(p)
    assert list(got) == list(PARAM_SHAPES)


def _graph_payload(model: bytes) -> bytes:
    """The GraphProto bytes of a model_proto() result."""
    from tone_amd.onnx_weights import _fields
    for f, wt, v in _fields(memoryview(model)):
        if f == 7:
            return bytes(v)
    raise AssertionError("no graph")


# ---- BatchNorm identity only for a fused pair; one key per shared constant ------------------
def test_unfused_batchnorm_with_anonymous_inputs_raises(tmp_path):
    """A graph that keeps a BatchNormalization node whose parameters cannot be attributed (anonymous inputs
    behind an unknown op) must not load with an identity norm: the parameters stay missing and the loader
    raises."""
    w = {k: v.astype(np.float16).astype(np.float32) for k, v in synthetic_weights(2).items()}
    base = _graph_payload(export_like_graph(w))
    bn = "encoder.layers.4.conv.batch_norm"
    extra = _ld(1, node_proto("/_model/encoder/layers.4/conv/batch_norm/BatchNormalization", "BatchNormalization",
                              ["x", "opaque_g", "opaque_b", "opaque_m", "opaque_v"], [bn + "_out"]))
    p = tmp_path / "model.onnx"
    p.write_bytes(_vi(1, 8) + _ld(7, base + extra))
    with pytest.raises(ValueError, match="batch_norm"):
        load_onnx_weights(p)


def test_shared_constant_written_under_one_key(tmp_path):
    """One folded constant consumed by two scoped nodes (a MatMul, and an Add in another module) is attributed
    to the first successful parameter only."""
    from tone_amd.onnx_weights import onnx_state_dict, read_onnx_graph
    v = np.arange(384, dtype=np.float32)
    inits = [tensor_proto("onnx::Shared_1", v)]
    nodes = [node_proto("/_model/encoder/layers.0/feed_forward1/linear2/Add", "Add", ["x", "onnx::Shared_1"], ["a"]),
             node_proto("/_model/encoder/layers.1/feed_forward1/linear2/Add", "Add", ["y", "onnx::Shared_1"], ["b"])]
    p = tmp_path / "m.onnx"
    p.write_bytes(model_proto(inits, nodes))
    t, n = read_onnx_graph(p)
    sd = onnx_state_dict(t, n)
    keys = [k for k in sd if k.endswith("feed_forward1.linear2.bias")]
    assert len(keys) == 1, keys
