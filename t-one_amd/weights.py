"""Weight catalogue, deterministic synthetic weights and checkpoint loading.

Parameter names follow the reference ``state_dict`` of ``Tone`` (``tone/nn/model.py:39-41``):
``encoder.*`` is ``Encoder`` (``tone/nn/modules/conformer.py:102-135``) and ``decoder.*`` is
``ConvASRDecoder`` (``conformer.py:334-336``).  The HF ``ToneForCTC`` checkpoint prefixes every
key with ``tone.`` (``tone/training/model_wrapper.py:134-166``); :func:`normalize_keys` strips it.

Real ``t-tech/T-one`` weights are not available offline, so tests, the bench and
``smoke()`` use :func:`synthetic_weights`: a counter-based splitmix64 generator keyed by
(seed, parameter name, element index).  It is order independent and reproducible in any
language, so no multi-hundred-MB fixture has to be committed.
"""

from __future__ import annotations

import zlib
from collections import OrderedDict
from pathlib import Path

import numpy as np

from . import config as C

_MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _param_shapes() -> "OrderedDict[str, tuple[int, ...]]":
    """Every floating parameter/buffer the acoustic path reads, with its reference shape."""
    d = C.D_MODEL
    s: "OrderedDict[str, tuple[int, ...]]" = OrderedDict()
    pe = "encoder.pre_encode."
    s[pe + "pre_norm.weight"] = (C.N_MELS,)
    cin = 1
    for i in range(2):
        co = C.SUB_CH[i]
        kt, kf = C.SUB_K[i]
        s[pe + f"conv.{i}.0.weight"] = (co, cin, kt, kf)
        s[pe + f"conv.{i}.0.bias"] = (co,)
        for b in ("weight", "bias", "running_mean", "running_var"):
            s[pe + f"conv.{i}.1.{b}"] = (co,)
        cin = co
    s[pe + "out.weight"] = (d, C.SUB_OUT_IN)
    s[pe + "out_norm.weight"] = (d,)
    tr = "encoder.temportal_reduction."   # sic: the reference attribute name (conformer.py:114)
    s[tr + "conv.weight"] = (4 * d, 1, C.REDUCTION_KERNEL)
    s[tr + "conv.bias"] = (4 * d,)
    s[tr + "conv_pw.weight"] = (d, 4 * d, 1)
    s[tr + "conv_pw.bias"] = (d,)
    for L in range(C.N_LAYERS):
        p = f"encoder.layers.{L}."
        for ff in ("feed_forward1", "feed_forward2"):
            s[p + f"norm_{ff}.weight"] = (d,)
            s[p + f"{ff}.linear1.weight"] = (C.D_FF, d)
            s[p + f"{ff}.linear1.bias"] = (C.D_FF,)
            s[p + f"{ff}.linearv.weight"] = (C.D_FF, d)
            s[p + f"{ff}.linearv.bias"] = (C.D_FF,)
            s[p + f"{ff}.linear2.weight"] = (d, C.D_FF)
            s[p + f"{ff}.linear2.bias"] = (d,)
        s[p + "norm_self_att.weight"] = (d,)
        s[p + "self_attn.linear_v.weight"] = (d, d)
        s[p + "self_attn.linear_v.bias"] = (d,)
        s[p + "self_attn.linear_out.weight"] = (d, d)
        s[p + "self_attn.linear_out.bias"] = (d,)
        if C.RECOMPUTE_SCORES[L]:
            s[p + "self_attn.linear_q.weight"] = (d, d)
            s[p + "self_attn.linear_q.bias"] = (d,)
            s[p + "self_attn.linear_k.weight"] = (d, d)
            s[p + "self_attn.linear_k.bias"] = (d,)
            for ln in ("q_ln", "k_ln"):
                s[p + f"self_attn.{ln}.weight"] = (C.D_HEAD,)
                s[p + f"self_attn.{ln}.bias"] = (C.D_HEAD,)
        s[p + "norm_conv.weight"] = (d,)
        s[p + "conv.pointwise_conv1.weight"] = (2 * d, d, 1)
        s[p + "conv.pointwise_conv1.bias"] = (2 * d,)
        s[p + "conv.depthwise_conv.conv.weight"] = (d, 1, C.CONV_KERNEL)
        s[p + "conv.depthwise_conv.conv.bias"] = (d,)
        for b in ("weight", "bias", "running_mean", "running_var"):
            s[p + f"conv.batch_norm.{b}"] = (d,)
        s[p + "conv.pointwise_conv2.weight"] = (d, d, 1)
        s[p + "conv.pointwise_conv2.bias"] = (d,)
        s[p + "norm_out.weight"] = (d,)
    s["decoder.decoder_layers.0.weight"] = (C.VOCAB, d, 1)
    s["decoder.decoder_layers.0.bias"] = (C.VOCAB,)
    return s


PARAM_SHAPES = _param_shapes()
N_PARAMS = int(sum(int(np.prod(v)) for v in PARAM_SHAPES.values()))


def _splitmix_uniform(seed: int, name: str, n: int) -> np.ndarray:
    """n uniforms in [-1, 1) from splitmix64(seed ^ crc32(name) * golden + index)."""
    key = (np.uint64(seed & 0xFFFFFFFF) << np.uint64(32)) ^ np.uint64(zlib.crc32(name.encode()))
    with np.errstate(over="ignore"):
        z = key * np.uint64(0x9E3779B97F4A7C15) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    # top 24 bits -> exact float32 in [0, 1)
    u = (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return (2.0 * u - 1.0).astype(np.float32)


def _fan_in(shape: tuple[int, ...]) -> int:
    return int(np.prod(shape[1:])) if len(shape) > 1 else 1


def synthetic_weights(seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Deterministic random-init weights of the T-one architecture (float32).

    Matrices/convs are U(-1,1)/sqrt(fan_in) (the torch default init family); biases 0.1*U;
    norm gains 1 + 0.1*U; BatchNorm running_var in [0.5, 1.5].  The CTC head is scaled x4 so
    logits are peaky enough for greedy argmax to be a meaningful parity check.
    """
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, shape in PARAM_SHAPES.items():
        n = int(np.prod(shape))
        u = _splitmix_uniform(seed, name, n).reshape(shape)
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "running_var":
            w = 1.0 + 0.5 * u
        elif leaf == "running_mean":
            w = 0.1 * u
        elif leaf == "bias":
            w = 0.1 * u
        elif len(shape) == 1:     # RMSNorm / LayerNorm / BatchNorm gains
            w = 1.0 + 0.1 * u
        else:
            w = u / np.float32(np.sqrt(_fan_in(shape)))
            if name.startswith("decoder."):
                w = w * np.float32(4.0)
        out[name] = np.ascontiguousarray(w.astype(np.float32))
    return out


def normalize_keys(sd: dict) -> "OrderedDict[str, np.ndarray]":
    """Map a reference checkpoint (``Tone`` or HF ``ToneForCTC`` keys) onto PARAM_SHAPES names."""
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for k, v in sd.items():
        kk = k
        for pfx in ("_model.", "tone."):   # ModelToExport._model (tone/scripts/export.py:144); HF ToneForCTC.tone
            if kk.startswith(pfx):
                kk = kk[len(pfx):]
        if kk.endswith("num_batches_tracked"):
            continue
        if kk not in PARAM_SHAPES:
            continue
        arr = np.asarray(v.detach().cpu().float().numpy() if hasattr(v, "detach") else v, dtype=np.float32)
        if tuple(arr.shape) != PARAM_SHAPES[kk]:
            raise ValueError(f"weight {k}: shape {arr.shape} != expected {PARAM_SHAPES[kk]}")
        out[kk] = np.ascontiguousarray(arr)
    missing = [k for k in PARAM_SHAPES if k not in out]
    if missing:
        raise ValueError(f"checkpoint is missing {len(missing)} tensors, e.g. {missing[:3]}")
    return OrderedDict((k, out[k]) for k in PARAM_SHAPES)


def load_weights(path: str | Path) -> "OrderedDict[str, np.ndarray]":
    """Load weights from ``model.safetensors`` / ``*.npz`` / ``*.pt`` (weights_only) /
    ``model.onnx`` (graph initializers, :mod:`tone_amd.onnx_weights`) or a directory holding one.

    Only loaders that execute nothing from the file are used (safetensors, numpy without
    pickle, ``torch.load(weights_only=True)``).
    """
    p = Path(path)
    if p.is_dir():
        for cand in ("model.safetensors", "weights.npz", "pytorch_model.bin", "model.onnx"):
            if (p / cand).exists():
                return load_weights(p / cand)
        raise FileNotFoundError(f"no model.safetensors / weights.npz / pytorch_model.bin / model.onnx in {p}")
    if not p.exists():
        raise FileNotFoundError(f"weight file {p} does not exist")
    if p.suffix == ".onnx":
        from .onnx_weights import load_onnx_weights
        return load_onnx_weights(p)
    if p.suffix == ".safetensors":
        from safetensors.numpy import load_file
        return normalize_keys(load_file(str(p)))
    if p.suffix == ".npz":
        with np.load(str(p), allow_pickle=False) as z:
            return normalize_keys({k: z[k] for k in z.files})
    if p.suffix in (".pt", ".pth", ".bin"):
        import torch
        return normalize_keys(torch.load(str(p), map_location="cpu", weights_only=True))
    raise ValueError(f"unsupported weight file {p} (use .safetensors, .npz, .pt or .onnx)")
