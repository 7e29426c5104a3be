"""CPU oracle of the EXPORTED graph's numerics (TEST INFRASTRUCTURE ONLY).

Like ``tone_oracle.py`` this module is a checker: only ``tests/`` (and the bench's optional CPU leg) may
import it, never the product path.

``ToneOracleFP16`` restates one streaming step as ``tone/scripts/export.py`` traces it into the ONNX graph
that ``onnx_wrapper`` runs: ``Tone.forward_for_export`` (tone/nn/model.py:101-206) under
``torch.amp.autocast("cpu", dtype=torch.float16)`` (export.py:411) with the export's fp32 LayerNorm patch
(export.py:28-34).  Every rounding point comes from the op trace of the reference itself
(``tests/golden/op_trace_fp16.txt``, written by ``tests/golden/make_golden_fp16.py --trace``):

* front end: fp32, features -> fp16 (feats.py:95-133), as ``ToneOracle``;
* every Linear / Conv1d / Conv2d: weights and bias -> fp16, fp32 accumulate, output -> fp16
  (autocast's lower-precision op list);
* every elementwise op on fp16 tensors (SiLU, GLU, the SwiGLU product, BatchNorm, x0.5, residual adds,
  the upsampling add, the score scaling) computes in fp32 and rounds its output to fp16;
* RMSNorm: fp32 inside, fp16 out (submodules.py:34-54);
* q/k LayerNorm: fp32 in and out (the export patch); RoPE in fp32; q, k -> fp16 as the score matmul's
  operands; scores, softmax and P.V in fp16 (``avoid_float16_autocast_context``,
  tone/nn/torch_utils.py:10-34, checks the CUDA autocast state and does nothing on the CPU trace);
* log_softmax of the fp16 logits: the CPU kernel keeps the exp-sum and its log in fp16
  (checked bit for bit against torch here), output fp16 -> ``.float()`` (model.py:196).

GEMMs accumulate in float32 through numpy's sgemm, which reproduces torch's CPU fp16 ``addmm`` bit for bit
(same MKL kernel on the upcast operands); ``acc="f64"`` accumulates in float64 instead -- the same rounding
points with a different summation order, the measure of how far any other correct implementation (ORT's
MLAS kernels, the MI355X path) can drift from the torch trace by fp16 rounding flips alone.

Pinned to the reference by ``tests/golden/golden_fp16.npz`` (tests/test_oracle.py).
"""

from __future__ import annotations

import math

import numpy as np

import tone_amd.config as C
from tone_oracle import F32, StreamState, ToneOracle, layernorm


def h(x) -> np.ndarray:
    """Round to fp16, keep float32 storage."""
    return np.asarray(x, dtype=np.float32).astype(np.float16).astype(F32)


class ToneOracleFP16(ToneOracle):
    """One streaming step with the fp16-autocast export's rounding points."""

    def __init__(self, weights: dict, acc: str = "f32"):
        super().__init__(weights, round_feats=True)
        assert acc in ("f32", "f64")
        self.acc = np.float32 if acc == "f32" else np.float64
        self.H = {k: h(v) for k, v in self.W.items()}          # autocast casts every weight / bias to fp16

    # --- primitives ----------------------------------------------------------------------------
    def mm(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        return (a.astype(self.acc) @ b.astype(self.acc)).astype(F32)

    def lin(self, x: np.ndarray, name: str, bias: bool = True) -> np.ndarray:
        """nn.Linear / 1x1 Conv1d under autocast: fp16 operands, fp32 accumulate, + fp16 bias, -> fp16."""
        w = self.H[name + ".weight"]
        y = self.mm(x, w.reshape(w.shape[0], -1).T)
        if bias:
            y = y + self.H[name + ".bias"]
        return h(y)

    @staticmethod
    def rms(x: np.ndarray, w: np.ndarray) -> np.ndarray:
        """RMSNorm (submodules.py:34-54): fp32 inside, returned in the input dtype (fp16)."""
        norm = np.sqrt(np.sum(x * x, axis=-1, keepdims=True, dtype=F32))
        rms = norm * np.float32(x.shape[-1] ** -0.5)
        return h(w * (x / (rms + np.float32(C.RMS_EPS))))

    @staticmethod
    def silu(x: np.ndarray) -> np.ndarray:
        return h(x / (np.float32(1) + np.exp(-x)))

    def bn(self, x: np.ndarray, pfx: str, axis: int) -> np.ndarray:
        """Eval BatchNorm of an fp16 tensor with fp32 statistics (the CPU kernel's alpha / beta form), -> fp16."""
        W = self.W
        shape = [1] * x.ndim
        shape[axis] = -1
        inv = np.float32(1) / np.sqrt(W[pfx + "running_var"] + np.float32(C.BN_EPS))
        al = inv * W[pfx + "weight"]
        be = W[pfx + "bias"] - W[pfx + "running_mean"] * al
        return h(x * al.reshape(shape) + be.reshape(shape))

    @staticmethod
    def softmax16(x: np.ndarray) -> np.ndarray:
        m = x.max(axis=-1, keepdims=True)
        e = np.exp(x - m)
        return h(e / e.sum(axis=-1, keepdims=True))

    # --- a3: convolutional subsampling (conformer_blocks.py:614-653) ---------------------------
    def pre_encode(self, feats: np.ndarray, st: StreamState, nst: dict) -> np.ndarray:
        W, H = self.W, self.H
        pe = "encoder.pre_encode."
        x = self.rms(feats.astype(F32), W[pe + "pre_norm.weight"])                      # (B, 30, 64) fp16
        b = x.shape[0]
        cat1 = np.concatenate([st.sub1[:, 0].astype(F32), x], axis=1)
        nst["sub1"] = cat1[:, None, -C.SUB1_STATE:].astype(np.float16)
        mt = x.shape[1]
        win = np.lib.stride_tricks.sliding_window_view(cat1, C.SUB_K[0], axis=(1, 2))
        w1 = H[pe + "conv.0.0.weight"].reshape(C.SUB_CH[0], -1)
        y1 = h(self.mm(win.reshape(b, mt, C.SUB1_F, -1), w1.T) + H[pe + "conv.0.0.bias"])
        y1 = self.silu(self.bn(y1, pe + "conv.0.1.", axis=3))
        y1 = np.ascontiguousarray(y1.transpose(0, 3, 1, 2))                               # (B,32,mt,44)
        cat2 = np.concatenate([st.sub2.astype(F32), y1], axis=2)
        nst["sub2"] = cat2[:, :, -C.SUB2_STATE:].astype(np.float16)
        win2 = np.lib.stride_tricks.sliding_window_view(cat2, C.SUB_K[1], axis=(2, 3))[:, :, :: C.SUB_STRIDE[1][0]]
        t_out = win2.shape[2]
        a2 = np.ascontiguousarray(win2.transpose(0, 2, 3, 1, 4, 5)).reshape(b, t_out, C.SUB2_F, -1)
        w2 = H[pe + "conv.1.0.weight"].reshape(C.SUB_CH[1], -1)
        y2 = h(self.mm(a2, w2.T) + H[pe + "conv.1.0.bias"])
        y2 = self.silu(self.bn(y2, pe + "conv.1.1.", axis=3))
        flat = np.ascontiguousarray(y2.transpose(0, 1, 3, 2)).reshape(b, t_out, C.SUB_OUT_IN)
        x = self.lin(flat, pe + "out", bias=False)
        return self.rms(x, W[pe + "out_norm.weight"])

    # --- a5: SwiGLU FFN (conformer_blocks.py:468-482) ------------------------------------------
    def ffn(self, x: np.ndarray, p: str) -> np.ndarray:
        g = self.silu(self.lin(x, p + "linear1"))
        return self.lin(h(g * self.lin(x, p + "linearv")), p + "linear2")

    # --- a6-a8: RoPE MHSA (conformer_blocks.py:688-726, submodules.py:204-303) -----------------
    def mhsa(self, hn: np.ndarray, L: int, st: StreamState, nst: dict, shared: dict) -> np.ndarray:
        W = self.W
        p = f"encoder.layers.{L}.self_attn."
        b, t, d = hn.shape
        S = C.mhsa_cache_rows(L)
        if S:
            cache = st.mhsa[:, L - C.MHSA_STATELESS, -S:].astype(F32)
            kv = np.concatenate([cache, hn], axis=1)
            new = np.concatenate([cache[:, t:], hn[:, :t]], axis=1)
            padded = np.zeros((b, C.MHSA_STATE, d), F32)
            padded[:, C.MHSA_STATE - S:] = new
            nst.setdefault("mhsa", [None] * C.N_MHSA_LAYERS)[L - C.MHSA_STATELESS] = padded.astype(np.float16)
        else:
            kv = hn
        tk = kv.shape[1]
        hd, dk = C.N_HEADS, C.D_HEAD
        v = self.lin(kv, p + "linear_v").reshape(b, tk, hd, dk).transpose(0, 2, 1, 3)
        if C.RECOMPUTE_SCORES[L]:
            q = self.lin(hn, p + "linear_q").reshape(b, t, hd, dk)
            k = self.lin(kv, p + "linear_k").reshape(b, tk, hd, dk)
            q = layernorm(q, W[p + "q_ln.weight"], W[p + "q_ln.bias"]).transpose(0, 2, 1, 3)   # fp32 (export patch)
            k = layernorm(k, W[p + "k_ln.weight"], W[p + "k_ln.bias"]).transpose(0, 2, 1, 3)
            q = h(self._rope(q, 0))
            k = h(self._rope(k, S))
            scores = h(h(self.mm(q, k.transpose(0, 1, 3, 2))) / np.float32(math.sqrt(dk)))
            shared["scores"] = scores
        else:
            scores = shared["scores"]
        if S:
            mask = self._mask(L, st, t, S)
            attn = np.where(mask[:, None], np.float32(0), self.softmax16(np.where(mask[:, None], np.float32(-10000), scores)))
        else:
            attn = self.softmax16(scores)
        ctx = h(self.mm(attn, v)).transpose(0, 2, 1, 3).reshape(b, t, d)
        return self.lin(ctx, p + "linear_out")

    # --- a9: convolution module (conformer_blocks.py:403-436, submodules.py:346-402) -----------
    def conv_module(self, hn: np.ndarray, L: int, st: StreamState, nst: dict) -> np.ndarray:
        H = self.H
        p = f"encoder.layers.{L}.conv."
        y = self.lin(hn, p + "pointwise_conv1")
        d = C.D_MODEL
        u = h(y[..., :d] * (np.float32(1) / (np.float32(1) + np.exp(-y[..., d:]))))          # GLU
        cat = np.concatenate([st.conv[:, L].astype(F32), u.transpose(0, 2, 1)], axis=2)
        nst.setdefault("conv", [None] * C.N_LAYERS)[L] = cat[:, :, -C.CONV_STATE:].astype(np.float16)
        win = np.lib.stride_tricks.sliding_window_view(cat, C.CONV_KERNEL, axis=2)           # (B,384,T,31)
        w = H[p + "depthwise_conv.conv.weight"][:, 0].astype(self.acc)
        dw = np.einsum("bctk,ck->bct", win.astype(self.acc), w).astype(F32)
        dw = h(dw + H[p + "depthwise_conv.conv.bias"][None, :, None])
        dw = self.silu(self.bn(dw, p + "batch_norm.", axis=1))
        return self.lin(dw.transpose(0, 2, 1), p + "pointwise_conv2")

    # --- a10: macaron layer (conformer_blocks.py:799-836) ---------------------------------------
    def layer(self, x: np.ndarray, L: int, st: StreamState, nst: dict, shared: dict) -> np.ndarray:
        W = self.W
        p = f"encoder.layers.{L}."
        r = x
        r = h(r + h(self.ffn(self.rms(r, W[p + "norm_feed_forward1.weight"]), p + "feed_forward1.") * np.float32(0.5)))
        r = h(r + self.mhsa(self.rms(r, W[p + "norm_self_att.weight"]), L, st, nst, shared))
        r = h(r + self.conv_module(self.rms(r, W[p + "norm_conv.weight"]), L, st, nst))
        r = h(r + h(self.ffn(self.rms(r, W[p + "norm_feed_forward2.weight"]), p + "feed_forward2.") * np.float32(0.5)))
        return self.rms(r, W[p + "norm_out.weight"])

    # --- a11: causal temporal reduction (conformer_blocks.py:874-911) ---------------------------
    def reduce(self, x: np.ndarray, st: StreamState, nst: dict) -> np.ndarray:
        H = self.H
        tr = "encoder.temportal_reduction."
        xt = x.transpose(0, 2, 1)
        cat = np.concatenate([st.reduction.astype(F32), xt], axis=2)
        nst["reduction"] = cat[:, :, -C.RED_STATE:].astype(np.float16)
        w = H[tr + "conv.weight"][:, 0].astype(self.acc)
        src = np.repeat(cat, 4, axis=1)
        win = np.lib.stride_tricks.sliding_window_view(src, C.REDUCTION_KERNEL, axis=2)[:, :, :: C.REDUCTION_FACTOR]
        y = h(np.einsum("botk,ok->bot", win.astype(self.acc), w).astype(F32) + H[tr + "conv.bias"][None, :, None])
        return self.lin(y.transpose(0, 2, 1), tr + "conv_pw")

    # --- a14: CTC head (conformer.py:338-354) ----------------------------------------------------
    def head(self, x: np.ndarray) -> np.ndarray:
        z = self.lin(x, "decoder.decoder_layers.0")
        m = z.max(axis=-1, keepdims=True)
        lse = h(np.log(h(np.exp(z - m).sum(axis=-1, keepdims=True))))   # the CPU kernel's fp16 sum and log
        return h(z - m - lse)

    # --- the whole encoder ------------------------------------------------------------------------
    def encode(self, feats: np.ndarray, st: StreamState, nst: dict, trace: list | None = None) -> np.ndarray:
        x = self.pre_encode(feats, st, nst)
        if trace is not None:
            trace.append(x)
        shared: dict = {}
        residual = None
        for L in range(C.N_LAYERS):
            x = self.layer(x, L, st, nst, shared)
            if L == C.REDUCTION_POS:
                residual = x
                x = self.reduce(x, st, nst)
            if L == C.UPSAMPLE_POS:
                rep = np.repeat(x, C.REDUCTION_FACTOR, axis=1)
                up = np.zeros_like(residual)
                n = min(rep.shape[1], residual.shape[1])
                up[:, :n] = rep[:, :n]
                x = h(up + residual)
            if trace is not None:
                trace.append(x)
        return x
