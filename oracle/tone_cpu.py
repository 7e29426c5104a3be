"""CPU side-by-side: the T-one streaming step restated with torch CPU ops (TEST / BENCH INFRASTRUCTURE).

This is the ``cpu_baseline`` leg of ``bench.py`` (BASELINE.md 4 / SURVEY.md 8d: "time a compiled CPU
restatement at B = 1 and B = 256 with the core count stated").  It is NOT the reference code and not
the product path: it restates the same arithmetic as :mod:`tone_oracle` (the numpy checker, which
cites the reference file:line of every stage) with batched torch CPU kernels -- oneDNN/MKL GEMMs and
convolutions, intra-op threads = the cores given -- so the CPU number is what a tuned CPU server
would get, not what a numpy loop gets.  BatchNorm is folded into the preceding convolution and the
SwiGLU/GLU pairs are fused into one GEMM each, as a CPU inference engine would.

Numerics: fp32 with the reference's fp16 rounding points (PCM, features, carried state), so it agrees
with :class:`tone_oracle.ToneOracle` to fp32 reassociation error (tests/test_cpu_baseline.py).
Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import this module.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

import tone_amd.config as C
from tone_oracle import forward_basis, mel_filterbank, rope_tables


def _t(a) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float32)))


class ToneCPU:
    """One streaming step, batched, torch fp32 on the host CPU."""

    def __init__(self, weights: dict):
        W = {k: _t(v) for k, v in weights.items()}
        self.basis = _t(forward_basis())            # (162, 160)
        self.fbank = _t(mel_filterbank())           # (64, 81)
        pe = "encoder.pre_encode."
        self.pre_norm = W[pe + "pre_norm.weight"]
        self.out_norm = W[pe + "out_norm.weight"]
        self.c1w, self.c1b = self._fold_bn(W, pe + "conv.0.0.", pe + "conv.0.1.")
        self.c2w, self.c2b = self._fold_bn(W, pe + "conv.1.0.", pe + "conv.1.1.")
        self.sub_out = W[pe + "out.weight"]
        self.layers = []
        for L in range(C.N_LAYERS):
            p = f"encoder.layers.{L}."
            lw = {"norms": [W[p + n + ".weight"] for n in
                            ("norm_feed_forward1", "norm_self_att", "norm_conv", "norm_feed_forward2", "norm_out")]}
            for f in ("feed_forward1", "feed_forward2"):
                q = p + f + "."
                lw[f] = (torch.cat([W[q + "linear1.weight"], W[q + "linearv.weight"]]),
                         torch.cat([W[q + "linear1.bias"], W[q + "linearv.bias"]]),
                         W[q + "linear2.weight"], W[q + "linear2.bias"])
            a = p + "self_attn."
            lw["v"] = (W[a + "linear_v.weight"], W[a + "linear_v.bias"])
            if C.RECOMPUTE_SCORES[L]:
                lw["q"] = (W[a + "linear_q.weight"], W[a + "linear_q.bias"])
                lw["k"] = (W[a + "linear_k.weight"], W[a + "linear_k.bias"])
                lw["ln"] = (W[a + "q_ln.weight"], W[a + "q_ln.bias"], W[a + "k_ln.weight"], W[a + "k_ln.bias"])
            lw["out"] = (W[a + "linear_out.weight"], W[a + "linear_out.bias"])
            c = p + "conv."
            lw["pw1"] = (W[c + "pointwise_conv1.weight"].reshape(2 * C.D_MODEL, C.D_MODEL), W[c + "pointwise_conv1.bias"])
            lw["dw"] = self._fold_bn(W, c + "depthwise_conv.conv.", c + "batch_norm.")
            lw["pw2"] = (W[c + "pointwise_conv2.weight"].reshape(C.D_MODEL, C.D_MODEL), W[c + "pointwise_conv2.bias"])
            self.layers.append(lw)
        tr = "encoder.temportal_reduction."
        self.red = (W[tr + "conv.weight"], W[tr + "conv.bias"],
                    W[tr + "conv_pw.weight"].reshape(C.D_MODEL, -1), W[tr + "conv_pw.bias"])
        self.head_w = W["decoder.decoder_layers.0.weight"].reshape(C.VOCAB, C.D_MODEL)
        self.head_b = W["decoder.decoder_layers.0.bias"]
        self.rope = {}
        for n, off in ((10, 0), (5, 0), (20, 15), (40, 30)):
            cos, sin = rope_tables(n, off)
            self.rope[(n, off)] = (_t(cos), _t(sin))

    @staticmethod
    def _fold_bn(W, conv, bn):
        g = W[bn + "weight"] / torch.sqrt(W[bn + "running_var"] + C.BN_EPS)
        w = W[conv + "weight"] * g.reshape(-1, *([1] * (W[conv + "weight"].dim() - 1)))
        b = (W[conv + "bias"] - W[bn + "running_mean"]) * g + W[bn + "bias"]
        return w.contiguous(), b.contiguous()

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _rms(x, w):
        return w * (x / (torch.linalg.vector_norm(x, dim=-1, keepdim=True) * (x.shape[-1] ** -0.5) + C.RMS_EPS))

    def _rot(self, x, n, off):
        cos, sin = self.rope[(n, off)]
        r = x[..., : C.ROPE_DIM]
        h = C.ROPE_DIM // 2
        rot = torch.cat([-r[..., h:], r[..., :h]], dim=-1)
        return torch.cat([r * cos + rot * sin, x[..., C.ROPE_DIM:]], dim=-1)

    def step(self, pcm: torch.Tensor, state: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """pcm (B, 2400) int32, state (B, 219729) fp16 -> (logprobs (B,10,35) fp32, next state fp16)."""
        with torch.no_grad():
            return self._step(pcm, state)

    def _step(self, pcm, state):
        b = pcm.shape[0]
        sec = {k: state[:, o: o + int(np.prod(s))].reshape((b,) + s) for k, (o, s) in C.STATE_SECTIONS.items()}
        nxt = torch.empty_like(state)
        nsec = {k: nxt[:, o: o + int(np.prod(s))].reshape((b,) + s) for k, (o, s) in C.STATE_SECTIONS.items()}
        # front end
        wav = (pcm.float() / 32767.0).half()
        x = torch.cat([sec["preproc"], wav], dim=1)
        nsec["preproc"].copy_(x[:, -C.PREPROC_STATE:])
        frames = x.float().unfold(1, C.WIN_LENGTH, C.HOP_LENGTH)                        # (B, 30, 160)
        spec = frames @ self.basis.T
        power = spec[..., : C.N_BINS] ** 2 + spec[..., C.N_BINS:] ** 2
        feats = torch.log(power @ self.fbank.T + C.LOG_GUARD).half().float()            # (B, 30, 64)
        # subsampling
        x = self._rms(feats, self.pre_norm)
        cat1 = torch.cat([sec["sub1"][:, 0].float(), x], dim=1)                           # (B, 40, 64)
        nsec["sub1"].copy_(cat1[:, None, -C.SUB1_STATE:])
        y1 = F.silu(F.conv2d(cat1[:, None], self.c1w, self.c1b))                          # (B, 32, 30, 44)
        cat2 = torch.cat([sec["sub2"].float(), y1], dim=2)                                # (B, 32, 38, 44)
        nsec["sub2"].copy_(cat2[:, :, -C.SUB2_STATE:])
        y2 = F.silu(F.conv2d(cat2, self.c2w, self.c2b, stride=C.SUB_STRIDE[1]))           # (B, 64, 10, 34)
        flat = y2.permute(0, 2, 1, 3).reshape(b, C.CHUNK_FRAMES, C.SUB_OUT_IN)
        x = self._rms(F.linear(flat, self.sub_out), self.out_norm)
        # encoder
        mhsa_len = sec["mhsa_len"][:, 0].float()
        scores = residual = None
        for L, lw in enumerate(self.layers):
            r = x
            r = r + 0.5 * self._ffn(self._rms(r, lw["norms"][0]), lw["feed_forward1"])
            att, scores = self._mhsa(self._rms(r, lw["norms"][1]), L, lw, sec, nsec, scores, mhsa_len)
            r = r + att
            r = r + self._conv(self._rms(r, lw["norms"][2]), L, lw, sec, nsec)
            r = r + 0.5 * self._ffn(self._rms(r, lw["norms"][3]), lw["feed_forward2"])
            x = self._rms(r, lw["norms"][4])
            if L == C.REDUCTION_POS:
                residual = x
                cw, cb, pw, pb = self.red
                cat = torch.cat([sec["reduction"].float(), x.transpose(1, 2)], dim=2)      # (B, 384, 11)
                nsec["reduction"].copy_(cat[:, :, -C.RED_STATE:])
                y = F.conv1d(cat, cw, cb, stride=C.REDUCTION_FACTOR, groups=C.D_MODEL)      # (B, 1536, 5)
                x = F.linear(y.transpose(1, 2).contiguous(), pw, pb)
            if L == C.UPSAMPLE_POS:
                x = x.repeat_interleave(C.REDUCTION_FACTOR, dim=1)[:, : residual.shape[1]] + residual
        nsec["mhsa_len"].copy_(torch.clamp(mhsa_len + C.CHUNK_FRAMES, max=C.MHSA_STATE)[:, None].half())
        logp = F.log_softmax(F.linear(x, self.head_w, self.head_b), dim=-1)
        return logp, nxt

    @staticmethod
    def _ffn(x, w):
        w1v, b1v, w2, b2 = w
        h = F.linear(x, w1v, b1v)
        g, v = h.chunk(2, dim=-1)
        return F.linear(F.silu(g) * v, w2, b2)

    def _mhsa(self, h, L, lw, sec, nsec, scores, mhsa_len):
        b, t, d = h.shape
        S = C.mhsa_cache_rows(L)
        if S:
            cache = sec["mhsa"][:, L - C.MHSA_STATELESS, -S:].float()
            kv = torch.cat([cache, h], dim=1)
            dst = nsec["mhsa"][:, L - C.MHSA_STATELESS]
            dst[:, : C.MHSA_STATE - S] = 0
            dst[:, C.MHSA_STATE - S:] = kv[:, t: t + S]
        else:
            kv = h
        tk = kv.shape[1]
        hd, dk = C.N_HEADS, C.D_HEAD
        v = F.linear(kv, *lw["v"]).reshape(b, tk, hd, dk).transpose(1, 2)
        if C.RECOMPUTE_SCORES[L]:
            qw, qb, kw, kb = lw["ln"]
            q = F.layer_norm(F.linear(h, *lw["q"]).reshape(b, t, hd, dk), (dk,), qw, qb, C.LN_EPS).transpose(1, 2)
            k = F.layer_norm(F.linear(kv, *lw["k"]).reshape(b, tk, hd, dk), (dk,), kw, kb, C.LN_EPS).transpose(1, 2)
            q = self._rot(q, t, 0)
            k = self._rot(k, tk, S)
            scores = (q @ k.transpose(-1, -2)) / math.sqrt(dk)
        if S:
            off = C.MHSA_STATE - mhsa_len
            if C.REDUCTION_POS < L <= C.UPSAMPLE_POS:
                off = torch.floor(off / C.REDUCTION_FACTOR)
            j = torch.arange(S + t, dtype=torch.float32)
            i = torch.arange(t, dtype=torch.float32) + S
            mask = ~((i[None, :, None] >= off[:, None, None]) & (j[None, None, :] >= off[:, None, None]))
            attn = torch.softmax(scores.masked_fill(mask[:, None], -10000.0), dim=-1).masked_fill(mask[:, None], 0.0)
        else:
            attn = torch.softmax(scores, dim=-1)
        ctx = (attn @ v).transpose(1, 2).reshape(b, t, d)
        return F.linear(ctx, *lw["out"]), scores

    @staticmethod
    def _conv(h, L, lw, sec, nsec):
        u = F.glu(F.linear(h, *lw["pw1"]), dim=-1)                                          # (B, T, 384)
        cat = torch.cat([sec["conv"][:, L].float(), u.transpose(1, 2)], dim=2)              # (B, 384, 30 + T)
        nsec["conv"][:, L].copy_(cat[:, :, -C.CONV_STATE:])
        dw = F.silu(F.conv1d(cat, lw["dw"][0], lw["dw"][1], groups=C.D_MODEL))             # (B, 384, T)
        return F.linear(dw.transpose(1, 2).contiguous(), *lw["pw2"])
