"""CPU oracle: a numpy restatement of ONE T-one streaming step (TEST INFRASTRUCTURE ONLY).

This module is the checker for the HIP path.  Only ``tests/``, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of ``bench.py`` may import it; the product path never does.

It restates ``Tone.forward_for_export`` (``tone/nn/model.py:101-206``) in float32 with the
reference's fp16 rounding points:

  #1  PCM int32 / 32767 -> fp16                         (model.py:165)
  #2  log-mel features  -> fp16                         (feats.py:102, ``.to(waveform.dtype)``)
  #3  every carried state tensor -> fp16 at the boundary (onnx_wrapper.py:115-121, the ONNX I/O
      dtype; ``tone/scripts/export.py:454-455``)

Everything between those points is float32, like the reference torch modules run on CPU.

Parity pin: ``tests/golden/`` holds vectors produced by the reference's own modules
(``tone/nn/modules/{feats,conformer,conformer_blocks,submodules}.py`` imported from
``/root/reference``; torchaudio's ``melscale_fbanks`` restated because torchaudio is absent)
by ``tests/golden/make_golden.py``; ``tests/test_oracle.py`` checks this oracle against them.
Against the real ORT fp16 graph and the real weights the oracle is *parity unpinned*
(neither is available offline).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

import tone_amd.config as C

F32 = np.float32


# ----------------------------------------------------------------------------------------------
# front-end constants
# ----------------------------------------------------------------------------------------------
def hann_window_f32(n: int) -> np.ndarray:
    """torch.hann_window(n, periodic=False) in float32 (feats.py:60)."""
    k = np.arange(n, dtype=np.float32) * np.float32(2.0 * math.pi / (n - 1))
    return (np.float32(0.5) - np.float32(0.5) * np.cos(k)).astype(F32)


def forward_basis() -> np.ndarray:
    """The (162, 160) float32 DFT basis with Hann window and per-frame pre-emphasis folded in
    (FilterbankFeatures._compute_forward_basis, feats.py:66-80).  Row r < 81 is Re, r >= 81 Im."""
    n = C.N_FFT
    kk = np.arange(n, dtype=np.float64)
    ang = -2.0 * math.pi * np.outer(kk, kk) / n           # fft(eye(n)) rows
    four = np.exp(1j * ang)[: n // 2 + 1]                  # (81, 160)
    fb = np.concatenate([four.real, four.imag], axis=0).T  # (160, 162)
    fb = fb * hann_window_f32(C.WIN_LENGTH).astype(np.float64)[:, None]
    p = np.eye(C.WIN_LENGTH)
    p -= np.diag(np.full(C.WIN_LENGTH - 1, C.PREEMPH), 1)
    p[0, 0] -= C.PREEMPH
    fb = p @ fb
    return np.ascontiguousarray(fb.T.astype(F32))            # (162, 160)


def _hz_to_mel_slaney(f: float) -> float:
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = math.log(6.4) / 27.0
    if f >= min_log_hz:
        mels = min_log_mel + math.log(f / min_log_hz) / logstep
    return mels


def mel_filterbank() -> np.ndarray:
    """(64, 81) float32 Slaney-scale, Slaney-normalised triangular filters.

    Restates torchaudio 2.7.1 ``functional.melscale_fbanks(n_freqs=81, f_min=0, f_max=4000,
    n_mels=64, sample_rate=8000, norm="slaney", mel_scale="slaney")`` as called at
    feats.py:83-93 (torchaudio is not vendored and not installed; version from poetry.lock).
    """
    n_freqs, n_mels = C.N_BINS, C.N_MELS
    all_freqs = np.linspace(0, C.SAMPLE_RATE // 2, n_freqs, dtype=np.float32)
    m_min, m_max = _hz_to_mel_slaney(0.0), _hz_to_mel_slaney(C.SAMPLE_RATE / 2)
    m_pts = np.linspace(m_min, m_max, n_mels + 2, dtype=np.float32)
    f_sp = np.float32(200.0 / 3)
    min_log_hz, min_log_mel = np.float32(1000.0), np.float32(1000.0 / (200.0 / 3))
    logstep = np.float32(math.log(6.4) / 27.0)
    f_pts = (f_sp * m_pts).astype(F32)
    lt = m_pts >= min_log_mel
    f_pts[lt] = (min_log_hz * np.exp(logstep * (m_pts[lt] - min_log_mel))).astype(F32)
    f_diff = (f_pts[1:] - f_pts[:-1]).astype(F32)
    slopes = (f_pts[None, :] - all_freqs[:, None]).astype(F32)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = np.maximum(np.float32(0), np.minimum(down, up)).astype(F32)
    enorm = (2.0 / (f_pts[2: n_mels + 2] - f_pts[:n_mels])).astype(F32)
    fb = (fb * enorm[None, :]).astype(F32)
    return np.ascontiguousarray(fb.T)                        # (64, 81)


def rope_tables(n_pos: int, offset: int) -> tuple[np.ndarray, np.ndarray]:
    """cos/sin (n_pos, 32) for positions -offset .. n_pos-offset-1 (submodules.py:120-140)."""
    inv_freq = (1.0 / (np.float32(C.ROPE_BASE) ** (np.arange(0, C.ROPE_DIM, 2, dtype=np.float32) / np.float32(C.ROPE_DIM)))).astype(F32)
    pos = np.arange(-offset, n_pos - offset, dtype=np.float32)
    freqs = np.outer(pos, inv_freq).astype(F32)
    emb = np.concatenate([freqs, freqs], axis=1)
    return np.cos(emb).astype(F32), np.sin(emb).astype(F32)


# ----------------------------------------------------------------------------------------------
# primitives
# ----------------------------------------------------------------------------------------------
def rmsnorm(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """RMSNorm with eps outside the sqrt (submodules.py:34-54)."""
    x = x.astype(F32)
    norm = np.sqrt(np.sum(x * x, axis=-1, keepdims=True, dtype=F32))
    rms = norm * np.float32(x.shape[-1] ** -0.5)
    return (w * (x / (rms + np.float32(C.RMS_EPS)))).astype(F32)


def layernorm(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    mu = x.mean(axis=-1, keepdims=True, dtype=F32)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True, dtype=F32)
    return ((x - mu) / np.sqrt(var + np.float32(C.LN_EPS)) * w + b).astype(F32)


def silu(x: np.ndarray) -> np.ndarray:
    return (x / (np.float32(1) + np.exp(-x))).astype(F32)


def sigmoid(x: np.ndarray) -> np.ndarray:
    return (np.float32(1) / (np.float32(1) + np.exp(-x))).astype(F32)


def linear(x: np.ndarray, w: np.ndarray, b: np.ndarray | None = None) -> np.ndarray:
    y = x @ w.reshape(w.shape[0], -1).T
    if b is not None:
        y = y + b
    return y.astype(F32)


def bn_eval(x: np.ndarray, W: dict, pfx: str, axis: int) -> np.ndarray:
    shape = [1] * x.ndim
    shape[axis] = -1
    g = W[pfx + "weight"].reshape(shape)
    b = W[pfx + "bias"].reshape(shape)
    m = W[pfx + "running_mean"].reshape(shape)
    v = W[pfx + "running_var"].reshape(shape)
    return ((x - m) / np.sqrt(v + np.float32(C.BN_EPS)) * g + b).astype(F32)


def softmax(x: np.ndarray) -> np.ndarray:
    m = x.max(axis=-1, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis=-1, keepdims=True)).astype(F32)


def fp16(x: np.ndarray) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).astype(np.float16)


# ----------------------------------------------------------------------------------------------
# state
# ----------------------------------------------------------------------------------------------
@dataclass
class StreamState:
    """The seven state tensors of one batch, float16, batch-first (model.py:101-113)."""

    preproc: np.ndarray   # (B, 80)
    mhsa: np.ndarray      # (B, 2, 30, 384)
    conv: np.ndarray      # (B, 16, 384, 30)
    mhsa_len: np.ndarray  # (B, 1)
    sub1: np.ndarray      # (B, 1, 10, 64)
    sub2: np.ndarray      # (B, 32, 8, 44)
    reduction: np.ndarray  # (B, 384, 1)

    @classmethod
    def zeros(cls, b: int) -> "StreamState":
        return cls.unflatten(np.zeros((b, C.STATE_SIZE), np.float16))

    @classmethod
    def unflatten(cls, flat: np.ndarray) -> "StreamState":
        b = flat.shape[0]
        parts = {}
        for name, (off, shp) in C.STATE_SECTIONS.items():
            n = int(np.prod(shp))
            parts[name] = flat[:, off: off + n].reshape((b,) + shp)
        return cls(**parts)

    def flatten(self) -> np.ndarray:
        b = self.preproc.shape[0]
        out = np.empty((b, C.STATE_SIZE), np.float16)
        for name, (off, shp) in C.STATE_SECTIONS.items():
            n = int(np.prod(shp))
            out[:, off: off + n] = getattr(self, name).reshape(b, n)
        return out


# ----------------------------------------------------------------------------------------------
# the step
# ----------------------------------------------------------------------------------------------
class ToneOracle:
    """One streaming step of the acoustic path, float32 numpy."""

    def __init__(self, weights: dict, round_feats: bool = True):
        """``round_feats=False`` skips rounding point #2 (features -> fp16): what
        ``Tone.forward_for_export`` computes when handed float32 states (its preprocessor then
        returns float32 features), used to pin the oracle against tests/golden/golden_fx.npz."""
        self.W = {k: np.asarray(v, dtype=F32) for k, v in weights.items()}
        self.round_feats = round_feats
        self.basis = forward_basis()
        self.fbank = mel_filterbank()

    # --- a1/a2: PCM -> fp16 -> log-mel (model.py:164-169, feats.py:95-102,118-133) ----------
    def mel(self, pcm: np.ndarray, pre_state: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """pcm (B, 2400) int -> feats (B, 30, 64) fp16, next preproc state (B, 80) fp16."""
        wav = fp16(pcm.astype(F32) / np.float32(32767))
        x = np.concatenate([pre_state.astype(np.float16), wav], axis=1)            # (B, 2480) fp16
        nxt = x[:, -C.PREPROC_STATE:].copy()
        xf = x.astype(F32)
        frames = np.lib.stride_tricks.sliding_window_view(xf, C.WIN_LENGTH, axis=1)[:, :: C.HOP_LENGTH]
        spec = frames @ self.basis.T                                                # (B, 30, 162)
        power = spec[..., : C.N_BINS] ** 2 + spec[..., C.N_BINS:] ** 2             # (B, 30, 81)
        mel = power @ self.fbank.T                                                  # (B, 30, 64)
        feats = np.log(mel + np.float32(C.LOG_GUARD)).astype(F32)
        return (fp16(feats) if self.round_feats else feats), nxt

    # --- a3: convolutional subsampling (conformer_blocks.py:614-653) ------------------------
    def pre_encode(self, feats: np.ndarray, st: StreamState, nst: dict) -> np.ndarray:
        W = self.W
        pe = "encoder.pre_encode."
        x = rmsnorm(feats.astype(F32), W[pe + "pre_norm.weight"])                  # (B, 30, 64)
        b = x.shape[0]
        cat1 = np.concatenate([st.sub1[:, 0].astype(F32), x], axis=1)              # (B, 40, 64)
        nst["sub1"] = fp16(cat1[:, None, -C.SUB1_STATE:])
        kt, kf = C.SUB_K[0]
        mt = x.shape[1]                                                              # 30 (300 ms) | 40 (400 ms)
        win = np.lib.stride_tricks.sliding_window_view(cat1, (kt, kf), axis=(1, 2))  # (B,mt,44,11,21)
        w1 = W[pe + "conv.0.0.weight"].reshape(C.SUB_CH[0], -1)
        y1 = win.reshape(b, mt, C.SUB1_F, -1) @ w1.T + W[pe + "conv.0.0.bias"]       # (B,mt,44,32)
        y1 = silu(bn_eval(y1, W, pe + "conv.0.1.", axis=3))
        y1 = np.ascontiguousarray(y1.transpose(0, 3, 1, 2))                          # (B,32,30,44)
        cat2 = np.concatenate([st.sub2.astype(F32), y1], axis=2)                     # (B,32,38,44)
        nst["sub2"] = fp16(cat2[:, :, -C.SUB2_STATE:])
        kt, kf = C.SUB_K[1]
        win2 = np.lib.stride_tricks.sliding_window_view(cat2, (kt, kf), axis=(2, 3))[:, :, :: C.SUB_STRIDE[1][0]]
        # win2: (B, 32, T, 34, 11, 11) -> (B, T, 34, 32*11*11); T = 10 | 13 (a 400 ms chunk leaves row 47 unread)
        t_out = win2.shape[2]
        a2 = np.ascontiguousarray(win2.transpose(0, 2, 3, 1, 4, 5)).reshape(b, t_out, C.SUB2_F, -1)
        w2 = W[pe + "conv.1.0.weight"].reshape(C.SUB_CH[1], -1)
        y2 = a2 @ w2.T + W[pe + "conv.1.0.bias"]                                    # (B,10,34,64)
        y2 = silu(bn_eval(y2, W, pe + "conv.1.1.", axis=3))
        flat = np.ascontiguousarray(y2.transpose(0, 1, 3, 2)).reshape(b, t_out, C.SUB_OUT_IN)  # c*34+f
        x = linear(flat, W[pe + "out.weight"])
        return rmsnorm(x, W[pe + "out_norm.weight"])

    # --- a5: SwiGLU FFN (conformer_blocks.py:468-482) ---------------------------------------
    def ffn(self, x: np.ndarray, p: str) -> np.ndarray:
        W = self.W
        gate = silu(linear(x, W[p + "linear1.weight"], W[p + "linear1.bias"]))
        return linear(gate * linear(x, W[p + "linearv.weight"], W[p + "linearv.bias"]),
                      W[p + "linear2.weight"], W[p + "linear2.bias"])

    # --- a6-a8: RoPE MHSA with input cache and shared scores ---------------------------------
    def mhsa(self, h: np.ndarray, L: int, st: StreamState, nst: dict, shared: dict) -> np.ndarray:
        W = self.W
        p = f"encoder.layers.{L}.self_attn."
        b, t, d = h.shape
        S = C.mhsa_cache_rows(L)
        if S:
            # update_before_layer slices the cache to its last S rows (conformer_blocks.py:147-148);
            # update_state appends the normed input (submodules.py:295-302); update_after_layer
            # left-pads the new S-row cache to 30 (conformer_blocks.py:161-163).
            cache = st.mhsa[:, L - C.MHSA_STATELESS, -S:].astype(F32)
            kv = np.concatenate([cache, h], axis=1)                                  # (B, S+T, D)
            new = np.concatenate([cache[:, t:], h[:, :t]], axis=1)                   # (B, S, D)
            padded = np.zeros((b, C.MHSA_STATE, d), F32)
            padded[:, C.MHSA_STATE - S:] = new
            nst.setdefault("mhsa", [None] * C.N_MHSA_LAYERS)[L - C.MHSA_STATELESS] = fp16(padded)
        else:
            kv = h
        tk = kv.shape[1]
        hd, dk = C.N_HEADS, C.D_HEAD
        v = linear(kv, W[p + "linear_v.weight"], W[p + "linear_v.bias"]).reshape(b, tk, hd, dk).transpose(0, 2, 1, 3)
        if C.RECOMPUTE_SCORES[L]:
            q = linear(h, W[p + "linear_q.weight"], W[p + "linear_q.bias"]).reshape(b, t, hd, dk)
            k = linear(kv, W[p + "linear_k.weight"], W[p + "linear_k.bias"]).reshape(b, tk, hd, dk)
            q = layernorm(q, W[p + "q_ln.weight"], W[p + "q_ln.bias"]).transpose(0, 2, 1, 3)
            k = layernorm(k, W[p + "k_ln.weight"], W[p + "k_ln.bias"]).transpose(0, 2, 1, 3)
            q = self._rope(q, 0)
            k = self._rope(k, S)
            scores = (q @ k.transpose(0, 1, 3, 2)) / np.float32(math.sqrt(dk))     # (B, H, T, S+T)
            shared["scores"] = scores
        else:
            scores = shared["scores"]                                                # reused (conformer_blocks.py:150-152,719)
        if S:
            mask = self._mask(L, st, t, S)                                           # (B, T, S+T)
            sc = np.where(mask[:, None], np.float32(-10000), scores)
            attn = np.where(mask[:, None], np.float32(0), softmax(sc))
        else:
            attn = softmax(scores)
        ctx = (attn @ v).transpose(0, 2, 1, 3).reshape(b, t, d)
        return linear(ctx, W[p + "linear_out.weight"], W[p + "linear_out.bias"])

    @staticmethod
    def _rope(x: np.ndarray, offset: int) -> np.ndarray:
        """Partial RoPE on dims [0, 32) of each head (submodules.py:78-157)."""
        n = x.shape[2]
        cos, sin = rope_tables(n, offset)
        r = x[..., : C.ROPE_DIM]
        half = C.ROPE_DIM // 2
        rot = np.concatenate([-r[..., half:], r[..., :half]], axis=-1)
        out = x.copy()
        out[..., : C.ROPE_DIM] = r * cos + rot * sin
        return out.astype(F32)

    @staticmethod
    def _mask(L: int, st: StreamState, t: int, S: int) -> np.ndarray:
        """Streaming attention mask of layers 14/15 (EncoderState.create_masks / _update_masks,
        conformer_blocks.py:197-349): with offset = 30 - mhsa_len (floor-divided by the
        reduction factor inside the reduced block) a (query i, key j) pair is masked iff key
        position j or query position S+i lies before the offset."""
        mlen = st.mhsa_len[:, 0].astype(F32)
        off = np.float32(C.MHSA_STATE) - mlen
        if C.REDUCTION_POS < L <= C.UPSAMPLE_POS:
            off = np.floor(off / np.float32(C.REDUCTION_FACTOR))
        j = np.arange(S + t, dtype=F32)
        i = np.arange(t, dtype=F32) + np.float32(S)
        kvalid = j[None, :] >= off[:, None]                   # (B, S+T)
        qvalid = i[None, :] >= off[:, None]                   # (B, T)
        return ~(qvalid[:, :, None] & kvalid[:, None, :])

    # --- a9: convolution module (conformer_blocks.py:403-436, submodules.py:346-402) ---------
    def conv_module(self, h: np.ndarray, L: int, st: StreamState, nst: dict) -> np.ndarray:
        W = self.W
        p = f"encoder.layers.{L}.conv."
        y = linear(h, W[p + "pointwise_conv1.weight"], W[p + "pointwise_conv1.bias"])   # (B,T,768)
        d = C.D_MODEL
        u = y[..., :d] * sigmoid(y[..., d:])                                             # GLU
        cat = np.concatenate([st.conv[:, L].astype(F32), u.transpose(0, 2, 1)], axis=2)  # (B,384,30+T)
        nst.setdefault("conv", [None] * C.N_LAYERS)[L] = fp16(cat[:, :, -C.CONV_STATE:])
        win = np.lib.stride_tricks.sliding_window_view(cat, C.CONV_KERNEL, axis=2)       # (B,384,T,31)
        dw = np.einsum("bctk,ck->bct", win, W[p + "depthwise_conv.conv.weight"][:, 0]) \
            + W[p + "depthwise_conv.conv.bias"][None, :, None]
        dw = silu(bn_eval(dw.astype(F32), W, p + "batch_norm.", axis=1))
        return linear(dw.transpose(0, 2, 1), W[p + "pointwise_conv2.weight"], W[p + "pointwise_conv2.bias"])

    # --- a10: one macaron Conformer layer (conformer_blocks.py:799-836) ----------------------
    def layer(self, x: np.ndarray, L: int, st: StreamState, nst: dict, shared: dict) -> np.ndarray:
        W = self.W
        p = f"encoder.layers.{L}."
        r = x
        r = r + self.ffn(rmsnorm(r, W[p + "norm_feed_forward1.weight"]), p + "feed_forward1.") * np.float32(0.5)
        r = r + self.mhsa(rmsnorm(r, W[p + "norm_self_att.weight"]), L, st, nst, shared)
        r = r + self.conv_module(rmsnorm(r, W[p + "norm_conv.weight"]), L, st, nst)
        r = r + self.ffn(rmsnorm(r, W[p + "norm_feed_forward2.weight"]), p + "feed_forward2.") * np.float32(0.5)
        return rmsnorm(r, W[p + "norm_out.weight"])

    # --- a11: causal temporal reduction (conformer_blocks.py:874-911) ------------------------
    def reduce(self, x: np.ndarray, st: StreamState, nst: dict) -> np.ndarray:
        W = self.W
        tr = "encoder.temportal_reduction."
        xt = x.transpose(0, 2, 1)                                                    # (B,384,10)
        cat = np.concatenate([st.reduction.astype(F32), xt], axis=2)                 # (B,384,11)
        nst["reduction"] = fp16(cat[:, :, -C.RED_STATE:])
        w = W[tr + "conv.weight"][:, 0]                                              # (1536, 3)
        src = np.repeat(cat, 4, axis=1)                                              # group g -> outs 4g..4g+3
        win = np.lib.stride_tricks.sliding_window_view(src, C.REDUCTION_KERNEL, axis=2)[:, :, :: C.REDUCTION_FACTOR]
        y = np.einsum("botk,ok->bot", win, w) + W[tr + "conv.bias"][None, :, None]  # (B,1536,5)
        return linear(y.transpose(0, 2, 1).astype(F32), W[tr + "conv_pw.weight"], W[tr + "conv_pw.bias"])

    # --- a14: CTC head (conformer.py:338-354) -------------------------------------------------
    def head(self, x: np.ndarray) -> np.ndarray:
        W = self.W
        z = linear(x, W["decoder.decoder_layers.0.weight"], W["decoder.decoder_layers.0.bias"])
        m = z.max(axis=-1, keepdims=True)
        return (z - m - np.log(np.exp(z - m).sum(axis=-1, keepdims=True))).astype(F32)

    # --- the whole step ---------------------------------------------------------------------
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
                # TemporalUpsampling (conformer_blocks.py:955-988): repeat x2, right-pad 1, trim to T,
                # +residual (the pad frame is live for T = 13: 2 x 6 = 12 < 13)
                rep = np.repeat(x, C.REDUCTION_FACTOR, axis=1)
                up = np.zeros_like(residual)
                n = min(rep.shape[1], residual.shape[1])
                up[:, :n] = rep[:, :n]
                x = up + residual
            if trace is not None:
                trace.append(x)
        return x

    def step(self, pcm: np.ndarray, state: np.ndarray | None = None, trace: list | None = None
             ) -> tuple[np.ndarray, np.ndarray]:
        """pcm (B, 2400 | 3200 [,1]) int32, flat state (B, 219729) fp16 | None -> (logprobs fp32, state fp16).
        A 3200-sample (400 ms) chunk gives 13 frames; the state layout is the same.

        ``trace`` (optional list) receives the stage outputs the HIP path exposes for debugging:
        [feats (B,30,64), pre-encode output (B,10,384), layer 0 output, ..., layer 15 output]."""
        pcm = np.asarray(pcm)
        pcm = pcm.reshape(pcm.shape[0], -1)
        if pcm.shape[1] not in (2400, 3200):
            raise ValueError(f"chunk of {pcm.shape[1]} samples (2400 or 3200)")
        b = pcm.shape[0]
        st = StreamState.zeros(b) if state is None else StreamState.unflatten(np.asarray(state, np.float16))
        nst: dict = {}
        feats, nst["preproc"] = self.mel(pcm, st.preproc)
        if trace is not None:
            trace.append(feats.astype(F32))
        x = self.encode(feats, st, nst, trace)
        logp = self.head(x)
        nxt = StreamState(
            preproc=nst["preproc"],
            mhsa=np.stack(nst["mhsa"], axis=1),
            conv=np.stack(nst["conv"], axis=1),
            mhsa_len=fp16(np.minimum(st.mhsa_len.astype(F32) + logp.shape[1], C.MHSA_STATE)),
            sub1=nst["sub1"],
            sub2=nst["sub2"],
            reduction=nst["reduction"],
        )
        return logp, nxt.flatten()
