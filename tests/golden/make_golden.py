"""Generate the golden vectors in tests/golden/ from the REFERENCE's own torch modules.

Run in the build container (needs /root/reference, which never travels to the GPU box):

    python tests/golden/make_golden.py

What runs is the reference code itself -- ``FilterbankFeatures.forward_streaming``
(tone/nn/modules/feats.py:118-133), ``Encoder.forward`` + ``EncoderState.next``
(tone/nn/modules/conformer.py:148-233, conformer_blocks.py:178-195) and
``ConvASRDecoder.forward`` (conformer.py:338-354) -- composed exactly as
``Tone.forward_for_export`` does (tone/nn/model.py:162-205), with two adaptations:

* ``tone/__init__.py`` is bypassed (it imports onnxruntime/pyctcdecode/kenlm/miniaudio, absent here)
  by registering a bare ``tone`` package whose ``__path__`` is the reference directory.
* torchaudio is absent, so ``torchaudio.functional.melscale_fbanks`` is provided by a stub that
  restates torchaudio 2.7.1's Slaney implementation (the only torchaudio call, feats.py:84-92).
* the encoder runs in float32 on the fp16-rounded features (the ONNX graph would run it under fp16
  autocast, export.py:411, which CPU torch cannot); states cross the step boundary as fp16.

Weights are ``tone_amd.weights.synthetic_weights(seed=0)`` (real weights are not available offline).
"""

from __future__ import annotations

import math
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

import tone_amd.config as C  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402


def _install_stubs() -> None:
    pkg = types.ModuleType("tone")
    pkg.__path__ = [str(REF / "tone")]
    sys.modules["tone"] = pkg

    ta = types.ModuleType("torchaudio")
    taf = types.ModuleType("torchaudio.functional")

    def _hz_to_mel(freq: float) -> float:
        f_sp = 200.0 / 3
        mels = freq / f_sp
        min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
        if freq >= min_log_hz:
            mels = min_log_mel + math.log(freq / min_log_hz) / logstep
        return mels

    def _mel_to_hz(mels: torch.Tensor) -> torch.Tensor:
        f_sp = 200.0 / 3
        freqs = f_sp * mels
        min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
        log_t = mels >= min_log_mel
        freqs[log_t] = min_log_hz * torch.exp(logstep * (mels[log_t] - min_log_mel))
        return freqs

    def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate, norm=None, mel_scale="htk"):
        assert norm == "slaney" and mel_scale == "slaney" and f_min == 0
        all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
        m_pts = torch.linspace(_hz_to_mel(f_min), _hz_to_mel(f_max), n_mels + 2)
        f_pts = _mel_to_hz(m_pts)
        f_diff = f_pts[1:] - f_pts[:-1]
        slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
        down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
        up = slopes[:, 2:] / f_diff[1:]
        fb = torch.max(torch.zeros(1), torch.min(down, up))
        enorm = 2.0 / (f_pts[2: n_mels + 2] - f_pts[:n_mels])
        return fb * enorm.unsqueeze(0)

    taf.melscale_fbanks = melscale_fbanks
    ta.functional = taf
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.functional"] = taf


ENCODER_PARAMS = {  # tone/training/model_wrapper.py:37-75
    "feat_in": 64, "n_layers": 16, "subsampling_conv_channels": [32, 64],
    "subsampling_kernel_size": [[11, 21], [11, 11]], "subsampling_strides": [[1, 1], [3, 1]],
    "ff_expansion_factor": 4, "n_heads": 8, "conv_kernel_size": 31, "dropout": 0.1,
    "dropout_att": 0.1, "mhsa_stateless_layers": 14, "rope_dim": 32,
    "should_recompute_att_scores": list(C.RECOMPUTE_SCORES), "mhsa_state_size": 30,
    "chunk_size": 10, "d_model": 384, "reduction_factor": 2, "reduction_kernel_size": 3,
    "reduction_position": 6, "upsample_position": 14,
}


class RefStep:
    """Tone.forward_for_export (model.py:162-205) on the reference modules, fp32 between fp16 I/O."""

    def __init__(self, seed: int = 0):
        _install_stubs()
        from tone.nn.modules.conformer import ConvASRDecoder, Encoder
        from tone.nn.modules.feats import FilterbankFeatures

        self.pre = FilterbankFeatures(sample_rate=8000, window_size=0.02, window_stride=0.01, n_fft=160, n_mels=64)
        self.enc = Encoder(**ENCODER_PARAMS).eval()
        self.dec = ConvASRDecoder(feat_in=384, vocabulary=list(C.LABELS)).eval()
        W = synthetic_weights(seed)
        enc_sd = {k[len("encoder."):]: torch.from_numpy(v) for k, v in W.items() if k.startswith("encoder.")}
        for k, v in self.enc.state_dict().items():
            if k.endswith("num_batches_tracked"):
                enc_sd[k] = v
        self.enc.load_state_dict(enc_sd, strict=True)
        dec_sd = {k[len("decoder."):]: torch.from_numpy(v) for k, v in W.items() if k.startswith("decoder.")}
        self.dec.load_state_dict(dec_sd, strict=True)

    @torch.no_grad()
    def mel(self, pcm: np.ndarray, pre_state: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        wav = (torch.from_numpy(pcm.astype(np.int32)).float() / torch.iinfo(torch.int16).max).half()
        feats, st = self.pre.forward_streaming(waveform=wav, state=torch.from_numpy(pre_state))
        return feats.numpy(), st.numpy()

    @torch.no_grad()
    def step(self, pcm: np.ndarray, flat_state: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        b = pcm.shape[0]
        sec = {}
        for name, (off, shp) in C.STATE_SECTIONS.items():
            n = int(np.prod(shp))
            sec[name] = torch.from_numpy(flat_state[:, off: off + n].reshape((b,) + shp).copy())
        feats, pre_next = self.mel(pcm, sec["preproc"].numpy())
        feats = torch.from_numpy(feats).float()
        out, _ = self.enc(
            audio_signal=feats, length=None,
            state_mhsa=sec["mhsa"].float().transpose(0, 1),
            state_conv=sec["conv"].float().transpose(0, 1),
            state_mhsa_len=sec["mhsa_len"].float()[:, 0],
            state_subsampling_1=sec["sub1"].float(),
            state_subsampling_2=sec["sub2"].float(),
            state_reduction=sec["reduction"].float(),
        )
        nxt = self.enc.state.next()
        logp = self.dec(encoder_output=out).float().numpy()
        parts = {
            "preproc": torch.from_numpy(pre_next),
            "mhsa": nxt.mhsa.transpose(0, 1),
            "conv": nxt.conv.transpose(0, 1),
            "mhsa_len": nxt.mhsa_len.unsqueeze(-1),
            "sub1": nxt.subsampling[0],
            "sub2": nxt.subsampling[1],
            "reduction": nxt.reduction,
        }
        flat = np.empty((b, C.STATE_SIZE), np.float16)
        for name, (off, shp) in C.STATE_SECTIONS.items():
            n = int(np.prod(shp))
            flat[:, off: off + n] = parts[name].reshape(b, n).half().numpy()
        return logp, flat


def synthetic_pcm(rng: np.random.Generator, b: int, n_chunks: int, silence: float = 0.2) -> np.ndarray:
    """Gaussian sigma=3000 clipped to int16, with a share of all-zero chunks."""
    x = np.clip(np.round(rng.normal(0.0, 3000.0, size=(b, n_chunks, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767)
    x[rng.random((b, n_chunks)) < silence] = 0
    return x.astype(np.int32)


STATE_SAMPLE_STRIDE = 61   # sample every 61st state element (covers every section)


def main() -> None:
    torch.set_num_threads(8)
    ref = RefStep(seed=0)
    rng = np.random.default_rng(20260115)

    # F3: log-mel front-end, 4 streams x 3 chunks, includes an extreme-amplitude stream
    pcm_m = synthetic_pcm(rng, 4, 3, silence=0.0)
    pcm_m[3] = np.where(rng.random((3, 2400)) < 0.5, -32768, 32767)
    pcm_m[2, 1] = 0
    st = np.zeros((4, C.PREPROC_STATE), np.float16)
    feats = []
    for c in range(3):
        f, st = ref.mel(pcm_m[:, c], st)
        feats.append(f)
    np.savez_compressed(HERE / "golden_mel.npz", pcm=pcm_m.astype(np.int16), feats=np.stack(feats, 1))

    # F1: full streaming step, 4 streams x 6 chunks, stream s restarts (zero state) until chunk s,
    # so one batch mixes mhsa_len 0/10/20/30.
    B, N = 4, 6
    pcm = synthetic_pcm(rng, B, N)
    state = np.zeros((B, C.STATE_SIZE), np.float16)
    logps, samples, sums = [], [], []
    idx = np.arange(0, C.STATE_SIZE, STATE_SAMPLE_STRIDE)
    for c in range(N):
        for s in range(B):
            if s > c:
                state[s] = 0
        logp, state = ref.step(pcm[:, c], state)
        logps.append(logp)
        samples.append(state[:, idx])
        sec_sums = []
        for name, (off, shp) in C.STATE_SECTIONS.items():
            n = int(np.prod(shp))
            sec_sums.append(np.abs(state[:, off: off + n].astype(np.float64)).sum(axis=1))
        sums.append(np.stack(sec_sums, 1))
    np.savez_compressed(
        HERE / "golden_stream.npz",
        pcm=pcm.astype(np.int16), logprobs=np.stack(logps, 1), state_samples=np.stack(samples, 1),
        state_abs_sums=np.stack(sums, 1), sample_stride=np.array(STATE_SAMPLE_STRIDE),
        final_state_stream0=state[0],
    )
    print("wrote", [p.name for p in HERE.glob("golden_*.npz")])


if __name__ == "__main__":
    main()
