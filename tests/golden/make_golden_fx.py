"""Golden vectors from the reference's own ``Tone.forward_for_export`` (tone/nn/model.py:101-206).

Run in the build container (needs /root/reference; the output fixtures travel, the reference does not):

    python tests/golden/make_golden_fx.py

``tone.nn.model.Tone`` is built from the reference modules (``tone/__init__.py`` bypassed and
torchaudio's ``melscale_fbanks`` restated, as in make_golden.py) with ``synthetic_weights(0)`` and
``forward_for_export`` is called directly, two ways:

* ``fp32``  -- autocast off, every state handed in as float32 (the fp16 values of the flat state).
  The preprocessor state is then float32 too, so ``FilterbankFeatures`` keeps the features in
  float32: this is the exported arithmetic without rounding point #2 (features -> fp16).
* ``fp16``  -- under ``torch.autocast(device, dtype=torch.float16)`` with fp16 states, exactly as
  tone/scripts/export.py:411 traces the ONNX graph (CPU autocast here; ORT's kernels may round
  differently, so this is the graph's *semantics*, not ORT's bits).

Fixtures (tests/golden/golden_fx.npz):

* ``stream_*``: the 4 streams x 6 chunks of golden_stream.npz (staggered restarts, mhsa_len 0..30
  mixed) stepped through both modes, logprobs per chunk.
* ``step_*``: one step from a carried state (the fp32 chain's state after chunk 3, stored in full):
  pcm, state_in, logprobs, next state (every 7th element), and the encoder's stage outputs (pre-encode, every layer,
  the reduction output at layer 6 and the upsampled sum at layer 14) captured with forward hooks --
  the per-stage pin of the oracle (tests/test_oracle.py).
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
sys.path.insert(0, str(HERE))

import tone_amd.config as C  # noqa: E402
from make_golden import ENCODER_PARAMS, _install_stubs  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402

STATE_SAMPLE = 7    # next-state fixtures keep every 7th element (covers every section)
SECTIONS = ["preproc", "mhsa", "conv", "mhsa_len", "sub1", "sub2", "reduction"]


def build_tone(seed: int = 0):
    _install_stubs()
    from tone.nn.model import Tone

    fe = dict(sample_rate=8000, window_size=0.02, window_stride=0.01, n_fft=160, n_mels=64)  # model_wrapper.py:28-35
    m = Tone(fe, ENCODER_PARAMS, dict(feat_in=384, vocabulary=list(C.LABELS))).eval()
    W = synthetic_weights(seed)
    sd = {}
    for k, v in m.state_dict().items():
        if k in W:
            sd[k] = torch.from_numpy(W[k])
        elif k.endswith("num_batches_tracked") or k.startswith("preprocessor."):
            sd[k] = v                        # BN counters; the preprocessor's DFT basis / fbank buffers
        else:
            raise KeyError(k)
    m.load_state_dict(sd, strict=True)
    return m


def split_state(flat: np.ndarray, dt) -> list:
    b = flat.shape[0]
    out = []
    for name in SECTIONS:
        off, shp = C.STATE_SECTIONS[name]
        n = int(np.prod(shp))
        out.append(torch.from_numpy(flat[:, off: off + n].reshape((b,) + shp).astype(dt)))
    return out


@torch.no_grad()
def fx_step(m, pcm: np.ndarray, flat: np.ndarray, fp16: bool):
    """One forward_for_export call; returns (logprobs fp32, next flat state fp16)."""
    b = pcm.shape[0]
    st = split_state(flat, np.float16 if fp16 else np.float32)
    x = torch.from_numpy(np.ascontiguousarray(pcm.reshape(b, -1, 1)).astype(np.int32))
    with torch.autocast("cpu", dtype=torch.float16, enabled=fp16):
        out = m.forward_for_export(x, None, *st)
    nxt = np.empty((b, C.STATE_SIZE), np.float16)
    for name, t in zip(SECTIONS, out[1:]):
        off, shp = C.STATE_SECTIONS[name]
        n = int(np.prod(shp))
        nxt[:, off: off + n] = t.reshape(b, n).half().numpy()
    return out[0].float().numpy(), nxt


def capture_stages(m):
    """Forward hooks giving the oracle's trace order: pre-encode, then each layer's output with the
    reduction (after layer 6) / upsampling (after layer 14) applied."""
    rec: dict = {}

    def hook(key):
        def f(_mod, _inp, out):
            rec[key] = (out[0] if isinstance(out, tuple) else out).float().numpy().copy()
        return f

    hs = [m.encoder.pre_encode.register_forward_hook(hook("pre")),
          m.encoder.temportal_reduction.register_forward_hook(hook("red")),
          m.encoder.temporal_upsample.register_forward_hook(hook("up"))]
    hs += [m.encoder.layers[i].register_forward_hook(hook(i)) for i in range(C.N_LAYERS)]

    def stages():
        out = [rec["pre"]]
        for i in range(C.N_LAYERS):
            out.append(rec["red"] if i == C.REDUCTION_POS else rec["up"] if i == C.UPSAMPLE_POS else rec[i])
        return out

    return hs, stages


def main() -> None:
    torch.set_num_threads(8)
    m = build_tone(0)
    g = np.load(HERE / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    res = {}
    states = {}
    for mode in ("fp32", "fp16"):
        state = np.zeros((B, C.STATE_SIZE), np.float16)
        lps = []
        for c in range(N):
            state[np.arange(B) > c] = 0
            if mode == "fp32" and c == 4:
                states["step_in"] = state.copy()
            lp, state = fx_step(m, pcm[:, c], state, mode == "fp16")
            lps.append(lp)
        res[f"stream_{mode}_logprobs"] = np.stack(lps, 1)

    # one step from a carried state, every stage captured (fp32 mode)
    st_in = states["step_in"]
    hs, stages = capture_stages(m)
    lp, nxt = fx_step(m, pcm[:, 4], st_in, False)
    st = stages()
    for h in hs:
        h.remove()
    stage_arr = np.zeros((B, len(st), C.CHUNK_FRAMES, C.D_MODEL), np.float32)
    for i, a in enumerate(st):
        stage_arr[:, i, : a.shape[1]] = a
    lp16, nxt16 = fx_step(m, pcm[:, 4], st_in, True)
    np.savez_compressed(
        HERE / "golden_fx.npz",
        stream_pcm_source=np.array("golden_stream.npz"),
        step_pcm=pcm[:, 4].astype(np.int16), step_state_in=st_in, step_logprobs_fp32=lp,
        step_state_out_fp32=nxt[:, ::STATE_SAMPLE], step_stages_fp32=stage_arr, step_logprobs_fp16=lp16,
        step_state_out_fp16=nxt16[:, ::STATE_SAMPLE], state_sample=np.array(STATE_SAMPLE), **res,
    )
    print("wrote golden_fx.npz; fp16-vs-fp32 stream max |dlogp| =",
          float(np.abs(res["stream_fp16_logprobs"] - res["stream_fp32_logprobs"]).max()))


if __name__ == "__main__":
    main()
