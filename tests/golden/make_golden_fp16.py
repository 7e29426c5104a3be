"""Golden vectors of the EXPORTED graph's numerics: ``Tone.forward_for_export`` under fp16 autocast with the
export's LayerNorm patch -- what ``onnx_wrapper`` runs (tone/onnx_wrapper.py:84-123 executes the graph that
tone/scripts/export.py traces).

Run in the build container (needs /root/reference; the fixture travels, the reference does not):

    python tests/golden/make_golden_fp16.py

How the export traces the step (and so what this script reproduces, on CPU like the export itself -- the
model is loaded by ``ToneForCTC.from_pretrained`` and never moved to a GPU, export.py:143-145):

* ``torch.amp.autocast("cpu", dtype=torch.float16)`` around ``forward_for_export`` (export.py:411).  Linear,
  Conv and matmul run in fp16 (weights cast to fp16, outputs fp16); every elementwise op on an fp16 tensor
  rounds to fp16; RMSNorm computes in fp32 and returns fp16 (submodules.py:34-54); the front end is fp32 up
  to the fp16 features (feats.py).  ``avoid_float16_autocast_context`` (tone/nn/torch_utils.py:10-34) and
  the fp32 cast at conformer_blocks.py:708-713 test the *CUDA* autocast state, so on a CPU trace they do
  nothing: attention runs in fp16 too (scores, softmax, P.V).
* ``torch.nn.functional.layer_norm`` replaced by ``layer_norm(inputs.float(), ...)`` before tracing
  (export.py:28-34, 466-467): the q/k LayerNorms take and return fp32, so RoPE runs on fp32 values and
  q/k round to fp16 only as the score matmul's operands.
* fp16 states in and out (export.py:454-455).

``tests/golden/op_trace_fp16.txt`` (written by ``--trace``) lists every aten op of one step with its input
and output dtypes -- the rounding points ``oracle/tone_oracle_fp16.py`` restates.

Fixture (tests/golden/golden_fp16.npz), ``synthetic_weights(0)``:

* ``stream_logprobs``: the 4 streams x 6 chunks of golden_stream.npz (staggered restarts, mhsa_len 0..30).
* ``step_*``: one step from the fp16 chain's own state after chunk 3, with every encoder stage (pre-encode,
  each layer, reduction / upsampling) captured by forward hooks as the fp16 values the graph carries, the
  features, and every 7th element of the next state.
* ``audio_logprobs``: the reference's example utterance (audio_short, 300 ms padding each side as
  pipeline.py:191 does) chunk by chunk at B = 1.
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
from make_golden_fx import STATE_SAMPLE, build_tone, capture_stages, split_state, SECTIONS  # noqa: E402

_old_layer_norm = torch.nn.functional.layer_norm


def _export_layer_norm(inputs, *args, **kwargs):
    """tone/scripts/export.py:28-34: LayerNorm in float32 for the ONNX export."""
    return _old_layer_norm(inputs.float(), *args, **kwargs)


@torch.no_grad()
def export_step(m, pcm: np.ndarray, flat: np.ndarray):
    """One forward_for_export call with the export's numerics; (logprobs fp32, next flat state fp16)."""
    b = pcm.shape[0]
    st = split_state(flat, np.float16)
    x = torch.from_numpy(np.ascontiguousarray(pcm.reshape(b, -1, 1)).astype(np.int32))
    torch.nn.functional.layer_norm = _export_layer_norm
    try:
        with torch.autocast("cpu", dtype=torch.float16):
            out = m.forward_for_export(x, None, *st)
    finally:
        torch.nn.functional.layer_norm = _old_layer_norm
    nxt = np.empty((b, C.STATE_SIZE), np.float16)
    for name, t in zip(SECTIONS, out[1:]):
        off, shp = C.STATE_SECTIONS[name]
        n = int(np.prod(shp))
        nxt[:, off: off + n] = t.reshape(b, n).half().numpy()
    return out[0].float().numpy(), nxt


def write_trace(m, pcm, flat, path: Path) -> None:
    """Every aten op of one step with its module and dtypes (the rounding points)."""
    from torch.utils._python_dispatch import TorchDispatchMode

    stack: list = []
    hooks = []
    for n, mod in m.named_modules():
        if n.count(".") <= 4:
            hooks.append(mod.register_forward_pre_hook(lambda _m, _i, n=n: stack.append(n)))
            hooks.append(mod.register_forward_hook(lambda _m, _i, _o: (stack.pop(), None)[1]))
    lines: list = []

    def dt(x):
        if isinstance(x, torch.Tensor):
            return f"{str(x.dtype)[6:]}{tuple(x.shape)}"
        if isinstance(x, (list, tuple)):
            return [dt(y) for y in x if isinstance(y, torch.Tensor)]
        return None

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            ins = [d for d in (dt(a) for a in args) if d]
            lines.append(f"{stack[-1] if stack else '-'} {func.__name__} {ins} -> {dt(out)}")
            return out

    with Log():
        export_step(m, pcm, flat)
    for h in hooks:
        h.remove()
    path.write_text("\n".join(lines) + "\n")


def main() -> None:
    torch.set_num_threads(8)
    m = build_tone(0)
    g = np.load(HERE / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    state = np.zeros((B, C.STATE_SIZE), np.float16)
    lps, step_in = [], None
    for c in range(N):
        state[np.arange(B) > c] = 0
        if c == 4:
            step_in = state.copy()
        lp, state = export_step(m, pcm[:, c], state)
        lps.append(lp)
    stream = np.stack(lps, 1)

    hs, stages = capture_stages(m)
    feats_rec = {}

    def grab(_m, _a, kw):
        feats_rec["f"] = kw["audio_signal"].float().numpy().copy()

    hf = m.encoder.register_forward_pre_hook(grab, with_kwargs=True)
    lp, nxt = export_step(m, pcm[:, 4], step_in)
    st = stages()
    for h in hs + [hf]:
        h.remove()
    stage_arr = np.zeros((B, len(st), C.CHUNK_FRAMES, C.D_MODEL), np.float32)
    for i, a in enumerate(st):
        stage_arr[:, i, : a.shape[1]] = a

    audio = np.load(HERE / "audio_short_pcm.npy").astype(np.int32)
    padded = np.pad(audio, (2400, 2400))                       # pipeline.py:191 PADDING
    padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
    ast = np.zeros((1, C.STATE_SIZE), np.float16)
    alps = []
    for ch in padded:
        lpa, ast = export_step(m, ch[None], ast)
        alps.append(lpa[0])

    if "--trace" in sys.argv:
        write_trace(m, pcm[:1, 4], step_in[:1], HERE / "op_trace_fp16.txt")
    np.savez_compressed(
        HERE / "golden_fp16.npz",
        stream_logprobs=stream, step_pcm=pcm[:, 4].astype(np.int16), step_state_in=step_in,
        step_feats=feats_rec["f"].astype(np.float16), step_stages=stage_arr.astype(np.float16),
        step_logprobs=lp, step_state_out=nxt[:, ::STATE_SAMPLE], state_sample=np.array(STATE_SAMPLE),
        audio_logprobs=np.stack(alps),
    )
    old = np.load(HERE / "golden_fx.npz")["stream_fp16_logprobs"]
    print("wrote golden_fp16.npz; vs golden_fx fp16 (LayerNorm unpatched) max |dlogp| =",
          float(np.abs(stream - old).max()), "; audio chunks", len(alps))


if __name__ == "__main__":
    main()
