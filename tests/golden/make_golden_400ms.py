"""Golden vectors of the 400 ms chunk variant from the reference's own ``Tone.forward_for_export``
(3200-sample chunks: 40 mel frames, 13 acoustic frames, 6 in the reduced block, the upsampling pad
frame live -- tone/nn/modules/conformer_blocks.py:978-981; the chunk length the Triton ensemble
serves, triton/ensemble/config.pbtxt:12-18, and tone/scripts/export.py exports with
chunk_duration_ms=400).

Run in the build container (needs /root/reference; the fixture travels, the reference does not):

    python tests/golden/make_golden_400ms.py

Same construction as make_golden_fx.py (fp32 mode: states handed in as float32, autocast off):
4 streams x 5 chunks, stream s restarting from the zero state until chunk s (mhsa_len 0/13/26/30
mixed in one batch), logprobs per chunk, and one step from a carried state with every encoder stage.
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
from make_golden_fx import STATE_SAMPLE, build_tone, capture_stages, fx_step  # noqa: E402

CHUNK = 3200


def main() -> None:
    torch.set_num_threads(8)
    m = build_tone(0)
    rng = np.random.default_rng(400)
    B, N = 4, 5
    pcm = np.clip(np.round(rng.normal(0, 3000, (B, N, CHUNK))), -32768, 32767).astype(np.int32)
    pcm[1, 2] = 0                                                         # a silent chunk
    state = np.zeros((B, C.STATE_SIZE), np.float16)
    lps, step_in = [], None
    for c in range(N):
        state[np.arange(B) > c] = 0
        if c == 3:
            step_in = state.copy()
        lp, state = fx_step(m, pcm[:, c], state, False)
        lps.append(lp)
    hs, stages = capture_stages(m)
    lp, nxt = fx_step(m, pcm[:, 3], step_in, False)
    st = stages()
    for h in hs:
        h.remove()
    T = lp.shape[1]
    stage_arr = np.zeros((B, len(st), T, C.D_MODEL), np.float32)
    for i, a in enumerate(st):
        stage_arr[:, i, : a.shape[1]] = a
    np.savez_compressed(
        HERE / "golden_400ms.npz",
        pcm=pcm.astype(np.int16), logprobs=np.stack(lps, 1), step_state_in=step_in, step_logprobs=lp,
        step_state_out=nxt[:, ::STATE_SAMPLE], step_stages=stage_arr, state_sample=np.array(STATE_SAMPLE),
    )
    print("wrote golden_400ms.npz", np.stack(lps, 1).shape)


if __name__ == "__main__":
    main()
