"""Measure the bf16 (or PREC=fp8) mode (BASELINE config 3) against the fp32 oracle: B = 2048, 10 stateful chunks,
stream s starts (zero state) at chunk s % 4; 64 sampled streams checked every chunk.  Also the
greedy decode of the example audio in bf16 vs the oracle decode of the fp32 oracle logprobs.
Prints JSON (used to set the bounds in tests/test_gpu_parity.py)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tone_amd.config as C  # noqa: E402
from tone_amd.model import ToneSession  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402
from tone_oracle import ToneOracle  # noqa: E402
import tone_decode_oracle as O  # noqa: E402

w = synthetic_weights(0)
orc = ToneOracle(w)
B, N = 2048, 10
PREC = os.environ.get("PREC", "bf16")
pick = np.arange(0, B, 32)
rng = np.random.default_rng(41)
s = ToneSession(w, precision=PREC, max_batch=B)
st = torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device="cuda:0")
st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
off = np.arange(B) % 4
rows = []
for c in range(N):
    x = np.clip(np.round(rng.normal(0, 3000, (B, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767)
    x[rng.random(B) < 0.2] = 0
    x = x.astype(np.int32)
    st[torch.from_numpy(off == c).cuda()] = 0
    st_o[off[pick] == c] = 0
    lp, st = s.step(torch.from_numpy(x).cuda(), st)
    lp = lp.cpu().numpy()[pick]
    lpo, st_o = orc.step(x[pick], st_o)
    live = off[pick] <= c
    d = np.abs(lp - lpo)[live]
    srt = np.sort(lpo[live], -1)
    clear = (srt[..., -1] - srt[..., -2]) > 0.1
    rows.append({"chunk": c, "max": float(d.max()), "p99": float(np.percentile(d, 99)), "median": float(np.median(d)),
                 "argmax_agree": float(np.mean(lp[live].argmax(-1) == lpo[live].argmax(-1))),
                 "argmax_agree_margin_0.1": float(np.mean((lp[live].argmax(-1) == lpo[live].argmax(-1))[clear]))})
s.close()
# example audio decode
audio = np.load(os.path.join(ROOT, "tests", "golden", "audio_short_pcm.npy")).astype(np.int32)
padded = np.pad(audio, (O.PADDING, O.PADDING))
padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
res = {}
for prec in (PREC, "fp32"):
    s = ToneSession(w, precision=prec, max_batch=1)
    state, sto, so, got, want, toks_g, toks_o = None, None, None, [], [], [], []
    for i, ch in enumerate(padded):
        lp, state = s.step(torch.from_numpy(ch[None]).cuda(), state)
        lp = lp.cpu().numpy()[0]
        lpo, so = orc.step(ch[None], so)
        out, sto_ = O.pipeline_step(lp, sto, i == len(padded) - 1)
        sto = sto_
        got += out
        toks_g.append(lp.argmax(-1)); toks_o.append(lpo[0].argmax(-1))
        if prec == "bf16":
            pass
    st2 = None
    so = None
    for i, ch in enumerate(padded):
        lpo, so = orc.step(ch[None], so)
        out, st2 = O.pipeline_step(lpo[0], st2, i == len(padded) - 1)
        want += out
    s.close()
    tg, to = np.concatenate(toks_g), np.concatenate(toks_o)
    res[prec] = {"phrases_identical": got == want, "n_phrases": len(want), "frame_token_agree": float(np.mean(tg == to)),
                 "got": [p[0] for p in got][:5], "want": [p[0] for p in want][:5]}
print(json.dumps({"stagger": rows, "example_audio": res}))
