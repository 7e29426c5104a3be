"""Experiment: the B = 256 fp32 step as K independent sessions of 256 / K streams each, replayed
concurrently on K HIP streams (each session's graph on its own stream), vs one session of 256.
Prints one JSON line per K: real-time streams and ms per (whole-batch) step."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tone_amd.config as C  # noqa: E402
from tone_amd.model import ToneSession  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402


def run(k: int, total: int, steps: int, precision: str) -> dict:
    dev = torch.device("cuda:0")
    w = synthetic_weights(0)
    b = total // k
    sess = [ToneSession(w, device=0, precision=precision, max_batch=b, graph=True) for _ in range(k)]
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    rng = np.random.default_rng(1)
    pcm = [torch.from_numpy(np.clip(rng.normal(0, 3000, (4, b, C.AUDIO_CHUNK_SAMPLES)), -32768, 32767)
                            .astype(np.int32)).to(dev) for _ in range(k)]
    slabs = [[torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=dev) for _ in range(2)] for _ in range(k)]
    logp = [torch.zeros((b, C.CHUNK_FRAMES, C.VOCAB), dtype=torch.float32, device=dev) for _ in range(k)]

    def step(i):
        for j in range(k):
            with torch.cuda.stream(streams[j]):
                sess[j].run(pcm[j][i % 4], slabs[j][i % 2], logp[j], slabs[j][1 - i % 2], stream=streams[j])

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    for s in sess:
        s.close()
    return {"sessions": k, "streams_per_session": b, "ms_per_step": round(dt * 1e3, 4),
            "rt_streams": round(total / dt * 0.3, 1), "precision": precision}


if __name__ == "__main__":
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    for k in (1, 2, 4):
        print(json.dumps(run(k, total, 200, prec)), flush=True)
