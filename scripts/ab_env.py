"""In-step A/B of environment-selected routes (one ToneSession per route, same process, interleaved rounds):
per-family us/step with HIP events and the graph-replayed step time.
Usage: AB_BATCH=2048 AB_PREC=bf16 python scripts/ab_env.py "" "TONE_SWIGLU_T=1" ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tone_amd.config as C  # noqa: E402
from tone_amd.model import ToneSession  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402

B = int(os.environ.get("AB_BATCH", "2048"))
PREC = os.environ.get("AB_PREC", "bf16")
routes = sys.argv[1:]
w = synthetic_weights(0)
rng = np.random.default_rng(0)
pcm = torch.from_numpy(np.clip(rng.normal(0, 3000, (B, 2400)), -32768, 32767).astype(np.int32)).cuda()
fams = ["gemm_ffn_up", "gemm_ffn_down", "gemm_qkv", "gemm_attn_out", "gemm_pw1", "gemm_pw2"]
keys = {kv.split("=")[0] for r in routes for kv in r.split(",") if kv}
for rnd in range(2):
    for r in routes:
        for k in keys:
            os.environ.pop(k, None)
        for kv in (x for x in r.split(",") if x):
            k, v = kv.split("=")
            os.environ[k] = v
        s = ToneSession(w, precision=PREC, max_batch=B)
        st = torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device="cuda")
        for _ in range(3):
            _, st = s.step(pcm, st)
        s.set_timing(True)
        for _ in range(10):
            _, st = s.step(pcm, st)
        torch.cuda.synchronize()
        out = {f: round(s.kernel_us(f)[0] * s.kernel_us(f)[1] / 10, 1) for f in fams}
        s.set_timing(False)
        s.set_graph(True)
        sig = torch.empty_like(pcm); sig.copy_(pcm)
        a = torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device="cuda"); b = torch.empty_like(a)
        lp = torch.empty((B, 10, 35), device="cuda")
        strm = torch.cuda.Stream()
        with torch.cuda.stream(strm):
            for i in range(5):
                s.run(sig, a, lp, b, stream=strm); a, b = b, a
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(strm):
            e0.record(strm)
            for i in range(50):
                s.run(sig, a, lp, b, stream=strm); a, b = b, a
            e1.record(strm)
        torch.cuda.synchronize()
        print(json.dumps({"route": r, "batch": B, "prec": PREC, "round": rnd, "step_ms": round(e0.elapsed_time(e1) / 50, 4),
                          "families": out}), flush=True)
        s.close()
