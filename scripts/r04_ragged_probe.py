import sys, os, numpy as np
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "oracle"), os.path.join(os.getcwd(), "tests")]
import tone_amd.config as C
from tone_amd.model import ToneSession
from tone_amd.weights import synthetic_weights
from tone_oracle import ToneOracle
from test_gpu_parity import synthetic_pcm, gpu_step
w = synthetic_weights(0); orc = ToneOracle(w)
for b in (1000, 2048):
    s = ToneSession(w, precision="fp8", max_batch=b)
    rng = np.random.default_rng(41)
    pick = np.unique(np.r_[np.arange(0, b, 50), b - 1])
    st = np.zeros((b, C.STATE_SIZE), np.float16); st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
    for c in range(2):
        pcm = synthetic_pcm(rng, b)
        lp_g, st = gpu_step(s, pcm, st)
        lp_o, st_o = orc.step(pcm[pick], st_o)
        d = np.abs(lp_g[pick] - lp_o)
        print(os.environ.get("TONEHIP_LIB", "cur"), b, c, "max %.3f p99 %.3f agree %.4f" % (d.max(), np.percentile(d, 99), np.mean(lp_g[pick].argmax(-1) == lp_o.argmax(-1))), flush=True)
    s.close()
