"""HIP path vs the CPU oracle (and the reference golden vectors) on a real MI355X.

Tolerances (north_star): logprobs within 1e-3 abs fp32, greedy argmax identical wherever the
oracle's top-2 margin exceeds the tolerance; states are fp16 at the boundary, compared to a few
fp16 ulps.  The bf16-MFMA mode is checked against a looser bound (documented in DESIGN.md).
"""

from pathlib import Path

import numpy as np
import pytest

import tone_amd.config as C
from tone_amd.weights import synthetic_weights

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).parent / "golden"
LOGP_TOL = 1e-3


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(0)


@pytest.fixture(scope="module")
def oracle(weights):
    from tone_oracle import ToneOracle
    return ToneOracle(weights)


@pytest.fixture(scope="module")
def sess(weights):
    _gpu()
    from tone_amd.model import ToneSession
    s = ToneSession(weights, device=0, precision="fp32", max_batch=256)
    yield s
    s.close()


def synthetic_pcm(rng, b, silence=0.2):
    x = np.clip(np.round(rng.normal(0.0, 3000.0, size=(b, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767)
    x[rng.random(b) < silence] = 0
    return x.astype(np.int32)


def gpu_step(sess, pcm, state):
    dev = sess.dev
    sig = torch.from_numpy(np.ascontiguousarray(pcm.reshape(pcm.shape[0], -1))).to(dev)
    st = torch.from_numpy(np.ascontiguousarray(state)).to(dev)
    logp, nst = sess.step(sig, st)
    torch.cuda.synchronize()
    return logp.cpu().numpy(), nst.cpu().numpy()


def assert_logp_close(lp, ref, tol=LOGP_TOL, what=""):
    d = np.abs(lp - ref)
    assert d.max() < tol, f"{what} max |dlogp| = {d.max():.3g}"
    srt = np.sort(ref, axis=-1)
    clear = (srt[..., -1] - srt[..., -2]) > 2 * tol
    np.testing.assert_array_equal(lp.argmax(-1)[clear], ref.argmax(-1)[clear], err_msg=f"{what} greedy argmax")


def assert_state_close(st, ref, what=""):
    a, b = st.astype(np.float32), ref.astype(np.float32)
    d = np.abs(a - b)
    ulp = np.abs(np.spacing(ref)).astype(np.float32)
    frac_close = np.mean(d <= 2 * ulp)
    assert d.max() < 2e-2 and frac_close > 0.995, f"{what} state max diff {d.max():.3g}, within 2 ulp {frac_close:.4f}"


def test_stagewise_parity(sess, oracle):
    """Every stage of one step (front end, pre-encode, each Conformer layer) vs the oracle trace,
    from a non-trivial carried state (the step after a first chunk)."""
    rng = np.random.default_rng(7)
    b = 4
    _, st0 = oracle.step(synthetic_pcm(rng, b, 0.0), None)
    pcm = synthetic_pcm(rng, b, 0.0)
    trace = []
    oracle.step(pcm, st0, trace=trace)
    errs = []
    try:
        for stage, ref in enumerate(trace):
            sess.debug_stop(stage)
            gpu_step(sess, pcm, st0)
            if stage == 0:
                got = sess.debug_read("feats", (b, C.MEL_FRAMES, C.N_MELS))
            else:
                layer = stage - 2
                reduced = C.REDUCTION_POS <= layer < C.UPSAMPLE_POS
                got = sess.debug_read("rB", (b, 5, C.D_MODEL)) if reduced else sess.debug_read("rA", (b, 10, C.D_MODEL))
            errs.append(float(np.abs(got - ref).max()))
    finally:
        sess.debug_stop(-1)
    names = ["feats", "pre_encode"] + [f"layer{i}" for i in range(16)]
    report = ", ".join(f"{n}={e:.2e}" for n, e in zip(names, errs))
    assert max(errs) < 5e-3, report


def test_golden_stream_parity(sess, oracle):
    """The reference's own golden vectors (4 streams x 6 chunks, mhsa_len 0..30 mixed)."""
    g = np.load(GOLDEN / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    st_gpu = np.zeros((B, C.STATE_SIZE), np.float16)
    st_orc = st_gpu.copy()
    for c in range(N):
        st_gpu[np.arange(B) > c] = 0
        st_orc[np.arange(B) > c] = 0
        lp_o, st_o = oracle.step(pcm[:, c], st_gpu)       # oracle from the GPU's state: per-step error
        lp_g, st_g = gpu_step(sess, pcm[:, c], st_gpu)
        assert_logp_close(lp_g, lp_o, what=f"chunk {c} vs oracle")
        assert_logp_close(lp_g, g["logprobs"][:, c], what=f"chunk {c} vs reference golden")
        assert_state_close(st_g, st_o, what=f"chunk {c}")
        st_gpu = st_g


def test_example_audio_parity(sess, oracle):
    """The reference's example utterance (tests/golden/audio_short_pcm.npy: the MD5-pinned decode of
    tone/demo/audio_examples/audio_short.flac) fed as the pipeline feeds it -- 300 ms of padding on
    both sides, whole 2400-sample chunks (tone/pipeline.py:178-200) -- beside its polarity-inverted
    copy; every chunk's logprobs vs the oracle stepped from the same state, <= 1e-3."""
    pcm = np.load(GOLDEN / "audio_short_pcm.npy").astype(np.int32)
    a = np.pad(pcm, (C.AUDIO_CHUNK_SAMPLES, C.AUDIO_CHUNK_SAMPLES))
    a = np.pad(a, (0, -len(a) % C.AUDIO_CHUNK_SAMPLES)).reshape(-1, C.AUDIO_CHUNK_SAMPLES)
    chunks = np.stack([a, np.clip(-a, -32768, 32767)], 1)
    st = np.zeros((2, C.STATE_SIZE), np.float16)
    for c in range(len(chunks)):
        lp_g, st_g = gpu_step(sess, chunks[c], st)
        lp_o, st_o = oracle.step(chunks[c], st)
        assert_logp_close(lp_g, lp_o, what=f"example audio chunk {c}")
        assert_state_close(st_g, st_o, what=f"example audio chunk {c}")
        st = st_g


def test_b256_parity(sess, oracle):
    """BASELINE config 2: batch 256, fp32, logprobs vs the CPU oracle <= 1e-3 over 3 chunks."""
    rng = np.random.default_rng(11)
    b = 256
    st = np.zeros((b, C.STATE_SIZE), np.float16)
    for c in range(3):
        pcm = synthetic_pcm(rng, b)
        lp_g, st_g = gpu_step(sess, pcm, st)
        lp_o, st_o = oracle.step(pcm, st)
        assert_logp_close(lp_g, lp_o, what=f"B=256 chunk {c}")
        assert_state_close(st_g, st_o, what=f"B=256 chunk {c}")
        st = st_g


def test_edge_inputs(sess, oracle):
    """Full-scale square wave, silence, single-sample spikes; stream of length 1 (B=1)."""
    pcm = np.zeros((3, C.AUDIO_CHUNK_SAMPLES), np.int32)
    pcm[0] = np.where(np.arange(2400) % 7 < 3, -32768, 32767)
    pcm[2, ::97] = 32767
    st = np.zeros((3, C.STATE_SIZE), np.float16)
    for c in range(2):
        lp_g, st_g = gpu_step(sess, pcm, st)
        lp_o, st_o = oracle.step(pcm, st)
        assert_logp_close(lp_g, lp_o, what=f"edge chunk {c}")
        st = st_g
    lp1, _ = gpu_step(sess, pcm[:1], np.zeros((1, C.STATE_SIZE), np.float16))
    lpb, _ = gpu_step(sess, pcm, np.zeros((3, C.STATE_SIZE), np.float16))
    assert np.abs(lp1 - lpb[:1]).max() < 1e-5


def test_streams_independent_and_deterministic(sess):
    rng = np.random.default_rng(3)
    b = 6
    pcm = synthetic_pcm(rng, b, 0.0)
    st = np.zeros((b, C.STATE_SIZE), np.float16)
    _, st = gpu_step(sess, pcm, st)
    lp_a, st_a = gpu_step(sess, pcm, st)
    lp_b, st_b = gpu_step(sess, pcm, st)
    np.testing.assert_array_equal(lp_a, lp_b)
    np.testing.assert_array_equal(st_a, st_b)
    for s in (0, 3, 5):
        lp_s, st_s = gpu_step(sess, pcm[s:s + 1], st[s:s + 1])
        assert np.abs(lp_s - lp_a[s:s + 1]).max() < 1e-5
        assert np.abs(st_s.astype(np.float32) - st_a[s:s + 1].astype(np.float32)).max() <= 1e-3


def test_graph_replay_and_slots_match_eager(sess):
    rng = np.random.default_rng(5)
    b = 8
    dev = sess.dev
    sig = torch.from_numpy(synthetic_pcm(rng, b, 0.0)).to(dev)
    st_in = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=dev)
    st_e = torch.empty_like(st_in)
    lp_e = torch.empty((b, 10, 35), dtype=torch.float32, device=dev)
    sess.run(sig, st_in, lp_e, st_e)
    # hipGraph replay (captured on a side stream)
    stream = torch.cuda.Stream(dev)
    st_g = torch.empty_like(st_in)
    lp_g = torch.empty_like(lp_e)
    sess.set_graph(True)
    try:
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            for _ in range(3):
                sess.run(sig, st_in, lp_g, st_g, stream=stream)
        stream.synchronize()
    finally:
        sess.set_graph(False)
    assert torch.equal(lp_e, lp_g) and torch.equal(st_e, st_g)
    # device-resident slab, streams scattered over slots
    n_slots = 20
    slots = torch.tensor([3, 17, 0, 9, 11, 4, 19, 7], dtype=torch.int32, device=dev)
    slab_in = torch.zeros((n_slots, C.STATE_SIZE + 47), dtype=torch.float16, device=dev)   # padded stride
    slab_out = torch.zeros_like(slab_in)
    lp_s = torch.empty_like(lp_e)
    sess.run_slots(sig, slots, slab_in, slab_out, lp_s)
    torch.cuda.synchronize()
    assert torch.equal(lp_s, lp_e)
    assert torch.equal(slab_out[slots.long(), : C.STATE_SIZE], st_e)


def test_numpy_dropin_matches_session(weights):
    _gpu()
    from tone_amd.model import StreamingCTCModel, ToneSession
    model = StreamingCTCModel(ToneSession(weights, max_batch=4))
    rng = np.random.default_rng(9)
    chunk = synthetic_pcm(rng, 6, 0.0)[:, :, None]            # batch 6 > max_batch 4: split
    lp, st = model.forward(chunk)
    assert lp.shape == (6, 10, 35) and lp.dtype == np.float32
    assert st.shape == (6, C.STATE_SIZE) and st.dtype == np.float16
    lp2, st2 = model.forward(chunk, st)
    s = model.session
    ref_a, _ = gpu_step(s, chunk[:4, :, 0], st[:4])
    ref_b, _ = gpu_step(s, chunk[4:, :, 0], st[4:])
    np.testing.assert_allclose(lp2, np.concatenate([ref_a, ref_b]), atol=1e-6)
    with pytest.raises(ValueError):
        model.forward(chunk.astype(np.int64))
    model.session.close()


def test_fp32_split_vs_fp32_mfma(weights, oracle):
    """The default fp32 path computes its GEMMs as exact 3-way bf16 splits on the bf16 MFMA
    (gemm_t.hip gemm_x3); "fp32-mfma" uses v_mfma_f32_32x32x2_f32.  Both must meet the fp32 bar
    against the oracle, and the split path must be no less accurate than the exact-fp32 MFMA one."""
    _gpu()
    from tone_amd.model import ToneSession
    rng = np.random.default_rng(21)
    b = 32
    pcm = [synthetic_pcm(rng, b) for _ in range(3)]
    errs = {}
    for prec in ("fp32", "fp32-mfma"):
        s = ToneSession(weights, precision=prec, max_batch=b)
        st = np.zeros((b, C.STATE_SIZE), np.float16)
        worst = 0.0
        for c in range(3):
            lp_g, st_g = gpu_step(s, pcm[c], st)
            lp_o, st_o = oracle.step(pcm[c], st)
            assert_logp_close(lp_g, lp_o, what=f"{prec} chunk {c}")
            assert_state_close(st_g, st_o, what=f"{prec} chunk {c}")
            worst = max(worst, float(np.abs(lp_g - lp_o).max()))
            st = st_g
        s.close()
        errs[prec] = worst
    assert errs["fp32"] <= 2 * errs["fp32-mfma"] + 1e-5, errs


# bf16 bounds, measured (scripts/bf16_measure.py, profiles/r02_bf16_bounds.json): B = 2048, 10 stateful
# chunks, staggered starts, 64 sampled streams -- max |dlogp| 0.043-0.051 per chunk, p99 0.030-0.032,
# argmax 100 % identical.  Bounds: max 0.08, p99 0.05, argmax identical wherever the oracle's top-2 margin
# exceeds 0.1 and >= 99.5 % overall.
BF16_MAX, BF16_P99, BF16_MARGIN = 0.08, 0.05, 0.1


# fp8 (MXFP8 q/k/v + FFN GEMMs, BASELINE config 5) bounds, measured the same way (PREC=fp8
# scripts/bf16_measure.py, profiles/r02_fp8_bounds.json): max |dlogp| 0.36-0.43 per chunk, p99 0.27-0.30,
# argmax 99.8-100 % identical.  Bounds: max 0.6, p99 0.4, argmax identical where the margin exceeds 1.0
# and >= 99 % overall.
FP8_MAX, FP8_P99, FP8_MARGIN = 0.6, 0.4, 1.0


def assert_bf16_close(lp, ref, what="", bounds=(BF16_MAX, BF16_P99, BF16_MARGIN), agree=0.995):
    mx, p99, margin = bounds
    d = np.abs(lp - ref)
    assert d.max() < mx and np.percentile(d, 99) < p99, f"{what} max {d.max():.3g} p99 {np.percentile(d, 99):.3g}"
    srt = np.sort(ref, axis=-1)
    clear = (srt[..., -1] - srt[..., -2]) > margin
    np.testing.assert_array_equal(lp.argmax(-1)[clear], ref.argmax(-1)[clear], err_msg=f"{what} argmax")
    assert np.mean(lp.argmax(-1) == ref.argmax(-1)) >= agree, what


def test_bf16_mode_close_to_oracle(weights, oracle):
    """BASELINE config 3 arithmetic: bf16 MFMA operands, fp32 accumulate/norms/softmax (small batch)."""
    _gpu()
    from tone_amd.model import ToneSession
    s = ToneSession(weights, precision="bf16", max_batch=64)
    rng = np.random.default_rng(13)
    b = 32
    st = np.zeros((b, C.STATE_SIZE), np.float16)
    st_o = st.copy()
    for c in range(3):
        pcm = synthetic_pcm(rng, b)
        lp_g, st = gpu_step(s, pcm, st)
        lp_o, st_o = oracle.step(pcm, st_o)
        assert_bf16_close(lp_g, lp_o, f"chunk {c}")
    s.close()


@pytest.mark.parametrize("b", [3, 64])
def test_bf16_pre_encode_stage(weights, oracle, b):
    """bf16 front end + subsampling (sub_conv_bf16: conv1 + conv2 from one LDS slab, Linear, out_norm) vs the
    oracle's pre-encode output from a carried state: relative L2 error at bf16 level, and per frame the largest
    element error against that frame's largest value (a race or a wrong tile shows as O(1) there).  Measured on
    MI355X (scripts/probe_preencode.py, profiles/r05_probe_preencode.txt): relative L2 0.0042, worst frame 0.0062."""
    _gpu()
    from tone_amd.model import ToneSession
    s = ToneSession(weights, precision="bf16", max_batch=b)
    rng = np.random.default_rng(23)
    _, st0 = oracle.step(synthetic_pcm(rng, b, 0.0), None)
    pcm = synthetic_pcm(rng, b, 0.0)
    trace = []
    oracle.step(pcm, st0, trace=trace)
    try:
        s.debug_stop(1)
        gpu_step(s, pcm, st0)
        got = s.debug_read("rA", (b, 10, C.D_MODEL))
    finally:
        s.debug_stop(-1)
        s.close()
    ref = trace[1]
    rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    frame = float((np.abs(got - ref).max(-1) / np.abs(ref).max(-1)).max())
    assert rel < 1e-2 and frame < 2e-2, (rel, frame)


@pytest.mark.parametrize("prec,b,n", [("bf16", 512, 10), ("bf16", 2048, 10), ("bf16", 4096, 10), ("fp8", 4096, 10)])
def test_large_batch_staggered_streams(weights, oracle, prec, b, n):
    """The bench's own workloads with the oracle: config 4's per-GPU shard at N = 8 (bf16, B = 512),
    BASELINE config 3 (bf16, B = 2048) and the
    N = 1 legs of configs 4 / 5 (bf16 / fp8 at B = 4096, the batch bench.py times), 10 stateful 300 ms chunks,
    stream s starting (zero state) at chunk s % 4; 64 sampled streams stepped independently by the oracle
    (its own fp32 state chain, not the device state) and compared every chunk.  These batches route FFN up
    (and, from B = 1536, pw1) to the X-stationary kernels (gemm_xs in bf16, gemm_xs8 in fp8) and the other
    MXFP8 GEMMs to their 256-row X tiles, which the smaller tests do not reach at the same tile counts."""
    _gpu()
    from tone_amd.model import ToneSession
    pick = np.arange(0, b, b // 64)
    s = ToneSession(weights, precision=prec, max_batch=b)
    rng = np.random.default_rng(17)
    off = np.arange(b) % 4
    st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
    st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
    bounds = (BF16_MAX, BF16_P99, BF16_MARGIN) if prec == "bf16" else (FP8_MAX, FP8_P99, FP8_MARGIN)
    try:
        for c in range(n):
            pcm = synthetic_pcm(rng, b)
            st[torch.from_numpy(off == c).to(s.dev)] = 0
            st_o[off[pick] == c] = 0
            lp, st = s.step(torch.from_numpy(pcm).to(s.dev), st)
            lp_o, st_o = oracle.step(pcm[pick], st_o)
            live = off[pick] <= c
            assert_bf16_close(lp.cpu().numpy()[pick][live], lp_o[live], f"{prec} B={b} chunk {c}", bounds,
                              0.995 if prec == "bf16" else 0.99)
    finally:
        s.close()


def test_fp8_staggered_streams(weights, oracle):
    """BASELINE config 5 arithmetic (MXFP8 q/k/v + FFN GEMMs, everything else as bf16 mode): B = 512, 6
    stateful chunks with staggered starts, 32 sampled streams against the fp32 oracle's own state chain."""
    _gpu()
    from tone_amd.model import ToneSession
    b, n = 512, 6
    pick = np.arange(0, b, 16)
    s = ToneSession(weights, precision="fp8", max_batch=b)
    rng = np.random.default_rng(37)
    off = np.arange(b) % 4
    st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
    st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
    try:
        for c in range(n):
            pcm = synthetic_pcm(rng, b)
            st[torch.from_numpy(off == c).to(s.dev)] = 0
            st_o[off[pick] == c] = 0
            lp, st = s.step(torch.from_numpy(pcm).to(s.dev), st)
            lp_o, st_o = oracle.step(pcm[pick], st_o)
            live = off[pick] <= c
            assert_bf16_close(lp.cpu().numpy()[pick][live], lp_o[live], f"chunk {c}", (FP8_MAX, FP8_P99, FP8_MARGIN), 0.99)
    finally:
        s.close()


_FP8_PROBE = """
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[2]]
import tone_amd.config as C
from tone_amd.model import ToneSession
from tone_amd.weights import synthetic_weights
b = 64
s = ToneSession(synthetic_weights(0), precision="fp8", max_batch=b)
rng = np.random.default_rng(5)
st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
pcm = [np.clip(np.round(rng.normal(0, 3000, (b, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767).astype(np.int32)
       for _ in range(3)]
out = {}
lp = []
for c in range(3):
    if c == 2:   # chunk 2 (carried state): the first FFN1 operand, stopped right after the pre-encode norm, and
        m = b * 10   # layer 0's FFN2 operand, stopped right after pw2
        for tag, stop in (("norm", 1), ("pw2", 100)):
            s.debug_stop(stop)
            s.step(torch.from_numpy(pcm[c]).to(s.dev), st)
            out[tag + "_a8"] = s.debug_read("a8", (m, 384), np.uint8)
            out[tag + "_a8s"] = s.debug_read("a8s", (m, 12), np.uint8)
            out[tag + "_ss"] = s.debug_read("ss8", (m, 12)).sum(axis=1)
            out[tag + "_xb"] = s.debug_read("xbA", (m, 384), np.uint16)
        s.debug_stop(-1)
    l, st = s.step(torch.from_numpy(pcm[c]).to(s.dev), st)
    lp.append(l.cpu().numpy())
out["lp"] = np.stack(lp)
np.savez(sys.argv[1], **out)
"""


def mx_quant_ref(xb: np.ndarray):
    """quant_mx_kernel (gemm_mx.hip) restated on the host for a bf16 [M][384] operand (raw bits): per 32-column block
    E = clamp(biased exponent of max |v| - 7, 1, 254) (round 6: one binade of headroom, common.h mx_exp), values
    v * 2^(127 - E) (all below 256, so the +-448 clamp never acts) rounded to OCP e4m3 (round to nearest even, torch's
    float8_e4m3fn cast), and the row's sum of squares."""
    import torch
    m = xb.shape[0]
    v = (xb.astype(np.uint32) << 16).view(np.float32).reshape(m, 12, 32)
    amax = np.abs(v).max(axis=2)
    e = np.clip(((amax.view(np.uint32) >> 23) & 0xFF).astype(np.int64) - 7, 1, 254)
    inv = ((254 - e).astype(np.uint32) << 23).view(np.float32)
    y = np.clip(v * inv[..., None], np.float32(-448), np.float32(448)).astype(np.float32)
    q = torch.from_numpy(y.reshape(m, 384)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    ss = (v.astype(np.float64) ** 2).sum(axis=(1, 2))
    return q, e.astype(np.uint8), ss


def test_fp8_norm_quant_fusion_matches_quant_mx(tmp_path):
    """fp8 mode: the RMSNorm kernels that feed a layer's FFN1, FFN1's down-projection (before q|k|v) and pw2 (before
    FFN2) emit the next MX GEMM's MXFP8 operand themselves (TONE_FP8_NORMQ=1; the RESID epilogues of gemm_glds and
    gemm_mx).  That operand must equal what quant_mx makes from the bf16 shadow: e4m3 values and E8M0 scales bit
    for bit, the row's sum of squares (slab slots added) up to its summation order.
    * after the pre-encode norm (the step's first MXFP8 operand): fused run against the separate-launch run
      (TONE_FP8_NORMQ=0), bit for bit;
    * after layer 0's pw2: the fused run's operand against quant_mx restated on the host from the same run's shadow
      (the two runs no longer share that shadow: FFN1 down's fused operand feeds q|k|v a row factor summed in a
      different order, and its last bits move a few bf16 roundings downstream);
    * the logprobs of both runs (3 stateful chunks) stay within the fp8 bounds of each other."""
    _gpu()
    import os
    import subprocess
    import sys
    root = str(Path(__file__).resolve().parents[1])
    res = {}
    for flag in ("1", "0"):
        f = tmp_path / f"probe{flag}.npz"
        env = dict(os.environ, TONE_FP8_NORMQ=flag)
        subprocess.run([sys.executable, "-c", _FP8_PROBE, str(f), root], env=env, check=True, timeout=240)
        res[flag] = np.load(f)
    np.testing.assert_array_equal(res["1"]["norm_a8"], res["0"]["norm_a8"], err_msg="norm")
    np.testing.assert_array_equal(res["1"]["norm_a8s"], res["0"]["norm_a8s"], err_msg="norm")
    np.testing.assert_allclose(res["1"]["norm_ss"], res["0"]["norm_ss"], rtol=2e-6, err_msg="norm")
    for flag in ("1", "0"):   # each run's operand against the host quantization of its own shadow
        for tag in ("norm", "pw2"):
            q, e, ss = mx_quant_ref(res[flag][tag + "_xb"])
            np.testing.assert_array_equal(res[flag][tag + "_a8"], q, err_msg=f"{tag} NORMQ={flag}")
            np.testing.assert_array_equal(res[flag][tag + "_a8s"], e, err_msg=f"{tag} NORMQ={flag}")
            np.testing.assert_allclose(res[flag][tag + "_ss"], ss, rtol=2e-6, err_msg=f"{tag} NORMQ={flag}")
    assert_bf16_close(res["1"]["lp"], res["0"]["lp"], "fused vs separate", (FP8_MAX, FP8_P99, FP8_MARGIN), 0.99)


@pytest.mark.parametrize("prec,b", [("fp32", 300), ("bf16", 1000), ("fp8", 1000)])
def test_ragged_batches(weights, oracle, prec, b):
    """Batch sizes that are not multiples of any GEMM tile and cross the launchers' routing thresholds:
    partial last M-tiles (M = 10 B, 5 B in the reduced block, B (S + T) for the k|v projections of layers
    14 / 15), the fp32 ring kernel's M >= 4096 route, gemm_p / MX tiles at a non-multiple of 256.  Two
    stateful chunks; fp32 compares every stream at the 1e-3 bar, bf16 / fp8 sampled streams (always
    including the last one) at their measured bounds."""
    _gpu()
    from tone_amd.model import ToneSession
    s = ToneSession(weights, precision=prec, max_batch=b)
    rng = np.random.default_rng(41)
    pick = np.arange(b) if prec == "fp32" else np.unique(np.r_[np.arange(0, b, 50), b - 1])
    st = np.zeros((b, C.STATE_SIZE), np.float16)
    st_o = np.zeros((len(pick), C.STATE_SIZE), np.float16)
    try:
        for c in range(2):
            pcm = synthetic_pcm(rng, b)
            lp_g, st = gpu_step(s, pcm, st)
            if prec == "fp32":
                lp_o, st_ref = oracle.step(pcm, st_o)
                assert_logp_close(lp_g, lp_o, what=f"B={b} chunk {c}")
                assert_state_close(st, st_ref, what=f"B={b} chunk {c}")
                st_o = st.copy()            # next oracle step from the device state: per-step error
            else:
                lp_o, st_o = oracle.step(pcm[pick], st_o)
                bounds = (BF16_MAX, BF16_P99, BF16_MARGIN) if prec == "bf16" else (FP8_MAX, FP8_P99, FP8_MARGIN)
                # fp8, overall argmax agreement on these 21 x 10 frames: the first chunk (zero state) has many
                # near-tie frames -- measured 0.9905 (fp32 residual stream) and 0.981 (fp16, this tree) at B = 1000,
                # 0.9929 at B = 2048 for both, 1.0 on the second chunk (scripts/r04_ragged_probe.py,
                # profiles/r04_ragged_probe.txt); every flip is below the 1.0 margin, which stays strict
                # fp8: at most 4 flips of the 210 frames (the measured 0.981), all below the strict 1.0 margin
                agree = 0.995 if prec == "bf16" else 1.0 - 4.5 / lp_o[..., 0].size
                assert_bf16_close(lp_g[pick], lp_o, f"{prec} B={b} chunk {c}", bounds, agree)
    finally:
        s.close()


@pytest.mark.parametrize("prec", ["bf16", "fp8"])
def test_low_precision_example_audio_greedy_decode(weights, oracle, prec):
    """Greedy decode of the reference's example utterance in bf16 / fp8 mode against the oracle decode of the
    fp32 oracle's logprobs: every frame's greedy token wherever the oracle's top-2 margin exceeds the mode's
    bound (a frame at a token change can sit 0.09 nats from a tie -- chunk 20 frame 8 here -- well inside fp8's
    measured error), the same phrase texts, and phrase times within one 30 ms frame."""
    _gpu()
    import tone_decode_oracle as O
    from tone_amd.model import ToneSession
    audio = np.load(GOLDEN / "audio_short_pcm.npy").astype(np.int32)
    padded = np.pad(audio, (O.PADDING, O.PADDING))
    padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
    s = ToneSession(weights, precision=prec, max_batch=1)
    try:
        state, so, sg, sw, got, want = None, None, None, None, [], []
        for i, ch in enumerate(padded):
            lp, state = s.step(torch.from_numpy(ch[None]).to(s.dev), state)
            lp = lp.cpu().numpy()[0]
            lpo, so = oracle.step(ch[None], so)
            bounds = (BF16_MAX, BF16_P99, BF16_MARGIN) if prec == "bf16" else (FP8_MAX, FP8_P99, FP8_MARGIN)
            srt = np.sort(lpo[0], axis=-1)
            clear = (srt[:, -1] - srt[:, -2]) > bounds[2]
            np.testing.assert_array_equal(lp.argmax(-1)[clear], lpo[0].argmax(-1)[clear], err_msg=f"chunk {i}")
            assert np.abs(lp - lpo[0]).max() < bounds[0], f"chunk {i}"
            out, sg = O.pipeline_step(lp, sg, i == len(padded) - 1)
            got += out
            out, sw = O.pipeline_step(lpo[0], sw, i == len(padded) - 1)
            want += out
    finally:
        s.close()
    assert [p[0] for p in got] == [p[0] for p in want] and len(want) > 0
    np.testing.assert_allclose([p[1:] for p in got], [p[1:] for p in want], atol=0.03 + 1e-9)


@pytest.mark.gpu
def test_fp32_pre_encode_split_vs_mfma(weights, oracle):
    """fp32 front end + subsampling from a carried state, split mode (conv2 on the two-slab
    conv2_p3 kernel, 6 bf16 products per MAC) and exact-fp32-MFMA mode (implicit GEMM) vs the
    oracle's pre-encode output: both at fp32 level, the split no worse than 2x the fp32 MFMA."""
    _gpu()
    from tone_amd.model import ToneSession
    rng = np.random.default_rng(29)
    b = 5
    _, st0 = oracle.step(synthetic_pcm(rng, b, 0.0), None)
    pcm = synthetic_pcm(rng, b, 0.0)
    trace = []
    oracle.step(pcm, st0, trace=trace)
    ref = trace[1]
    rel = {}
    for prec in ("fp32", "fp32-mfma"):
        s = ToneSession(weights, precision=prec, max_batch=8)
        try:
            s.debug_stop(1)
            gpu_step(s, pcm, st0)
            got = s.debug_read("rA", (b, 10, C.D_MODEL))
        finally:
            s.debug_stop(-1)
            s.close()
        rel[prec] = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    print("pre-encode relative L2 error:", rel)
    assert rel["fp32"] < 1e-4, rel
    assert rel["fp32"] <= 2 * rel["fp32-mfma"] + 1e-6, rel


def test_hip_vs_forward_for_export(sess):
    """The HIP fp32 path on the golden streams (4 x 6 chunks, staggered restarts) against the reference's
    own Tone.forward_for_export (tests/golden/golden_fx.npz), argmax identical to both of its modes.
    * fp32 mode of the golden (fp16 states, features NOT rounded to fp16): the HIP path rounds the
      features to fp16 at the ONNX boundary (the export's fp16 `signal` path), and that rounding point alone
      moves the logprobs by 1.85e-3 -- the oracle with the same rounding differs from this golden by
      1.854e-3, the HIP path by 1.868e-3 (measured on the MI355X).  Bound 2.5e-3; the 1e-3 arithmetic bar
      is held against the oracle with identical rounding points (test_golden_stream, <= 1e-3).
    * fp16-autocast graph (golden_fx, LayerNorm unpatched): the stated 2.5e-2 delta (measured 1.58e-2)."""
    g, gs = np.load(GOLDEN / "golden_fx.npz"), np.load(GOLDEN / "golden_stream.npz")
    pcm = gs["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    st = np.zeros((B, C.STATE_SIZE), np.float16)
    d32 = d16 = 0.0
    for c in range(N):
        st[np.arange(B) > c] = 0
        lp, st = gpu_step(sess, pcm[:, c], st)
        r32, r16 = g["stream_fp32_logprobs"][:, c], g["stream_fp16_logprobs"][:, c]
        d32, d16 = max(d32, float(np.abs(lp - r32).max())), max(d16, float(np.abs(lp - r16).max()))
        np.testing.assert_array_equal(lp.argmax(-1), r32.argmax(-1))
        np.testing.assert_array_equal(lp.argmax(-1), r16.argmax(-1))
    print(f"HIP fp32 vs forward_for_export: fp32 {d32:.3g}, fp16-autocast {d16:.3g}")
    assert d32 < 2.5e-3 and d16 < 2.5e-2, (d32, d16)


def test_hip_vs_exported_fp16_graph(sess):
    """The HIP fp32 path against the EXPORTED graph's numerics (golden_fp16.npz: forward_for_export under the
    export's fp16 autocast and fp32 LayerNorm patch, what onnx_wrapper runs) on the golden streams and on the
    reference's example utterance chunk by chunk.  The floor for this comparison is measured, not chosen
    (tests/test_oracle.py::test_fp16_summation_order_floor): two fp16 implementations with identical rounding
    points but different summation orders differ by 1.56e-2 max / 3.1e-3 mean; the fp32 oracle sits at 1.9e-2 /
    3.6e-3 (streams) and 1.7e-2 / 3.6e-3 (audio).  Bounds: max 2.5e-2, mean 5e-3, argmax identical everywhere
    (the audio's smallest top-2 margin in the graph is 0.09)."""
    g, gs = np.load(GOLDEN / "golden_fp16.npz"), np.load(GOLDEN / "golden_stream.npz")
    pcm = gs["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    st = np.zeros((B, C.STATE_SIZE), np.float16)
    ds = []
    for c in range(N):
        st[np.arange(B) > c] = 0
        lp, st = gpu_step(sess, pcm[:, c], st)
        ref = g["stream_logprobs"][:, c]
        ds.append(np.abs(lp - ref))
        np.testing.assert_array_equal(lp.argmax(-1), ref.argmax(-1))
    audio = np.load(GOLDEN / "audio_short_pcm.npy").astype(np.int32)
    padded = np.pad(audio, (2400, 2400))
    padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
    st1 = np.zeros((1, C.STATE_SIZE), np.float16)
    for i, ch in enumerate(padded):
        lp, st1 = gpu_step(sess, ch[None], st1)
        ref = g["audio_logprobs"][i]
        ds.append(np.abs(lp[0] - ref))
        np.testing.assert_array_equal(lp[0].argmax(-1), ref.argmax(-1))
    d = np.concatenate([x.ravel() for x in ds])
    print(f"HIP fp32 vs exported fp16 graph: max {d.max():.3g}, mean {d.mean():.3g}")
    assert d.max() < 2.5e-2 and d.mean() < 5e-3, (d.max(), d.mean())


# bf16 / fp8 modes against the exported fp16 graph (golden_fp16.npz): both keep the residual stream in fp16 as that
# graph does.  Measured on the MI355X (profiles/r05_lowprec_bounds.log): bf16 max 0.051 / mean 0.0105 / 0 argmax
# flips of 480 frames, fp8 max 0.42 / mean 0.088 / 1 flip; bounds about 1.5x the measured max / mean.
FP16_GRAPH_BOUNDS = {"bf16": (0.08, 0.016), "fp8": (0.6, 0.13)}


@pytest.mark.parametrize("prec", ["bf16", "fp8"])
def test_lowprec_vs_exported_fp16_graph(weights, prec):
    """The bf16 / fp8 modes (fp16 residual stream, as the exported graph keeps it, tone/scripts/export.py:411) against
    the EXPORTED graph's numerics on the golden streams and the reference's example utterance, chunk by chunk: max and
    mean |dlogp| within the mode's bound, greedy argmax identical wherever the graph's top-2 margin exceeds the mode's
    argmax margin (BF16_MARGIN / FP8_MARGIN)."""
    _gpu()
    from tone_amd.model import ToneSession
    g, gs = np.load(GOLDEN / "golden_fp16.npz"), np.load(GOLDEN / "golden_stream.npz")
    margin = BF16_MARGIN if prec == "bf16" else FP8_MARGIN
    s = ToneSession(weights, precision=prec, max_batch=4)
    ds, flips, frames = [], 0, 0

    def check(lp, ref, what):
        nonlocal flips, frames
        ds.append(np.abs(lp - ref).ravel())
        srt = np.sort(ref, axis=-1)
        clear = (srt[..., -1] - srt[..., -2]) > margin
        np.testing.assert_array_equal(lp.argmax(-1)[clear], ref.argmax(-1)[clear], err_msg=what)
        flips += int((lp.argmax(-1) != ref.argmax(-1)).sum())
        frames += lp[..., 0].size

    try:
        pcm = gs["pcm"].astype(np.int32)
        B, N = pcm.shape[:2]
        st = np.zeros((B, C.STATE_SIZE), np.float16)
        for c in range(N):
            st[np.arange(B) > c] = 0
            lp, st = gpu_step(s, pcm[:, c], st)
            check(lp, g["stream_logprobs"][:, c], f"{prec} stream chunk {c}")
        audio = np.load(GOLDEN / "audio_short_pcm.npy").astype(np.int32)
        padded = np.pad(audio, (2400, 2400))
        padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
        st1 = np.zeros((1, C.STATE_SIZE), np.float16)
        for i, ch in enumerate(padded):
            lp, st1 = gpu_step(s, ch[None], st1)
            check(lp[0], g["audio_logprobs"][i], f"{prec} audio chunk {i}")
    finally:
        s.close()
    d = np.concatenate(ds)
    print(f"HIP {prec} vs exported fp16 graph: max {d.max():.3g}, mean {d.mean():.3g}, p99 {np.percentile(d, 99):.3g}, "
          f"argmax flips {flips}/{frames}")
    mx, mean = FP16_GRAPH_BOUNDS[prec]
    assert d.max() < mx and d.mean() < mean, (d.max(), d.mean())
    assert flips <= 0.005 * frames, (flips, frames)


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp8"])
def test_nan_propagates(weights, prec):
    """A NaN inside the step reaches the logprobs in every precision: one NaN in an FFN up-projection
    bias makes one column of the SwiGLU output NaN, which fp8 mode quantizes to MXFP8 inside the GEMM epilogue --
    that quantization must encode it as the e4m3 NaN, not clamp it to a finite -448."""
    _gpu()
    from tone_amd.model import ToneSession
    w = dict(weights)
    b = w["encoder.layers.3.feed_forward1.linear1.bias"].copy()
    b[5] = np.nan
    w["encoder.layers.3.feed_forward1.linear1.bias"] = b
    s = ToneSession(w, precision=prec, max_batch=4)
    try:
        lp, _ = gpu_step(s, synthetic_pcm(np.random.default_rng(2), 4, 0.0), np.zeros((4, C.STATE_SIZE), np.float16))
    finally:
        s.close()
    assert np.isnan(lp).all(), f"{prec}: {np.isnan(lp).mean():.3f} of the logprobs are NaN"


@pytest.mark.parametrize("prec,b,bound", [("bf16", 4096, 0.03), ("fp8", 4096, 0.15), ("bf16", 2048, 0.03)])
def test_lowprec_stagewise_large_batch(weights, oracle, prec, b, bound):
    """bf16 / fp8 at the bench's batches (the large-batch routes: gemm_xw / gemm_xs8, gemm_rp / gemm_rp_mx, dwconv,
    sub_conv, the recomputing attention), stage by stage against the oracle on 8 sampled streams from a carried state:
    per (stream, frame) row the largest element error over the row's largest value.  Measured on MI355X
    (scripts/probe_stagewise_lowprec.py, profiles/r05_probe_stagewise_lowprec.txt): bf16 <= 0.008 at every stage, fp8
    <= 0.058 (growing through the layers); the bounds are ~4x / ~2.5x that -- far tighter than the step tests'
    logprob bounds (fp8 max 0.6).  (The gemm_rp_mx race that test_gpu_kernels.py catches did not show on these
    sampled rows in the step: the build before its fix passes this test too, profiles/r05_stagewise_prev.log.)"""
    _gpu()
    import torch
    from tone_amd.model import ToneSession
    s = ToneSession(weights, precision=prec, max_batch=b)
    rng = np.random.default_rng(31)
    pick = np.sort(rng.choice(b, 8, replace=False))
    pcm0 = synthetic_pcm(rng, b, 0.0)
    pcm1 = synthetic_pcm(rng, b, 0.0)
    worst = []
    try:
        st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16, device=s.dev)
        _, st = s.step(torch.from_numpy(pcm0).to(s.dev), st)
        trace = []
        oracle.step(pcm1[pick], st.cpu().numpy()[pick], trace=trace)
        for stage, ref in enumerate(trace):
            if stage == 0:
                continue
            s.debug_stop(stage)
            s.step(torch.from_numpy(pcm1).to(s.dev), st.clone())
            layer = stage - 2
            reduced = C.REDUCTION_POS <= layer < C.UPSAMPLE_POS
            got = s.debug_read("rB" if reduced else "rA", (b, 5 if reduced else 10, C.D_MODEL))[pick]
            worst.append(float((np.abs(got - ref).max(-1) / np.abs(ref).max(-1)).max()))
    finally:
        s.debug_stop(-1)
        s.close()
    assert max(worst) < bound, " ".join(f"{i + 1}:{v:.3f}" for i, v in enumerate(worst))
