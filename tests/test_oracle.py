"""The CPU oracle against the golden vectors made by the reference's own modules (CPU only)."""

from pathlib import Path

import numpy as np
import pytest

import tone_amd.config as C
from tone_amd.weights import PARAM_SHAPES, synthetic_weights
from tone_oracle import StreamState, ToneOracle

GOLDEN = Path(__file__).parent / "golden"


@pytest.fixture(scope="module")
def oracle():
    return ToneOracle(synthetic_weights(0))


def test_mel_matches_reference_features(oracle):
    """FilterbankFeatures.forward_streaming (feats.py:118-133) vectors: fp16 features agree to one
    fp16 ulp or 1e-4 absolute near log(mel) = 0 (the conv1d summation order differs), and almost
    all bit-exactly."""
    g = np.load(GOLDEN / "golden_mel.npz")
    pcm, ref = g["pcm"].astype(np.int32), g["feats"]              # ref: (B, chunks, 64, 30) fp16
    st = np.zeros((pcm.shape[0], C.PREPROC_STATE), np.float16)
    for c in range(pcm.shape[1]):
        feats, st = oracle.mel(pcm[:, c], st)
        r = ref[:, c].transpose(0, 2, 1).astype(np.float32)
        f = feats.astype(np.float32)
        ulp = np.abs(np.spacing(r.astype(np.float16)).astype(np.float32))
        assert np.all(np.abs(f - r) <= np.maximum(ulp, 1e-4))
        assert np.mean(f == r) > 0.99


def test_stream_matches_reference_step(oracle):
    """Tone.forward_for_export composed from the reference modules: 4 streams x 6 chunks with
    staggered restarts (mhsa_len 0..30 mixed in one batch).

    Bound 5e-4 (measured 3.7e-4 at chunk 3).  It is not arithmetic error -- one step from a shared
    state agrees to 1.3e-5 (test_oracle_step_matches_forward_for_export) -- but fp16 rounding-boundary
    flips: a feature or state value whose fp32 pre-image differs in the last bits can round to the
    neighbouring fp16 value (~0.2 % of state elements per step), and each flip moves later logprobs by
    ~1e-4.  Chunk 0 (zero state, only the feature rounding) is already 1.3e-4."""
    g = np.load(GOLDEN / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    idx = np.arange(0, C.STATE_SIZE, int(g["sample_stride"]))
    state = np.zeros((B, C.STATE_SIZE), np.float16)
    for c in range(N):
        state[np.arange(B) > c] = 0
        logp, state = oracle.step(pcm[:, c], state)
        ref = g["logprobs"][:, c]
        assert np.abs(logp - ref).max() < 5e-4
        np.testing.assert_array_equal(logp.argmax(-1), ref.argmax(-1))
        ds = np.abs(state[:, idx].astype(np.float32) - g["state_samples"][:, c].astype(np.float32))
        assert ds.max() <= 4e-3
    fs = g["final_state_stream0"].astype(np.float32)
    d = np.abs(state[0].astype(np.float32) - fs)
    assert d.max() <= 8e-3 and np.mean(d == 0) > 0.9


def test_state_layout_roundtrip():
    rng = np.random.default_rng(0)
    flat = rng.standard_normal((3, C.STATE_SIZE)).astype(np.float16)
    st = StreamState.unflatten(flat)
    assert st.mhsa.shape == (3, 2, 30, 384) and st.conv.shape == (3, 16, 384, 30)
    assert st.sub2.shape == (3, 32, 8, 44) and st.reduction.shape == (3, 384, 1)
    np.testing.assert_array_equal(st.flatten(), flat)
    assert sum(int(np.prod(s)) for _, s in C.STATE_SECTIONS.values()) == C.STATE_SIZE


def test_streams_are_independent(oracle):
    """No cross-stream arithmetic: a batch equals each stream run alone."""
    rng = np.random.default_rng(1)
    pcm = np.clip(rng.normal(0, 3000, (3, 2, 2400)), -32768, 32767).astype(np.int32)
    st = np.zeros((3, C.STATE_SIZE), np.float16)
    lp_b, st_b = oracle.step(pcm[:, 0], st)
    lp_b, st_b = oracle.step(pcm[:, 1], st_b)
    for s in range(3):
        lp, st1 = oracle.step(pcm[s:s + 1, 0], None)
        lp, st1 = oracle.step(pcm[s:s + 1, 1], st1)
        assert np.abs(lp - lp_b[s:s + 1]).max() < 1e-4
        assert np.abs(st1.astype(np.float32) - st_b[s:s + 1].astype(np.float32)).max() < 4e-3


def test_mhsa_len_progression(oracle):
    """EncoderState.next: mhsa_len = min(mhsa_len + 10, 30) (conformer_blocks.py:191)."""
    pcm = np.zeros((1, 2400), np.int32)
    st = None
    seen = []
    for _ in range(5):
        _, st = oracle.step(pcm, st)
        seen.append(float(st[0, C.OFF_MHSA_LEN]))
    assert seen == [10.0, 20.0, 30.0, 30.0, 30.0]


def test_layer14_cache_is_left_padded(oracle):
    """Layer 14 keeps 15 rows, stored left-padded with zeros to 30 (conformer_blocks.py:161-163)."""
    rng = np.random.default_rng(2)
    pcm = np.clip(rng.normal(0, 3000, (2, 2400)), -32768, 32767).astype(np.int32)
    _, st = oracle.step(pcm, None)
    s = StreamState.unflatten(st)
    assert np.all(s.mhsa[:, 0, :15] == 0)
    assert np.any(s.mhsa[:, 0, 15:] != 0)
    assert np.any(s.mhsa[:, 1] != 0)


def test_synthetic_weights_cover_reference_catalogue():
    w = synthetic_weights(0)
    assert list(w) == list(PARAM_SHAPES)
    for k, v in w.items():
        assert v.shape == PARAM_SHAPES[k] and v.dtype == np.float32 and np.isfinite(v).all()
    assert np.all(w["encoder.layers.3.conv.batch_norm.running_var"] > 0)
    # deterministic and seed dependent
    np.testing.assert_array_equal(w["decoder.decoder_layers.0.weight"], synthetic_weights(0)["decoder.decoder_layers.0.weight"])
    assert not np.array_equal(w["decoder.decoder_layers.0.weight"], synthetic_weights(1)["decoder.decoder_layers.0.weight"])


# ---- pinned to Tone.forward_for_export itself (tests/golden/make_golden_fx.py) --------------------
FX = GOLDEN / "golden_fx.npz"


def test_oracle_step_matches_forward_for_export():
    """One step from a carried state through the reference's own forward_for_export (fp32, no
    feature rounding): every encoder stage within 2e-5 abs (measured 6.7e-6 on values up to 5.7),
    logprobs within 5e-5 (measured 1.3e-5), next state within one fp16 ulp (or 8e-6) with >= 99.5 % of the
    sampled elements bit-identical (measured 99.8 %)."""
    g = np.load(FX)
    orc = ToneOracle(synthetic_weights(0), round_feats=False)
    trace = []
    lp, st = orc.step(g["step_pcm"].astype(np.int32), g["step_state_in"], trace=trace)
    for i, t in enumerate(trace[1:]):
        ref = g["step_stages_fp32"][:, i, : t.shape[1]]
        assert np.abs(t - ref).max() < 2e-5, f"stage {i}: {np.abs(t - ref).max():.3g}"
    assert np.abs(lp - g["step_logprobs_fp32"]).max() < 5e-5
    ss = int(g["state_sample"])
    got, ref = st[:, ::ss].astype(np.float32), g["step_state_out_fp32"].astype(np.float32)
    d = np.abs(got - ref)
    # one fp16 ulp, or 8e-6 absolute for small values whose fp32 pre-image carries cancellation error
    assert np.all(d <= np.maximum(np.abs(np.spacing(g["step_state_out_fp32"])).astype(np.float32), 8e-6))
    assert np.mean(d == 0) >= 0.995


def test_oracle_stream_matches_forward_for_export():
    """The 6-chunk staggered streams through forward_for_export (fp32): <= 3e-4 (measured 1.6e-4,
    fp16 state-rounding flips accumulating as above), argmax identical."""
    g, gs = np.load(FX), np.load(GOLDEN / "golden_stream.npz")
    pcm = gs["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    orc = ToneOracle(synthetic_weights(0), round_feats=False)
    st = np.zeros((B, C.STATE_SIZE), np.float16)
    for c in range(N):
        st[np.arange(B) > c] = 0
        lp, st = orc.step(pcm[:, c], st)
        ref = g["stream_fp32_logprobs"][:, c]
        assert np.abs(lp - ref).max() < 3e-4
        np.testing.assert_array_equal(lp.argmax(-1), ref.argmax(-1))


def test_fp16_graph_delta_is_stated(oracle):
    """forward_for_export under fp16 autocast with fp16 states (the ONNX export's semantics,
    tone/scripts/export.py:411) vs the fp32 arithmetic the oracle and the HIP path implement:
    measured 1.6e-2 max |dlogp| over the streams (1.7e-2 for one step), argmax identical.  So 1e-3
    against an fp16 ORT graph is below that graph's own rounding noise; the bar is held against the
    fp32 restatement instead, and this bound (2.5e-2) is the stated
    fp16-graph delta."""
    g, gs = np.load(FX), np.load(GOLDEN / "golden_stream.npz")
    pcm = gs["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    st = np.zeros((B, C.STATE_SIZE), np.float16)
    worst = 0.0
    for c in range(N):
        st[np.arange(B) > c] = 0
        lp, st = oracle.step(pcm[:, c], st)
        ref = g["stream_fp16_logprobs"][:, c]
        worst = max(worst, float(np.abs(lp - ref).max()))
        np.testing.assert_array_equal(lp.argmax(-1), ref.argmax(-1))
    assert 1e-3 < worst < 2.5e-2, worst


# ---- the 400 ms chunk variant, pinned to forward_for_export (tests/golden/make_golden_400ms.py) ----------
def test_oracle_400ms_step_matches_forward_for_export():
    """3200-sample chunk from a carried state: 40 mel frames, 13 frames, 6 in the reduced block, the
    upsampling pad frame live; every stage within 2e-5, logprobs within 5e-5, next state within one
    fp16 ulp (or 8e-6) with >= 99.5 % bit-identical (the bounds of the 300 ms pin above)."""
    g = np.load(GOLDEN / "golden_400ms.npz")
    orc = ToneOracle(synthetic_weights(0), round_feats=False)
    trace = []
    lp, st = orc.step(g["pcm"][:, 3].astype(np.int32), g["step_state_in"], trace=trace)
    assert lp.shape == (4, 13, 35)
    for i, t in enumerate(trace[1:]):
        ref = g["step_stages"][:, i, : t.shape[1]]
        assert t.shape[1] == (6 if 7 <= i <= 14 else 13), (i, t.shape)
        assert np.abs(t - ref).max() < 2e-5, f"stage {i}: {np.abs(t - ref).max():.3g}"
    assert np.abs(lp - g["step_logprobs"]).max() < 5e-5
    ss = int(g["state_sample"])
    got, ref = st[:, ::ss].astype(np.float32), g["step_state_out"].astype(np.float32)
    d = np.abs(got - ref)
    assert np.all(d <= np.maximum(np.abs(np.spacing(g["step_state_out"])).astype(np.float32), 8e-6))
    assert np.mean(d == 0) >= 0.995


def test_oracle_400ms_stream_matches_forward_for_export():
    """4 streams x 5 chunks of 400 ms with staggered restarts (mhsa_len 0 / 13 / 26 / 30 in one batch)."""
    g = np.load(GOLDEN / "golden_400ms.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    orc = ToneOracle(synthetic_weights(0), round_feats=False)
    st = np.zeros((B, C.STATE_SIZE), np.float16)
    for c in range(N):
        st[np.arange(B) > c] = 0
        lp, st = orc.step(pcm[:, c], st)
        ref = g["logprobs"][:, c]
        assert np.abs(lp - ref).max() < 3e-4, (c, np.abs(lp - ref).max())
        np.testing.assert_array_equal(lp.argmax(-1), ref.argmax(-1))


# ---- the exported graph's fp16 numerics (tests/golden/make_golden_fp16.py, oracle/tone_oracle_fp16.py) ----
def _h(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def test_fp16_rounding_semantics_match_torch_cpu():
    """The rounding points tone_oracle_fp16 restates, checked bit for bit against torch's own CPU fp16 kernels
    (the ones the export traced): fp16 addmm = fp32-accumulated product + fp16 bias rounded once; true
    division by a Python scalar; softmax with an fp32 sum; log_softmax with the exp-sum AND its log kept in
    fp16.  SiLU / GLU / BatchNorm are the fp32 formula rounded once (a handful of last-bit exp differences)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.normal(0, 3, (64, 384)).astype(np.float16))
    xf = x.float().numpy()
    w = torch.from_numpy(rng.normal(0, 0.05, (256, 384)).astype(np.float16))
    b = torch.from_numpy(rng.normal(0, 0.1, 256).astype(np.float16))
    np.testing.assert_array_equal(torch.addmm(b, x, w.T).float().numpy(),
                                  _h(xf @ w.float().numpy().T + b.float().numpy()))
    np.testing.assert_array_equal((x / np.sqrt(48.0)).float().numpy(), _h(xf / np.float32(np.sqrt(48.0))))
    m = xf.max(-1, keepdims=True)
    e = np.exp(xf - m)
    np.testing.assert_array_equal(torch.softmax(x, -1).float().numpy(), _h(e / e.sum(-1, keepdims=True)))
    lse = _h(np.log(_h(e.sum(-1, keepdims=True))))
    np.testing.assert_array_equal(torch.log_softmax(x, -1).float().numpy(), _h(xf - m - lse))
    silu = torch.nn.functional.silu(x).float().numpy()
    assert np.mean(silu != _h(xf / (np.float32(1) + np.exp(-xf)))) < 1e-3


@pytest.fixture(scope="module")
def fp16_runs():
    """The golden streams through the fp16 oracle with fp32 (numpy sgemm, torch's order) and fp64 accumulation."""
    from tone_oracle_fp16 import ToneOracleFP16
    g = np.load(GOLDEN / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    W = synthetic_weights(0)
    out = {}
    for acc in ("f32", "f64"):
        orc = ToneOracleFP16(W, acc)
        st = np.zeros((B, C.STATE_SIZE), np.float16)
        lps = []
        for c in range(N):
            st[np.arange(B) > c] = 0
            lp, st = orc.step(pcm[:, c], st)
            lps.append(lp)
        out[acc] = np.stack(lps, 1)
    return out


def test_fp16_oracle_matches_exported_graph(fp16_runs):
    """tone_oracle_fp16 against Tone.forward_for_export with the export's numerics (golden_fp16.npz): every
    logprob within two fp16 ulps of the graph's (|lp| < 16: 2 x 7.8e-3), mean 3.1e-3 measured, ~42 % of the
    logprobs bit-identical, argmax identical everywhere.  The oracle has the graph's rounding points; what it
    cannot have is the exporting machine's summation order inside each conv / GEMM (numpy's sgemm equals torch's
    addmm, its im2col convolutions do not equal oneDNN's), and an fp32 last-bit difference in front of an fp16
    rounding point lands on the neighbouring fp16 value -- see the floor test below."""
    ref = np.load(GOLDEN / "golden_fp16.npz")["stream_logprobs"]
    d = np.abs(fp16_runs["f32"] - ref)
    assert d.max() <= 2 * 7.8125e-3 and d.mean() < 5e-3, (d.max(), d.mean())
    assert np.mean(d == 0) > 0.3
    np.testing.assert_array_equal(fp16_runs["f32"].argmax(-1), ref.argmax(-1))


def test_fp16_summation_order_floor(fp16_runs):
    """The measured floor of "<= 1e-3 against the fp16 graph": two implementations with IDENTICAL rounding
    points that differ only in the summation order inside the contractions (fp32 vs fp64 accumulation) already
    disagree by 1.56e-2 max, 3.1e-3 mean (p99 1.2e-2) on these streams -- as far apart as either is from the
    torch trace.  The first divergence is the first rounding point: 0.09 % of the fp16 features (7 of 7680
    values in one step) round the other way, and every later fp16 rounding multiplies the flips (30 % of the
    pre-encode output differs by one ulp).  So no implementation short of a bitwise clone of the exporting
    machine's kernels -- ORT's MLAS kernels included -- can hold 1e-3 against the fp16 graph; the 1e-3 bar
    is held against the fp32 semantics (test_stream_matches_reference_step, GPU test_golden_stream_parity)."""
    d = np.abs(fp16_runs["f32"] - fp16_runs["f64"])
    assert 5e-3 < d.max() <= 2 * 7.8125e-3 and d.mean() > 1e-3, (d.max(), d.mean())
    np.testing.assert_array_equal(fp16_runs["f32"].argmax(-1), fp16_runs["f64"].argmax(-1))


def test_fp16_oracle_stages_track_the_graph():
    """One step from a carried state, stage by stage against the graph's own fp16 values (forward hooks):
    features >= 99.8 % bit-identical; the encoder stages drift by flips alone -- relative L2 error growing
    from 2.8e-4 (pre-encode) to 1.3e-3 (layer 13), max 8.8e-3 on values up to 5.8 (a few fp16 ulps), about
    one fp16 half-ulp of relative error per layer."""
    from tone_oracle_fp16 import ToneOracleFP16
    g = np.load(GOLDEN / "golden_fp16.npz")
    trace = []
    ToneOracleFP16(synthetic_weights(0)).step(g["step_pcm"].astype(np.int32), g["step_state_in"], trace=trace)
    feats = g["step_feats"].astype(np.float32).transpose(0, 2, 1)
    assert np.mean(trace[0] == feats) > 0.998
    ref = g["step_stages"].astype(np.float32)
    for i, t in enumerate(trace[1:]):
        r = ref[:, i, : t.shape[1]]
        rel = np.linalg.norm(t - r) / np.linalg.norm(r)
        assert rel < 2.5e-3 and np.abs(t - r).max() < 1.6e-2, f"stage {i}: rel {rel:.3g}"
