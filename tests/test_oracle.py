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
    staggered restarts (mhsa_len 0..30 mixed in one batch)."""
    g = np.load(GOLDEN / "golden_stream.npz")
    pcm = g["pcm"].astype(np.int32)
    B, N = pcm.shape[:2]
    idx = np.arange(0, C.STATE_SIZE, int(g["sample_stride"]))
    state = np.zeros((B, C.STATE_SIZE), np.float16)
    for c in range(N):
        state[np.arange(B) > c] = 0
        logp, state = oracle.step(pcm[:, c], state)
        ref = g["logprobs"][:, c]
        assert np.abs(logp - ref).max() < 1e-3
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
