"""Decode side: device frame info, frame-based splitter + greedy decoder,
multi-stream slot pipeline.

CPU: the oracle restatement (oracle/tone_decode_oracle.py) against the reference splitter's own
outputs (tests/golden/golden_decode.npz, made by tests/golden/make_golden_decode.py), and the
product's frame-based splitter (tone_amd.pipeline) against the same fixture.
GPU: frame_info from the head kernel against argmax / threshold of the logprobs it wrote, and the
slot pipeline (idle streams, late joins) against per-stream sequential runs.
"""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

import tone_decode_oracle as O
from tone_amd import pipeline as P

GOLD = Path(__file__).parent / "golden" / "golden_decode.npz"


def _golden():
    g = np.load(GOLD)
    phrases = json.loads(bytes(g["phrases"]).decode())
    offs = np.concatenate([[0], np.cumsum(g["lengths"])])
    streams = [g["logprobs"][offs[i]:offs[i + 1]] for i in range(len(g["lengths"]))]
    return streams, phrases


def test_oracle_matches_reference_splitter_and_decoder():
    streams, want = _golden()
    got = []
    for si, lp in enumerate(streams):
        st, n = None, len(lp) // 10
        for c in range(n):
            out, st = O.splitter_step(lp[10 * c:10 * c + 10], st, c == n - 1)
            for plp, s, e in out:
                t0, t1 = O.phrase_times(s, e)
                got.append({"stream": si, "chunk": c, "text": O.greedy_text(plp), "start_frame": s, "end_frame": e,
                            "start_time": t0, "end_time": t1, "n_logprob_rows": len(plp)})
    assert len(want) >= 40
    assert got == want


def test_frame_splitter_matches_reference():
    """tone_amd.pipeline on (argmax, speech) frames == the reference splitter + greedy decoder on logprobs."""
    streams, want = _golden()
    got = []
    for si, lp in enumerate(streams):
        st, n = None, len(lp) // 10
        toks = np.argmax(lp, axis=-1).astype(np.int32)
        speech = np.exp(lp[:, -2:]).sum(axis=-1) <= 0.9
        info = toks | (speech.astype(np.int32) << 8)
        for c in range(n):
            t, sp = P.decode_frame_info(info[10 * c:10 * c + 10])
            found, st = P.split_frames(t, sp, st, is_last=c == n - 1)
            for ptok, s, e in found:
                t0, t1 = P.phrase_times(s, e)
                got.append({"stream": si, "chunk": c, "text": P.greedy_text(ptok), "start_frame": s, "end_frame": e,
                            "start_time": t0, "end_time": t1, "n_logprob_rows": len(ptok)})
    assert got == want


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_frame_splitter_random_vs_oracle(seed):
    """Random speech/silence masks (short silences, 19/20/21-frame edges, > 2000-frame speech)."""
    rng = np.random.default_rng(seed)
    n = 4200 + 10 * int(rng.integers(0, 50))
    speech = np.zeros(n, bool)
    t = 0
    while t < n:
        run = int(rng.choice([rng.integers(1, 25), rng.integers(2000, 2300)], p=[0.9, 0.1]))
        speech[t:t + run] = bool(rng.integers(2))
        t += run
    toks = rng.integers(0, 35, n).astype(np.int32)
    # logprobs consistent with (toks, speech) for the oracle: blank/space mass decides speech
    lp = np.full((n, 35), -30.0, np.float32)
    lp[np.arange(n), toks] = -0.01
    lp[:, 34] = np.where(speech, -30.0, -0.01)
    lp[~speech & (toks != 34), toks[~speech & (toks != 34)]] = -5.0
    speech = np.exp(lp[:, -2:]).sum(-1) <= np.float32(0.9)     # the head kernel's flag rule
    st_o, st_p = None, None
    for c in range(n // 10):
        last = c == n // 10 - 1
        o, st_o = O.splitter_step(lp[10 * c:10 * c + 10], st_o, last)
        p, st_p = P.split_frames(np.argmax(lp[10 * c:10 * c + 10], -1), speech[10 * c:10 * c + 10], st_p, is_last=last)
        assert [(s, e) for _, s, e in o] == [(s, e) for _, s, e in p]
        assert [O.greedy_text(a) for a, _, _ in o] == [P.greedy_text(a) for a, _, _ in p]
        assert st_o.offset == st_p.offset and len(st_o.past) == len(st_p.tokens)


def test_greedy_text_rules():
    assert P.greedy_text(np.array([34, 0, 0, 34, 0, 33, 33, 1, 34])) == "аа б"
    assert P.greedy_text(np.array([], np.int32)) == ""
    assert P.greedy_text(np.array([33, 33, 34])) == ""


# --------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def session():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from tone_amd.model import ToneSession
    from tone_amd.weights import synthetic_weights
    return ToneSession(synthetic_weights(0), device=0, precision="fp32", max_batch=8)


def _pcm(rng, b):
    x = np.clip(rng.normal(0, 3000, (b, 2400)), -32768, 32767).astype(np.int32)
    x[rng.random(b) < 0.2] = 0
    return x


@pytest.mark.gpu
def test_frame_info_matches_logprobs(session):
    import torch
    rng = np.random.default_rng(5)
    info = torch.full((8, 10), -1, dtype=torch.int32, device=session.dev)
    session.set_frame_info(info)
    try:
        state = None
        for _ in range(3):
            sig = torch.from_numpy(_pcm(rng, 8)).to(session.dev)
            logp, state = session.step(sig, state)
            lp = logp.cpu().numpy()
            got = info.cpu().numpy()
            assert np.array_equal(got & 0xFF, np.argmax(lp, -1))
            ssum = np.exp(lp[..., -2:]).sum(-1)
            flag = (got >> 8).astype(bool)
            mism = flag != (ssum <= np.float32(0.9))
            assert not np.any(mism & (np.abs(ssum - 0.9) > 1e-6))
    finally:
        session.set_frame_info(None)


@pytest.mark.gpu
def test_slot_pipeline_matches_sequential_streams(session):
    import torch
    rng = np.random.default_rng(11)
    pipe = P.StreamingGreedyPipeline(session, n_slots=4)
    try:
        sched = [["A", "B"], ["A", "B", "C"], ["A", "C"], ["A", "B", "C"], ["B"], ["A", "B", "C"]]
        audio = {k: [_pcm(rng, 1)[0] for _ in range(6)] for k in "ABC"}
        slot = {}
        used = {k: 0 for k in "ABC"}
        step_logp = []
        for names in sched:
            for k in names:
                if k not in slot:
                    slot[k] = pipe.open_stream()
            chunks = np.stack([audio[k][used[k]] for k in names])
            phrases = pipe.forward(chunks, [slot[k] for k in names])
            lp = pipe._logp[:len(names)].cpu().numpy()
            step_logp.append({k: lp[i] for i, k in enumerate(names)})
            for i, k in enumerate(names):
                used[k] += 1
            assert len(phrases) == len(names)
        # sequential per-stream reference on the same session (B = 1, device state chain)
        session.set_frame_info(None)
        for k in "ABC":
            state, j = None, 0
            for rec in step_logp:
                if k not in rec:
                    continue
                logp, state = session.step(torch.from_numpy(audio[k][j][None]).to(session.dev), state)
                np.testing.assert_allclose(rec[k], logp.cpu().numpy()[0], atol=1e-4, rtol=0)
                j += 1
    finally:
        session.set_frame_info(None)


def _example_audio():
    return np.load(Path(__file__).parent / "golden" / "audio_short_pcm.npy").astype(np.int32)


def _noise_audio():
    rng = np.random.default_rng(3)
    audio = np.clip(rng.normal(0, 2500, 8000 * 4), -32768, 32767).astype(np.int32)
    audio[8000:16000] = 0
    return audio


@pytest.mark.gpu
@pytest.mark.parametrize("make_audio", [_noise_audio, _example_audio], ids=["noise", "example_audio"])
def test_forward_offline_matches_oracle_decode(session, make_audio):
    """Offline decoding of one utterance (synthetic, and the reference's example audio_short.flac):
    phrases from device frame info == the oracle's splitter + greedy decoder run on the device
    logprobs of the same steps."""
    import torch
    audio = make_audio()
    pipe = P.StreamingGreedyPipeline(session, n_slots=2)
    got = pipe.forward_offline(audio)
    # replay: same chunks through session.step, oracle decode on the logprobs
    padded = np.pad(audio, (P.PADDING, P.PADDING))
    padded = np.pad(padded, (0, -len(padded) % 2400)).reshape(-1, 2400)
    session.set_frame_info(None)
    state, st, want = None, None, []
    for i, ch in enumerate(padded):
        logp, state = session.step(torch.from_numpy(ch[None]).to(session.dev), state)
        out, st = O.pipeline_step(logp.cpu().numpy()[0], st, i == len(padded) - 1)
        want += out
    assert [(p.text, p.start_time, p.end_time) for p in got] == want


# --------------------------------------------------------------------------- scheduler (CPU)
class _FakePipe:
    """Stands in for StreamingGreedyPipeline: records every batch the scheduler forms."""

    def __init__(self, max_batch):
        self.session = type("S", (), {"max_batch": max_batch})()
        self.batches, self.open, self._next = [], set(), 0

    def open_stream(self):
        self._next += 1
        self.open.add(self._next)
        return self._next

    def close_stream(self, slot):
        self.open.remove(slot)

    def forward(self, chunks, slots, is_last):
        assert len(slots) == len(set(slots)) <= self.session.max_batch
        self.batches.append((list(slots), [int(c[0]) for c in chunks], list(is_last)))
        return [[P.TextPhrase(f"{s}:{int(c[0])}", 0.0, 0.0)] for s, c in zip(slots, chunks)]


def test_scheduler_packs_oldest_first_one_chunk_per_stream():
    pipe = _FakePipe(max_batch=2)
    sch = P.StreamScheduler(pipe)
    ch = lambda v: np.full(2400, v, np.int32)   # noqa: E731
    sch.submit("a", ch(1))
    sch.submit("a", ch(2))
    sch.submit("b", ch(10))
    sch.submit("c", ch(20), is_last=True)
    sch.submit("a", ch(3), is_last=True)
    with pytest.raises(ValueError):
        sch.submit("c", ch(21))                   # after its last chunk
    out1 = sch.step()                             # oldest waiting: a(1), b(10)
    assert sorted(out1) == ["a", "b"] and pipe.batches[-1][1] == [1, 10]
    out2 = sch.step()                             # a(2) (seq 1) before c(20) (seq 3)
    assert pipe.batches[-1][1] == [2, 20] and pipe.batches[-1][2] == [False, True]
    assert "c" in out2 and sch.active_streams == 2   # c closed after its last chunk
    out3 = sch.step()
    assert pipe.batches[-1][1] == [3] and list(out3) == ["a"]
    assert sch.step() == {} and sch.pending == 0 and sch.active_streams == 1   # b stays open, idle
    with pytest.raises(ValueError):
        sch.submit("b", np.zeros(2399, np.int32))


# --------------------------------------------------------------------------- slots vs oracle (GPU)
@pytest.fixture(scope="module")
def oracle():
    from tone_oracle import ToneOracle
    from tone_amd.weights import synthetic_weights
    return ToneOracle(synthetic_weights(0))


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [True, False])
def test_ping_pong_rows_vs_oracle(session, oracle, resident):
    """Streams that join late and sit idle for several steps (their rows untouched, no state copy):
    every stepping stream's logprobs vs the oracle stepped from that stream's device state, <= 1e-3;
    idle streams' states bit-identical across the steps they skip.  Both state forms: resident (conv caches in
    rings, run_ring; state_of exports) and flat ping-pong rows (run_rows)."""
    import torch
    rng = np.random.default_rng(19)
    pipe = P.StreamingGreedyPipeline(session, n_slots=6, resident=resident)
    try:
        sched = [["A"], ["A", "B"], ["B", "C", "D"], ["A", "D"], ["A", "B", "C", "D"], ["C"], ["A", "B", "C", "D"]]
        slot = {}
        for names in sched:
            for k in names:
                if k not in slot:
                    slot[k] = pipe.open_stream()
            idle = {k: pipe.state_of(s).clone() for k, s in slot.items() if k not in names}
            before = np.stack([pipe.state_of(slot[k]).cpu().numpy() for k in names])
            chunks = _pcm(rng, len(names))
            pipe.forward(chunks, [slot[k] for k in names])
            lp = pipe._logp[:len(names)].cpu().numpy()
            lp_o, st_o = oracle.step(chunks, before)
            assert np.abs(lp - lp_o).max() < 1e-3, np.abs(lp - lp_o).max()
            after = np.stack([pipe.state_of(slot[k]).cpu().numpy() for k in names]).astype(np.float32)
            assert np.mean(np.abs(after - st_o.astype(np.float32)) <= 2 * np.abs(np.spacing(st_o)).astype(np.float32)) > 0.995
            for k, t in idle.items():
                assert torch.equal(pipe.state_of(slot[k]), t), f"idle stream {k} state changed"
    finally:
        session.set_frame_info(None)


@pytest.mark.gpu
def test_scheduler_matches_single_stream_decode(session):
    """Uneven arrivals through StreamScheduler (max_batch 3 < 5 streams, streams start and end at
    different steps) give each stream the same phrases as decoding it alone."""
    rng = np.random.default_rng(23)
    audio = {}
    for k in range(5):
        a = np.clip(rng.normal(0, 2500, 2400 * int(rng.integers(3, 9))), -32768, 32767).astype(np.int32)
        a[2400:2400 * 2] = 0
        audio[k] = a.reshape(-1, 2400)
    pipe = P.StreamingGreedyPipeline(session, n_slots=8)
    sch = P.StreamScheduler(pipe, max_batch=3)
    try:
        pos = {k: 0 for k in audio}
        got = {k: [] for k in audio}
        t = 0
        while any(pos[k] < len(audio[k]) for k in audio):
            for k in audio:       # stream k delivers a chunk every (k % 2 + 1) ticks, starting at tick k
                if t >= k and (t - k) % (k % 2 + 1) == 0 and pos[k] < len(audio[k]):
                    sch.submit(k, audio[k][pos[k]], is_last=pos[k] == len(audio[k]) - 1)
                    pos[k] += 1
            for k, ph in sch.step().items():
                got[k] += ph
            t += 1
        for k, ph in sch.drain().items():
            got[k] += ph
        assert sch.active_streams == 0
        for k in audio:
            want = []
            s = pipe.open_stream()
            for i, ch in enumerate(audio[k]):
                want += pipe.forward(ch[None], [s], [i == len(audio[k]) - 1])[0]
            pipe.close_stream(s)
            assert [(p.text, p.start_time, p.end_time) for p in got[k]] == \
                   [(p.text, p.start_time, p.end_time) for p in want]
    finally:
        session.set_frame_info(None)


# --------------------------------------------------------------------------- host decoder wiring
def test_frames_to_phrases_with_host_decoder_matches_greedy():
    """The logprob-row payload path (for a host beam decoder such as the reference's KenLM
    BeamSearchCTCDecoder) cuts the same phrases as the token path, and with the greedy host decoder
    gives the same texts."""
    rng = np.random.default_rng(5)
    logp = np.log(rng.dirichlet(np.ones(35) * 0.3, size=(9, 10))).astype(np.float32)
    speech = rng.random((9, 10)) < 0.6
    speech[3:6] = False
    dec = P.GreedyLogprobDecoder()
    st_t, st_l, got_t, got_l = None, P.FrameSplitterState(tokens=np.zeros((0, 35), np.float32)), [], []
    for c in range(9):
        a, st_t = P.frames_to_phrases(logp[c].argmax(-1).astype(np.int32), speech[c], st_t, is_last=c == 8)
        b, st_l = P.frames_to_phrases(logp[c], speech[c], st_l, is_last=c == 8, decode=dec.forward)
        got_t += a
        got_l += b
    assert got_t == got_l and len(got_t) >= 2
    with pytest.raises(ValueError):
        dec.forward(np.zeros((3, 34), np.float32))


@pytest.mark.gpu
def test_host_decoder_pipeline_matches_device_greedy(session):
    """StreamingGreedyPipeline with a host decoder (logprobs to the host, phrase rows to
    decoder.forward -- the KenLM wiring) == the device greedy path on the same audio."""
    audio = _noise_audio()
    try:
        want = P.StreamingGreedyPipeline(session, n_slots=1).forward_offline(audio)
        got = P.StreamingGreedyPipeline(session, n_slots=1, decoder=P.GreedyLogprobDecoder()).forward_offline(audio)
    finally:
        session.set_frame_info(None)
    assert [(p.text, p.start_time, p.end_time) for p in got] == [(p.text, p.start_time, p.end_time) for p in want]
