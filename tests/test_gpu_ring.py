"""The resident state form (tone_session_run_ring, include/tonehip.h) against the flat form, on a real MI355X.

The resident form keeps each stream's conv-module caches in a time-major ring updated in place (only the T new frames
written per step) and the other sections in ping-pong slab rows; its arithmetic is the flat form's, so over several
stateful chunks the logprobs must be bit-identical to ``run`` on the flat state, and the exported state must equal the
flat state bit for bit (both directions of the conversion included).  Streams that sit out a step keep their row and
ring untouched; a stream re-imported mid-way (counter back to 0, phases reset) continues identically.
"""

import numpy as np
import pytest

import tone_amd.config as C
from tone_amd.weights import synthetic_weights

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(0)


def _pcm(rng, n, b, chunk):
    x = np.clip(np.round(rng.normal(0.0, 3000.0, size=(n, b, chunk))), -32768, 32767)
    x[rng.random((n, b)) < 0.2] = 0
    return x.astype(np.int32)


@pytest.mark.parametrize("precision,B,chunk,graph", [("bf16", 512, 2400, True), ("fp8", 512, 2400, True),
                                                      ("fp32", 64, 2400, False), ("fp32", 32, 3200, True),
                                                      ("fp32", 3, 2400, True), ("bf16", 2048, 2400, True)])
def test_ring_matches_flat(weights, precision, B, chunk, graph):
    _gpu()
    from tone_amd.model import ToneSession

    s = ToneSession(weights, device=0, precision=precision, max_batch=B, graph=graph, chunk_samples=chunk)
    dev = s.dev
    try:
        n_chunks = 12 if B <= 512 else 7            # > 30 / T steps: every ring phase is visited at T = 5 / 10
        pcm = torch.from_numpy(_pcm(np.random.default_rng(5), n_chunks, B, chunk)).to(dev)
        # flat reference: ping-pong over two (B, 219729) buffers
        st = [torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev) for _ in range(2)]
        lp_flat = []
        lp = torch.empty((B, s.frames, C.VOCAB), dtype=torch.float32, device=dev)
        half = n_chunks // 2
        for i in range(n_chunks):
            s.run(pcm[i], st[i % 2], lp, st[(i + 1) % 2])
            lp_flat.append(lp.clone())
            if i == half - 1:
                flat_mid = st[(i + 1) % 2].clone()
        flat_final = st[n_chunks % 2].clone()
        # resident form from the zero state: rows 2 p(b) / 2 p(b) + 1 of one slab, rings in a shuffled order
        perm = torch.from_numpy(np.random.default_rng(1).permutation(B).astype(np.int32)).to(dev)
        rows = [2 * perm, 2 * perm + 1]
        ring_ids = torch.from_numpy(np.random.default_rng(2).permutation(B + 3).astype(np.int32)[:B]).to(dev)
        slab = torch.full((2 * B, C.STATE_SIZE), float("nan"), dtype=torch.float16, device=dev)
        rings = torch.full((B + 3, s.ring_elems), float("nan"), dtype=torch.float16, device=dev)
        s.ring_import(torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev), slab, rows[0], rings, ring_ids)
        for i in range(n_chunks):
            if i == half:
                # export, compare with the flat state at this point, re-import (counter 0: the phases restart)
                mid = s.ring_export(slab, rows[i % 2], rings, ring_ids)
                torch.cuda.synchronize()
                assert torch.equal(mid.view(torch.int16), flat_mid.view(torch.int16)), "mid-way export"
                s.ring_import(mid, slab, rows[i % 2], rings, ring_ids)
            s.run_ring(pcm[i], rows[i % 2], rows[(i + 1) % 2], slab, rings, ring_ids, lp)
            torch.cuda.synchronize()
            assert torch.equal(lp, lp_flat[i]), f"chunk {i}: max |dlogp| {float((lp - lp_flat[i]).abs().max()):.3g}"
        out = s.ring_export(slab, rows[n_chunks % 2], rings, ring_ids)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16), flat_final.view(torch.int16)), \
            f"{int((out.view(torch.int16) != flat_final.view(torch.int16)).sum())} state elements differ"
    finally:
        s.close()


def test_ring_mid_export_matches_flat_state(weights):
    """The state exported after k steps equals the flat form's state after k steps, for every k (300 ms, bf16)."""
    _gpu()
    from tone_amd.model import ToneSession

    B, n = 96, 7
    s = ToneSession(weights, device=0, precision="bf16", max_batch=B)
    dev = s.dev
    try:
        pcm = torch.from_numpy(_pcm(np.random.default_rng(9), n, B, 2400)).to(dev)
        a = torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev)
        b = torch.empty_like(a)
        lp = torch.empty((B, s.frames, C.VOCAB), dtype=torch.float32, device=dev)
        idx = torch.arange(B, dtype=torch.int32, device=dev)
        rows = [idx, idx + B]
        slab = torch.zeros((2 * B, C.STATE_SIZE), dtype=torch.float16, device=dev)
        rings = torch.zeros((B, s.ring_elems), dtype=torch.float16, device=dev)
        s.ring_import(a, slab, rows[0], rings, idx)
        for i in range(n):
            s.run(pcm[i], a, lp, b)
            a, b = b, a
            s.run_ring(pcm[i], rows[i % 2], rows[(i + 1) % 2], slab, rings, idx, lp)
            got = s.ring_export(slab, rows[(i + 1) % 2], rings, idx)
            torch.cuda.synchronize()
            assert torch.equal(got.view(torch.int16), a.view(torch.int16)), f"step {i}"
    finally:
        s.close()


def test_ring_idle_streams_untouched(weights):
    """A step over a subset of streams leaves the other streams' rows and rings exactly as they were."""
    _gpu()
    from tone_amd.model import ToneSession

    B = 64
    s = ToneSession(weights, device=0, precision="bf16", max_batch=B)
    dev = s.dev
    try:
        idx = torch.arange(B, dtype=torch.int32, device=dev)
        slab = torch.zeros((2 * B, C.STATE_SIZE), dtype=torch.float16, device=dev)
        rings = torch.zeros((B, s.ring_elems), dtype=torch.float16, device=dev)
        rng = np.random.default_rng(3)
        init = torch.from_numpy((rng.standard_normal((B, C.STATE_SIZE)) * 0.5).astype(np.float16)).to(dev)
        init[:, C.STATE_SECTIONS["mhsa_len"][0]] = 10.0
        s.ring_import(init, slab, idx, rings, idx)
        torch.cuda.synchronize()
        slab0, rings0 = slab.clone(), rings.clone()
        act = torch.arange(0, B, 2, dtype=torch.int32, device=dev)          # the even streams step
        pcm = torch.from_numpy(_pcm(rng, 1, act.numel(), 2400)[0]).to(dev)
        lp = torch.empty((act.numel(), s.frames, C.VOCAB), dtype=torch.float32, device=dev)
        s.run_ring(pcm, act, act + B, slab, rings, act, lp)
        torch.cuda.synchronize()
        odd = torch.arange(1, B, 2, device=dev)
        assert torch.equal(slab[odd].view(torch.int16), slab0[odd].view(torch.int16))
        assert torch.equal(slab[odd + B].view(torch.int16), slab0[odd + B].view(torch.int16))
        assert torch.equal(rings[odd].view(torch.int16), rings0[odd].view(torch.int16))
        assert not torch.equal(rings[act.long()].view(torch.int16), rings0[act.long()].view(torch.int16))
    finally:
        s.close()
