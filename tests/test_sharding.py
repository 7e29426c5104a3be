"""The N>1 path on CPU: world_size 2 over gloo, streams sharded in contiguous blocks, each rank
runs the step on its shard (the numpy oracle stands in for the GPU here), logprobs all-gathered in
stream order; the gathered batch equals the single-process batch."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tone_amd.shard import gather_logprobs, shard_bounds, shard_sizes


def test_shard_bounds_cover_and_balance():
    for n in (0, 1, 5, 512, 4096, 4097):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sz = shard_sizes(n, w)
            assert max(sz) - min(sz) <= 1
    assert shard_bounds(4096, 8, 3) == (1536, 2048)      # 512 streams per GPU (BASELINE config 4)
    with pytest.raises(ValueError):
        shard_bounds(4, 2, 2)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_streams, pcm, ref_logp, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [root, os.path.join(root, "oracle")]
        from tone_amd.weights import synthetic_weights
        from tone_oracle import ToneOracle

        s, e = shard_bounds(n_streams, world, rank)
        orc = ToneOracle(synthetic_weights(0))
        st = None
        for c in range(pcm.shape[0]):
            lp, st = orc.step(pcm[c, s:e], st)
        full = gather_logprobs(torch.from_numpy(lp), n_streams)
        err = float(np.abs(full.numpy() - ref_logp).max())
        result_q.put((rank, err, tuple(full.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_streams", [4, 5])
def test_gloo_world2_gather_matches_single_process(n_streams):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle")]
    from tone_amd.weights import synthetic_weights
    from tone_oracle import ToneOracle

    rng = np.random.default_rng(4)
    pcm = np.clip(rng.normal(0, 3000, (2, n_streams, 2400)), -32768, 32767).astype(np.int32)
    orc = ToneOracle(synthetic_weights(0))
    st = None
    for c in range(2):
        ref, st = orc.step(pcm[c], st)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_streams, pcm, ref, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, shape in res:
        assert shape == (n_streams, 10, 35)
        assert err < 1e-4, (rank, err)


def _bcast_worker(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tone_amd.shard import broadcast_weights
        from tone_amd.weights import synthetic_weights
        w = broadcast_weights(synthetic_weights(0) if rank == 0 else None)
        ref = synthetic_weights(0)
        ok = list(w) == list(ref) and all(np.array_equal(w[k], ref[k]) for k in ref)
        result_q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_weight_broadcast():
    """One checkpoint load on rank 0, broadcast once: every rank holds the identical replica."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res
