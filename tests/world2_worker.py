"""One rank of the world-2 sharded run (launched by tests/test_multi_gpu.py through torchrun; not a
test module itself).  Every rank drives a real ToneSession on the one GPU of the box, the checkpoint
comes from rank 0 by broadcast, the streams are split with shard_bounds, each rank steps its shard
for several stateful chunks, and the logprobs are all-gathered in stream order over gloo.  Rank 0
then checks the gathered batch against the single-process HIP batch and the CPU oracle and writes
the result as JSON to argv[1]."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import tone_amd.config as C  # noqa: E402
from tone_amd.model import ToneSession  # noqa: E402
from tone_amd.shard import broadcast_weights, gather_logprobs, shard_bounds  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402

N_STREAMS, N_CHUNKS = 7, 3


def main(out_path: str) -> None:
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    w = broadcast_weights(synthetic_weights(0) if rank == 0 else None)
    rng = np.random.default_rng(31)
    pcm = np.clip(np.round(rng.normal(0, 3000, (N_CHUNKS, N_STREAMS, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767)
    pcm = pcm.astype(np.int32)
    s, e = shard_bounds(N_STREAMS, world, rank)
    sess = ToneSession(w, device=0, precision="fp32", max_batch=N_STREAMS)
    st = torch.zeros((e - s, C.STATE_SIZE), dtype=torch.float16, device="cuda:0")
    gathered = []
    for c in range(N_CHUNKS):
        lp, st = sess.step(torch.from_numpy(pcm[c, s:e]).cuda(), st)
        gathered.append(gather_logprobs(lp.cpu(), N_STREAMS).numpy())
    if rank == 0:
        from tone_oracle import ToneOracle
        ref_sess = ToneSession(synthetic_weights(0), device=0, precision="fp32", max_batch=N_STREAMS)
        orc = ToneOracle(synthetic_weights(0))
        st1 = torch.zeros((N_STREAMS, C.STATE_SIZE), dtype=torch.float16, device="cuda:0")
        sto = None
        d_single = d_oracle = 0.0
        for c in range(N_CHUNKS):
            lp1, st1 = ref_sess.step(torch.from_numpy(pcm[c]).cuda(), st1)
            lpo, sto = orc.step(pcm[c], sto)
            d_single = max(d_single, float(np.abs(gathered[c] - lp1.cpu().numpy()).max()))
            d_oracle = max(d_oracle, float(np.abs(gathered[c] - lpo).max()))
        with open(out_path, "w") as fh:
            json.dump({"world": world, "shape": list(gathered[0].shape), "d_single": d_single,
                       "d_oracle": d_oracle}, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
