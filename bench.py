"""Throughput of the MI355X streaming acoustic path (BASELINE.json metric).

A step = one streaming step (PCM chunk + carried state -> logprobs + next state) for every
stream of the batch, inputs resident in HBM, states ping-ponged between two device slabs, the
whole step replayed as one hipGraph.  With --gpus N (one process per GPU, torchrun) every rank
runs its own shard of streams (weak scaling, no data-path collective) and the per-step logprobs
are all-gathered to every rank over RCCL (the host-decoding exchange).

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tone_amd.config as C  # noqa: E402
from tone_amd.model import ToneSession  # noqa: E402
from tone_amd.shard import gather_logprobs  # noqa: E402
from tone_amd.weights import synthetic_weights  # noqa: E402

METRIC = "real-time-factor & streams/sec/node, 300 ms chunk, batch=1..4096"
PEAK_TFLOPS = {"fp32": 157.3, "fp32-mfma": 157.3, "bf16": 2500.0}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
# "fp32" runs its GEMMs as exact 3-way bf16 splits: 6 bf16 MFMA products per fp32 multiply-add, so the
# matrix pipe's own ceiling for that arithmetic is the bf16 dense peak / 6
SPLIT_PIPE_PEAK = 2500.0 / 6
HBM_PEAK_GBS = 8000.0

# GEMM families and their algorithmic FLOP per step (per stream-chunk, x batch), for the roofline
GEMM_FAMILIES = ["gemm_ffn_up", "gemm_ffn_down", "gemm_qkv", "gemm_attn_out", "gemm_pw1", "gemm_pw2",
                 "gemm_sub_out", "gemm_reduce"]


def family_flops_per_stream() -> dict:
    d, ff = C.D_MODEL, C.D_FF
    frames = [C.layer_frames(l) for l in range(C.N_LAYERS)]
    f = {k: 0 for k in GEMM_FAMILIES}
    for l, t in enumerate(frames):
        f["gemm_ffn_up"] += 2 * (2 * t * d * 2 * ff)
        f["gemm_ffn_down"] += 2 * (2 * t * ff * d)
        s = C.mhsa_cache_rows(l)
        if l < C.MHSA_STATELESS:
            f["gemm_qkv"] += 2 * t * d * (3 * d if C.RECOMPUTE_SCORES[l] else d)
        else:
            f["gemm_qkv"] += 2 * t * d * d + 2 * (s + t) * d * 2 * d
        f["gemm_attn_out"] += 2 * t * d * d
        f["gemm_pw1"] += 2 * t * d * 2 * d
        f["gemm_pw2"] += 2 * t * d * d
    f["gemm_sub_out"] = 2 * 10 * C.SUB_OUT_IN * d
    f["gemm_reduce"] = 2 * 5 * 4 * d * d
    return f


def measured_traffic(family: str, precision: str, batch: int):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (scripts/pmc_traffic.sh + scripts/traffic_summary.py: FETCH_SIZE x2 + WRITE_SIZE, gfx950
    correction), or (None, None) when no summary exists for this precision / batch."""
    path = os.path.join(ROOT, "profiles", f"r01_traffic_{precision}_b{batch}.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    if t.get("kernel") != family:
        return None, None
    return int(t["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)


def algo_bytes(family: str, precision: str, batch: int) -> float:
    """Algorithmic HBM bytes per launch of a GEMM family: A read + W read + C write, averaged over the
    family's launches in one step (only the FFN up-projection is modelled)."""
    if family != "gemm_ffn_up":
        return 0.0
    e = 2 if precision == "bf16" else 4
    d, ff = C.D_MODEL, C.D_FF
    per = [e * (batch * C.layer_frames(l) * d + 2 * ff * d + batch * C.layer_frames(l) * ff)
           for l in range(C.N_LAYERS) for _ in range(2)]
    return sum(per) / len(per)


def synthetic_pcm(rng, b, n_chunks, silence=0.2):
    """Gaussian sigma=3000 clipped to int16, 20 % silent chunks."""
    x = np.clip(np.round(rng.normal(0.0, 3000.0, size=(n_chunks, b, C.AUDIO_CHUNK_SAMPLES))), -32768, 32767)
    x[rng.random((n_chunks, b)) < silence] = 0
    return x.astype(np.int32)


def cpu_baseline(budget_s: float, batch: int) -> dict:
    """The CPU oracle (numpy port of the reference step) on a bounded sample, this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from tone_oracle import ToneOracle
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = os.cpu_count() or 1
    orc = ToneOracle(synthetic_weights(0))
    rng = np.random.default_rng(1)
    pcm = synthetic_pcm(rng, batch, 4)
    st = None
    orc.step(pcm[0], st)  # warm-up
    t0 = time.perf_counter()
    n = 0
    while True:
        _, st = orc.step(pcm[n % 4], st)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = (time.perf_counter() - t0) / n
    return {"value": round(batch * C.AUDIO_CHUNK_SAMPLES / C.SAMPLE_RATE / dt, 2), "unit": "real-time streams",
            "chunks_per_s": round(batch / dt, 2), "ms_per_step": round(dt * 1e3, 2), "cores": int(threads),
            "kind": "port",
            "sample": f"numpy oracle (oracle/tone_oracle.py), batch {batch}, {n} stateful steps, fp32"}


def measure(args, B, precision, dev, local, world, rank, pg, with_roofline=True):
    """Time args.steps streaming steps of B streams per GPU; returns (elapsed_s, roofline dict | None)."""
    sess = ToneSession(synthetic_weights(0), device=local, precision=precision, max_batch=B,
                       graph=not args.no_graph)
    rng = np.random.default_rng(1000 + rank)
    pcm = torch.from_numpy(synthetic_pcm(rng, B, args.chunks)).to(dev)             # (chunks, B, 2400)
    slabs = [torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev) for _ in range(2)]
    signal = torch.empty((B, C.AUDIO_CHUNK_SAMPLES), dtype=torch.int32, device=dev)   # audio lands here
    logp = torch.empty((B, C.CHUNK_FRAMES, C.VOCAB), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)

    def step(i: int) -> None:
        signal.copy_(pcm[i % args.chunks], non_blocking=True)
        sess.run(signal, slabs[i % 2], logp, slabs[(i + 1) % 2], stream=stream)
        if pg is not None:   # host-decoding exchange: every rank's logprobs, in stream order
            gather_logprobs(logp, world * B)

    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for i in range(args.warmup, args.warmup + args.steps):
            step(i)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- roofline of the dominant kernel: per-kernel HIP events on the launch stream -----------
    roof = None
    if rank == 0 and with_roofline:
        sess.set_graph(False)
        sess.set_timing(True)
        with torch.cuda.stream(stream):
            for i in range(args.steps):
                signal.copy_(pcm[i % args.chunks], non_blocking=True)
                sess.run(signal, slabs[i % 2], logp, slabs[(i + 1) % 2], stream=stream)
        torch.cuda.synchronize()
        per_stream = family_flops_per_stream()
        fams = {}
        for fam in GEMM_FAMILIES:
            us, n = sess.kernel_us(fam)
            if n:
                fams[fam] = {"avg_us": us, "launches_per_step": n / args.steps,
                             "flop_per_launch": per_stream[fam] * B / (n / args.steps)}
        sess.set_timing(False)
        dom = max(fams, key=lambda k: fams[k]["avg_us"] * fams[k]["launches_per_step"])
        f = fams[dom]
        achieved = f["flop_per_launch"] / (f["avg_us"] * 1e-6) / 1e12
        peak = PEAK_TFLOPS[precision]
        traffic, tsrc = measured_traffic(dom, precision, B)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": tsrc, "algo_bytes": int(algo_bytes(dom, precision, B)),
                "avg_us": round(f["avg_us"], 2), "flop_per_launch": int(f["flop_per_launch"]),
                "step_tflops": round(C.FLOP_PER_CHUNK * B / (elapsed / args.steps) / 1e12, 2),
                "families_us_per_step": {k: round(v["avg_us"] * v["launches_per_step"], 1) for k, v in fams.items()}}
        if precision == "fp32":
            roof["gemm_arith"] = ("fp32 as exact 3-way bf16 splits, 6 products per multiply-add on "
                                  "v_mfma_f32_32x32x16_bf16 (fp32-accurate; tests/test_gpu_parity.py)")
            roof["pipe_peak"] = round(SPLIT_PIPE_PEAK, 1)
            roof["pipe_frac"] = round(achieved / SPLIT_PIPE_PEAK, 4)
    sess.close()
    del slabs, pcm
    torch.cuda.empty_cache()
    return elapsed, roof


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="streams per GPU (BASELINE config 2: 256)")
    ap.add_argument("--precision", choices=["fp32", "fp32-mfma", "bf16"], default="fp32")
    ap.add_argument("--chunks", type=int, default=10, help="distinct 300 ms chunks cycled per stream")
    ap.add_argument("--cpu-baseline-s", type=float, default=12.0, help="CPU oracle budget (0 = skip)")
    ap.add_argument("--cpu-baseline-batch", type=int, default=32)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--alt", type=int, default=1, help="also measure BASELINE config 3 (bf16, B=2048) at N=1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torchrun)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        pg = dist

    B = args.batch
    elapsed, roof = measure(args, B, args.precision, dev, local, world, rank, pg)
    ms_step = elapsed / args.steps * 1e3
    chunks_s = world * B / (elapsed / args.steps)
    streams = chunks_s * C.AUDIO_CHUNK_SAMPLES / C.SAMPLE_RATE

    # BASELINE config 3 (1 GPU, batch 2048, bf16 MFMA, stateful) reported beside the headline
    alt = None
    if world == 1 and args.alt:
        e2, r2 = measure(args, 2048, "bf16", dev, local, world, rank, pg)
        cs2 = 2048 / (e2 / args.steps)
        alt = {"workload": "BASELINE config 3: streaming step, batch 2048, bf16 MFMA GEMMs, stateful 300 ms chunks",
               "value": round(cs2 * C.AUDIO_CHUNK_SAMPLES / C.SAMPLE_RATE, 1), "unit": "real-time streams",
               "ms_per_step": round(e2 / args.steps * 1e3, 4), "chunks_per_s": round(cs2, 1),
               "rtf": round(e2 / args.steps * 1e3 / 300.0, 5), "dtype": "bf16", "roofline": r2}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_s > 0:
        cpu = cpu_baseline(args.cpu_baseline_s, args.cpu_baseline_batch)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(streams, 1),
            "unit": "real-time streams (300 ms chunks/s x 0.3 s)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (Gaussian sigma=3000 int16 PCM, 20% silent chunks; random-init T-one weights)",
            "config": {"workload": "BASELINE config 2: streaming step, batch 256/GPU, fp32, stateful 300 ms chunks"
                       if args.precision == "fp32" and B == 256 else
                       f"streaming step, batch {B}/GPU, {args.precision}, stateful 300 ms chunks",
                       "model": "T-one 71.7M (16-layer chunked Conformer, d384)",
                       "batch_per_gpu": B, "global_batch": world * B, "chunk_ms": 300,
                       "parallelism": f"dp{world}", "graph": not args.no_graph},
            "chunks_per_s": round(chunks_s, 1),
            "rtf": round(ms_step / 300.0, 5),
            "roofline": roof,
            "cpu_baseline": cpu,
            "alt_workloads": [alt] if alt else [],
        }
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()   # rank 0 finishes its roofline pass before any rank tears the communicator down
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
