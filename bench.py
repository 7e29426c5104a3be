"""Throughput of the MI355X streaming acoustic path (BASELINE.json metric).

A step = one streaming step (PCM chunk + carried state -> logprobs + next state) for every
stream of the batch, inputs resident in HBM, the state in the resident form a server keeps
(conv caches in per-stream rings updated in place, the other sections ping-ponged between two
slab rows; ``--state flat``: the boundary's (B, 219729) state ping-ponged between two buffers;
bit-identical results), the whole step replayed as one hipGraph.  With --gpus N (one process per GPU, torchrun) every rank
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
from tone_amd.weights import synthetic_weights  # noqa: E402

METRIC = "real-time-factor & streams/sec/node, 300 ms chunk, batch=1..4096"
PEAK_TFLOPS = {"fp32": 157.3, "fp32-mfma": 157.3, "bf16": 2500.0, "fp8": 5000.0}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
# "fp32" runs its GEMMs as exact 3-way bf16 splits: 6 bf16 MFMA products per fp32 multiply-add, so the
# matrix pipe's own ceiling for that arithmetic is the bf16 dense peak / 6
SPLIT_PIPE_PEAK = 2500.0 / 6
HBM_PEAK_GBS = 8000.0

# GEMM families and their algorithmic FLOP per step (per stream-chunk, x batch), for the roofline
GEMM_FAMILIES = ["gemm_ffn_up", "gemm_ffn_down", "gemm_qkv", "gemm_attn_out", "gemm_pw1", "gemm_pw2",
                 "gemm_sub_out", "gemm_reduce"]


def family_flops_per_stream(T: int = C.CHUNK_FRAMES) -> dict:
    """Algorithmic FLOP per stream-chunk of each GEMM family; T = 10 (300 ms) or 13 (400 ms) frames,
    Tr = (T + 1 - 3) // 2 + 1 inside the reduced block (layers 7..14)."""
    d, ff = C.D_MODEL, C.D_FF
    tr = (T + 1 - 3) // 2 + 1
    frames = [tr if C.REDUCTION_POS < l <= C.UPSAMPLE_POS else T for l in range(C.N_LAYERS)]
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
    f["gemm_sub_out"] = 2 * T * C.SUB_OUT_IN * d
    f["gemm_reduce"] = 2 * tr * 4 * d * d
    return f


def family_bytes_per_stream(T: int = C.CHUNK_FRAMES, precision: str = "fp32") -> dict:
    """Algorithmic HBM bytes per stream-chunk of each GEMM family as the session runs it: A read + W read
    (amortised over the batch: added by the caller) + C write, + the residual read/write and the bf16
    shadow for RESID outputs.  Element sizes follow the precision: fp32 mode reads fp32 activations and an fp32
    residual stream; bf16 mode bf16 activation shadows, bf16 FFN hidden and q/k/v, and the residual stream in fp16
    (read + written: 4 B per element, plus the 2 B shadow); fp8 mode as bf16 with e4m3 (+1/32 scale) for the FFN
    and q/k/v operands, and the RESID epilogues that feed an MX GEMM (FFN1 down of layers 0-13, pw2) also write the
    shadow's MXFP8 form and its sum-of-squares slab (12 floats per row)."""
    d, ff = C.D_MODEL, C.D_FF
    tr = (T + 1 - 3) // 2 + 1
    lp = precision in ("bf16", "fp8")
    f8 = precision == "fp8"
    ea = 2 if lp else 4                                   # activation operand
    e8 = 1 + 1 / 32 if f8 else ea                         # MX operand (FFN, q/k/v in fp8 mode)
    eh = 1 + 1 / 32 if f8 else ea                         # FFN hidden h
    sh = 2 if lp else 0                                   # bf16 shadow of a residual output
    er = 2 if lp else 4                                   # residual stream element (fp16 / fp32)
    q8 = (1 + 1 / 32 + 4 * 12 / d) if f8 else 0.0         # MXFP8 shadow + sum-of-squares slab, per element
    f = {k: 0.0 for k in GEMM_FAMILIES}
    for l in range(C.N_LAYERS):
        t = tr if C.REDUCTION_POS < l <= C.UPSAMPLE_POS else T
        s = C.mhsa_cache_rows(l)
        f["gemm_ffn_up"] += 2 * t * (d * e8 + ff * eh)
        f["gemm_ffn_down"] += 2 * t * (ff * eh + d * (2 * er + sh)) + (t * d * q8 if l < C.MHSA_STATELESS else 0)
        if l < C.MHSA_STATELESS:
            f["gemm_qkv"] += t * d * (e8 + (3 if C.RECOMPUTE_SCORES[l] else 1) * ea)
        else:
            f["gemm_qkv"] += t * d * (e8 + ea) + (s + t) * d * (e8 + 2 * ea)
        f["gemm_attn_out"] += t * d * (ea + 2 * er + sh)
        f["gemm_pw1"] += t * d * (ea + 4)
        f["gemm_pw2"] += t * d * (ea + 2 * er + sh + q8)
    f["gemm_sub_out"] = T * (C.SUB_OUT_IN * ea + d * er)
    f["gemm_reduce"] = tr * (4 * d * ea + d * (er + sh))
    return f


def family_weight_bytes(precision: str = "fp32") -> dict:
    """Weight bytes each GEMM family reads per step (every launch reads its W once)."""
    d, ff = C.D_MODEL, C.D_FF
    ew = 2 if precision in ("bf16", "fp8") else 4
    e8 = 1 + 1 / 32 if precision == "fp8" else ew
    nl = C.N_LAYERS
    qkv = sum((3 * d * d if C.RECOMPUTE_SCORES[l] else d * d) if l < C.MHSA_STATELESS else 3 * d * d for l in range(nl))
    return {"gemm_ffn_up": nl * 2 * 2 * ff * d * e8, "gemm_ffn_down": nl * 2 * ff * d * e8, "gemm_qkv": qkv * e8,
            "gemm_attn_out": nl * d * d * ew, "gemm_pw1": nl * 2 * d * d * ew, "gemm_pw2": nl * d * d * ew,
            "gemm_sub_out": C.SUB_OUT_IN * d * ew, "gemm_reduce": 4 * d * d * ew}


# launches per 300 ms step of each family (session.hip enqueue_step): two FFNs per layer, q/k/v as one launch
# in layers 0..13 and two (q; k|v) in 14/15
FAMILY_LAUNCHES = {"gemm_ffn_up": 2 * C.N_LAYERS, "gemm_ffn_down": 2 * C.N_LAYERS,
                   "gemm_qkv": C.MHSA_STATELESS + 2 * (C.N_LAYERS - C.MHSA_STATELESS),
                   "gemm_attn_out": C.N_LAYERS, "gemm_pw1": C.N_LAYERS, "gemm_pw2": C.N_LAYERS,
                   "gemm_sub_out": 1, "gemm_reduce": 1}
# the residual-output (EPI_RESID) GEMMs: one kernel family in the traffic summary, the HBM-bound one
RESID_FAMILIES = ("gemm_ffn_down", "gemm_attn_out", "gemm_pw2")


def measured_traffic(family: str, precision: str, batch: int):
    """HBM bytes per launch of a GEMM family ("gemm_ffn_up", or "resid" = every EPI_RESID launch) from the
    committed rocprofv3 PMC summary (scripts/pmc_traffic.sh + scripts/traffic_summary.py: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950 correction), or (None, None) when no summary covers this precision / batch / family."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):   # the newest round's summary first
        path = os.path.join(ROOT, "profiles", f"{rnd}_traffic_{precision}_b{batch}.json")
        try:
            with open(path) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        fam = t.get("families", {}).get(family)
        if fam is None and t.get("kernel") == family:
            fam = t
        if fam is None:
            continue
        return int(fam["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def algo_bytes(family: str, precision: str, batch: int, T: int = C.CHUNK_FRAMES) -> float:
    """Algorithmic HBM bytes per launch of a GEMM family, averaged over the family's launches in one step:
    activations in and out at the precision's element sizes (family_bytes_per_stream: fp8 operands at
    1 + 1/32 B per element, bf16 at 2, fp32 at 4; residual in/out fp32 + bf16 shadow for RESID outputs) x
    batch, plus the weights every launch reads once.  family "resid" = the three EPI_RESID families together
    (FFN down, attn-out, pw2), the unit the PMC summary measures."""
    pb, wb = family_bytes_per_stream(T, precision), family_weight_bytes(precision)
    fams = RESID_FAMILIES if family == "resid" else (family,)
    tot = sum(pb[f] * batch + wb[f] for f in fams)
    return tot / sum(FAMILY_LAUNCHES[f] for f in fams)


def synthetic_pcm(rng, b, n_chunks, silence=0.2, chunk=C.AUDIO_CHUNK_SAMPLES):
    """Gaussian sigma=3000 clipped to int16, 20 % silent chunks."""
    x = np.clip(np.round(rng.normal(0.0, 3000.0, size=(n_chunks, b, chunk))), -32768, 32767)
    x[rng.random((n_chunks, b)) < silence] = 0
    return x.astype(np.int32)


def cpu_baseline(budget_s: float) -> dict:
    """BASELINE.md 4 / SURVEY.md 8d CPU side-by-side: the step restated with batched torch CPU kernels
    (oracle/tone_cpu.py: oneDNN/MKL GEMMs and convolutions, BatchNorm folded, fp32 with the reference's
    fp16 rounding points) timed on this host's cores at B = 1 and B = 256, ``budget_s`` of stateful
    steps each (after one warm-up step); median and p99 per step."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from tone_cpu import ToneCPU
    cores = torch.get_num_threads()
    cpu = ToneCPU(synthetic_weights(0))
    out = {}
    for b in (1, 256):
        pcm = torch.from_numpy(synthetic_pcm(np.random.default_rng(1), b, 4))
        st = torch.zeros((b, C.STATE_SIZE), dtype=torch.float16)
        _, st = cpu.step(pcm[0], st)       # warm-up
        ts = []
        t_end = time.perf_counter() + budget_s
        while time.perf_counter() < t_end or len(ts) < 3:
            t0 = time.perf_counter()
            _, st = cpu.step(pcm[len(ts) % 4], st)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        out[f"b{b}"] = {"value": round(b * C.AUDIO_CHUNK_SAMPLES / C.SAMPLE_RATE / med, 2), "median_ms": round(med * 1e3, 2),
                        "p99_ms": round(float(np.percentile(ts, 99)) * 1e3, 2), "steps": len(ts)}
    return {"value": out["b256"]["value"], "unit": "real-time streams", "cores": int(cores), "kind": "port",
            "batch": 256, "per_batch": out,
            "sample": f"torch-CPU restatement (oracle/tone_cpu.py), fp32, stateful synthetic chunks, about {budget_s:g} s "
                      f"of steps at each of B = 1 and B = 256 on {cores} threads; value = B = 256 median"}


_WEIGHTS = None


def replica_weights(pg, dev):
    """The checkpoint on this rank: built once on rank 0 and broadcast to the others (RCCL)."""
    global _WEIGHTS
    if _WEIGHTS is None:
        if pg is None:
            _WEIGHTS = synthetic_weights(0)
        else:
            from tone_amd.shard import broadcast_weights
            _WEIGHTS = broadcast_weights(synthetic_weights(0) if pg.get_rank() == 0 else None,
                                         device=dev if pg.get_backend() == "nccl" else None)
    return _WEIGHTS


def measure(args, B, precision, dev, local, world, rank, pg, with_roofline=True, cap=None, chunk=C.AUDIO_CHUNK_SAMPLES):
    """Time args.steps streaming steps of B streams on this GPU; returns a dict with the max-over-ranks
    elapsed time, per-step percentiles (HIP events on the launch stream) and the roofline (rank 0).

    With pg (N > 1) each step's logprobs are all-gathered to every rank (the host-decoding exchange,
    SURVEY.md 8e) on a separate stream, overlapped with the next step: logprobs are double-buffered and
    step i + 2 waits only for the gather that read its buffer.  ``cap`` (largest shard) pads unequal
    shards so the collective has equal parts."""
    cap = cap or B
    sess = ToneSession(replica_weights(pg, dev), device=local, precision=precision, max_batch=B,
                       graph=not args.no_graph, chunk_samples=chunk)
    fr = sess.frames
    rng = np.random.default_rng(1000 + rank)
    pcm = torch.from_numpy(synthetic_pcm(rng, B, args.chunks, chunk=chunk)).to(dev)   # (chunks, B, chunk)
    ring = args.state == "ring"
    if ring:
        # the resident state a server keeps (include/tonehip.h tone_session_run_ring): the conv caches in per-stream rings
        # updated in place, the other sections in two ping-pong rows per stream of one slab; imported from the zero state
        slab = torch.zeros((2 * B, C.STATE_SIZE), dtype=torch.float16, device=dev)
        rings = torch.zeros((B, sess.ring_elems), dtype=torch.float16, device=dev)
        ids = torch.arange(B, dtype=torch.int32, device=dev)
        rows = [ids, ids + B]
        sess.ring_import(torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev), slab, rows[0], rings, ids)
        slabs = None
    else:
        slabs = [torch.zeros((B, C.STATE_SIZE), dtype=torch.float16, device=dev) for _ in range(2)]

    def run_step(i: int, lp) -> None:
        if ring:
            sess.run_ring(signal, rows[i % 2], rows[(i + 1) % 2], slab, rings, ids, lp, stream=stream, check=False)
        else:
            sess.run(signal, slabs[i % 2], lp, slabs[(i + 1) % 2], stream=stream)

    signal = torch.empty((B, chunk), dtype=torch.int32, device=dev)   # audio lands here
    logp = [torch.zeros((cap, fr, C.VOCAB), dtype=torch.float32, device=dev) for _ in range(2)]
    gathered = [torch.empty((world * cap, fr, C.VOCAB), dtype=torch.float32, device=dev)
                for _ in range(2)] if pg is not None else None
    stream = torch.cuda.Stream(dev)
    comm = torch.cuda.Stream(dev) if pg is not None else None
    freed = [None, None]          # event: the gather that last read logp[k] is done

    def step(i: int) -> None:
        k = i % 2
        if freed[k] is not None:
            stream.wait_event(freed[k])
        signal.copy_(pcm[i % args.chunks], non_blocking=True)
        run_step(i, logp[k][:B])
        if pg is not None:
            ready = stream.record_event()
            with torch.cuda.stream(comm):
                comm.wait_event(ready)
                if args.dist_backend == "gloo":      # one-GPU rehearsal: gloo gathers host tensors
                    comm.synchronize()
                    host = torch.empty((world * cap, fr, C.VOCAB), dtype=torch.float32)
                    pg.all_gather_into_tensor(host, logp[k].cpu())
                    gathered[k].copy_(host)
                else:
                    pg.all_gather_into_tensor(gathered[k], logp[k])
                freed[k] = comm.record_event()

    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for i in range(args.warmup, args.warmup + args.steps):
            ev[i - args.warmup].record(stream)
            step(i)
        ev[-1].record(stream)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pg is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        elapsed = float(t.item())
    per_step = np.array([ev[j].elapsed_time(ev[j + 1]) for j in range(args.steps)])
    res = {"elapsed": elapsed, "median_ms": round(float(np.median(per_step)), 4),
           "p99_ms": round(float(np.percentile(per_step, 99)), 4)}

    # ---- roofline of the dominant kernel: per-kernel HIP events on the launch stream -----------
    res["roofline"] = None
    if rank == 0 and with_roofline:
        sess.set_graph(False)
        sess.set_timing(True)
        with torch.cuda.stream(stream):
            for i in range(args.steps):
                signal.copy_(pcm[i % args.chunks], non_blocking=True)
                run_step(args.warmup + args.steps + i, logp[0][:B])
        torch.cuda.synchronize()
        per_stream = family_flops_per_stream(fr)
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
        traffic, tsrc = measured_traffic(dom, precision, B) if chunk == 2400 else (None, None)
        gemm_us = sum(v["avg_us"] * v["launches_per_step"] for v in fams.values())
        gemm_flop = sum(per_stream.values()) * B
        # per-family roofline: the larger of the MFMA floor (algorithmic FLOP / dense peak of the dtype)
        # and the HBM floor (algorithmic bytes / 8 TB/s) is the family's bound; frac = that floor / time
        pb, wb = family_bytes_per_stream(fr, precision), family_weight_bytes(precision)
        fam_roof, floor_sum = {}, 0.0
        for k, v in fams.items():
            us = v["avg_us"] * v["launches_per_step"]
            t_mfma = per_stream[k] * B / (peak * 1e12) * 1e6
            t_hbm = (pb[k] * B + wb[k]) / (HBM_PEAK_GBS * 1e9) * 1e6
            bnd = "mfma" if t_mfma >= t_hbm else "hbm"
            fl = max(t_mfma, t_hbm)
            floor_sum += fl
            fam_roof[k] = {"us_per_step": round(us, 1), "bound": bnd, "floor_us": round(fl, 1),
                           "frac": round(fl / us, 3), "gb_per_step": round((pb[k] * B + wb[k]) / 1e9, 4)}
        # the residual-output family (FFN down, attn-out, pw2: every EPI_RESID launch, the unit the PMC summary
        # measures): its algorithmic bytes per launch / mean launch time against 8 TB/s, its PMC traffic per launch,
        # and its bound from the same two floors as gemm_families (HBM in the bf16 / fp8 modes, MFMA in fp32)
        resid = None
        rf = [k for k in RESID_FAMILIES if k in fams]
        if rf:
            r_launch = sum(fams[k]["launches_per_step"] for k in rf)
            r_us = sum(fams[k]["avg_us"] * fams[k]["launches_per_step"] for k in rf) / r_launch
            r_bytes = algo_bytes("resid", precision, B, fr)
            r_tm = sum(per_stream[k] * B for k in rf) / r_launch / (peak * 1e12) * 1e6
            r_th = r_bytes / (HBM_PEAK_GBS * 1e9) * 1e6
            r_traffic, r_src = measured_traffic("resid", precision, B) if chunk == 2400 else (None, None)
            resid = {"bound": "mfma" if r_tm >= r_th else "hbm", "kernels": "EPI_RESID launches (FFN down, attn-out, pw2)",
                     "launches_per_step": r_launch, "avg_us": round(r_us, 2), "algo_bytes": int(r_bytes),
                     "achieved": round(r_bytes / (r_us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "hbm_frac": round(r_bytes / (r_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                     "frac": round(max(r_tm, r_th) / r_us, 4), "traffic": r_traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": r_src,
                     "traffic_over_algo": round(r_traffic / r_bytes, 3) if r_traffic else None}
        a_bytes = algo_bytes(dom, precision, B, fr)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": tsrc, "algo_bytes": int(a_bytes),
                "traffic_over_algo": round(traffic / a_bytes, 3) if traffic else None,
                "resid_family": resid,
                "avg_us": round(f["avg_us"], 2), "flop_per_launch": int(f["flop_per_launch"]),
                "step_tflops": round(C.FLOP_PER_CHUNK * B / (elapsed / args.steps) / 1e12, 2) if chunk == 2400 else None,
                "encoder_gemm_tflops": round(gemm_flop / (gemm_us * 1e-6) / 1e12, 2),
                "encoder_gemm_frac": round(gemm_flop / (gemm_us * 1e-6) / 1e12 / peak, 4),
                "step_io_gbs": round(B * (C.IO_BYTES_PER_CHUNK + 4 * (chunk - 2400) + 4 * (fr - 10) * 35)
                                     / (elapsed / args.steps) / 1e9, 1),
                "families_us_per_step": {k: round(v["avg_us"] * v["launches_per_step"], 1) for k, v in fams.items()},
                "gemm_families": fam_roof,
                "gemm_roofline_frac": round(floor_sum / gemm_us, 4)}
        if precision == "fp32":
            roof["gemm_arith"] = ("fp32 as exact 3-way bf16 splits, 6 products per multiply-add on "
                                  "v_mfma_f32_32x32x16_bf16 (fp32-accurate; tests/test_gpu_parity.py)")
            roof["pipe_peak"] = round(SPLIT_PIPE_PEAK, 1)
            roof["pipe_frac"] = round(achieved / SPLIT_PIPE_PEAK, 4)
        res["roofline"] = roof
    sess.close()
    del slabs, pcm, logp, gathered
    if ring:
        del slab, rings
    torch.cuda.empty_cache()
    return res


def dropin_latency_b1(dev_index: int, calls: int = 200) -> dict:
    """Per-call latency of the numpy drop-in at B = 1, the reference pipeline's call pattern
    (tone/pipeline.py:146): StreamingCTCModel.forward with host chunk + host state in and host logprobs + next
    state out (the 440 KB state crosses PCIe both ways every call, as with ORT's CUDA execution provider), next
    to the device-resident step (ToneSession.run, eager launches) of the same batch."""
    from tone_amd.model import StreamingCTCModel
    sess = ToneSession(replica_weights(None, None), device=dev_index, precision="fp32", max_batch=1)
    model = StreamingCTCModel(sess)          # eager launches (a graph replay measured 1.01 vs 0.97 ms per step)
    pcm = synthetic_pcm(np.random.default_rng(7), 1, 8)[:, :, :, None]      # (chunks, 1, 2400, 1)
    st = None
    for i in range(5):
        _, st = model.forward(pcm[i % 8], st)
    ts = []
    for i in range(calls):
        t0 = time.perf_counter()
        _, st = model.forward(pcm[i % 8], st)
        ts.append(time.perf_counter() - t0)
    dev = sess.dev
    sig = torch.from_numpy(pcm[0, :, :, 0]).to(dev)
    s_in = torch.zeros((1, C.STATE_SIZE), dtype=torch.float16, device=dev)
    s_out, lp = torch.empty_like(s_in), torch.empty((1, sess.frames, C.VOCAB), dtype=torch.float32, device=dev)
    for i in range(6):
        sess.run(sig, s_in if i % 2 == 0 else s_out, lp, s_out if i % 2 == 0 else s_in)
    torch.cuda.synchronize()
    td = []
    for i in range(calls):
        t0 = time.perf_counter()
        sess.run(sig, s_in if i % 2 == 0 else s_out, lp, s_out if i % 2 == 0 else s_in)
        torch.cuda.synchronize()
        td.append(time.perf_counter() - t0)
    sess.close()
    return {"batch": 1, "calls": calls, "dropin_numpy_median_ms": round(float(np.median(ts)) * 1e3, 3),
            "dropin_numpy_p99_ms": round(float(np.percentile(ts, 99)) * 1e3, 3),
            "device_step_median_ms": round(float(np.median(td)) * 1e3, 3),
            "device_step_p99_ms": round(float(np.percentile(td, 99)) * 1e3, 3),
            "what": "StreamingCTCModel.forward at B = 1 (host I/O, as pipeline.py:146 calls it) vs ToneSession.run "
                    "with device-resident I/O (eager launches + sync; a graph replay measured 1.01 vs 0.97 ms), fp32"}


def workload_line(name, res, n_streams, steps, dtype, chunk=C.AUDIO_CHUNK_SAMPLES, **extra):
    dt = res["elapsed"] / steps
    chunk_ms = chunk * 1000.0 / C.SAMPLE_RATE
    return {"workload": name, "value": round(n_streams / dt * chunk / C.SAMPLE_RATE, 1),
            "unit": "real-time streams", "ms_per_step": round(dt * 1e3, 4), "median_ms": res["median_ms"],
            "p99_ms": res["p99_ms"], "chunks_per_s": round(n_streams / dt, 1), "rtf": round(dt * 1e3 / chunk_ms, 5),
            "dtype": dtype, **extra, "roofline": res["roofline"]}


_ROOF_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_unit", "traffic_source",
              "algo_bytes", "traffic_over_algo", "avg_us", "flop_per_launch", "step_tflops", "encoder_gemm_tflops",
              "encoder_gemm_frac", "gemm_roofline_frac", "step_io_gbs", "pipe_peak", "pipe_frac")
_RESID_KEYS = ("bound", "avg_us", "achieved", "hbm_frac", "frac", "traffic", "traffic_over_algo")


def summary_roofline(roof: dict | None, alt: bool = False) -> dict | None:
    """The roofline fields the printed line keeps (the per-family tables stay in the detail file)."""
    if roof is None:
        return None
    keys = ("kernel", "achieved", "peak", "frac", "avg_us", "encoder_gemm_frac", "traffic_over_algo") if alt else _ROOF_KEYS
    out = {k: roof[k] for k in keys if k in roof}
    if roof.get("resid_family"):
        out["resid_family"] = {k: roof["resid_family"][k] for k in _RESID_KEYS if k in roof["resid_family"]}
    return out


def summary_line(out: dict, detail: str | None) -> dict:
    s = {k: v for k, v in out.items() if k not in ("roofline", "alt_workloads", "cpu_baseline")}
    s["roofline"] = summary_roofline(out["roofline"])
    cpu = out["cpu_baseline"]
    s["cpu_baseline"] = None if cpu is None else {k: v for k, v in cpu.items() if k != "per_batch"} | {
        "b1": cpu["per_batch"]["b1"]["value"] if "b1" in cpu.get("per_batch", {}) else None}
    s["alt_workloads"] = [{"workload": a["workload"].split(":")[0], "value": a["value"], "ms_per_step": a["ms_per_step"],
                           "dtype": a["dtype"], "n_gpus": a.get("n_gpus"), "batch_per_gpu": a.get("batch_per_gpu"),
                           "global_batch": a.get("global_batch"), "scaling": a.get("scaling"),
                           "roofline": summary_roofline(a["roofline"], alt=True)} for a in out["alt_workloads"]]
    s["detail"] = detail
    return s


def rank_envs(n: int, port: int, base_env: dict | None = None) -> list[dict]:
    """The environment of each of n rank processes, as torchrun would set it (one process per GPU, rendezvous on
    127.0.0.1)."""
    base = dict(os.environ if base_env is None else base_env)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def spawn_ranks(n: int, argv: list[str], timeout_s: float | None = None, script: str | None = None) -> int:
    """``python bench.py --gpus N`` without torchrun: start the N rank processes as children of this one (which has
    not touched the GPU) and wait for them.  Rank 0's stdout (the JSON line) is passed through; if any rank fails,
    the others are terminated (they would block in a collective) and the first failing exit status is returned."""
    import signal
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-u", script or os.path.abspath(__file__)] + argv
    procs = [subprocess.Popen(cmd, env=e, cwd=ROOT, start_new_session=True,
                              stdout=None if r == 0 else subprocess.DEVNULL)
             for r, e in enumerate(rank_envs(n, port))]
    t_end = None if timeout_s is None else time.monotonic() + timeout_s

    def stop_ranks(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    # the ranks run in their own sessions: if this parent is terminated or interrupted (a driver's own timeout,
    # Ctrl-C), take them down with it instead of leaving them holding the GPUs
    def on_signal(signum, _frame):
        stop_ranks(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                stop_ranks(signal.SIGKILL)
        os._exit(128 + signum)

    prev = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    status = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and status == 0:
            status = bad[0]
        if all(c is not None for c in codes):
            break
        if bad or (t_end is not None and time.monotonic() > t_end):
            status = status or 124
            stop_ranks(signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    stop_ranks(signal.SIGKILL)
                    p.wait()
            break
        time.sleep(0.2)
    for sg, h in prev.items():
        signal.signal(sg, h)
    if status < 0:
        status = 128 - status          # killed by a signal
    if status:
        print(f"bench.py: a rank failed (exit status {status})", file=sys.stderr)
    return status


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300, help="timed steps (300 x 3.6 ms: a window of about 1 s)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="streams per GPU, weak scaling (BASELINE config 2: 256)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="total streams split over the GPUs, strong scaling (BASELINE config 4: 4096); "
                         "replaces --batch for the headline")
    ap.add_argument("--precision", choices=["fp32", "fp32-mfma", "bf16", "fp8"], default="fp32")
    ap.add_argument("--chunks", type=int, default=10, help="distinct 300 ms chunks cycled per stream")
    ap.add_argument("--chunk-samples", type=int, default=C.AUDIO_CHUNK_SAMPLES, choices=[2400, 3200],
                    help="headline leg's chunk: 2400 (300 ms, BASELINE) or 3200 (the 400 ms variant; A/B runs)")
    ap.add_argument("--cpu-baseline-s", type=float, default=8.0, help="CPU baseline budget per batch (0 = skip)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--state", choices=["ring", "flat"], default="ring",
                    help="ring: the resident state form a server keeps (conv caches in per-stream rings updated in place, "
                         "tone_session_run_ring); flat: the (B, 219729) boundary state ping-ponged between two buffers "
                         "(tone_session_run).  Bit-identical results (tests/test_gpu_ring.py)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse N > 1 on one GPU (ranks share the card, collectives staged through host)")
    ap.add_argument("--alt", type=int, default=1, help="also measure BASELINE config 3 (bf16, B=2048) and the 400 ms "
                                                       "variant (fp32, B=256) at N=1")
    ap.add_argument("--config4", type=int, default=4096,
                    help="also measure BASELINE config 4: this many streams in total, sharded over the N GPUs, "
                         "bf16, logprobs all-gathered (0 = skip)")
    ap.add_argument("--config5", type=int, default=4096,
                    help="also measure BASELINE config 5's device step: this many streams sharded over the N GPUs, "
                         "MXFP8 q/k/v + FFN GEMMs, logprobs all-gathered (0 = skip)")
    ap.add_argument("--dist-always", action="store_true",
                    help="initialise the process group even at N = 1 (torchrun --nproc-per-node 1): the weight broadcast, "
                         "the per-step logprob all-gather and the max-over-ranks reduction then run through RCCL on one GPU")
    ap.add_argument("--spawn-timeout", type=float, default=1500.0,
                    help="--gpus N > 1 without torchrun: seconds before the spawned ranks are terminated")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the full per-family roofline of every leg (the printed line carries a summary)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched as plain `python bench.py --gpus N`: this process starts the N ranks itself (before any GPU call)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.spawn_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (launch N>1 with torchrun)")
    if args.dist_backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1 or args.dist_always:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        pg = dist

    from tone_amd.shard import shard_sizes
    if args.global_batch:
        sizes = shard_sizes(args.global_batch, world)
        B, cap, total, scaling = sizes[rank], max(sizes), args.global_batch, "strong"
    else:
        B, cap, total, scaling = args.batch, args.batch, world * args.batch, "weak"
    res = measure(args, B, args.precision, dev, local, world, rank, pg, cap=cap, chunk=args.chunk_samples)
    ms_step = res["elapsed"] / args.steps * 1e3
    chunks_s = total / (res["elapsed"] / args.steps)
    streams = chunks_s * args.chunk_samples / C.SAMPLE_RATE

    alts = []
    # BASELINE config 3 (1 GPU, batch 2048, bf16 MFMA, stateful) reported beside the headline
    if world == 1 and args.alt:
        r2 = measure(args, 2048, "bf16", dev, local, world, rank, pg)
        alts.append(workload_line("BASELINE config 3: streaming step, batch 2048, bf16 MFMA GEMMs, stateful 300 ms "
                                  "chunks", r2, 2048, args.steps, "bf16", n_gpus=1, scaling="n/a"))
        # the 400 ms chunk variant (3200 samples -> 13 frames), config 2's batch and dtype
        r400 = measure(args, 256, "fp32", dev, local, world, rank, pg, chunk=3200)
        alts.append(workload_line("400 ms chunk variant: streaming step, batch 256, fp32, stateful 3200-sample chunks "
                                  "(13 frames per step)", r400, 256, args.steps, "fp32", chunk=3200, n_gpus=1,
                                  scaling="n/a"))
    # BASELINE config 4 (4096 streams over the node's GPUs, strong scaling, RCCL all-gather of logprobs)
    if args.config4 and not (args.global_batch == args.config4 and args.precision == "bf16"):
        sizes = shard_sizes(args.config4, world)
        r4 = measure(args, sizes[rank], "bf16", dev, local, world, rank, pg, cap=max(sizes))
        alts.append(workload_line(
            f"BASELINE config 4: {args.config4} streams sharded {max(sizes)}/GPU over {world} GPU(s), bf16 MFMA "
            f"GEMMs, RCCL all-gather of logprobs per step (overlapped), strong scaling", r4, args.config4,
            args.steps, "bf16", n_gpus=world, global_batch=args.config4, batch_per_gpu=max(sizes), scaling="strong"))

    # BASELINE config 5 (4096 streams, fp8 MFMA on the q/k/v and FFN weights); the host KenLM beam search
    # consumes the gathered logprobs outside the device step (pipeline.StreamingGreedyPipeline(decoder=...))
    if args.config5:
        sizes = shard_sizes(args.config5, world)
        r5 = measure(args, sizes[rank], "fp8", dev, local, world, rank, pg, cap=max(sizes))
        alts.append(workload_line(
            f"BASELINE config 5 (device step): {args.config5} streams sharded {max(sizes)}/GPU over {world} GPU(s), "
            f"MXFP8 (e4m3 + E8M0 per 32) q/k/v and FFN GEMMs on v_mfma_scale_f32_16x16x128_f8f6f4, bf16 elsewhere, "
            f"RCCL all-gather of logprobs per step; the host KenLM beam decode of the gathered logprobs is not in "
            f"the timed step (pyctcdecode/kenlm are not installed)", r5, args.config5, args.steps, "fp8", n_gpus=world,
            global_batch=args.config5, batch_per_gpu=max(sizes), scaling="strong"))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_s > 0:
        cpu = cpu_baseline(args.cpu_baseline_s)
    lat = dropin_latency_b1(local) if rank == 0 and world == 1 and args.alt else None

    if rank == 0:
        if args.global_batch:
            wl = (f"streaming step, {total} streams sharded {cap}/GPU over {world} GPU(s), {args.precision}, "
                  f"stateful 300 ms chunks, strong scaling")
        elif args.precision == "fp32" and B == 256:
            wl = "BASELINE config 2: streaming step, batch 256/GPU, fp32, stateful 300 ms chunks"
        else:
            wl = f"streaming step, batch {B}/GPU, {args.precision}, stateful 300 ms chunks"
        out = {
            "metric": METRIC,
            "value": round(streams, 1),
            "unit": "real-time streams (300 ms chunks/s x 0.3 s)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "median_ms": res["median_ms"],
            "p99_ms": res["p99_ms"],
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (Gaussian sigma=3000 int16 PCM, 20% silent chunks; random-init T-one weights)",
            "config": {"workload": wl, "model": "T-one 71.7M (16-layer chunked Conformer, d384)",
                       "batch_per_gpu": cap, "global_batch": total, "chunk_ms": 300,
                       "parallelism": f"dp{world}", "graph": not args.no_graph,
                       "state": ("resident: conv caches in per-stream rings updated in place, other sections in "
                                 "ping-pong slab rows (run_ring)") if args.state == "ring"
                       else "flat (B, 219729) fp16, ping-pong buffers (run)",
                       "collective": "RCCL all_gather_into_tensor of logprobs per step, overlapped" if pg is not None
                       else None},
            "chunks_per_s": round(chunks_s, 1),
            "rtf": round(ms_step / 300.0, 5),
            "roofline": res["roofline"],
            "cpu_baseline": cpu,
            "latency_b1": lat,
            "alt_workloads": alts,
        }
        # the full line (per-family rooflines of every leg) goes to a file; the printed line carries a summary
        # short enough for a driver's stdout tail to hold all of it
        detail = None
        if args.detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
                with open(args.detail, "w") as fh:
                    json.dump(out, fh, indent=1)
                detail = os.path.relpath(os.path.abspath(args.detail), ROOT)
            except OSError:
                detail = None
        print(json.dumps(summary_line(out, detail)), flush=True)
    if pg is not None:
        pg.barrier()   # rank 0 finishes its roofline pass before any rank tears the communicator down
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
