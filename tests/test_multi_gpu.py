"""World-2 runs on the one GPU of the box: real ToneSessions per rank (tests/world2_worker.py) and
bench.py's N > 1 path (weight broadcast, strong-scaling shards, double-buffered all-gather) rehearsed
with the gloo backend, since RCCL needs one card per rank.  Both are started as child processes of
torchrun (never exec'd from this process)."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, timeout, nproc=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="4")
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_world2_sessions_gather_matches_single_process(tmp_path):
    out = tmp_path / "w2.json"
    r = _torchrun([os.path.join(ROOT, "tests", "world2_worker.py"), str(out)], timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["shape"] == [7, 10, 35]
    # the gathered shards equal the one-process batch up to summation order: streams are independent, but the GEMM
    # routing depends on the row count (3-4 streams per rank = M <= 64 routes to the small-M tiles, 7 streams does not)
    assert res["d_single"] <= 1e-4, res
    assert res["d_oracle"] < 1e-3, res


@pytest.mark.gpu
def test_bench_world2_strong_scaling_rehearsal():
    r = _torchrun(["bench.py", "--gpus", "2", "--dist-backend", "gloo", "--global-batch", "64", "--steps", "4",
                   "--warmup", "1", "--alt", "0", "--config4", "32", "--config5", "32", "--cpu-baseline-s", "0"],
                  timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["config"]["global_batch"] == 64
    assert out["config"]["batch_per_gpu"] == 32 and out["value"] > 0
    c4, c5 = out["alt_workloads"]
    assert c4["global_batch"] == 32 and c4["batch_per_gpu"] == 16 and c4["scaling"] == "strong"
    assert c5["dtype"] == "fp8" and c5["batch_per_gpu"] == 16 and c5["value"] > 0


@pytest.mark.gpu
def test_bench_rccl_world1():
    """bench.py's collective path through RCCL itself (the nccl backend) on the box's one GPU: world size 1, so the
    weight broadcast, the double-buffered logprob all-gather on the comm stream and the max-over-ranks all_reduce
    run as real RCCL calls (two ranks would need two cards)."""
    r = _torchrun(["bench.py", "--gpus", "1", "--dist-always", "--dist-backend", "nccl", "--steps", "6", "--warmup", "2",
                   "--alt", "0", "--config4", "64", "--config5", "64", "--cpu-baseline-s", "0", "--batch", "64"],
                  timeout=240, nproc=1)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert out["config"]["collective"] and "RCCL" in out["config"]["collective"]
    c4, c5 = out["alt_workloads"]
    assert c4["value"] > 0 and c5["value"] > 0 and c5["dtype"] == "fp8"


@pytest.mark.gpu
def test_bench_gpus2_without_torchrun(tmp_path):
    """The driver's launch form: plain `python bench.py --gpus 2` (no torchrun, WORLD_SIZE unset) starts its two
    rank processes itself (gloo here: the box has one card) and prints one line with n_gpus 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "4"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--steps", "4",
                        "--warmup", "1", "--batch", "16", "--alt", "0", "--config4", "64", "--config5", "0",
                        "--cpu-baseline-s", "0", "--detail", str(tmp_path / "detail.json")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["config"]["global_batch"] == 32 and out["value"] > 0
    (c4,) = out["alt_workloads"]
    assert c4["n_gpus"] == 2 and c4["batch_per_gpu"] == 32 and c4["value"] > 0
    full = json.loads((tmp_path / "detail.json").read_text())
    assert "gemm_families" in full["roofline"] and full["value"] == out["value"]
