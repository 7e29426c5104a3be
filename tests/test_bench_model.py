"""bench.py's roofline model (CPU): the GEMM families' algorithmic FLOP and HBM bytes per stream-chunk."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402


def test_gemm_flops_per_stream_chunk():
    """1.093 GFLOP of dense GEMMs per 300 ms stream-chunk; the 400 ms chunk adds frames."""
    f10, f13 = bench.family_flops_per_stream(10), bench.family_flops_per_stream(13)
    assert abs(sum(f10.values()) / 1e9 - 1.093) < 0.005
    assert f10["gemm_ffn_up"] == 2 * f10["gemm_ffn_down"]
    assert all(f13[k] > f10[k] for k in f10)


def test_family_bytes_and_bounds():
    """bf16 activations halve the activation bytes (RESID outputs stay fp32, plus a bf16 shadow); at
    BASELINE config 3 (bf16, B = 2048) the FFN up-projection is MFMA-bound and the residual (RESID)
    projections are HBM-bound; at config 2 (fp32, B = 256) every family is MFMA-bound on the 157 TF fp32
    peak."""
    b32, b16 = bench.family_bytes_per_stream(10, "fp32"), bench.family_bytes_per_stream(10, "bf16")
    assert all(b16[k] <= b32[k] for k in b32) and b16["gemm_ffn_up"] < b32["gemm_ffn_up"]

    def bound(prec, B):
        pb, wb, fl = bench.family_bytes_per_stream(10, prec), bench.family_weight_bytes(prec), bench.family_flops_per_stream(10)
        return {k: "mfma" if fl[k] * B / (bench.PEAK_TFLOPS[prec] * 1e12) >= (pb[k] * B + wb[k]) / (bench.HBM_PEAK_GBS * 1e9)
                else "hbm" for k in fl}

    b = bound("bf16", 2048)
    assert b["gemm_ffn_up"] == "mfma"
    assert b["gemm_ffn_down"] == b["gemm_attn_out"] == b["gemm_pw2"] == "hbm"
    assert set(bound("fp32", 256).values()) == {"mfma"}


def test_algo_bytes_per_launch_by_precision():
    """The dominant kernel's algorithmic bytes per launch (bench.algo_bytes): the FFN up-projection at
    B = 4096 reads X and writes h at 2 B per element in bf16 and at 1 + 1/32 B (e4m3 + one E8M0 scale per
    32) in fp8, plus the 2.36 MB bf16 / 1.22 MB MXFP8 weight matrix; fp32 at 4 B."""
    d, ff, B = 384, 1536, 4096
    rows = sum(B * (5 if 6 < l <= 14 else 10) for l in range(16)) * 2 / 32      # mean rows per FFN launch
    e8 = 1 + 1 / 32
    want = {"fp32": 4 * rows * (d + ff) + 4 * 2 * ff * d, "bf16": 2 * rows * (d + ff) + 2 * 2 * ff * d,
            "fp8": e8 * rows * (d + ff) + e8 * 2 * ff * d}
    for prec, w in want.items():
        assert abs(bench.algo_bytes("gemm_ffn_up", prec, B) - w) / w < 1e-9, prec
    assert 61e6 < bench.algo_bytes("gemm_ffn_up", "fp8", B) < 63e6       # ~62 MB, not 240.6 MB
    assert bench.algo_bytes("gemm_ffn_up", "fp8", B) < bench.algo_bytes("gemm_ffn_up", "bf16", B) / 1.9


def test_algo_bytes_resid_family():
    """The EPI_RESID family (FFN down, attn-out, pw2 as one kernel family, 64 launches per step): A read at
    the operand size, the residual stream read and written (fp32 in fp32 mode, fp16 in the bf16 / fp8 modes), the
    bf16 shadow (bf16 / fp8 modes), in fp8 mode the MXFP8 shadow + sum-of-squares slab written by FFN1 down of layers
    0-13 and by pw2, W once."""
    d, ff, B = 384, 1536, 2048
    for prec, ea, eh, er, sh in (("bf16", 2, 2, 2, 2), ("fp8", 2, 1 + 1 / 32, 2, 2), ("fp32", 4, 4, 4, 0)):
        q8 = (1 + 1 / 32 + 48 / d) if prec == "fp8" else 0.0
        tot = 0.0
        for l in range(16):
            rows = B * (5 if 6 < l <= 14 else 10)
            tot += 2 * rows * (ff * eh + d * (2 * er + sh))    # two FFN downs
            tot += rows * d * q8 if l < 14 else 0.0            # FFN1 down feeds q|k|v (fp8)
            tot += 2 * rows * (d * ea + d * (2 * er + sh))     # attn-out + pw2
            tot += rows * d * q8                               # pw2 feeds FFN2 (fp8)
        ew, e8 = (4, 4) if prec == "fp32" else (2, eh)
        tot += 16 * (2 * ff * d * e8 + 2 * d * d * ew)
        got = bench.algo_bytes("resid", prec, B)
        assert abs(got - tot / 64) / (tot / 64) < 1e-9, prec
    assert bench.FAMILY_LAUNCHES["gemm_ffn_down"] + bench.FAMILY_LAUNCHES["gemm_attn_out"] + \
        bench.FAMILY_LAUNCHES["gemm_pw2"] == 64


def test_measured_traffic_not_below_algorithmic():
    """Every committed PMC traffic summary that bench.py quotes must be at least the algorithmic bytes of
    the launches it measures: a ratio below 1 means the bookkeeping is wrong."""
    import glob, json, os, re
    for path in sorted(glob.glob(os.path.join(bench.ROOT, "profiles", "r0[34]_traffic_*_b*.json"))):
        prec, b = re.search(r"traffic_(fp32|bf16|fp8)_b(\d+)\.json", path).groups()
        t = json.load(open(path))
        fams = t.get("families") or {"gemm_ffn_up": t}
        for fam, v in fams.items():
            ratio = v["traffic_bytes_per_launch"] / bench.algo_bytes(fam, prec, int(b))
            assert ratio >= 1.0, (path, fam, ratio)


def test_rank_envs_like_torchrun():
    envs = bench.rank_envs(4, 29512, {"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"] and all(e["WORLD_SIZE"] == "4" for e in envs)
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29512"
               and e["PATH"] == "/bin" for e in envs)


def test_spawn_ranks_passes_rank0_and_propagates_failure(tmp_path, capfd):
    """`bench.py --gpus N` without torchrun starts N children (no GPU here: a stand-in rank script); rank 0's
    stdout passes through, a failing rank's status comes back and the blocked ranks are terminated."""
    ok = tmp_path / "ok.py"
    ok.write_text("import os\nprint('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'])\n")
    assert bench.spawn_ranks(3, [], 60, script=str(ok)) == 0
    out = capfd.readouterr().out
    assert "rank 0 of 3" in out and "rank 1" not in out          # only rank 0's stdout is passed through
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(120)\n")
    t0 = __import__("time").monotonic()
    assert bench.spawn_ranks(2, [], 60, script=str(bad)) == 3
    assert __import__("time").monotonic() - t0 < 30                # rank 0 was terminated, not waited for
    hang = tmp_path / "hang.py"
    hang.write_text("import time\ntime.sleep(120)\n")
    assert bench.spawn_ranks(2, [], 2, script=str(hang)) == 124


def test_spawn_ranks_parent_signal_stops_ranks(tmp_path):
    """A parent terminated while its ranks run (a driver's own timeout) takes the rank process groups with it."""
    import signal
    import subprocess
    import sys
    import time

    hang = tmp_path / "hang.py"
    hang.write_text("import os, time\nopen(os.environ['PIDDIR'] + '/' + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
                    "time.sleep(120)\n")
    parent = tmp_path / "parent.py"
    parent.write_text(f"import sys\nsys.path.insert(0, {repr(bench.ROOT)})\nimport bench\n"
                      f"sys.exit(bench.spawn_ranks(2, [], 100, script={repr(str(hang))}))\n")
    p = subprocess.Popen([sys.executable, str(parent)], env=dict(__import__("os").environ, PIDDIR=str(tmp_path)))
    t_end = time.monotonic() + 60
    while not all((tmp_path / r).exists() and (tmp_path / r).read_text() for r in "01"):
        assert time.monotonic() < t_end and p.poll() is None
        time.sleep(0.1)
    pids = [int((tmp_path / r).read_text()) for r in "01"]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for pid in pids:        # the ranks are gone (reaped by the parent before it exited)
        t_end = time.monotonic() + 10
        while True:
            try:
                __import__("os").kill(pid, 0)
            except ProcessLookupError:
                break
            assert time.monotonic() < t_end, pid
            time.sleep(0.1)


def test_summary_line_fits_driver_tail():
    """The printed line keeps every leg's value / ms_per_step / roofline fraction and stays well inside the
    driver's ~8 KB stdout tail; the per-family tables go to the detail file."""
    fams = {f: {"us_per_step": 1.0, "bound": "hbm", "floor_us": 1.0, "frac": 0.5, "gb_per_step": 0.1}
            for f in bench.GEMM_FAMILIES}
    roof = {k: 1.0 for k in bench._ROOF_KEYS} | {"kernel": "gemm_ffn_up", "unit": "TFLOP/s", "bound": "mfma",
                                                  "traffic_source": "profiles/r05_traffic_fp32_b256.json",
                                                  "gemm_families": fams, "families_us_per_step": {f: 1.0 for f in fams},
                                                  "resid_family": {k: 1.0 for k in bench._RESID_KEYS} | {"kernels": "x" * 80}}
    alt = {"workload": "BASELINE config 4: " + "y" * 200, "value": 1.0, "ms_per_step": 1.0, "dtype": "bf16", "n_gpus": 8,
           "batch_per_gpu": 512, "global_batch": 4096, "scaling": "strong", "roofline": roof}
    out = {"metric": bench.METRIC, "value": 1.0, "roofline": roof, "alt_workloads": [alt] * 4,
           "cpu_baseline": {"value": 1.0, "unit": "real-time streams", "cores": 16, "kind": "port", "sample": "z" * 200,
                            "per_batch": {"b1": {"value": 20.0}, "b256": {"value": 190.0}}},
           "latency_b1": {"device_step_median_ms": 1.0, "what": "w" * 200}, "config": {"workload": "c" * 100}}
    s = bench.summary_line(out, "gpurun_out/bench_detail.json")
    txt = __import__("json").dumps(s)
    assert len(txt) < 6000, len(txt)
    assert s["roofline"]["frac"] == 1.0 and "gemm_families" not in s["roofline"]
    assert [a["workload"] for a in s["alt_workloads"]] == ["BASELINE config 4"] * 4
    assert all(a["roofline"]["encoder_gemm_frac"] == 1.0 and a["roofline"]["resid_family"]["hbm_frac"] == 1.0
               for a in s["alt_workloads"])
    assert s["cpu_baseline"]["cores"] == 16 and s["cpu_baseline"]["b1"] == 20.0 and s["detail"]
