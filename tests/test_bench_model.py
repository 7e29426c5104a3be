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
