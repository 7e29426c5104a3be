"""Kernel-level numerics on the GPU: each hand-written GEMM route against a naive GPU reference of the same op.

`t-one_amd/gemm_bench` (tools/gemm_bench.hip, built by `__graft_entry__.build()`) feeds one kernel seeded synthetic
operands, runs it once, and compares every output element with a plain per-element fp64-accumulated reference kernel
over the same (bf16 / MXFP8-dequantized) operands: `max_rel_err` is the largest |out - ref| / (1 + |ref|) over the
output, `shadow_err` the same for the bf16 shadow a RESID launch also writes.  The step-level parity tests
(test_gpu_parity.py) bound whole-model logprobs; these catch a kernel that is wrong on some rows only -- e.g. the
fp8 row-panel RESID kernel once let the epilogue overwrite LDS that a slower wave was still reading when K = 384
(three K-tiles): max_rel_err 0.69-0.77 at M = 10240-20480 while the fp8 step tests stayed inside their bounds.
"""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.environ.get("TONE_GEMM_BENCH", os.path.join(ROOT, "t-one_amd", "gemm_bench"))   # override: A/B of a build


def _gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    if not os.path.exists(BENCH):
        pytest.fail("t-one_amd/gemm_bench is missing: run __graft_entry__.build()")


def _run(M, K, N, epi, variant, env):
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    out = subprocess.run([BENCH, str(M), str(K), str(N), str(epi), str(variant), "1", "2"], env=e,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert rows, out.stdout[-2000:]
    for r in rows:
        assert "error" not in r, r
    return rows[-1]


# (M, K): the fp8 / bf16 step's residual-output shapes (FFN down K = 1536, attn-out / pw2 K = 384) at B = 4096 / 2048
# / 1024 / 1638, i.e. both panel heights (160 / 80 rows) and the 48- / 64-row panels below
RESID_SHAPES = [(40960, 1536), (40960, 384), (20480, 1536), (20480, 384), (16384, 384), (10240, 384)]


@pytest.mark.parametrize("M,K", RESID_SHAPES)
def test_rp_mx_resid_matches_reference(M, K):
    """fp8 mode: gemm_rp_mx (MXFP8 operands, fp16 residual in place, bf16 shadow) at every routed panel height."""
    _gpu()
    r = _run(M, K, 384, 1, 99, {"RPMX": 1, "RES16": 1})
    assert r["max_rel_err"] < 2e-3, r


@pytest.mark.parametrize("M,K", RESID_SHAPES)
def test_rp_bf16_resid_matches_reference(M, K):
    """bf16 mode: gemm_rp (auto panel height) on the same shapes; the bf16 shadow within its own rounding."""
    _gpu()
    r = _run(M, K, 384, 1, 90, {"RES16": 1})
    assert r["max_rel_err"] < 2e-3 and r["shadow_err"] < 1e-2, r


@pytest.mark.parametrize("M,N,epi", [(40960, 3072, 2), (20480, 3072, 2), (4096, 3072, 2), (40960, 768, 3)])
def test_xw_matches_reference(M, N, epi):
    """bf16 gemm_xw (K = 384, folded RMSNorm row factor): FFN up SwiGLU and pw1 GLU, bf16 output."""
    _gpu()
    r = _run(M, 384, N, epi, -300, {"ROWSCALE": 1})
    assert r["max_rel_err"] < 1e-2, r


@pytest.mark.parametrize("M", [40960, 20480, 4096])
def test_xs8_swiglu_matches_reference(M):
    """fp8 gemm_xs8 (FFN up SwiGLU with the MXFP8 quantization of h in its epilogue): the error is the MXFP8
    rounding of the output (measured 0.08-0.19); a wrong tile or row reads as ~1."""
    _gpu()
    r = _run(M, 384, 3072, 2, 98, {"ROWSCALE": 1})
    assert r["max_rel_err"] < 0.3, r


# the fp32 step's GEMMs through gemm()'s own routing (gemm_x3 tiles, its 3-way split K at 400 ms, gemm_r3, gemm_sm at
# M <= 64), full fp32 operands against the fp64 reference: (K, N, epi, row factor) of FFN up, FFN down, attn-out / pw2,
# pw1 and q|k|v, at B = 256 (T = 10 / 5), 400 ms (T = 13 / 6) and the drop-in's B = 1 / 6
FP32_OPS = [(384, 3072, 2, 1), (1536, 384, 1, 0), (384, 384, 1, 0), (384, 768, 3, 1), (384, 1152, 0, 1)]


@pytest.mark.parametrize("M", [2560, 1280, 3328, 1536, 60, 10])
@pytest.mark.parametrize("K,N,epi,rs", FP32_OPS)
def test_fp32_routes_match_reference(M, K, N, epi, rs):
    _gpu()
    r = _run(M, K, N, epi, -2, {"FULLF32": 1, "NOC2": 1, "ROWSCALE": rs})
    assert r["max_rel_err"] < 2e-5, r


# the bf16 step's GEMMs through gemm()'s routing below the large-batch kernels (gemm_glds, gemm_t; B = 512 .. 1638)
@pytest.mark.parametrize("M", [10240, 5120, 2560])
@pytest.mark.parametrize("K,N,epi,rs", FP32_OPS)
def test_bf16_routes_match_reference(M, K, N, epi, rs):
    _gpu()
    r = _run(M, K, N, epi, -1, {"RES16": int(epi == 1), "ROWSCALE": rs})   # the fp16 residual on RESID only
    assert r["max_rel_err"] < 1e-2, r


# fp8 mode below the row-panel / X-stationary routes: the persistent MXFP8 kernel (gemm_mx) for q|k|v (fp32 out),
# FFN down (fp16 residual) and FFN up (SwiGLU -> MXFP8 h: its rounding, as for gemm_xs8)
@pytest.mark.parametrize("M", [10240, 5120, 2560])
@pytest.mark.parametrize("K,N,epi,rs,tol", [(384, 1152, 0, 1, 2e-3), (1536, 384, 1, 0, 2e-3), (384, 3072, 2, 1, 0.3)])
def test_mx_routes_match_reference(M, K, N, epi, rs, tol):
    _gpu()
    r = _run(M, K, N, epi, 99, {"RES16": int(epi == 1), "ROWSCALE": rs})
    assert r["max_rel_err"] < tol, r
