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
CHECK = os.environ.get("TONE_KERNEL_CHECK", os.path.join(ROOT, "t-one_amd", "kernel_check"))


def _gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    if not os.path.exists(BENCH) or not os.path.exists(CHECK):
        pytest.fail("t-one_amd/gemm_bench or kernel_check is missing: run __graft_entry__.build()")


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


# the fused block-final RMSNorm (NORM) and the shadow's MXFP8 form + sum-of-squares slab (Q8) of the row-panel kernels,
# at the heights the step routes them (M >= 16384): the normalized rows against the reference normalized the same way
# (norm_ref_kernel: the residual sum rounded to fp16, then w v / (||v|| / sqrt(384) + 1e-8) in fp64), the MXFP8 bytes
# against quant_mx over the kernel's own shadow, byte for byte, and the slab's row factor against quant_mx's
RP_FUSED_SHAPES = [(40960, 1536), (40960, 384), (20480, 1536), (20480, 384), (16384, 384)]


@pytest.mark.parametrize("M,K", RP_FUSED_SHAPES)
@pytest.mark.parametrize("norm,q8", [(1, 0), (0, 1), (1, 1)])
def test_rp_bf16_norm_q8_matches_reference(M, K, norm, q8):
    _gpu()
    r = _run(M, K, 384, 1, 90, {"RES16": 1, "NORMW": norm, "Q8": q8})
    assert r["norm"] == norm and r["max_rel_err"] < 3e-3 and r["shadow_err"] < 1.2e-2, r
    if q8:
        assert r["q8_bad"] == 0 and r["q8_inv_err"] < 1e-5, r


@pytest.mark.parametrize("M,K", RP_FUSED_SHAPES)
@pytest.mark.parametrize("norm,q8", [(1, 0), (0, 1), (1, 1)])
def test_rp_mx_norm_q8_matches_reference(M, K, norm, q8):
    _gpu()
    r = _run(M, K, 384, 1, 99, {"RPMX": 1, "RES16": 1, "NORMW": norm, "Q8": q8})
    assert r["norm"] == norm and r["max_rel_err"] < 3e-3, r
    if q8:
        assert r["q8_bad"] == 0 and r["q8_inv_err"] < 1e-5, r


@pytest.mark.parametrize("M,N,epi", [(40960, 3072, 2), (20480, 3072, 2), (4096, 3072, 2), (40960, 768, 3)])
def test_xw_matches_reference(M, N, epi):
    """bf16 gemm_xw (K = 384, folded RMSNorm row factor): FFN up SwiGLU and pw1 GLU, bf16 output."""
    _gpu()
    r = _run(M, 384, N, epi, -300, {"ROWSCALE": 1})
    assert r["max_rel_err"] < 1e-2, r


@pytest.mark.parametrize("M", [40960, 20480, 16384])
def test_xw_blocked_hidden_matches_reference(M):
    """bf16 FFN up writing h in 32 x 32 tiles (common.h hblk_off, the session's layout from M = 16384): the output read
    back through the inverse map equals the reference, i.e. every element lands where the consumer reads it."""
    _gpu()
    r = _run(M, 384, 3072, 2, -300, {"ROWSCALE": 1, "HBLK": 1})
    assert r["hblk"] == 1 and r["max_rel_err"] < 1e-2, r


@pytest.mark.parametrize("M", [40960, 20480, 16384])
@pytest.mark.parametrize("norm", [0, 1])
def test_rp_blocked_hidden_matches_reference(M, norm):
    """bf16 FFN down (gemm_rp) reading h in 32 x 32 tiles, with and without the fused norm (FFN2 down)."""
    _gpu()
    r = _run(M, 1536, 384, 1, 90, {"RES16": 1, "HBLK": 1, "NORMW": norm})
    assert r["hblk"] == 1 and r["max_rel_err"] < 3e-3 and r["shadow_err"] < 1.2e-2, r


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


# fp32 mode's N = 384 projections where the session routes them to gemm_d3 (gemm_d3_routed: attn-out / pw2 K = 384, FFN
# down K = 1536, M = B T from 65 to 4096): A and W fragment-packed (common.h xpk_off / wpk_off; the padding rows of A's
# last 32-row block NaN, so a read of them that reached an output would show), through gemm()'s own routing, full fp32
# operands against fp64
@pytest.mark.parametrize("M", [2560, 1280, 3328, 1536, 640, 320, 100])
@pytest.mark.parametrize("K,epi", [(384, 1), (1536, 1), (1536, 0)])
def test_fp32_d3_packed_matches_reference(M, K, epi):
    """... RESID (attn-out, pw2, FFN down) and STORE (the reduction's 1x1, K = 1536), with the packed copy of C that the
    next rowscale projection reads (GemmArgs::CP) checked through the inverse map."""
    _gpu()
    r = _run(M, K, 384, epi, -499, {"FULLF32": 1, "NOC2": 1, "PACKX": 1, "CPOUT": 1})
    assert r["max_rel_err"] < 2e-5 and 0 <= r["cp_err"] < 2e-5, r


# the rowscale projections on gemm_d3n over the packed copy of the residual stream (folded-norm row factor from the
# packed rows): FFN up (SwiGLU, h written packed for FFN down), pw1 (GLU), q|k|v (layers 0 / 7), v (the shared layers)
@pytest.mark.parametrize("M", [2560, 1280, 3328, 1536, 640, 100])
@pytest.mark.parametrize("N,epi,cpack", [(3072, 2, 1), (768, 3, 0), (1152, 0, 0), (384, 0, 0)])
def test_fp32_d3n_rowscale_matches_reference(M, N, epi, cpack):
    _gpu()
    r = _run(M, 384, N, epi, -499, {"FULLF32": 1, "NOC2": 1, "PACKX": 1, "ROWSCALE": 1, "CPACK": cpack})
    assert r["max_rel_err"] < 2e-5, r


# gemm_x3's two tile-to-XCD deals (TONE_X3_XCD: 2 M halves x 4 N quarters, the default, where the tile grid allows it;
# else the N-only split): every tile computed once and correctly under both (a deal that dropped or doubled a tile shows
# as a wrong block), at the fp32 step's FFN up / q|k|v heights -- M = 3328 / 1536 have an odd M-tile count and take the
# N-only split either way
@pytest.mark.parametrize("M", [2560, 1280, 3328, 1536])
@pytest.mark.parametrize("N,epi", [(3072, 2), (1152, 0)])
def test_fp32_x3_xcd_deals_match_reference(M, N, epi):
    _gpu()
    r = [_run(M, 384, N, epi, -2, {"FULLF32": 1, "NOC2": 1, "ROWSCALE": 1, "TONE_X3_XCD": x}) for x in (0, 1)]
    assert all(v["max_rel_err"] < 2e-5 for v in r) and r[0]["max_rel_err"] == r[1]["max_rel_err"], r


# ... and the producer side of FFN down's packed A: the fp32 SwiGLU epilogue (gemm_x3) writing h fragment-packed, read
# back through the inverse map
@pytest.mark.parametrize("M", [2560, 1280, 3328, 1536, 640, 100])
def test_fp32_swiglu_packed_output_matches_reference(M):
    _gpu()
    r = _run(M, 384, 3072, 2, -2, {"FULLF32": 1, "NOC2": 1, "ROWSCALE": 1, "CPACK": 1})
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


# ---- the non-GEMM kernels, every element (t-one_amd/kernel_check, tools/kernel_check.hip) ----------------------------
# One launch per check at the bench's batches (bf16 / fp8 modes: B = 4096 / 2048; fp32: B = 256 and the drop-in's B = 1),
# every output element against a naive fp64 GPU reference of the reference model's op over the kernel's own operands,
# and every element of every state row: the read rows unchanged, the written rows' owned sections equal to the
# reference (fp16 ulps; copies exact), everything else in them still the sentinel.


def _check(*args):
    out = subprocess.run([CHECK, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert rows, out.stdout[-2000:]
    r = rows[-1]
    assert r["nan"] == 0, r
    return r


def _state_ok(r, ulp=None, err=None):
    """ulp: largest fp16 ulp distance allowed (0: the sections are exact copies); err: largest |out - ref| / (1 + |ref|)
    (recomputed values: one fp16 rounding of a value the kernel computes in another order)."""
    assert r["state_in_changed"] == 0 and r["state_sentinel_bad"] == 0, r
    if ulp is not None:
        assert r["state_ulp"] <= ulp, r
    if err is not None:
        assert r["state_err"] < err, r


@pytest.mark.parametrize("B", [4096, 2048, 512])
def test_sub_conv_bf16_every_element(B):
    """bf16 / fp8 pre-encode at 300 ms (sub_conv_bf16: RMSNorm + conv1 + conv2 in one launch, conformer_blocks.py:631-641):
    the bf16 flat output within its rounding; the new sub1 / sub2 state rows within an fp16 ulp."""
    _gpu()
    r = _check("sub_conv", B)
    assert r["outputs"]["flat"] < 1e-2, r
    _state_ok(r, err=2e-3)


@pytest.mark.parametrize("check,B,tol", [("sub1_f32", 256, 2e-5), ("sub1_f32", 1, 2e-5), ("sub1_f32_400", 256, 2e-5),
                                         ("sub1_bf16_400", 4096, 1e-2), ("sub1_bf16_400", 2048, 1e-2)])
def test_sub1_every_element(check, B, tol):
    """conv1 alone (fp32 mode, and bf16 at 400 ms): the conv2 input x2 (carried rows + conv1) and the new states."""
    _gpu()
    r = _check(check, B)
    assert r["outputs"]["x2"] < tol, r
    _state_ok(r, err=2e-3)


@pytest.mark.parametrize("check,B,tol", [("conv2_f32", 256, 2e-5), ("conv2_f32", 6, 2e-5), ("conv2_f32", 1, 2e-5),
                                         ("conv2_f32_400", 256, 2e-5), ("conv2_bf16_400", 4096, 1e-2)])
def test_conv2_every_element(check, B, tol):
    """conv2 + BN + SiLU: conv2_p3 (fp32 split, B > 8), conv2_sm (exact fp32, B <= 8), the bf16 implicit GEMM (400 ms)."""
    _gpu()
    r = _check(check, B)
    assert r["outputs"]["flat"] < tol, r


# "_pk": fp32 with the output fragment-packed for gemm_d3 (common.h xpk_off; the step's layout at M = B T > 64), read
# back through the inverse map
DW_CASES = [(4096, t, "dwconv_bf16", 1e-2) for t in (10, 5, 13, 6)] + [(2048, 10, "dwconv_bf16", 1e-2)] + \
           [(256, t, "dwconv", 1e-5) for t in (10, 5, 13, 6)] + [(1, 10, "dwconv", 1e-5)] + \
           [(256, t, "dwconv_pk", 1e-5) for t in (10, 5, 13, 6)] + [(9, 10, "dwconv_pk", 1e-5)]   # B coprime with 7 (the check's row permutation)


@pytest.mark.parametrize("B,T,check,tol", DW_CASES)
def test_dwconv_every_element(B, T, check, tol):
    """Depthwise conv k31 + state + BN + SiLU (submodules.py:364-402): output, and the new conv state = exact copies."""
    _gpu()
    r = _check(check, B, T)
    assert r["outputs"]["out"] < tol, r
    _state_ok(r, 0)


@pytest.mark.parametrize("B,T,check,tol", [(4096, 10, "dwconv_ring_bf16", 1e-2), (4096, 5, "dwconv_ring_bf16", 1e-2),
                                            (2048, 13, "dwconv_ring_bf16", 1e-2), (2048, 6, "dwconv_ring_bf16", 1e-2),
                                            (256, 10, "dwconv_ring", 1e-5), (256, 5, "dwconv_ring", 1e-5),
                                            (1, 10, "dwconv_ring", 1e-5), (256, 10, "dwconv_ring_pk", 1e-5),
                                            (256, 5, "dwconv_ring_pk", 1e-5), (256, 13, "dwconv_ring_pk", 1e-5)])
def test_dwconv_ring_every_element(B, T, check, tol):
    """The resident-form depthwise conv (cache frame i at ring row (n T + i) mod 30, the T new frames written over the T
    oldest): output, and every byte of every ring (the other rows, layers and the unused ring unchanged)."""
    _gpu()
    r = _check(check, B, T)
    assert r["outputs"]["out"] < tol and r["outputs"]["ring_bad_bytes"] == 0, r


REC_TS = [(10, 0), (5, 0), (5, 15), (10, 30), (13, 0), (6, 0), (6, 15), (13, 30)]


@pytest.mark.parametrize("T,S", REC_TS)
@pytest.mark.parametrize("check,B,tol", [("attn_rec_bf16", 4096, 1e-2), ("attn_rec", 256, 5e-5), ("attn_rec_pk", 256, 5e-5)])
def test_attention_rec_every_element(T, S, check, B, tol):
    """Recomputing layers (q/k LayerNorm, RoPE, masked softmax, P V; submodules.py:204-271) for every instantiated
    (T, S); the probabilities the shared layers reuse, where written; no state write."""
    _gpu()
    r = _check(check, B, T, S)
    assert r["outputs"]["ctx"] < tol, r
    if "probs" in r["outputs"]:
        assert r["outputs"]["probs"] < 2e-5, r
    _state_ok(r, 0)


@pytest.mark.parametrize("T", [10, 5, 13, 6])
@pytest.mark.parametrize("check,B,tol", [("attn_shared_bf16", 4096, 1e-2), ("attn_shared", 256, 1e-5),
                                         ("attn_shared_pk", 256, 1e-5)])
def test_attention_shared_every_element(T, check, B, tol):
    _gpu()
    r = _check(check, B, T)
    assert r["outputs"]["ctx"] < tol, r
    _state_ok(r, 0)


@pytest.mark.parametrize("T,S", [(5, 15), (10, 30), (6, 15), (13, 30)])
@pytest.mark.parametrize("check,B,tol", [("kv_bf16", 4096, 1e-2), ("kv", 256, 1e-5)])
def test_kv_assemble_every_element(T, S, check, B, tol):
    """Layers 14 / 15 input cache (conformer_blocks.py:147-163): xn, kv = [cache ; xn], the new left-padded cache."""
    _gpu()
    r = _check(check, B, T, S)
    assert r["outputs"]["xn"] < tol and r["outputs"]["kv"] < tol, r
    _state_ok(r, 1)


@pytest.mark.parametrize("T,S", [(5, 15), (10, 30), (6, 15), (13, 30)])
@pytest.mark.parametrize("check,B,tol", [("kv_ring_bf16", 4096, 1e-2), ("kv_ring", 256, 1e-5), ("kv_ring", 1, 1e-5)])
def test_kv_assemble_ring_every_element(T, S, check, B, tol):
    """The resident-form MHSA cache: kv's cached rows from ring frames 30 - S .. 29 (row (n T + j) mod 30), the T new
    xn rows written over the T oldest ring rows; every element of every ring (conv layers and the other MHSA layer
    unchanged, the new rows within one fp16 rounding)."""
    _gpu()
    r = _check(check, B, T, S)
    assert r["outputs"]["xn"] < tol and r["outputs"]["kv"] < tol and r["outputs"]["ring_max_ulp"] <= 1, r


@pytest.mark.parametrize("T", [10, 13])
@pytest.mark.parametrize("check,B,tol", [("reduce_bf16", 4096, 1e-2), ("reduce", 256, 1e-5), ("reduce_pk", 256, 1e-5),
                                         ("reduce_pk", 13, 1e-5)])
def test_reduce_conv_every_element(T, check, B, tol):
    _gpu()
    r = _check(check, B, T)
    assert r["outputs"]["y"] < tol, r
    _state_ok(r, 0)


@pytest.mark.parametrize("T", [10, 13])
@pytest.mark.parametrize("check,B,tol", [("upsample_r16", 4096, 2e-3), ("upsample", 256, 1e-6), ("upsample_pk", 256, 1e-6)])
def test_upsample_add_every_element(T, check, B, tol):
    """... "_pk": also the packed copy of the sum (layer 15's FFN1 A on gemm_d3n)."""
    _gpu()
    r = _check(check, B, T)
    assert r["outputs"]["x"] < tol and r["outputs"]["shadow"] < 1e-2, r
    if check.endswith("_pk"):
        assert r["outputs"]["xp"] < tol, r


@pytest.mark.parametrize("check,rows", [("head_r16", 40960), ("head_r16", 20480), ("head_r16", 4097), ("head", 2560),
                                        ("head", 2570), ("head", 65), ("head", 60), ("head", 10)])
def test_head_every_element(check, rows):
    """CTC head + log_softmax + the greedy token / speech flag (head_mfma_kernel / head_kernel, and head_rows_kernel at
    <= 64 rows); row counts off the 32-row block included."""
    _gpu()
    r = _check(check, rows)
    assert r["outputs"]["logprobs"] < 5e-5 and r["outputs"]["frame_info_bad"] == 0, r


@pytest.mark.parametrize("check,rows,tol", [("rmsnorm_q8", 40960, 2e-3), ("rmsnorm_r16", 20480, 2e-3),
                                            ("rmsnorm", 2560, 1e-5), ("rmsnorm_pk", 2560, 1e-5), ("rmsnorm_pk", 100, 1e-5)])
def test_rmsnorm_every_element(check, rows, tol):
    _gpu()
    r = _check(check, rows)
    assert r["outputs"]["x"] < tol and r["outputs"]["shadow"] < 1e-2, r
    if check.endswith("_pk"):   # the packed copy (the next FFN up's A on gemm_d3n)
        assert r["outputs"]["xp"] < tol, r
    if "q8_bad_bytes" in r["outputs"]:
        assert r["outputs"]["q8_bad_bytes"] == 0 and r["outputs"]["q8_row_factor"] < 1e-5, r
