"""Vendor-library reference for the encoder's K = 384 / K = 1536 GEMM shapes on the MI355X: torch.matmul (hipBLASLt /
rocBLAS) on plain bf16 operands, and torch._scaled_mm on e4m3 where this build supports it.  No epilogue (no SwiGLU,
bias, residual or row factor), so these times are a floor for what the fused kernels do -- measurement only, nothing
here is on the product path."""
import json
import torch

dev = "cuda"


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


shapes = [("ffn_up", 40960, 384, 3072), ("ffn_up", 20480, 384, 3072), ("ffn_down", 40960, 1536, 384),
          ("ffn_down", 20480, 1536, 384), ("qkv", 40960, 384, 1152), ("attn_out", 40960, 384, 384),
          ("ffn_up", 2560, 384, 3072)]
for name, M, K, N in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    us = timeit(lambda: torch.matmul(a, w.t()))
    fl = 2.0 * M * N * K
    rec = {"shape": name, "M": M, "K": K, "N": N, "dtype": "bf16", "us": round(us, 2), "tflops": round(fl / us * 1e-6, 1)}
    print(json.dumps(rec), flush=True)
    try:
        a8 = a.to(torch.float8_e4m3fn)
        w8 = w.to(torch.float8_e4m3fn)
        one = torch.ones((), device=dev, dtype=torch.float32)
        us8 = timeit(lambda: torch._scaled_mm(a8, w8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
        print(json.dumps({**rec, "dtype": "e4m3 (per-tensor scale)", "us": round(us8, 2),
                          "tflops": round(fl / us8 * 1e-6, 1)}), flush=True)
    except Exception as ex:  # noqa: BLE001 - report and continue
        print(json.dumps({"shape": name, "dtype": "e4m3", "error": str(ex)[:200]}), flush=True)
