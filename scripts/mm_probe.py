"""Times torch (hipBLASLt) GEMMs at the encoder's shapes, as a practical ceiling for the hand-written GEMMs."""
import json, sys, torch
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[sys.argv[2] if len(sys.argv) > 2 else "bf16"]
out = []
for name, M, K, N in [("ffn_up", B * 10, 384, 3072), ("ffn_down", B * 10, 1536, 384), ("qkv", B * 10, 384, 1152),
                      ("attn_out", B * 10, 384, 384), ("pw1", B * 10, 384, 768), ("ffn_up_T5", B * 5, 384, 3072)]:
    a = torch.randn(M, K, device="cuda", dtype=dt)
    w = torch.randn(N, K, device="cuda", dtype=dt)
    for _ in range(3): torch.mm(a, w.t())
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(20): torch.mm(a, w.t())
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    out.append({"gemm": name, "M": M, "K": K, "N": N, "us": round(us, 1), "tflops": round(2 * M * K * N / us / 1e6, 1)})
print(json.dumps(out))
