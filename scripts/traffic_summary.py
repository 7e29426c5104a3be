"""Per-launch HBM traffic of two GEMM families from the PMC passes of scripts/pmc_traffic.sh: the FFN
up-projection (the only SWIGLU GEMM) and the residual-output GEMMs (every EPI_RESID launch: FFN down,
attn-out, pw2), recognised by kernel name and epilogue template argument.  FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM), so
fetch bytes = 2 x FETCH_SIZE x 1024.
Usage: python scripts/traffic_summary.py gpurun_out/pmc_<prec> <prec> <batch> > profiles/<file>.json"""
import csv, glob, json, re, sys

root, prec, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
UP = {  # SWIGLU instantiations: EPI_SWIGLU = 2
    "fp32": r"gemm_x3_kernel<tone::(?:\(anonymous namespace\)::)?XT<[^>]*>, 2,",
    "fp32-mfma": r"gemm_kernel<tone::(?:\(anonymous namespace\)::)?Tile<[^>]*>, 2,",
    "bf16": r"(gemm_t_kernel<tone::(?:\(anonymous namespace\)::)?TT<[^>]*>, 2,|gemm_x[sw]\d?_kernel<2, )",
    "fp8": r"(gemm_xs8_kernel<2, |gemm_mx_kernel<\d+, 2, )",
}[prec]
# EPI_RESID = 1, in any GEMM kernel family; every gemm_rp_kernel launch
RESID = (r"(gemm_x3_kernel<tone::(?:\(anonymous namespace\)::)?XT<[^>]*>, 1,|gemm_glds_kernel<tone::(?:\(anonymous namespace\)::)?Tile<[^>]*>, 1,|gemm_kernel<tone::(?:\(anonymous namespace\)::)?Tile<[^>]*>, 1,"
         r"|gemm_t_kernel<tone::(?:\(anonymous namespace\)::)?TT<[^>]*>, 1,|gemm_f32t_kernel<[^>]*>, 1,|gemm_mx_kernel<\d+, 1,"
         r"|gemm_rp_kernel<"     # the row-panel kernel (round 5) is RESID only
         r"|gemm_d3_kernel<\d+, \d+, \d+, \d+, 1,)")   # fp32 direct-load kernel (round 6): <WM, WN, WK, D, EPI, XP>


def per_launch(sub, pat):
    f = glob.glob(f"{root}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if re.search(pat, r["Kernel_Name"])]


def family(pat):
    fetch, write = per_launch("fetch", pat), per_launch("write", pat)
    if not fetch or not write:
        return None
    fb = 2 * 1024 * sum(fetch) / len(fetch)
    wb = 1024 * sum(write) / len(write)
    return {"launches_fetch": len(fetch), "launches_write": len(write), "fetch_bytes_per_launch": round(fb),
            "write_bytes_per_launch": round(wb), "traffic_bytes_per_launch": round(fb + wb)}


up, resid = family(UP), family(RESID)
out = {"kernel": "gemm_ffn_up", "precision": prec, "batch": batch, **(up or {}),
       "families": {k: v for k, v in (("gemm_ffn_up", up), ("resid", resid)) if v},
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes, eager launches; fetch x2 (gfx950)"}
print(json.dumps(out))
