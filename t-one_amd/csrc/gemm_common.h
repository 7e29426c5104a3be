// Helpers shared by the fp32-split / bf16 GEMM translation units (gemm_t.hip, gemm_pp.hip): vector types,
// LDS-DMA-friendly barrier, bf16 / split tile stores and the per-tile epilogue.
#pragma once
#include "common.h"
#include "kernels.h"

namespace tone {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBiasMax = 3072;   // largest N of the encoder (FFN up: W1|Wv)

template <int BNW_, int BMX_, int WN_, int WM_>
struct TT {
  static constexpr int BNW = BNW_, BMX = BMX_, WN = WN_, WM = WM_;
};

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const __bf16 ha = (__bf16)a, hb = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

__device__ __forceinline__ float sumsq8(bf16x8 v, float acc) {
  const bf16x2 p0 = __builtin_shufflevector(v, v, 0, 1), p1 = __builtin_shufflevector(v, v, 2, 3);
  const bf16x2 p2 = __builtin_shufflevector(v, v, 4, 5), p3 = __builtin_shufflevector(v, v, 6, 7);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p0, p0, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p1, p1, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p2, p2, acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(p3, p3, acc, false);
}

// bf16-output activations: v_exp_f32 + v_rcp_f32 (~1 ulp fp32, far below the bf16 rounding of the
// result) instead of the IEEE expf / division sequences
__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float fast_silu(float x) { return x * fast_sigmoid(x); }

__device__ __forceinline__ void barrier_lds() {   // keeps LDS-DMA in flight (no vmcnt(0) fence)
  // lgkmcnt(0) (vmcnt / expcnt at their maxima) as the builtin, so the compiler's wait-count pass knows every earlier
  // LDS read has completed: written as inline asm it was opaque to the pass, which then put a second lgkmcnt(0) in
  // front of the first use of a fragment read before the barrier -- and that one also drained every read issued
  // after the barrier (gemm_xs8: its deferred K-step waited on the next K-step's fragments and the bias)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// 16 values of one 32x32 D tile for this lane (row m fixed; columns c + (r&3) + 8(r>>2) + 4h) as
// bf16: pack to 4-element runs, swap runs between the lane halves (T21) so each lane owns 8
// contiguous elements, and store 2 x 16 B.  rowp points at column c of row m.  All lanes must
// execute the swaps; only the store is predicated.
__device__ __forceinline__ void store_tile_bf16(uint16_t* rowp, const float (&v)[16], int lh, bool ok, bool nt = false) {
  uint32_t px[4], py[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    px[g] = pk2(v[4 * g], v[4 * g + 1]);
    py[g] = pk2(v[4 * g + 2], v[4 * g + 3]);
  }
#pragma unroll
  for (int k = 0; k < 4; k += 2) {
    const auto rx = __builtin_amdgcn_permlane32_swap(px[k], px[k + 1], false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(py[k], py[k + 1], false, false);
    const u32x4 o = {rx[0], ry[0], rx[1], ry[1]};
    if (ok) {
      // nt: streaming output (the FFN intermediate h) kept from displacing the operands in L2
      if (nt) __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(rowp + 8 * k + 8 * lh));
      else *reinterpret_cast<u32x4*>(rowp + 8 * k + 8 * lh) = o;
    }
  }
}

// The same 16 values stored as their exact 3-term bf16 split into three planes `plane` apart.
__device__ __forceinline__ void store_tile_split(uint16_t* rowp, int64_t plane, const float (&v)[16], int lh, bool ok) {
  float t0[16], t1[16], t2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) split3_f(v[r], t0[r], t1[r], t2[r]);
  store_tile_bf16(rowp, t0, lh, ok);
  store_tile_bf16(rowp + plane, t1, lh, ok);
  store_tile_bf16(rowp + 2 * plane, t2, lh, ok);
}

// Per-tile epilogue shared by both kernels.  acc[i][j] is the wave's 32x32 D tile (n-tile i,
// m-tile j); rd[m - m0] the row-scale denominators, sb[n - n0] the bias (both LDS).
// tile_epilogue_inv: the same with the row factors 1 / rden of this lane's rows (row wm * WTM + 32 j + lr)
// already in registers.
// R16: the residual stream R / C is fp16 (bf16 / fp8 modes; compile-time, see gemm.hip gemm_epilogue)
template <int EPI, bool RS, int TI, int TJ, int WTN, int WTM, bool R16 = false>
__device__ __forceinline__ void tile_epilogue_inv(const GemmArgs& p, f32x16 (&acc)[TI][TJ], const float (&invj)[TJ],
                                                  const float* sb, int m0, int n0, int wn, int wm, int lr, int lh) {
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU);
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int ml = wm * WTM + 32 * j + lr, m = m0 + ml;
    const bool ok = m < p.M;
    const int64_t mrow = min(m, p.M - 1);
    const float inv = RS ? invj[j] : 1.0f;
    if constexpr (PAIRED) {
#pragma unroll
      for (int ip = 0; ip < TI / 2; ++ip) {
        const int nl = wn * WTN + 64 * ip;                   // g rows nl..nl+31, u rows nl+32..nl+63
        float o[16];
        if (p.c_bf16) {
          // bf16 output: v_exp_f32 / v_rcp_f32, value pairs (consecutive columns) as two-float vectors so the fused
          // multiply-adds and products issue as v_pk_* with the scalar form's per-element roundings
          typedef float f32x2e __attribute__((ext_vector_type(2)));
          const f32x2e inv2 = {inv, inv};
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int n = nl + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const f32x2e g = __builtin_elementwise_fma(f32x2e{acc[2 * ip][j][r], acc[2 * ip][j][r + 1]}, inv2,
                                                       f32x2e{sb[n], sb[n + 1]});
            const f32x2e u = __builtin_elementwise_fma(f32x2e{acc[2 * ip + 1][j][r], acc[2 * ip + 1][j][r + 1]}, inv2,
                                                       f32x2e{sb[n + 32], sb[n + 33]});
            const f32x2e z = (EPI == EPI_SWIGLU) ? g : u;
            const f32x2e t = z * -1.4426950408889634f;
            const f32x2e d = f32x2e{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
            const f32x2e sg = f32x2e{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
            const f32x2e y = (EPI == EPI_SWIGLU) ? g * sg * u : g * sg;
            o[r] = y.x;
            o[r + 1] = y.y;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int n = nl + (r & 3) + 8 * (r >> 2) + 4 * lh;
            const float g = fmaf(acc[2 * ip][j][r], inv, sb[n]);
            const float u = fmaf(acc[2 * ip + 1][j][r], inv, sb[n + 32]);
            o[r] = (EPI == EPI_SWIGLU) ? silu_f(g) * u : g * sigmoid_f(u);   // fp32 output: IEEE exp/div
          }
        }
        if (p.c_bf16) {
          store_tile_bf16(static_cast<uint16_t*>(p.C) + mrow * p.ldc + (n0 + nl) / 2, o, lh, ok, p.nt_store != 0);
        } else if (p.c_plane) {   // fp32 split mode: the next GEMM's A as 3 bf16 planes
          store_tile_split(static_cast<uint16_t*>(p.C) + mrow * p.ldc + (n0 + nl) / 2, p.c_plane, o, lh, ok);
        } else {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 w = {o[4 * g], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]};
            // c_packed: FFN down's A for gemm_d3 (common.h xpk_off; 4 consecutive columns stay one 16-byte run)
            const int col = (n0 + nl) / 2 + 8 * g + 4 * lh;
            if (ok) *reinterpret_cast<f32x4*>(static_cast<float*>(p.C) + act_off(mrow, col, (int)p.ldc, p.c_packed)) = w;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int nl = wn * WTN + 32 * i, nb = n0 + nl;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = fmaf(acc[i][j][r], inv, sb[nl + (r & 3) + 8 * (r >> 2) + 4 * lh]);
        if constexpr (EPI == EPI_RESID) {
          f32x4 rr[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) rr[g] = load_res4(p.R, mrow * p.ldr + nb + 8 * g + 4 * lh, R16);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 o;
            o.x = rr[g].x + p.alpha * v[4 * g];
            o.y = rr[g].y + p.alpha * v[4 * g + 1];
            o.z = rr[g].z + p.alpha * v[4 * g + 2];
            o.w = rr[g].w + p.alpha * v[4 * g + 3];
            v[4 * g] = o.x; v[4 * g + 1] = o.y; v[4 * g + 2] = o.z; v[4 * g + 3] = o.w;
            if (ok) store_res4(p.C, mrow * p.ldc + nb + 8 * g + 4 * lh, o, R16);
            // fp32: the packed copy the next rowscale projection reads (gemm_d3n; common.h xpk_off)
            if (!R16 && p.CP && ok) *reinterpret_cast<f32x4*>(p.CP + xpk_off(mrow, nb + 8 * g + 4 * lh, (int)p.ldc)) = o;
          }
          if (p.C2 && p.c2_plane) store_tile_split(p.C2 + mrow * p.ldc + nb, p.c2_plane, v, lh, ok);
          else if (p.C2) store_tile_bf16(p.C2 + mrow * p.ldc + nb, v, lh, ok);
        } else if (p.c_bf16) {
          store_tile_bf16(static_cast<uint16_t*>(p.C) + mrow * p.ldc + nb, v, lh, ok);
        } else {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 o = {v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
            if (ok) store_res4(p.C, mrow * p.ldc + nb + 8 * g + 4 * lh, o, R16);   // fp32 or fp16 residual
            if (!R16 && p.CP && ok) *reinterpret_cast<f32x4*>(p.CP + xpk_off(mrow, nb + 8 * g + 4 * lh, (int)p.ldc)) = o;
          }
          if (p.C2 && p.c2_plane) store_tile_split(p.C2 + mrow * p.ldc + nb, p.c2_plane, v, lh, ok);
          else if (p.C2) store_tile_bf16(p.C2 + mrow * p.ldc + nb, v, lh, ok);   // bf16 shadow (fp32 C)
        }
      }
    }
  }
}

template <int EPI, bool RS, int TI, int TJ, int WTN, int WTM, bool R16 = false>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& p, f32x16 (&acc)[TI][TJ], const float* rd, const float* sb,
                                              int m0, int n0, int wn, int wm, int lr, int lh) {
  float invj[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) invj[j] = RS ? 1.0f / rd[wm * WTM + 32 * j + lr] : 1.0f;
  tile_epilogue_inv<EPI, RS, TI, TJ, WTN, WTM, R16>(p, acc, invj, sb, m0, n0, wn, wm, lr, lh);
}


// 8 fp32 values -> their three bf16 terms (round-to-nearest-even at each level)
__device__ __forceinline__ void split3(const f32x4 a, const f32x4 b, bf16x8& h, bf16x8& m, bf16x8& l) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 x0 = (__bf16)x[e];
    const float r1 = x[e] - (float)x0;
    const __bf16 x1 = (__bf16)r1;
    const float r2 = r1 - (float)x1;
    h[e] = x0;
    m[e] = x1;
    l[e] = (__bf16)r2;
  }
}

}  // namespace
}  // namespace tone
