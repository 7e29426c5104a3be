// W-stationary bf16 GEMM for the K = 384 encoder projections at large batch (FFN up + SwiGLU, pw1 + GLU,
// q|k|v STORE), D[n][m] = W[n][:] . X[m][:] in the transposed orientation of gemm_t / gemm_xs.
//
// Why: both earlier large-batch kernels stream one operand through an LDS ring filled by
// LDS-DMA, with a workgroup barrier per K-tile or W tile -- gemm_t both operands, gemm_xs the W tiles -- and the
// ring fill (30-48 GB/s per CU under those barrier-paced bursts) plus the epilogue set their time (FFN up at
// M = 40960: 86 us of kernel time in the step for 96.6 GFLOP).  Here nothing is streamed through LDS:
//   * a workgroup owns a 192-row slice of W for the whole launch: loaded ONCE into LDS (192 x 768 B, rows padded
//     to 784 B so every ds_read_b128 of the 32x32x16 fragment map is conflict-free), followed by the only barrier;
//   * each of its 8 waves then walks its own 32-row X steps with plain global loads straight into registers (the
//     MFMA B fragments: 96 VGPRs), and multiplies them against the LDS-resident slice in three 64-row sub-tiles;
//     the next step's fragment ks is loaded as soon as the last sub-tile's MFMAs of K-step ks have read the
//     current one, so a step's X arrives during the previous step's last sub-tile;
//   * accumulators are double-buffered per sub-tile (2 x 32 VGPRs): the epilogue of sub-tile u - 1 (bias, row
//     factor, SwiGLU / GLU, bf16 pack + stores) is spread over the K-steps of sub-tile u; the row factor of the
//     folded RMSNorm is summed from the X fragments during a step's first sub-tile;
//   * the waves never meet again after the W load, so one wave's loads and epilogue run under the other SIMD
//     wave's MFMAs.
// Measured (tools/gemm_bench, profiles/r03_ws_sweep.jsonl, r03_ws_ablate.jsonl): equal to gemm_xs at M = 40960
// (123 vs 125 us), slower at M <= 20480; its ablations show the MFMAs (~53 us at the 32x32x16 shape's sustained
// 1.8 PF), the W fragment reads (~31) and the X loads (~16) adding up rather than overlapping.  Kept out of
// libtonehip.so; built into the microbenchmark only.
// Work split: N / 192 n-groups x (256 / n-groups) m-groups, one workgroup per CU; the workgroups of one m-group
// (same X rows, different W slices) sit on one XCD, so each X row comes from HBM once per launch and from that
// XCD's L2 for the other n-groups.  W is read from HBM/MALL once per XCD.
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

#include <type_traits>

namespace tone {
namespace {

constexpr int kWsK = 384;                 // K (d_model)
constexpr int kWsKS = kWsK / 16;          // 32x32x16 K-steps (24)
constexpr int kWsBN = 192;                // W rows per workgroup (LDS-resident)
constexpr int kWsSubN = 64;               // W rows per sub-tile (two 32-row n-tiles: one g | u block pair)
constexpr int kWsWaves = 8;
constexpr int kWsRowB = kWsK * 2 + 16;    // padded LDS row (784 B): consecutive rows 4 banks apart
constexpr int kWsLds = kWsBN * kWsRowB + kWsBN * 4;

typedef __bf16 bf16x8_w __attribute__((ext_vector_type(8)));
typedef float f32x16_w __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_w __attribute__((ext_vector_type(4)));
typedef float f32x4_w __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_w __attribute__((ext_vector_type(2)));

// OVL: double-buffered accumulators, each sub-tile's epilogue spread over the next sub-tile's K-steps (else: the
// epilogue right after its sub-tile, under the other wave of the SIMD).
// DBG (WS_ABLATE microbenchmark builds only): 1 no epilogue, 2 no MFMA, 4 no X loads after the first step
template <int EPI, bool RS, bool OBF, int DBG = 0, bool OVL = true>
__global__ void __launch_bounds__(kWsWaves * 64) gemm_ws_kernel(GemmArgs p, int gn, int gm) {
  static_assert(EPI == EPI_SWIGLU || EPI == EPI_GLU || EPI == EPI_STORE, "SWIGLU / GLU / STORE");
  constexpr bool PAIRED = (EPI != EPI_STORE);
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWsLds];
  float* sbias = reinterpret_cast<float*>(lds + kWsBN * kWsRowB);

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  // XCD-major workgroup order: blocks x, x + 8, ... run on XCD x; consecutive g share an m-group
  const int g = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int ng = g % gn, mg = g / gn;
  if (mg >= gm) return;                                            // workgroup-uniform
  const int steps = (p.M + 31) >> 5;
  const int s0 = (int)((int64_t)steps * mg / gm), s1 = (int)((int64_t)steps * (mg + 1) / gm);
  if (s0 >= s1) return;

  int st = s0 + wid;
  // 32-bit byte offsets from uniform bases (the operands and outputs stay below 4 GiB): one VGPR per pointer
  const char* __restrict__ Xb = static_cast<const char*>(p.A);
  const uint32_t ldx = (uint32_t)p.lda * 2u;
  // lane (lr, lh): X row 32 st + lr, k 16 ks + 8 lh .. +7 of K-step ks (the B fragment of v_mfma_f32_32x32x16_bf16)
  auto xoff = [&](int s) -> uint32_t { return (uint32_t)min(32 * s + lr, p.M - 1) * ldx + 16u * lh; };
  bf16x8_w xf[kWsKS];
  if (st < s1) {   // the first step's fragments, in flight with the W slice below
    const uint32_t xo = xoff(st);
#pragma unroll
    for (int ks = 0; ks < kWsKS; ++ks) xf[ks] = *reinterpret_cast<const bf16x8_w*>(Xb + xo + 32 * ks);
  }
  // the W slice (rows ng * 192 ..) and its bias into LDS, once: all 18 loads of a thread issued before its stores
  {
    constexpr int kPer = kWsBN * 48 / (kWsWaves * 64);
    static_assert(kPer * kWsWaves * 64 == kWsBN * 48, "whole chunks per thread");
    const uint8_t* Wg = static_cast<const uint8_t*>(p.W) + (int64_t)ng * kWsBN * (kWsK * 2);
    u32x4_w v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) v[i] = *reinterpret_cast<const u32x4_w*>(Wg + (int64_t)(tid + i * kWsWaves * 64) * 16);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int ci = tid + i * kWsWaves * 64, r = ci / 48, c = ci - r * 48;
      *reinterpret_cast<u32x4_w*>(lds + r * kWsRowB + c * 16) = v[i];
    }
    for (int i = tid; i < kWsBN; i += kWsWaves * 64) sbias[i] = p.bias ? p.bias[ng * kWsBN + i] : 0.f;
  }
  __syncthreads();
  if (st >= s1) return;                                            // wave-uniform; no barrier follows
  // A fragments: W row 32 t + lr of the sub-tile, same k range
  const uint8_t* wl = lds + lr * kWsRowB + 16 * lh;

  f32x16_w acc[2][2];                                              // [buffer][n-tile]
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[b][t] = f32x16_w{};

  // output rows of the current and the previous step (the previous step's last sub-tile drains during this
  // step's first): row base pointer, store predicate, folded-RMSNorm factor
  // (every lane stores: a row past M was computed from row M - 1's fragments, so it rewrites row M - 1's values)
  constexpr int kOutB = OBF ? 2 : 4;
  char* __restrict__ Cb = static_cast<char*>(p.C);
  const uint32_t ldcb = (uint32_t)p.ldc * kOutB;
  uint32_t cc = 0, cp = 0;
  float invc = 1.0f, invp = 1.0f;

  // folded-RMSNorm factor from the lane's half-row sum of squares (the two lane halves hold the two halves)
  auto row_factor = [&](float ss) __attribute__((always_inline)) {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(ss), __float_as_uint(ss), false, false);
    const float tot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    return 1.0f / (sqrtf(tot) * p.inv_sqrt_k + kRmsEps);
  };

  // part q (0..3) of sub-tile PJ's epilogue from accumulator buffer b (C row offset cb, row factor inv): the
  // lane's values r = 4q .. 4q+3 of each output n-tile are 4 consecutive columns, stored at once (8 B bf16 /
  // 16 B fp32), so no epilogue value outlives its part
  auto epi_part = [&](auto Bc, auto PJc, int q, uint32_t cb, float inv) __attribute__((always_inline)) {
    constexpr int b = decltype(Bc)::value;
    constexpr int pj = decltype(PJc)::value;
    constexpr int NT = PAIRED ? 1 : 2;                             // output n-tiles of 32 columns
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float o[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int r = 4 * q + rr, n = kWsSubN * pj + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if constexpr (PAIRED) {
          const float gv = fmaf(acc[b][0][r], inv, sbias[n]);
          const float uv = fmaf(acc[b][1][r], inv, sbias[n + 32]);
          if constexpr (OBF) o[rr] = (EPI == EPI_SWIGLU) ? fast_silu(gv) * uv : gv * fast_sigmoid(uv);
          else o[rr] = (EPI == EPI_SWIGLU) ? silu_f(gv) * uv : gv * sigmoid_f(uv);
        } else {
          o[rr] = fmaf(acc[b][t][r], inv, sbias[n]);
        }
      }
      // output columns: PAIRED (64 pj + 8 q + 4 lh) / 2-pair -> 32 pj + 8 q + 4 lh; STORE 64 pj + 32 t + 8 q + 4 lh
      const int col = (PAIRED ? 32 * pj : 64 * pj + 32 * t) + 8 * q + 4 * lh;
      char* cq = Cb + cb + col * kOutB;
      if constexpr (OBF) {
        const u32x2_w w = {pk2(o[0], o[1]), pk2(o[2], o[3])};
        *reinterpret_cast<u32x2_w*>(cq) = w;
      } else {
        *reinterpret_cast<f32x4_w*>(cq) = f32x4_w{o[0], o[1], o[2], o[3]};
      }
    }
  };

  // sub-tile J of the current step into accumulator buffer B while sub-tile (J + 2) % 3 drains from buffer B ^ 1
  // (J = 0: the previous step's last one, none for the first step: F).  J = 0 also sums the rows' squares; J = 2
  // reloads the fragments for the step after (clamped rows: past the wave's last step it reloads valid rows)
  auto sub = [&](auto Bc, auto Jc, auto Fc, uint32_t xn, float& ss) __attribute__((always_inline)) {
    constexpr int b = decltype(Bc)::value;
    constexpr int j = decltype(Jc)::value;
    constexpr bool F = decltype(Fc)::value;
    using PB = std::integral_constant<int, b ^ 1>;
    using PJ = std::integral_constant<int, (j + 2) % 3>;
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[b][t] = f32x16_w{};
    const uint8_t* wj = wl + (kWsSubN * j) * kWsRowB;
    bf16x8_w wa[2], wb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) wa[t] = *reinterpret_cast<const bf16x8_w*>(wj + 32 * t * kWsRowB);
#pragma unroll
    for (int ks = 0; ks < kWsKS; ++ks) {
      bf16x8_w(&cur)[2] = (ks & 1) ? wb : wa;
      bf16x8_w(&nxt)[2] = (ks & 1) ? wa : wb;
      if (ks + 1 < kWsKS) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          nxt[t] = *reinterpret_cast<const bf16x8_w*>(wj + 32 * t * kWsRowB + 32 * (ks + 1));
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if constexpr (DBG & 2) asm volatile("" ::"v"(cur[t]), "v"(xf[ks]));
        else acc[b][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur[t], xf[ks], acc[b][t], 0, 0, 0);
      }
      if constexpr (RS && j == 0) ss = sumsq8(xf[ks], ss);
      // the next step's fragment ks - 1: its last MFMA was issued one K-step (one sched_barrier) ago
      if constexpr (j == 2 && !(DBG & 4)) {
        if (ks > 0) xf[ks - 1] = *reinterpret_cast<const bf16x8_w*>(Xb + xn + 32 * (ks - 1));
      }
      // the previous sub-tile's epilogue, four parts spread over the K-steps
      if constexpr (OVL && !(DBG & 1) && !(F && j == 0)) {
        if (ks % 6 == 3) {
          if constexpr (j == 0) epi_part(PB{}, PJ{}, ks / 6, cp, invp);
          else epi_part(PB{}, PJ{}, ks / 6, cc, invc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep each K-step's reads, MFMAs and epilogue part together
    }
    if constexpr (j == 2 && !(DBG & 4))
      xf[kWsKS - 1] = *reinterpret_cast<const bf16x8_w*>(Xb + xn + 32 * (kWsKS - 1));
    if constexpr (!OVL) {
      if constexpr (RS && j == 0) invc = row_factor(ss);
      if constexpr (!(DBG & 1)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) epi_part(Bc, Jc, q, cc, invc);
      } else {
        asm volatile("" ::"v"(acc[b][0]), "v"(acc[b][1]));   // keep the MFMAs
      }
    }
  };

  // one 32-row step: sub-tiles 0, 1, 2 in buffers P, P ^ 1, P
  auto step = [&](auto Pc, auto Fc) __attribute__((always_inline)) {
    constexpr int P = decltype(Pc)::value;
    using FF = std::integral_constant<bool, false>;
    using B0 = std::integral_constant<int, OVL ? P : 0>;
    using B1 = std::integral_constant<int, OVL ? P ^ 1 : 0>;
    using J0 = std::integral_constant<int, 0>;
    using J1 = std::integral_constant<int, 1>;
    using J2 = std::integral_constant<int, 2>;
    const uint32_t xn = xoff(st + kWsWaves);
    cp = cc; invp = invc;
    cc = (uint32_t)min(32 * st + lr, p.M - 1) * ldcb + (uint32_t)(ng * (PAIRED ? kWsBN / 2 : kWsBN) * kOutB);
    float ss = 0.f;
    sub(B0{}, J0{}, Fc, xn, ss);
    if constexpr (RS && OVL) invc = row_factor(ss);
    sub(B1{}, J1{}, FF{}, xn, ss);
    sub(B0{}, J2{}, FF{}, xn, ss);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using FT = std::integral_constant<bool, true>;
  using FF = std::integral_constant<bool, false>;
  int last = 0;
  step(I0{}, FT{});
  st += kWsWaves;
  while (st < s1) {
    step(I1{}, FF{});
    last = 1;
    st += kWsWaves;
    if (st >= s1) break;
    step(I0{}, FF{});
    last = 0;
    st += kWsWaves;
  }
  // drain: sub-tile 2 of the last step sits in buffer `last`
  using J2 = std::integral_constant<int, 2>;
  if constexpr (!OVL) {
  } else if constexpr (DBG & 1) {   // keep the accumulators alive
    *reinterpret_cast<float*>(Cb + cc) = acc[0][0][0] + acc[1][0][0] + acc[0][1][5] + acc[1][1][7];
  } else if (last == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) epi_part(I0{}, J2{}, q, cc, invc);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) epi_part(I1{}, J2{}, q, cc, invc);
  }
}

template <int EPI, bool OVL>
hipError_t launch_ws(const GemmArgs& a, hipStream_t st) {
  const int gn = a.N / kWsBN, gm = 256 / gn;
  const dim3 grid(256), block(kWsWaves * 64);
#ifdef WS_ABLATE
  if constexpr (EPI == EPI_SWIGLU) {
    switch (a.rowscale && a.c_bf16 ? a.dbg : 0) {
#define WS_D(d) case d: hipLaunchKernelGGL((gemm_ws_kernel<EPI, true, true, d, OVL>), grid, block, 0, st, a, gn, gm); return hipGetLastError();
      WS_D(1) WS_D(2) WS_D(3) WS_D(4) WS_D(5) WS_D(6) WS_D(7)
#undef WS_D
      default: break;
    }
  }
#endif
  if (a.c_bf16) {
    if (a.rowscale) hipLaunchKernelGGL((gemm_ws_kernel<EPI, true, true, 0, OVL>), grid, block, 0, st, a, gn, gm);
    else hipLaunchKernelGGL((gemm_ws_kernel<EPI, false, true, 0, OVL>), grid, block, 0, st, a, gn, gm);
  } else {
    if (a.rowscale) hipLaunchKernelGGL((gemm_ws_kernel<EPI, true, false, 0, OVL>), grid, block, 0, st, a, gn, gm);
    else hipLaunchKernelGGL((gemm_ws_kernel<EPI, false, false, 0, OVL>), grid, block, 0, st, a, gn, gm);
  }
  return hipGetLastError();
}

}  // namespace

// variant 0: epilogue after each sub-tile (no spills); 1: double-buffered accumulators (spills a few registers)
hipError_t gemm_ws(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  if (!a.a_bf16 || a.K != kWsK || a.N % kWsBN || a.N / kWsBN > 256 || a.M <= 0 || a.rpg || a.lda % 8 ||
      a.ldc % 8 || a.k_split || a.C2 || a.c_plane || (int64_t)a.M * a.lda * 2 >= (1ll << 32) ||
      (int64_t)a.M * a.ldc * (a.c_bf16 ? 2 : 4) >= (1ll << 32))
    return hipErrorInvalidValue;
  const bool ovl = variant == 1;
  switch (epi) {
    case EPI_SWIGLU: return ovl ? launch_ws<EPI_SWIGLU, true>(a, st) : launch_ws<EPI_SWIGLU, false>(a, st);
    case EPI_GLU: return ovl ? launch_ws<EPI_GLU, true>(a, st) : launch_ws<EPI_GLU, false>(a, st);
    case EPI_STORE: return ovl ? launch_ws<EPI_STORE, true>(a, st) : launch_ws<EPI_STORE, false>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
