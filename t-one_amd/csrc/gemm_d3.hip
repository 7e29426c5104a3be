// fp32 mode (BASELINE config 2): the N = 384 projections of the small-M layers (attn-out, pw2, FFN down and the
// reduction's 1x1 at M = B T = 65 .. 4096) and pw1 with the operands read straight into registers -- no LDS staging of
// operands at all.
//
// gemm_x3 stages W's three bf16 planes and the fp32 X rows through an LDS-DMA ring paced by workgroup barriers; at
// these shapes a launch is 240-480 workgroups of a few K-steps each and that fill (~30-40 GB/s per CU) bounds it,
// while the XCD's L2 serves plain vector loads at several times that rate (MI355X_MICROARCH.md, L2 ~34.5 TB/s).
// gemm_d3: each wave owns one 32 x 32 output tile (or a 1/WK share of its K range) and loads, per pair of 16-deep
// K-steps, its X fragment (lane l: row m0 + (l & 31), 8 fp32 at K offset 8 (l >> 5) of each step, 4 x 16 B) and its W
// fragments (lane l: row n0 + (l & 31) of each bf16 plane, 8 values of each step, 6 x 16 B) D pairs ahead of their use,
// both fragment-packed (common.h xpk_off / wpk_off: each load instruction reads 1 KiB contiguous; row-major X, 32 row
// segments per instruction, measured 1.5-2x slower: profiles/r06_d3_probe.jsonl); X is split into its three bf16 terms
// in registers (split3, as gemm_x3) and each K-step takes gemm_x3's six products in gemm_x3's order (small terms
// first), so the arithmetic is gemm_x3's.  W (the 884 KiB of planes of a 384 x 384 layer) stays L2-resident; the
// workgroups that share X rows are dealt to one XCD.  With WK > 1 the K range is split over the workgroup's waves and
// the partials are added in LDS in a fixed order.  The epilogue is gemm_x3's (tile_epilogue), including the optional
// packed copy of C (GemmArgs::CP) that pw1 reads.
// gemm_d3n: the same per-wave stream with NT W tiles per wave and the folded-norm row factor (pw1's GLU).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

namespace tone {
namespace {

template <int WM, int WN, int WK, int D, int EPI, bool XP>
__global__ void __launch_bounds__(256) gemm_d3_kernel(GemmArgs p) {
  static_assert(WM * WN * WK == 4, "four waves per workgroup");
  constexpr int NWT = WM * WN;                      // output tiles per workgroup
  __shared__ float red[(WK > 1 ? (WK - 1) * NWT : 1) * 64 * 16];
  __shared__ float sbias[32 * WN];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wk = wid / NWT, wt = wid % NWT, wm = wt / WN, wn = wt % WN;
  const int nbn = p.N / (32 * WN), nbm = (p.M + 32 * WM - 1) / (32 * WM), total = nbn * nbm;
  int b = blockIdx.x;
  if ((total & 7) == 0) b = (b & 7) * (total >> 3) + (b >> 3);   // XCD b % 8: a contiguous run, the same X rows
  const int bm = b / nbn, bn = b % nbn;
  const int m0 = bm * 32 * WM + 32 * wm, n0 = bn * 32 * WN + 32 * wn;
  const int kpt = p.K / 32, kp = kpt / WK;          // K-step pairs in all / per wave
  if (tid < 32 * WN) sbias[tid] = p.bias ? p.bias[bn * 32 * WN + tid] : 0.0f;

  // X: packed, the 4 KiB block (row block, pair) read as four 1 KiB chunks; row-major (XP false), lane (h, r) reads row
  // m0 + r at columns 32 pair + 16 e + 8 h (4 x 16 B, 32 rows per instruction: slower, measured)
  const float* xr;
  int xs, xe, xo;
  if constexpr (XP) {
    // a wave whose 32 rows all lie past M (the grid's last workgroup) reads the last row block instead: its outputs
    // are all masked, and the packed buffer holds only ceil(M / 32) blocks
    xr = static_cast<const float*>(p.A) + ((int64_t)(min(m0, (p.M - 1) & ~31) >> 5) * kpt + wk * kp) * 1024 + lane * 4;
    xs = 1024; xe = 512; xo = 256;
  } else {
    xr = static_cast<const float*>(p.A) + (int64_t)min(m0 + lr, p.M - 1) * p.lda + wk * kp * 32 + 8 * lh;
    xs = 32; xe = 16; xo = 4;
  }
  // W: packed planes (common.h wpk_off), 6 KiB per (row block, pair)
  const uint16_t* wr = p.W3P + ((int64_t)(n0 >> 5) * kpt + wk * kp) * 3072 + lane * 8;

  f32x4 xb[D][4];
  u32x4 wb[D][3][2];
  // the loads of pair pp + D - 1 are issued while pair pp is consumed; the offsets pass through an empty asm so that the
  // compiler cannot prove a slot's value equal to a load of the current iteration (it then folded the pipeline back into
  // load-then-use), and offsets rather than pointers, which would lose their address space (flat loads)
  auto load = [&](int slot, int pp) {
    int ox = xs * pp, ow = 3072 * pp;
    asm volatile("" : "+s"(ox), "+s"(ow));
    const float* x = xr + ox;
    const uint16_t* w = wr + ow;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      xb[slot][2 * e] = *reinterpret_cast<const f32x4*>(x + xe * e);
      xb[slot][2 * e + 1] = *reinterpret_cast<const f32x4*>(x + xe * e + xo);
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) wb[slot][c >> 1][c & 1] = *reinterpret_cast<const u32x4*>(w + 512 * c);
  };

  f32x16 acc[1][1];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.0f;
#pragma unroll
  for (int j = 0; j < D - 1; ++j) load(j, min(j, kp - 1));
  for (int p0 = 0; p0 < kp; p0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      load((j + D - 1) % D, min(p0 + j + D - 1, kp - 1));   // the tail re-reads the last pair (an L1 hit), no branch
      __builtin_amdgcn_sched_barrier(0);                     // issued here, ahead of this pair's MFMAs
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        bf16x8 x0, x1, x2;
        split3(xb[j][2 * e], xb[j][2 * e + 1], x0, x1, x2);
        const bf16x8 w0 = __builtin_bit_cast(bf16x8, wb[j][0][e]);
        const bf16x8 w1 = __builtin_bit_cast(bf16x8, wb[j][1][e]);
        const bf16x8 w2 = __builtin_bit_cast(bf16x8, wb[j][2][e]);
        f32x16 a = acc[0][0];   // small terms first (gemm_x3's order)
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, x0, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x1, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x2, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x0, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x1, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x0, a, 0, 0, 0);
        acc[0][0] = a;
      }
    }
  }
  if constexpr (WK > 1) {
    if (wk > 0) {
      float* dst = red + ((wk - 1) * NWT + wt) * 64 * 16;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64 + lane] = acc[0][0][r];
    }
  }
  __syncthreads();   // sbias written; K-split partials in LDS
  if constexpr (WK > 1) {
    if (wk > 0) return;
#pragma unroll
    for (int g = 1; g < WK; ++g) {   // partials added in K order
      const float* src = red + ((g - 1) * NWT + wt) * 64 * 16;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][0][r] += src[r * 64 + lane];
    }
  }
  if (p.dbg & 8) return;   // microbenchmark: no epilogue
  const float inv1[1] = {1.0f};
  // D tile (n, m) = (W row, X row): gemm_x3's orientation, so its epilogue (wave tile 32 x 32 at this wave's m0 / n0)
  tile_epilogue_inv<EPI, false, 1, 1, 32, 32>(p, acc, inv1, sbias + 32 * wn, m0, n0, 0, 0, lr, lh);
}

// The wide form for the rowscale projections (FFN up SwiGLU, pw1 GLU, q|k|v): each wave owns NT 32-column W tiles of
// one 32-row X block, so one X fragment feeds NT x 6 products; the folded RMSNorm's row factor from the same X values
// (gemm_x3's formula); SWIGLU / GLU take the tiles in (g, u) pairs -- the session's 32-row interleave -- through
// gemm_x3's epilogue.  XP: X fragment-packed as in gemm_d3_kernel (the session's form: the residual stream's producers
// write a packed copy, GemmArgs::CP / rmsnorm / upsample_add), else row-major (SWIGLU only: measured ~5 % ahead of
// gemm_x3 at best, profiles/r06_d3n_sweep.jsonl, not routed).
template <int WM, int WN, int NT, int D, int EPI, bool RS, bool XP>
__global__ void __launch_bounds__(256) gemm_d3n_kernel(GemmArgs p) {
  static_assert(WM * WN == 4, "four waves per workgroup");
  static_assert((EPI != EPI_SWIGLU && EPI != EPI_GLU) || NT % 2 == 0, "paired epilogues take (g, u) tile pairs");
  __shared__ float sbias[32 * WN * NT];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wm = wid / WN, wn = wid % WN;
  const int nbn = p.N / (32 * WN * NT), nbm = (p.M + 32 * WM - 1) / (32 * WM), total = nbn * nbm;
  int b = blockIdx.x;
  if ((total & 7) == 0) b = (b & 7) * (total >> 3) + (b >> 3);   // XCD b % 8: a contiguous run, the same X rows
  const int bm = b / nbn, bn = b % nbn;
  const int m0 = bm * 32 * WM + 32 * wm, nw0 = bn * 32 * WN * NT, n0 = nw0 + 32 * NT * wn;
  const int kpt = p.K / 32;
  for (int t = tid; t < 32 * WN * NT; t += 256) sbias[t] = p.bias ? p.bias[nw0 + t] : 0.0f;

  const float* xr;
  int xs, xe, xo;
  if constexpr (XP) {
    xr = static_cast<const float*>(p.A) + (int64_t)(min(m0, (p.M - 1) & ~31) >> 5) * kpt * 1024 + lane * 4;
    xs = 1024; xe = 512; xo = 256;
  } else {
    xr = static_cast<const float*>(p.A) + (int64_t)min(m0 + lr, p.M - 1) * p.lda + 8 * lh;
    xs = 32; xe = 16; xo = 4;
  }
  const uint16_t* wr = p.W3P + (int64_t)(n0 >> 5) * kpt * 3072 + lane * 8;
  const int64_t wnt = (int64_t)kpt * 3072;   // elements from one 32-row W block to the next

  f32x4 xb[D][4];
  u32x4 wb[D][NT][6];
  auto load = [&](int slot, int pp) {   // as gemm_d3_kernel's
    int ox = xs * pp, ow = 3072 * pp;
    asm volatile("" : "+s"(ox), "+s"(ow));
    const float* x = xr + ox;
    const uint16_t* w = wr + ow;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      xb[slot][2 * e] = *reinterpret_cast<const f32x4*>(x + xe * e);
      xb[slot][2 * e + 1] = *reinterpret_cast<const f32x4*>(x + xe * e + xo);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int c = 0; c < 6; ++c) wb[slot][t][c] = *reinterpret_cast<const u32x4*>(w + t * wnt + 512 * c);
  };

  f32x16 acc[NT][1];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][0][r] = 0.0f;
  float ss = 0.0f;
#pragma unroll
  for (int j = 0; j < D - 1; ++j) load(j, min(j, kpt - 1));
  for (int p0 = 0; p0 < kpt; p0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      load((j + D - 1) % D, min(p0 + j + D - 1, kpt - 1));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x4 a = xb[j][2 * e], c = xb[j][2 * e + 1];
        if constexpr (RS) {
          ss = fmaf(a.x, a.x, ss); ss = fmaf(a.y, a.y, ss); ss = fmaf(a.z, a.z, ss); ss = fmaf(a.w, a.w, ss);
          ss = fmaf(c.x, c.x, ss); ss = fmaf(c.y, c.y, ss); ss = fmaf(c.z, c.z, ss); ss = fmaf(c.w, c.w, ss);
        }
        bf16x8 x0, x1, x2;
        split3(a, c, x0, x1, x2);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 w0 = __builtin_bit_cast(bf16x8, wb[j][t][e]);
          const bf16x8 w1 = __builtin_bit_cast(bf16x8, wb[j][t][2 + e]);
          const bf16x8 w2 = __builtin_bit_cast(bf16x8, wb[j][t][4 + e]);
          f32x16 v = acc[t][0];   // small terms first (gemm_x3's order)
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, x0, v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x1, v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x2, v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, x0, v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x1, v, 0, 0, 0);
          v = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, x0, v, 0, 0, 0);
          acc[t][0] = v;
        }
      }
    }
  }
  float invj[1] = {1.0f};
  if constexpr (RS) {   // gemm_x3's row factor: 1 / (||x|| / sqrt(K) + eps), the two lane halves' squares added
    const float t = ss + __shfl_xor(ss, 32, 64);
    invj[0] = 1.0f / (sqrtf(t) * p.inv_sqrt_k + kRmsEps);
  }
  __syncthreads();   // sbias
  if (p.dbg & 8) return;
  tile_epilogue_inv<EPI, RS, NT, 1, 32 * NT, 32>(p, acc, invj, sbias + 32 * NT * wn, m0, n0, 0, 0, lr, lh);
}

template <int WM, int WN, int NT, int D, int EPI, bool XP>
hipError_t launch_d3n_e(const GemmArgs& a, hipStream_t st) {
  const int nbn = a.N / (32 * WN * NT), nbm = (a.M + 32 * WM - 1) / (32 * WM);
  if (a.rowscale) hipLaunchKernelGGL((gemm_d3n_kernel<WM, WN, NT, D, EPI, true, XP>), dim3(nbn * nbm), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gemm_d3n_kernel<WM, WN, NT, D, EPI, false, XP>), dim3(nbn * nbm), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int WM, int WN, int NT, int D>
hipError_t launch_d3n(const GemmArgs& a, int epi, hipStream_t st) {
  if (a.N % (32 * WN * NT) != 0 || (a.K / 32) % D != 0) return hipErrorInvalidValue;
  if (!a.a_packed) return hipErrorInvalidValue;   // row-major A: ~5 % ahead of gemm_x3 at best, not kept
  if (epi == EPI_SWIGLU) return launch_d3n_e<WM, WN, NT, D, EPI_SWIGLU, true>(a, st);
  if (epi == EPI_GLU) return launch_d3n_e<WM, WN, NT, D, EPI_GLU, true>(a, st);
  if (epi == EPI_STORE) return launch_d3n_e<WM, WN, NT, D, EPI_STORE, true>(a, st);
  return hipErrorInvalidValue;
}

template <int WM, int WN, int WK, int D>
hipError_t launch_d3(const GemmArgs& a, int epi, hipStream_t st) {
  if (a.N % (32 * WN) != 0 || a.K % (32 * WK) != 0 || (a.K / (32 * WK)) % D != 0) return hipErrorInvalidValue;
  const int nbn = a.N / (32 * WN), nbm = (a.M + 32 * WM - 1) / (32 * WM);
  const dim3 grid(nbn * nbm), block(256);
  if (a.a_packed) {
    if (epi == EPI_RESID) hipLaunchKernelGGL((gemm_d3_kernel<WM, WN, WK, D, EPI_RESID, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_d3_kernel<WM, WN, WK, D, EPI_STORE, true>), grid, block, 0, st, a);
  } else {
    if (epi == EPI_RESID) hipLaunchKernelGGL((gemm_d3_kernel<WM, WN, WK, D, EPI_RESID, false>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_d3_kernel<WM, WN, WK, D, EPI_STORE, false>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace

bool gemm_d3_routed(int M, int K, int N) {
  return N == kD && (K == kD || K == kDff) && M > 64 && M <= 4096 && knobs().d3;
}

hipError_t gemm_d3(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  if (!a.W3P || !a.A || a.a_bf16 || a.c_bf16 || a.rowscale || a.rpg || a.a_plane || a.c_plane || a.res16 || a.C8 ||
      a.norm_w || a.h_blocked || a.c_packed || (epi != EPI_STORE && epi != EPI_RESID) || a.lda % 4 != 0 ||
      a.ldc % 4 != 0 || a.M <= 0 || (a.a_packed && a.lda != a.K))
    return hipErrorInvalidValue;
  if (variant < 0) {
    // by shape (scripts/d3_sweep.sh, profiles/r06_d3_sweep.jsonl, N = 384; the headline's two heights confirmed in the
    // step, profiles/step_r06_d3*_fp32_b256.txt): one 32 x 32 tile per workgroup with K split over its four waves (7)
    // wherever that many waves fit -- M = 100 .. 640, 1536 / 3328 (400 ms): 4.6-5.0 / 8.0-9.6 us at K = 384 / 1536
    // against 7.6-8.1 / 15.7-17.9 for gemm_x3 at M <= 640; two tiles with K split in two (3) at M = 1280 (6.7 / 14.2 vs
    // 8.8 / 20.0); four tiles, no split (4) at M = 2560 (10.1 / 23.2 vs 12.5 / 32.9).  In the fp32 B = 256 step (3)+(4)
    // took 945 us per step against 998 for the microbenchmark's per-shape best ((6) / (8): 9.8 / 23.1)
    if (a.M > 1024 && a.M <= 1280) variant = 3;
    else if (a.M > 2048 && a.M <= 3072) variant = 4;
    else variant = 7;
    static const int force = [] {
      const char* e = std::getenv("TONE_D3_V");   // experiments only: one variant for every shape
      return e && *e ? std::atoi(e) : -1;
    }();
    if (force >= 0) variant = force;
  }
  switch (variant) {
    case 0: return launch_d3<4, 1, 1, 4>(a, epi, st);
    case 1: return launch_d3<2, 2, 1, 4>(a, epi, st);
    case 2: return launch_d3<1, 4, 1, 4>(a, epi, st);
    case 3: return launch_d3<2, 1, 2, 3>(a, epi, st);
    case 4: return launch_d3<4, 1, 1, 3>(a, epi, st);
    case 5: return launch_d3<4, 1, 1, 6>(a, epi, st);
    case 6: return launch_d3<1, 2, 2, 3>(a, epi, st);
    case 7: return launch_d3<1, 1, 4, 3>(a, epi, st);
    case 8: return launch_d3<2, 2, 1, 6>(a, epi, st);
    case 9: return launch_d3<2, 1, 2, 6>(a, epi, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t gemm_d3n(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  if (!a.W3P || !a.A || a.a_bf16 || a.c_bf16 || a.rpg || a.a_plane || a.c_plane || a.res16 || a.C2 || a.C8 ||
      a.norm_w || a.h_blocked || (a.c_packed && epi != EPI_SWIGLU) || a.K % 32 != 0 || a.lda % 4 != 0 ||
      a.ldc % 4 != 0 || a.M <= 0 || (a.a_packed && a.lda != a.K))
    return hipErrorInvalidValue;
  // by shape (scripts/d3n_sweep.sh, profiles/r06_d3n_packed_sweep.jsonl, A packed, K = 384; in the step only pw1
  // gains, session.hip): four W tiles per wave over four row blocks (3) for FFN up (M = 2560 / 1280: 43.2 / 23.8 vs
  // 49.0 / 26.9 us on gemm_x3) and q|k|v at M >= 2048 (21.4 vs 24.9); two (2) for pw1 (14.6 / 13.0 vs 17.2 / 14.8) and
  // the rest (q|k|v at 1280: 13.7 vs 15.7)
  if (variant < 0) variant = (epi == EPI_SWIGLU || (a.N >= 1024 && a.M >= 2048)) ? 3 : 2;
  switch (variant) {   // the sweep's other arrangements (2 x 2 / 1 x 4 waves) were slower on every shape
    case 2: return launch_d3n<4, 1, 2, 3>(a, epi, st);
    case 3: return launch_d3n<4, 1, 4, 2>(a, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
