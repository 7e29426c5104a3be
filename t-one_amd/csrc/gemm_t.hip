// Persistent bf16 GEMM for the large-batch encoder projections, computed in the transposed
// orientation  D[n][m] = W[n][:] . X[m][:]  (n = output feature, m = frame row of the batch).
//
// Why transposed: in the v_mfma_f32_32x32x16_bf16 D layout each lane owns one column (here: one
// frame row m) and 4-element runs of rows (here: 4 consecutive output features), so the epilogue
// holds whole 8-byte bf16 / 16-byte fp32 runs of an output row per lane.  A v_permlane32_swap pair
// widens the bf16 runs to 16-byte stores.  The folded RMSNorm row scale is one value per lane.
//
// Structure (MI355X, one 8-wave workgroup per CU, 2 waves per SIMD):
//   * tile BNW x BMX (256 x 256 for the FFN up-projection, 128 x 256 for N = 384), BK = 64;
//   * both operands staged into LDS by global_load_lds_dwordx4 (1 KiB per wave instruction =
//     8 rows x 128 B), two 64 KiB stages, the DMA of K-step g+1 in flight while the MFMAs of
//     K-step g run; the XOR swizzle slot ^= (row >> 1) & 7 (applied to the per-lane SOURCE address)
//     makes every ds_read_b128 fragment read conflict-free for the 32x32x16 lane map;
//   * persistent over tiles: the K-step ring runs across tile boundaries, so the first K-step of
//     tile t+1 is already in LDS when tile t's epilogue runs (no per-tile prologue bubble);
//     tiles are dealt XCD-contiguously (an XCD's 32 CUs walk neighbouring tiles: the X row block
//     is fetched into that XCD's L2 once and reused by every N-tile);
//   * the bias vector lives in LDS for the whole launch and the row scales go through LDS, so the
//     epilogue issues no global load that would make hipcc drain the in-flight LDS-DMA.
// Epilogues (reference ops, see gemm.hip): STORE (+bias, bf16 out), RESID (fp32 R + alpha*(.),
// fp32 out + bf16 shadow), SWIGLU / GLU on W rows interleaved in 32-row blocks.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

#include "gemm_common.h"

namespace tone {
namespace {

template <class TL, int EPI, bool RS>
__global__ void __launch_bounds__(TL::WN * TL::WM * 64) gemm_t_kernel(GemmArgs p) {
  constexpr int BNW = TL::BNW, BMX = TL::BMX, WN = TL::WN, WM = TL::WM, NW = WN * WM, NT = NW * 64;
  constexpr int BK = 64, WTN = BNW / WN, WTM = BMX / WM, TI = WTN / 32, TJ = WTM / 32;
  constexpr int WP = BNW / 8 / NW, XP = BMX / 8 / NW;          // DMA wave-instructions per stage
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU);
  static_assert(WP >= 1 && XP >= 1 && BNW % (8 * NW) == 0 && BMX % (8 * NW) == 0, "tile/wave mismatch");
  static_assert(TI >= 1 && TJ >= 1, "wave tile >= 32x32");
  static_assert(!PAIRED || (TI % 2 == 0), "paired epilogues pair 32-row W blocks");
  static_assert(EPI == EPI_STORE || EPI == EPI_RESID || PAIRED, "STORE/RESID/SWIGLU/GLU");
  constexpr int STAGE = (BNW + BMX) * BK;                       // bf16 elements per stage
  // ONE LDS object: [2 stages][W rows | X rows][64] bf16, rden [2][BMX] fp32, bias [kBiasMax] fp32
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * STAGE + 2 * (2 * BMX) + 2 * kBiasMax];
  float* rden = reinterpret_cast<float*>(lds + 2 * STAGE);
  float* sbias = rden + 2 * BMX;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / WM, wm = wid % WM;
  const int lr = lane & 31, lh = lane >> 5, cs = (lr >> 1) & 7;
  const int ntn = p.N / BNW, ntm = (p.M + BMX - 1) / BMX, ntiles = ntn * ntm;
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (ntiles + 7) >> 3, tbeg = xcd * q, tend = min(ntiles, tbeg + q);
  const int nmine = (tbeg + jb < tend) ? (tend - tbeg - jb + nxb - 1) / nxb : 0;
  if (nmine <= 0) return;                                       // workgroup-uniform
  const int nk = p.K / BK, G = nmine * nk;
  const uint16_t* __restrict__ X = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);
  constexpr bool rs_on = RS;

  for (int i = tid; i < p.N; i += NT) sbias[i] = p.bias ? p.bias[i] : 0.f;
  __syncthreads();                                              // no DMA in flight yet

  auto tile_of = [&](int g, int& m0, int& n0) {
    const int t = tbeg + jb + (g / nk) * nxb;
    m0 = (t / ntn) * BMX;
    n0 = (t % ntn) * BNW;
  };
  auto stage = [&](int buf, int g) {
    int m0, n0;
    tile_of(g, m0, n0);
    const int k0 = (g % nk) * BK;
    uint16_t* base = lds + buf * STAGE;
    (void)base;
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int piece = wid + i * NW, row = piece * 8 + (lane >> 3);
      const uint16_t* src = W + (int64_t)(n0 + row) * p.K + k0 + (((lane & 7) ^ ((row >> 1) & 7)) << 3);
      lds_dma16(src, base + piece * 8 * BK);
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int piece = wid + i * NW, row = piece * 8 + (lane >> 3);
      const int gm = min(m0 + row, p.M - 1);
      const uint16_t* src = X + (int64_t)gm * p.lda + k0 + (((lane & 7) ^ ((row >> 1) & 7)) << 3);
      lds_dma16(src, base + (BNW + piece * 8) * BK);
    }
  };

  f32x16 acc[TI][TJ];
  float ss[TJ];
  auto zero = [&]() {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      ss[j] = 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
  };

  // One K-step on LDS buffer buf: every fragment of the step is read first (one counted LDS
  // wait per slice), then the MFMAs.
  auto compute = [&](int buf) {
    const uint16_t* base = lds + buf * STAGE;
    bf16x8 fa[BK / 16][TI], fb[BK / 16][TJ];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int off = ((2 * ks + lh) ^ cs) << 3;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        fb[ks][j] = *reinterpret_cast<const bf16x8*>(base + (BNW + wm * WTM + 32 * j + lr) * BK + off);
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[ks][i] = *reinterpret_cast<const bf16x8*>(base + (wn * WTN + 32 * i + lr) * BK + off);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs (hipcc sinks them to their uses)
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
      if constexpr (RS) {   // m-tile (wn % TJ)'s sum of squares (branch-free select on the uniform wn)
        bf16x8 bs = fb[ks][0];
#pragma unroll
        for (int j = 1; j < TJ; ++j) bs = (wn % TJ == j) ? fb[ks][j] : bs;
        ss[0] = sumsq8(bs, ss[0]);
      }
    }
  };

  auto epilogue = [&](int m0, int n0, const float* rd) {
    tile_epilogue<EPI, RS, TI, TJ, WTN, WTM>(p, acc, rd, sbias + n0, m0, n0, wn, wm, lr, lh);
  };

  auto publish_rden = [&](int par) {   // last K-step of a tile: row-scale denominators -> LDS
    const float t = ss[0] + __shfl_xor(ss[0], 32, 64);
    if (wn < TJ && lh == 0) rden[par * BMX + wm * WTM + 32 * (wn % TJ) + lr] = sqrtf(t) * p.inv_sqrt_k + kRmsEps;
  };

  zero();
  stage(0, 0);
  for (int g = 0; g < G; ++g) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stage g landed (and the last epilogue's stores)
    barrier_lds();                                      // ... for every wave; buffer (g+1)&1 is free
    if (g > 0 && g % nk == 0) {                         // previous tile done: its epilogue first
      int m0, n0;
      tile_of(g - 1, m0, n0);
      if (!(p.dbg & 1)) epilogue(m0, n0, rden + ((g / nk - 1) & 1) * BMX);
      zero();
    }
    if (g + 1 < G && !(p.dbg & 4)) stage((g + 1) & 1, g + 1);
    if (!(p.dbg & 2)) compute(g & 1);
    if (rs_on && g % nk == nk - 1) publish_rden((g / nk) & 1);
  }
  barrier_lds();
  {
    int m0, n0;
    tile_of(G - 1, m0, n0);
    if (!(p.dbg & 1)) epilogue(m0, n0, rden + ((G / nk - 1) & 1) * BMX);
    else if (acc[0][0][0] == 1234.5f) static_cast<float*>(p.C)[tid] = acc[TI - 1][TJ - 1][15];   // keep the MFMAs
  }
}

// ---------------------------------------------------------------------------------------------
// Two workgroups per CU: 4 waves (2 n x 2 m), tile BNW x BMX (256 x 128: wave tile 128 x 64),
// BK = 32 (64-byte LDS rows, swizzle slot ^= (row >> 2) & 3, conflict-free for the 32x32x16
// fragment reads), three LDS-DMA stages (two K-steps in flight).  One tile per workgroup; the two
// co-resident workgroups drift out of phase, so one's epilogue VALU and DMA waits overlap the
// other's MFMAs.  LDS per workgroup: 3 x 24 KiB stages + 1 KiB bias + 0.5 KiB row scales.
template <class TL, int EPI, bool RS>
__global__ void __launch_bounds__(256) gemm_t2_kernel(GemmArgs p) {
  constexpr int BNW = TL::BNW, BMX = TL::BMX, WN = TL::WN, WM = TL::WM, NW = WN * WM, NT = NW * 64;
  constexpr int BK = 32, S = 3, WTN = BNW / WN, WTM = BMX / WM, TI = WTN / 32, TJ = WTM / 32;
  constexpr int WP = BNW / 16 / NW, XP = BMX / 16 / NW, IPS = WP + XP;    // DMA wave-instructions per stage
  static_assert(NW == 4 && WP >= 1 && XP >= 1 && BNW % (16 * NW) == 0 && BMX % (16 * NW) == 0, "tile/wave mismatch");
  static_assert(WN >= TJ, "row-scale ownership: one m-tile per wave");
  constexpr int STAGE = (BNW + BMX) * BK;
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * STAGE + 2 * BNW + 2 * BMX];
  float* sbias = reinterpret_cast<float*>(lds + S * STAGE);
  float* rden = sbias + BNW;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / WM, wm = wid % WM;
  const int lr = lane & 31, lh = lane >> 5, cs = (lr >> 2) & 3;
  const int ntn = p.N / BNW;
  int wgid = blockIdx.x;
  {   // XCD-aware bijective remap: consecutive tiles (same X rows, all N-tiles) share an XCD's L2
    const int nwg = gridDim.x, xcd = wgid & 7, q = nwg >> 3, rr = nwg & 7;
    wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (wgid >> 3);
  }
  const int m0 = (wgid / ntn) * BMX, n0 = (wgid % ntn) * BNW;
  const int nk = p.K / BK;
  const uint16_t* __restrict__ X = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);

  for (int i = tid; i < BNW; i += NT) sbias[i] = p.bias ? p.bias[n0 + i] : 0.f;
  __syncthreads();                                              // before any DMA is in flight

  auto stage = [&](int buf, int kt) {
    const int k0 = kt * BK;
    uint16_t* base = lds + buf * STAGE;
    (void)base;
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int piece = wid + i * NW, row = piece * 16 + (lane >> 2);
      const uint16_t* src = W + (int64_t)(n0 + row) * p.K + k0 + (((lane & 3) ^ ((row >> 2) & 3)) << 3);
      lds_dma16(src, base + piece * 16 * BK);
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int piece = wid + i * NW, row = piece * 16 + (lane >> 2);
      const int gm = min(m0 + row, p.M - 1);
      const uint16_t* src = X + (int64_t)gm * p.lda + k0 + (((lane & 3) ^ ((row >> 2) & 3)) << 3);
      lds_dma16(src, base + (BNW + piece * 16) * BK);
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float ss = 0.f;

  auto compute = [&](int buf) {
    const uint16_t* base = lds + buf * STAGE;
    bf16x8 fa[BK / 16][TI], fb[BK / 16][TJ];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int off = ((2 * ks + lh) ^ cs) << 3;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        fb[ks][j] = *reinterpret_cast<const bf16x8*>(base + (BNW + wm * WTM + 32 * j + lr) * BK + off);
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[ks][i] = *reinterpret_cast<const bf16x8*>(base + (wn * WTN + 32 * i + lr) * BK + off);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks][i], fb[ks][j], acc[i][j], 0, 0, 0);
      if constexpr (RS) {
        bf16x8 bs = fb[ks][0];
#pragma unroll
        for (int j = 1; j < TJ; ++j) bs = (wn % TJ == j) ? fb[ks][j] : bs;
        ss = sumsq8(bs, ss);
      }
    }
  };

  stage(0, 0);
  if (nk > 1) stage(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPS) : "memory");   // stage kt landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();                        // visible to all waves; buffer (kt + 2) % S is free
    if (kt + 2 < nk) stage((kt + 2) % S, kt + 2);
    compute(kt % S);
  }
  if constexpr (RS) {
    const float t = ss + __shfl_xor(ss, 32, 64);
    if (wn < TJ && lh == 0) rden[wm * WTM + 32 * (wn % TJ) + lr] = sqrtf(t) * p.inv_sqrt_k + kRmsEps;
    barrier_lds();
  }
  tile_epilogue<EPI, RS, TI, TJ, WTN, WTM>(p, acc, rden, sbias, m0, n0, wn, wm, lr, lh);
}

// ---------------------------------------------------------------------------------------------
// fp32 projections with few output tiles (N = 384..1152 at B = 256: M = 2560 / 1280 frame rows).
// Exact-fp32 MFMA (v_mfma_f32_32x32x2_f32), transposed orientation like above, one 32x32 (or
// 32x64) accumulator tile per wave and the K range split over WK wave groups INSIDE the workgroup
// (partials reduced through LDS at the end) -- enough waves for 1024 SIMDs without a split-K
// workspace round trip or a second kernel.  K-step = WK x 32: each group's 32-float (128-byte) row
// slice is its own region of the stage, filled by LDS-DMA with the same slot swizzle as the bf16
// kernels (fragment reads: lane (row r, half h) takes float4 slot 2q + h, q = 0..3; both operands
// use the same k permutation, so the 4 MFMAs per float4 pair sum the right products).
template <int BNW_, int BMX_, int WN_, int WM_, int WK_>
struct FT {
  static constexpr int BNW = BNW_, BMX = BMX_, WN = WN_, WM = WM_, WK = WK_;
};

template <class TL, int EPI, bool RS, bool BF, bool R16 = false>
__global__ void __launch_bounds__(TL::WN * TL::WM * TL::WK * 64) gemm_f32t_kernel(GemmArgs p) {
  constexpr int BNW = TL::BNW, BMX = TL::BMX, WN = TL::WN, WM = TL::WM, WK = TL::WK;
  constexpr int NW = WN * WM * WK, NT = NW * 64, S = 3;
  constexpr int WTN = BNW / WN, WTM = BMX / WM, TI = WTN / 32, TJ = WTM / 32;
  using E = typename std::conditional<BF, uint16_t, float>::type;   // operand element (bf16 bits / fp32)
  constexpr int EPR = 128 / (int)sizeof(E);                     // elements per 128-byte row slice = K per group
  constexpr int EPS = 16 / (int)sizeof(E);                      // elements per 16-byte slot
  constexpr int GROUP = (BNW + BMX) * 32;                       // floats (= 128-byte rows) of one k-group's slice
  constexpr int STAGE = WK * GROUP;
  constexpr int PIECES = WK * (BNW + BMX) / 8, IPW = PIECES / NW;  // 1 KiB DMA instructions
  static_assert(PIECES % NW == 0 && IPW >= 1, "DMA pieces per wave");
  static_assert(WN >= TJ, "row-scale ownership");
  constexpr int RED = (WK - 1) * (NW / WK) * 64 * TI * TJ * 16;   // K-split partials (floats)
  constexpr int LDSF = (S * STAGE > RED ? S * STAGE : RED);
  __shared__ __attribute__((aligned(16))) float lds[LDSF + BNW + BMX + (WK - 1) * (NW / WK) * 64];
  float* sbias = lds + LDSF;
  float* rden = sbias + BNW;
  float* ssr = rden + BMX;                                      // K-split row sums of squares

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid / (WN * WM), wr = wid % (WN * WM), wn = wr / WM, wm = wr % WM;
  const int lr = lane & 31, lh = lane >> 5, cs = (lr >> 1) & 7;
  const int ntn = p.N / BNW;
  int wgid = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = wgid & 7, q = nwg >> 3, rr = nwg & 7;
    wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (wgid >> 3);
  }
  const int m0 = (wgid / ntn) * BMX, n0 = (wgid % ntn) * BNW;
  const int nk = p.K / (EPR * WK);
  const E* __restrict__ X = static_cast<const E*>(p.A);
  const E* __restrict__ W = static_cast<const E*>(p.W);

  for (int i = tid; i < BNW; i += NT) sbias[i] = p.bias ? p.bias[n0 + i] : 0.f;
  __syncthreads();

  auto stage = [&](int buf, int kt) {
    float* base = lds + buf * STAGE;
    (void)base;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int piece = wid + i * NW;                           // 8 rows x 128 B
      const int g = piece / ((BNW + BMX) / 8), pr = piece % ((BNW + BMX) / 8);
      const int row = pr * 8 + (lane >> 3);                     // row of [W rows | X rows]
      const int k0 = (kt * WK + g) * EPR + ((lane & 7) ^ ((row >> 1) & 7)) * EPS;
      const E* src = row < BNW ? W + (int64_t)(n0 + row) * p.K + k0
                               : X + (int64_t)min(m0 + row - BNW, p.M - 1) * p.lda + k0;
      lds_dma16(src, base + g * GROUP + pr * 8 * 32);
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float ss = 0.f;
  const int jss = wn % TJ;                                      // m-tile whose sum of squares this wave keeps

  auto compute = [&](int buf) {
    const float* base = lds + buf * STAGE + wk * GROUP;         // rows of 32 floats = 128 bytes
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int off = ((2 * q + lh) ^ cs) << 2;                 // float offset of the 16-byte slot
      if constexpr (BF) {
        bf16x8 fa[TI], fb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(base + (wn * WTN + 32 * i + lr) * 32 + off);
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(base + (BNW + wm * WTM + 32 * j + lr) * 32 + off);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        if constexpr (RS) {
          bf16x8 v = fb[0];
#pragma unroll
          for (int j = 1; j < TJ; ++j) v = (jss == j) ? fb[j] : v;
          ss = sumsq8(v, ss);
        }
      } else {
        f32x4 fa[TI], fb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) fa[i] = *reinterpret_cast<const f32x4*>(base + (wn * WTN + 32 * i + lr) * 32 + off);
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[j] = *reinterpret_cast<const f32x4*>(base + (BNW + wm * WTM + 32 * j + lr) * 32 + off);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0);
        if constexpr (RS) {
          f32x4 v = fb[0];
#pragma unroll
          for (int j = 1; j < TJ; ++j) v = (jss == j) ? fb[j] : v;
          ss = fmaf(v.x, v.x, ss); ss = fmaf(v.y, v.y, ss); ss = fmaf(v.z, v.z, ss); ss = fmaf(v.w, v.w, ss);
        }
      }
    }
  };

  stage(0, 0);
  if (nk > 1) stage(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds();
    if (kt + 2 < nk) stage((kt + 2) % S, kt + 2);
    compute(kt % S);
  }
  barrier_lds();                                                // stage buffers free: reuse for the partials
  if constexpr (WK > 1) {
    if (wk > 0) {
      float* dst = lds + ((wk - 1) * (NW / WK) + wr) * 64 * TI * TJ * 16;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            *reinterpret_cast<f32x4*>(dst + (((i * TJ + j) * 4 + r4) * 64 + lane) * 4) =
                f32x4{acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2], acc[i][j][4 * r4 + 3]};
      if (RS) ssr[((wk - 1) * (NW / WK) + wr) * 64 + lane] = ss;
    }
    barrier_lds();
    if (wk == 0) {
#pragma unroll
      for (int g = 1; g < WK; ++g) {
        const float* src = lds + ((g - 1) * (NW / WK) + wr) * 64 * TI * TJ * 16;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
              const f32x4 v = *reinterpret_cast<const f32x4*>(src + (((i * TJ + j) * 4 + r4) * 64 + lane) * 4);
              acc[i][j][4 * r4] += v.x; acc[i][j][4 * r4 + 1] += v.y; acc[i][j][4 * r4 + 2] += v.z; acc[i][j][4 * r4 + 3] += v.w;
            }
        if (RS) ss += ssr[((g - 1) * (NW / WK) + wr) * 64 + lane];
      }
    }
  }
  if constexpr (RS) {
    const float t = ss + __shfl_xor(ss, 32, 64);
    if (wk == 0 && wn < TJ && lh == 0) rden[wm * WTM + 32 * jss + lr] = sqrtf(t) * p.inv_sqrt_k + kRmsEps;
    barrier_lds();
  }
  if (wk == 0) tile_epilogue<EPI, RS, TI, TJ, WTN, WTM, R16>(p, acc, rden, sbias, m0, n0, wn, wm, lr, lh);
}

// ---------------------------------------------------------------------------------------------
// fp32 projections on the bf16 MFMA by exact operand splitting ("x3": three bf16 terms per fp32
// value, six cross products).
//
//   x = x0 + x1 + x2,  x0 = bf16_rn(x), x1 = bf16_rn(x - x0), x2 = bf16_rn(x - x0 - x1)
//
// Both residuals are exact in fp32 and three 8-bit significands cover fp32's 24:
// |x - x0 - x1 - x2| <= 2^-27 |x|.  A bf16 x bf16 product is exact in the MFMA's fp32 accumulator,
// so keeping the six products with i + j <= 2,
//
//   W.X = W0.X0 + W0.X1 + W1.X0 + W0.X2 + W1.X1 + W2.X0   (dropped terms <= 3 * 2^-26 |W||X|),
//
// is an fp32-accurate dot product (tests/test_gpu_parity.py::test_fp32_split_vs_fp32_mfma runs the
// whole step both ways against the oracle; tools/gemm_bench with FULLF32=1 compares both GEMMs
// with an fp64 reference).  Cost: 6 x 32 cycles per 32x32x16 step on v_mfma_f32_32x32x16_bf16
// against 8 x 64 on v_mfma_f32_32x32x2_f32 -- 2.67x the fp32 MFMA rate.
// W is constant: split once at upload into three bf16 planes [3][N][K] (session.hip upload_w).
// X stays fp32 in memory (its producers are unchanged) and is split in registers from its LDS
// fragment, 8 values per lane per 16-deep k-step, the VALU issued between the MFMAs.
// Structure as gemm_f32t_kernel above (transposed orientation, shared epilogue, in-workgroup K
// split over WK wave groups, LDS-DMA ring of S stages).  Per wave group and K-step (32 k) a stage
// holds the three W planes (BNW rows x 64 B each, 16-byte slot ^= (row >> 2) & 3) and X (BMX rows
// x 128 B fp32, slot ^= (row >> 1) & 7); both swizzles go on the per-lane DMA source address and
// are undone on the ds_read_b128.
template <int BNW_, int BMX_, int WN_, int WM_, int WK_, int S_>
struct XT {
  static constexpr int BNW = BNW_, BMX = BMX_, WN = WN_, WM = WM_, WK = WK_, S = S_;
};


// XS: X arrives pre-split (3 bf16 planes written by its producer, GemmArgs::a_plane) and is staged
// like W -- no split VALU in the loop; otherwise X is fp32 and split from its LDS fragment.
template <class TL, int EPI, bool RS, bool XS>
__global__ void __launch_bounds__(TL::WN * TL::WM * TL::WK * 64) gemm_x3_kernel(GemmArgs p) {
  constexpr int BNW = TL::BNW, BMX = TL::BMX, WN = TL::WN, WM = TL::WM, WK = TL::WK, S = TL::S;
  constexpr int NW = WN * WM * WK, NT = NW * 64;
  constexpr int WTN = BNW / WN, WTM = BMX / WM, TI = WTN / 32, TJ = WTM / 32;
  constexpr int WPL = BNW * 16;                                 // floats of one W plane slice (64-B rows)
  constexpr int XPL = BMX * 16;                                 // floats of one X plane slice (XS)
  constexpr int GROUP = 3 * WPL + (XS ? 3 * XPL : BMX * 32);    // floats of one wave group's slice
  constexpr int STAGE = WK * GROUP;
  constexpr int WPC = 3 * BNW / 16, XPC = XS ? 3 * BMX / 16 : BMX / 8;   // 1 KiB DMA pieces per group
  constexpr int NL = NW;                                        // waves issuing the LDS-DMA
  constexpr int PIECES = WK * (WPC + XPC), IPW = PIECES / NL;
  static_assert(PIECES % NL == 0 && IPW >= 1, "DMA pieces per wave");
  static_assert(TI >= 1 && TJ >= 1 && WN >= TJ, "wave tile / row-scale ownership");
  static_assert(S == 2 || S == 3, "2 or 3 LDS stages");
  constexpr int RED = (WK - 1) * (NW / WK) * 64 * TI * TJ * 16;  // K-split partials (floats)
  constexpr int LDSF = (S * STAGE > RED ? S * STAGE : RED);
  // ONE LDS object (a second __shared__ array beside LDS-DMA staging can cost a vmcnt(0) per step)
  __shared__ __attribute__((aligned(16))) float lds[LDSF + BNW + BMX + (WK - 1) * (NW / WK) * 64];
  float* sbias = lds + LDSF;
  float* rden = sbias + BNW;
  float* ssr = rden + BMX;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid / (WN * WM), wr = wid % (WN * WM), wn = wr / WM, wm = wr % WM;
  const int lr = lane & 31, lh = lane >> 5;
  const int ntn = p.N / BNW;
  int m0, n0;
  const int ntm = gridDim.x / ntn;
  if (p.xcd_mn && (ntn & 3) == 0 && (ntm & 1) == 0) {
    // XCDs as 2 (M halves) x 4 (N quarters): each XCD's L2 takes half of X and a quarter of the W planes (FFN up at
    // M = 2560: 15.7 + 14.2 MB of fills over the chip instead of 31.5 + 7.1 with the N-only split below)
    const int xcd = blockIdx.x & 7, li = blockIdx.x >> 3, nq = ntn >> 2, mh = ntm >> 1;
    m0 = ((xcd >> 2) * mh + li / nq) * BMX;
    n0 = ((xcd & 3) * nq + li % nq) * BNW;
  } else if ((ntn & 7) == 0) {
    // large W (FFN up: 7 MB of planes > one XCD's 4 MB L2): XCD x owns N-tiles [x*ntn/8, (x+1)*ntn/8)
    // for every M-tile, so each W plane row is fetched into one L2 only and the X tile is reused
    // by the XCD's N-tiles back to back
    const int npx = ntn >> 3, li = blockIdx.x >> 3;
    m0 = (li / npx) * BMX;
    n0 = ((blockIdx.x & 7) * npx + li % npx) * BNW;
  } else {  // XCD-contiguous tile order (bijective for any grid size): an XCD shares each X tile
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (blockIdx.x >> 3);
    m0 = (wgid / ntn) * BMX;
    n0 = (wgid % ntn) * BNW;
  }
  // split-K (GemmArgs::k_split > 0): this workgroup's K range is [y * k_split, (y + 1) * k_split),
  // its raw partial goes to slab y of C ([nsplit][M][ldc])
  const int kofs = p.k_split ? (int)blockIdx.y * p.k_split : 0;
  if (p.k_split) p.C = static_cast<float*>(p.C) + (int64_t)blockIdx.y * p.M * p.ldc;
  const int nk = (p.k_split ? p.k_split : p.K) / (32 * WK);
  const float* __restrict__ X = static_cast<const float*>(p.A);
  const uint16_t* __restrict__ X3 = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W3 = p.W3;
  const int64_t plane = (int64_t)p.N * p.K;

  for (int i = tid; i < BNW; i += NT) sbias[i] = p.bias ? p.bias[n0 + i] : 0.f;
  __syncthreads();

  auto stage = [&](int buf, int kt) {
    float* base = lds + buf * STAGE;
    (void)base;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int piece = wid + i * NL;                           // wave-uniform
      const int g = piece / (WPC + XPC), pr = piece % (WPC + XPC);
      const int kb = kofs + (kt * WK + g) * 32;
      const void* src;
      float* dst;
      if (pr < WPC) {                                           // 16 W rows x 64 B of plane pl
        const int pl = pr / (BNW / 16), rb = (pr % (BNW / 16)) * 16, row = rb + (lane >> 2);
        const int slot = (lane & 3) ^ ((row >> 2) & 3);
        src = W3 + pl * plane + (int64_t)(n0 + row) * p.K + kb + slot * 8;
        dst = base + g * GROUP + pl * WPL + rb * 16;
      } else if constexpr (XS) {                                // 16 X rows x 64 B of plane pl
        const int xp = pr - WPC, pl = xp / (BMX / 16), rb = (xp % (BMX / 16)) * 16, row = rb + (lane >> 2);
        const int slot = (lane & 3) ^ ((row >> 2) & 3);
        src = X3 + pl * p.a_plane + (int64_t)min(m0 + row, p.M - 1) * p.lda + kb + slot * 8;
        dst = base + g * GROUP + 3 * WPL + pl * XPL + rb * 16;
      } else {                                                  // 8 X rows x 128 B
        const int rb = (pr - WPC) * 8, row = rb + (lane >> 3);
        const int slot = (lane & 7) ^ ((row >> 1) & 7);
        src = X + (int64_t)min(m0 + row, p.M - 1) * p.lda + kb + slot * 4;
        dst = base + g * GROUP + 3 * WPL + rb * 32;
      }
      lds_dma16(src, dst);
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float ss = 0.f;
  const int jss = wn % TJ;                                      // m-tile whose sum of squares this wave keeps

  // One K-step: every fragment of both 16-deep halves is read first (one LDS wait), then per half
  // the X split (VALU) and the 6 x TI x TJ MFMAs, so the split of one half can issue under the
  // MFMAs of the other.
  auto compute = [&](int buf) {
    const float* base = lds + buf * STAGE + wk * GROUP;
    bf16x8 w[2][3][TI], xs[2][3][TJ];
    f32x4 xv[2][TJ][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j8 = 2 * q + lh;                                // 8-value block of the 32-k slice
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = wn * WTN + 32 * i + lr;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          w[q][pl][i] = *reinterpret_cast<const bf16x8*>(base + pl * WPL + row * 16 + ((j8 ^ ((row >> 2) & 3)) << 2));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        if constexpr (XS) {
          const int row = wm * WTM + 32 * j + lr;
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            xs[q][pl][j] = *reinterpret_cast<const bf16x8*>(base + 3 * WPL + pl * XPL + row * 16 + ((j8 ^ ((row >> 2) & 3)) << 2));
        } else {
          const int row = wm * WTM + 32 * j + lr, cs = (row >> 1) & 7;
          const float* xr = base + 3 * WPL + row * 32;
          xv[q][j][0] = *reinterpret_cast<const f32x4*>(xr + (((2 * j8) ^ cs) << 2));
          xv[q][j][1] = *reinterpret_cast<const f32x4*>(xr + (((2 * j8 + 1) ^ cs) << 2));
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead (hipcc sinks them to their uses)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if constexpr (XS) {
        if constexpr (RS) {   // ||x||^2 in fp32 from the reassembled values (x0 + x1 + x2 == x exactly)
          bf16x8 a0 = xs[q][0][0], a1 = xs[q][1][0], a2 = xs[q][2][0];
#pragma unroll
          for (int j = 1; j < TJ; ++j) {
            a0 = (jss == j) ? xs[q][0][j] : a0;
            a1 = (jss == j) ? xs[q][1][j] : a1;
            a2 = (jss == j) ? xs[q][2][j] : a2;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = ((float)a0[e] + (float)a1[e]) + (float)a2[e];
            ss = fmaf(v, v, ss);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < TJ; ++j) split3(xv[q][j][0], xv[q][j][1], xs[q][0][j], xs[q][1][j], xs[q][2][j]);
        if constexpr (RS) {
          f32x4 a = xv[q][0][0], b = xv[q][0][1];
#pragma unroll
          for (int j = 1; j < TJ; ++j) {
            a = (jss == j) ? xv[q][j][0] : a;
            b = (jss == j) ? xv[q][j][1] : b;
          }
          ss = fmaf(a.x, a.x, ss); ss = fmaf(a.y, a.y, ss); ss = fmaf(a.z, a.z, ss); ss = fmaf(a.w, a.w, ss);
          ss = fmaf(b.x, b.x, ss); ss = fmaf(b.y, b.y, ss); ss = fmaf(b.z, b.z, ss); ss = fmaf(b.w, b.w, ss);
        }
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {   // small terms first
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][2][i], xs[q][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][1][i], xs[q][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][0][i], xs[q][2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][1][i], xs[q][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][0][i], xs[q][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[q][0][i], xs[q][0][j], acc[i][j], 0, 0, 0);
        }
    }
  };

  // dbg 64 (set by launch_x3): static priority for the second-dispatched half of the waves, the arbitration
  // loser of every segment (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if ((p.dbg & 64) && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if constexpr (S == 3) {
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier_lds();                                            // buffer (kt+2)%3 was read in step kt-1
      if (kt + 2 < nk) stage((kt + 2) % 3, kt + 2);
      compute(kt % 3);
    }
  } else {
    stage(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier_lds();                                            // buffer (kt+1)&1 was read in step kt-1
      if (kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
      compute(kt & 1);
    }
  }
  barrier_lds();                                                // stage buffers free: reuse for the partials
  if constexpr (WK > 1) {
    if (wk > 0) {
      float* dst = lds + ((wk - 1) * (NW / WK) + wr) * 64 * TI * TJ * 16;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            *reinterpret_cast<f32x4*>(dst + (((i * TJ + j) * 4 + r4) * 64 + lane) * 4) =
                f32x4{acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2], acc[i][j][4 * r4 + 3]};
      if (RS) ssr[((wk - 1) * (NW / WK) + wr) * 64 + lane] = ss;
    }
    barrier_lds();
    if (wk == 0) {
#pragma unroll
      for (int g = 1; g < WK; ++g) {
        const float* src = lds + ((g - 1) * (NW / WK) + wr) * 64 * TI * TJ * 16;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
              const f32x4 v = *reinterpret_cast<const f32x4*>(src + (((i * TJ + j) * 4 + r4) * 64 + lane) * 4);
              acc[i][j][4 * r4] += v.x; acc[i][j][4 * r4 + 1] += v.y; acc[i][j][4 * r4 + 2] += v.z; acc[i][j][4 * r4 + 3] += v.w;
            }
        if (RS) ss += ssr[((g - 1) * (NW / WK) + wr) * 64 + lane];
      }
    }
  }
  if constexpr (RS) {
    const float t = ss + __shfl_xor(ss, 32, 64);
    if (wk == 0 && wn < TJ && lh == 0) rden[wm * WTM + 32 * jss + lr] = sqrtf(t) * p.inv_sqrt_k + kRmsEps;
    barrier_lds();
  }
  if (p.dbg & 8) return;                                        // microbenchmark: no epilogue
  if (wk == 0) tile_epilogue<EPI, RS, TI, TJ, WTN, WTM>(p, acc, rden, sbias, m0, n0, wn, wm, lr, lh);
}

template <class TL, int EPI>
hipError_t launch_x3(const GemmArgs& a0, hipStream_t st) {
  GemmArgs a = a0;
  // static priority for waves NW/2..: fp32 B = 256 step 3.616 -> 3.583 ms, FFN down 897 -> 871 us
  // (profiles/r02_ab_x3_prio.jsonl)
  a.dbg |= 64;
  a.xcd_mn = knobs().x3_xcd;
  const dim3 tiles((a.N / TL::BNW) * ((a.M + TL::BMX - 1) / TL::BMX), a.k_split ? a.K / a.k_split : 1);
  const dim3 block(TL::WN * TL::WM * TL::WK * 64);
  if (a.a_plane) {
    if (a.rowscale) hipLaunchKernelGGL((gemm_x3_kernel<TL, EPI, true, true>), tiles, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_x3_kernel<TL, EPI, false, true>), tiles, block, 0, st, a);
  } else {
    if (a.rowscale) hipLaunchKernelGGL((gemm_x3_kernel<TL, EPI, true, false>), tiles, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_x3_kernel<TL, EPI, false, false>), tiles, block, 0, st, a);
  }
  return hipGetLastError();
}

template <class TL>
hipError_t launch_x3_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (!a.W3 || a.a_bf16 || a.c_bf16 || a.rpg || a.M <= 0 || a.N % TL::BNW || a.K % (32 * TL::WK) || a.lda % 8 ||
      a.ldc % 8 || (a.c_plane && (a.c_plane % 8 || (epi != EPI_SWIGLU && epi != EPI_GLU))) || a.c2_plane % 8 ||
      a.a_plane % 8 || (a.k_split && (a.K % a.k_split || a.k_split % (32 * TL::WK) || a.rowscale || epi != EPI_STORE)))
    return hipErrorInvalidValue;
  constexpr bool pairable = (TL::BNW / TL::WN / 32) % 2 == 0;   // g/u 32-row blocks in one wave tile
  switch (epi) {
    case EPI_STORE: return launch_x3<TL, EPI_STORE>(a, st);
    case EPI_RESID: return launch_x3<TL, EPI_RESID>(a, st);
    case EPI_SWIGLU: if constexpr (pairable) return launch_x3<TL, EPI_SWIGLU>(a, st); else return hipErrorInvalidValue;
    case EPI_GLU: if constexpr (pairable) return launch_x3<TL, EPI_GLU>(a, st); else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 projections by exact splitting, both operands streamed as fp32 ("r3": K-tile ring).
//
// gemm_x3 stages W as its three bf16 planes (6 bytes per element) and X as fp32.  Here W is staged as
// fp32 too (4 bytes, split in registers like X): 4 (BN + BM) bytes per k instead of (6 BN + 4 BM), and
// the stages form a ring of R K-tiles (32 k = one 128-byte line per row) with up to R - 1 in flight.
//   * persistent over tiles, the ring runs across tile boundaries; tiles dealt XCD-contiguously;
//   * per wave and 16-deep half: the raw fp32 fragments of W and X are read (two ds_read_b128 per
//     row and lane, slot ^= (row >> 1) & 7 applied on the DMA source), split in registers into
//     their three bf16 terms, and the six products with i + j <= 2 go to v_mfma_f32_32x32x16_bf16
//     (the arithmetic of gemm_x3: fp32-accurate, see there);
//   * folded RMSNorm (RS): the row sum of squares from the raw X fragments, as in gemm_x3.
// Measured (tools/gemm_bench, scripts/r3_sweep.sh / r3_ablate.sh, profiles/r02_r3_*.jsonl): the ring's
// DMA alone (no reads, split or MFMA) fills at 38-48 GB/s per CU, and the extra split VALU costs more
// than the saved bytes on every B = 256 shape except the large-M k|v projections of layers 14 / 15,
// which is where gemm() routes it.
template <int BN_, int BM_, int WN_, int WM_, int R_, int NB_>
struct RT {
  static constexpr int BN = BN_, BM = BM_, WN = WN_, WM = WM_, R = R_, NB = NB_;
};

template <int N>
__device__ __forceinline__ void wait_vm_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(k * IPW) for a wave-uniform k in [0, KMAX]
template <int IPW, int KMAX>
__device__ __forceinline__ void wait_vm_tiles(int k) {
  if constexpr (KMAX >= 4) if (k >= 4) { wait_vm_n<4 * IPW>(); return; }
  if constexpr (KMAX >= 3) if (k == 3) { wait_vm_n<3 * IPW>(); return; }
  if constexpr (KMAX >= 2) if (k == 2) { wait_vm_n<2 * IPW>(); return; }
  if constexpr (KMAX >= 1) if (k == 1) { wait_vm_n<IPW>(); return; }
  wait_vm_n<0>();
}

// Software pipeline (one wave's instruction stream): the MFMAs of one 16-deep half run on operands
// split in the previous phase while the LDS reads and the split of the next half are issued between
// them, so the VALU and the LDS-DMA issue fill the MFMA shadow instead of following it:
//   phase A of K-tile t:  MFMA(t, h0)  ||  read + split (t, h1)
//   wait K-tile t + 1, barrier (every wave is past its reads of K-tile t), DMA K-tile t + R into t's slot
//   phase B of K-tile t:  MFMA(t, h1)  ||  read + split (t + 1, h0)
// The issue and read indices are clamped to the last K-tile, so every phase is branch-free and the
// barrier waits on a fixed vmcnt; the ring slots those clamped DMAs land in are never read again.
// DBG (microbenchmark ablations only): bit 0 no MFMA, bit 1 no split (fragments reinterpreted), bit 2 no
// LDS-DMA, bit 3 no epilogue; every accumulator stays live
template <class TL, int EPI, bool RS, int DBG = 0>
__global__ void __launch_bounds__(TL::WN * TL::WM * 64) gemm_r3_kernel(GemmArgs p) {
  constexpr int BN = TL::BN, BM = TL::BM, WN = TL::WN, WM = TL::WM, R = TL::R, NB = TL::NB;
  constexpr int NW = WN * WM, NT = NW * 64;
  constexpr int WTN = BN / WN, WTM = BM / WM, TI = WTN / 32, TJ = WTM / 32;
  constexpr int STAGE = (BN + BM) * 32;                          // floats of one K-tile
  constexpr int P = (BN + BM) / 8, IPW = P / NW;                 // 1 KiB pieces (8 rows x 128 B)
  static_assert(P % NW == 0 && TI >= 1 && TJ >= 1 && WN >= TJ, "pieces per wave / tile ownership");
  static_assert(R >= 3 && R <= 6 && (R - 2) * IPW <= 63, "ring depth / vmcnt range");
  __shared__ __attribute__((aligned(16))) float lds[R * STAGE + NB + BM];
  float* sbias = lds + R * STAGE;
  float* rden = sbias + NB;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / WM, wm = wid % WM, lr = lane & 31, lh = lane >> 5;
  const int ntn = p.N / BN, ntm = (p.M + BM - 1) / BM, ntiles = ntn * ntm;
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (ntiles + 7) >> 3, tbeg = xcd * q, tend = min(ntiles, tbeg + q);
  const int nmine = (tbeg + jb < tend) ? (tend - tbeg - jb + nxb - 1) / nxb : 0;
  for (int i = tid; i < p.N; i += NT) sbias[i] = p.bias ? p.bias[i] : 0.f;
  __syncthreads();
  if (nmine <= 0) return;                                        // workgroup-uniform
  const int nk = p.K / 32, G = nmine * nk;
  const float* __restrict__ W = static_cast<const float*>(p.W);
  const float* __restrict__ X = static_cast<const float*>(p.A);

  auto tile_of = [&](int u, int& m0, int& n0) {
    const int t = tbeg + jb + (u / nk) * nxb;
    m0 = (t / ntn) * BM;
    n0 = (t % ntn) * BN;
  };
  // per-lane source rows of this wave's pieces: W rows for pieces < BN / 8, X rows after (piece i of
  // every wave is a W piece iff i * NW < BN / 8: compile-time, so the issue is branch-free)
  static_assert((BN / 8) % NW == 0, "W / X pieces split at a wave boundary");
  auto issue = [&](int u) {
    if constexpr (DBG & 4) return;
    int m0, n0;
    tile_of(u, m0, n0);
    const int k0 = (u % nk) * 32;
    float* base = lds + (u % R) * STAGE;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int pc = wid + i * NW;                               // wave-uniform
      const int r = pc * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const float* src;
      if (i * NW < BN / 8) src = W + (int64_t)(n0 + r) * p.K + k0 + 4 * c;   // folds after unrolling
      else src = X + (int64_t)min(m0 + r - BN, p.M - 1) * p.lda + k0 + 4 * c;
      lds_dma16(src, base + pc * 256);
    }
  };

  struct Ops {
    bf16x8 w0[TI], w1[TI], w2[TI], x0[TJ], x1[TJ], x2[TJ];
  };
  // raw fp32 fragments of half h of the K-tile in `slot` -> their bf16 terms; returns the lane's
  // partial sum of squares of its X row (RS)
  auto read_split = [&](int slot, int h, Ops& o) -> float {
    if constexpr ((DBG & 16) != 0) return 0.f;                  // ablation: no LDS reads at all
    const float* base = lds + slot * STAGE;
    const int c0 = 4 * h + 2 * lh;                               // first 16-byte chunk of this lane's 8 k
    f32x4 wv[TI][2], xv[TJ][2];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = wn * WTN + 32 * i + lr, s = (row >> 1) & 7;
      wv[i][0] = *reinterpret_cast<const f32x4*>(base + row * 32 + ((c0 ^ s) << 2));
      wv[i][1] = *reinterpret_cast<const f32x4*>(base + row * 32 + (((c0 + 1) ^ s) << 2));
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int row = BN + wm * WTM + 32 * j + lr, s = (row >> 1) & 7;
      xv[j][0] = *reinterpret_cast<const f32x4*>(base + row * 32 + ((c0 ^ s) << 2));
      xv[j][1] = *reinterpret_cast<const f32x4*>(base + row * 32 + (((c0 + 1) ^ s) << 2));
    }
    if constexpr (DBG & 2) {
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        o.w0[i] = __builtin_bit_cast(bf16x8, wv[i][0]); o.w1[i] = __builtin_bit_cast(bf16x8, wv[i][1]); o.w2[i] = o.w0[i];
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        o.x0[j] = __builtin_bit_cast(bf16x8, xv[j][0]); o.x1[j] = __builtin_bit_cast(bf16x8, xv[j][1]); o.x2[j] = o.x1[j];
      }
    } else {
#pragma unroll
      for (int i = 0; i < TI; ++i) split3(wv[i][0], wv[i][1], o.w0[i], o.w1[i], o.w2[i]);
#pragma unroll
      for (int j = 0; j < TJ; ++j) split3(xv[j][0], xv[j][1], o.x0[j], o.x1[j], o.x2[j]);
    }
    float c = 0.f;
    if constexpr (RS) {
      const int jss = wn % TJ;                                   // m-tile whose sum of squares this wave keeps
      f32x4 a = xv[0][0], b = xv[0][1];
#pragma unroll
      for (int j = 1; j < TJ; ++j) {
        a = (jss == j) ? xv[j][0] : a;
        b = (jss == j) ? xv[j][1] : b;
      }
      c = a.x * a.x; c = fmaf(a.y, a.y, c); c = fmaf(a.z, a.z, c); c = fmaf(a.w, a.w, c);
      c = fmaf(b.x, b.x, c); c = fmaf(b.y, b.y, c); c = fmaf(b.z, b.z, c); c = fmaf(b.w, b.w, c);
    }
    return c;
  };

  f32x16 acc[TI][TJ];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };
  auto mfma = [&](const Ops& o) {
    if constexpr (DBG & 1) {   // no MFMA: fold the operands into the accumulators (keeps them live)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j][0] += __builtin_bit_cast(f32x4, o.w2[i]).x + __builtin_bit_cast(f32x4, o.x2[j]).x +
                          __builtin_bit_cast(f32x4, o.w1[i]).y + __builtin_bit_cast(f32x4, o.x1[j]).y +
                          __builtin_bit_cast(f32x4, o.w0[i]).z + __builtin_bit_cast(f32x4, o.x0[j]).z;
      return;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {   // small terms first
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w2[i], o.x0[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w1[i], o.x1[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w0[i], o.x2[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w1[i], o.x0[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w0[i], o.x1[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(o.w0[i], o.x0[j], acc[i][j], 0, 0, 0);
      }
  };
  // interleave hint for one phase: the LDS reads first, then MFMAs with the split VALU between them
  auto interleave = [&]() {
    constexpr int NM = (DBG & 1) ? 0 : 6 * TI * TJ;
    if constexpr (NM > 0) {
      __builtin_amdgcn_sched_group_barrier(0x100, 4 * (TI + TJ), 0);   // ds_read_b128
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                // MFMA (reads in flight)
#pragma unroll
      for (int k = 2; k < NM; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x002, (TI + TJ) * 22 / (NM - 2) + 1, 0);   // VALU
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
      }
    }
  };

  zero();
  float ss = 0.f, ss_next = 0.f;
  for (int u = 0; u < R; ++u) issue(min(u, G - 1));             // the ring starts full
  wait_vm_n<(R - 1) * IPW>();                                    // K-tile 0 landed (this wave's pieces)
  barrier_lds();
  Ops cur, nxt;
  ss += read_split(0, 0, cur);
  for (int t = 0; t < G; ++t) {
    const int slot = t % R;
    // phase A: MFMA (t, h0) || read + split (t, h1)
    __builtin_amdgcn_sched_barrier(0);
    ss += read_split(slot, 1, nxt);
    mfma(cur);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
    // K-tile t + 1 landed: R - 2 later K-tiles stay in flight (clamped DMAs included)
    wait_vm_n<(R - 2) * IPW>();
    barrier_lds();                                               // every wave past its reads of K-tile t
    issue(min(t + R, G - 1));                                    // into slot t % R
    __builtin_amdgcn_sched_barrier(0);
    // phase B: MFMA (t, h1) || read + split (t + 1, h0)
    const int tn = min(t + 1, G - 1);
    const bool last = (t % nk == nk - 1);                        // K-tile t ends a tile: t + 1 starts the next
    const float cn = read_split(tn % R, 0, nxt);
    mfma(cur);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    ss_next = last ? cn : ss_next;
    ss += last ? 0.f : cn;
    cur = nxt;
    if (last) {
      int m0, n0;
      tile_of(t, m0, n0);
      if constexpr (RS) {
        const float s2 = ss + __shfl_xor(ss, 32, 64);
        if (wn < TJ && lh == 0) rden[wm * WTM + 32 * wn + lr] = sqrtf(s2) * p.inv_sqrt_k + kRmsEps;
        barrier_lds();
        ss = ss_next;
      }
      if constexpr (DBG & 8) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)   // never true (alpha is finite): keeps every accumulator live
            if (p.alpha == -1.2345e30f) *reinterpret_cast<f32x16*>(static_cast<float*>(p.C) + 16 * (64 * (i * TJ + j) + lane)) = acc[i][j];
      } else {
        tile_epilogue<EPI, RS, TI, TJ, WTN, WTM>(p, acc, rden, sbias + n0, m0, n0, wn, wm, lr, lh);
      }
      zero();
    }
  }
  wait_vm_n<0>();                                                // no LDS-DMA outlives the workgroup
}

template <class TL, int EPI>
hipError_t launch_r3(const GemmArgs& a, hipStream_t st) {
  const int ntiles = (a.N / TL::BN) * ((a.M + TL::BM - 1) / TL::BM);
  int grid = 256;                                                // one workgroup per CU (LDS)
  const int need = ((ntiles + 7) / 8) * 8;
  if (grid > need) grid = need;
  const dim3 block(TL::WN * TL::WM * 64);
  if constexpr (EPI == EPI_RESID) {   // microbenchmark ablations (tools/gemm_bench, dbg bits)
    switch (a.dbg) {
      case 0: break;
      case 1: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 1>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 2: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 2>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 3: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 3>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 4: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 4>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 6: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 6>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 8: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 8>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 12: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 12>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 13: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 13>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 9: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 27>), dim3(grid), block, 0, st, a); return hipGetLastError();
      case 5: hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false, 25>), dim3(grid), block, 0, st, a); return hipGetLastError();
      default: return hipErrorInvalidValue;
    }
  }
  if (a.rowscale) hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, true>), dim3(grid), block, 0, st, a);
  else hipLaunchKernelGGL((gemm_r3_kernel<TL, EPI, false>), dim3(grid), block, 0, st, a);
  return hipGetLastError();
}

template <class TL>
hipError_t launch_r3_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (!a.W || a.a_bf16 || a.c_bf16 || a.rpg || a.k_split || a.a_plane || a.M <= 0 || a.N % TL::BN || a.N > TL::NB ||
      a.K % 32 || a.lda % 4 || a.ldc % 4 || (a.c_plane && (a.c_plane % 8 || (epi != EPI_SWIGLU && epi != EPI_GLU))) ||
      a.c2_plane % 8)
    return hipErrorInvalidValue;
  constexpr bool pairable = (TL::BN / TL::WN / 32) % 2 == 0;    // g/u 32-row blocks in one wave tile
  switch (epi) {
    case EPI_STORE: return launch_r3<TL, EPI_STORE>(a, st);
    case EPI_RESID: return launch_r3<TL, EPI_RESID>(a, st);
    case EPI_SWIGLU: if constexpr (pairable) return launch_r3<TL, EPI_SWIGLU>(a, st); else return hipErrorInvalidValue;
    case EPI_GLU: if constexpr (pairable) return launch_r3<TL, EPI_GLU>(a, st); else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

int num_cus_t() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

template <class TL, int EPI>
hipError_t launch_t(const GemmArgs& a, hipStream_t st) {
  static_assert(TL::WN >= TL::BMX / TL::WM / 32, "row-scale ownership: one m-tile per wave");
  const int ntiles = (a.N / TL::BNW) * ((a.M + TL::BMX - 1) / TL::BMX);
  int grid = num_cus_t();
  const int need = ((ntiles + 7) / 8) * 8;
  if (grid > need) grid = need;
  grid = (grid + 7) / 8 * 8;
  if (a.rowscale) hipLaunchKernelGGL((gemm_t_kernel<TL, EPI, true>), dim3(grid), dim3(TL::WN * TL::WM * 64), 0, st, a);
  else hipLaunchKernelGGL((gemm_t_kernel<TL, EPI, false>), dim3(grid), dim3(TL::WN * TL::WM * 64), 0, st, a);
  return hipGetLastError();
}

template <class TL>
hipError_t launch_t_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (a.N % TL::BNW || a.K % 64 || a.N > kBiasMax || a.rpg || a.M <= 0) return hipErrorInvalidValue;
  if (a.ldc % 8) return hipErrorInvalidValue;   // 16-byte epilogue stores
  switch (epi) {
    case EPI_STORE: return launch_t<TL, EPI_STORE>(a, st);
    case EPI_RESID: return a.c_bf16 ? hipErrorInvalidValue : launch_t<TL, EPI_RESID>(a, st);
    case EPI_SWIGLU: return launch_t<TL, EPI_SWIGLU>(a, st);
    case EPI_GLU: return launch_t<TL, EPI_GLU>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

template <class TL, int EPI>
hipError_t launch_t2(const GemmArgs& a, hipStream_t st) {
  const int tiles = (a.N / TL::BNW) * ((a.M + TL::BMX - 1) / TL::BMX);
  if (a.rowscale) hipLaunchKernelGGL((gemm_t2_kernel<TL, EPI, true>), dim3(tiles), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gemm_t2_kernel<TL, EPI, false>), dim3(tiles), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <class TL>
hipError_t launch_t2_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (a.N % TL::BNW || a.K % 32 || a.rpg || a.M <= 0) return hipErrorInvalidValue;
  if (a.ldc % 8) return hipErrorInvalidValue;   // 16-byte epilogue stores
  switch (epi) {
    case EPI_STORE: return launch_t2<TL, EPI_STORE>(a, st);
    case EPI_RESID: return a.c_bf16 ? hipErrorInvalidValue : launch_t2<TL, EPI_RESID>(a, st);
    case EPI_SWIGLU: return launch_t2<TL, EPI_SWIGLU>(a, st);
    case EPI_GLU: return launch_t2<TL, EPI_GLU>(a, st);
    default: return hipErrorInvalidValue;
  }
}

template <class TL, int EPI, bool BF>
hipError_t launch_f32t(const GemmArgs& a, hipStream_t st) {
  const int kg = BF ? 64 : 32;
  if (a.N % TL::BNW || a.K % (kg * TL::WK) || a.rpg || a.M <= 0 || (a.ldc % 8) || (a.lda % 8)) return hipErrorInvalidValue;
  const int tiles = (a.N / TL::BNW) * ((a.M + TL::BMX - 1) / TL::BMX);
  const dim3 block(TL::WN * TL::WM * TL::WK * 64);
  if (a.res16) {   // the bf16 / fp8 modes' fp16 residual stream: RESID, or the STORE that starts it
    if constexpr (BF && (EPI == EPI_STORE || EPI == EPI_RESID)) {
      if (a.rowscale || a.c_bf16) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_f32t_kernel<TL, EPI, false, BF, true>), dim3(tiles), block, 0, st, a);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (a.rowscale) hipLaunchKernelGGL((gemm_f32t_kernel<TL, EPI, true, BF>), dim3(tiles), block, 0, st, a);
  else hipLaunchKernelGGL((gemm_f32t_kernel<TL, EPI, false, BF>), dim3(tiles), block, 0, st, a);
  return hipGetLastError();
}

template <class TL, int EPI>
hipError_t launch_f32t(const GemmArgs& a, hipStream_t st) {
  if (a.a_bf16) return launch_f32t<TL, EPI, true>(a, st);
  if (a.c_bf16) return hipErrorInvalidValue;
  return launch_f32t<TL, EPI, false>(a, st);
}

template <class TL>
hipError_t launch_f32t_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (epi == EPI_RESID && a.c_bf16) return hipErrorInvalidValue;
  constexpr bool pairable = (TL::BNW / TL::WN / 32) % 2 == 0;   // g/u 32-row blocks in one wave tile
  switch (epi) {
    case EPI_STORE: return launch_f32t<TL, EPI_STORE>(a, st);
    case EPI_RESID: return launch_f32t<TL, EPI_RESID>(a, st);
    case EPI_SWIGLU: if constexpr (pairable) return launch_f32t<TL, EPI_SWIGLU>(a, st); else return hipErrorInvalidValue;
    case EPI_GLU: if constexpr (pairable) return launch_f32t<TL, EPI_GLU>(a, st); else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// fp32 variants: 0 = 64x64 tile, 8 waves (2n x 2m x 2k); 1 = 128x64 (paired epilogues), 8 waves;
// 2 = 64x64, 4 waves (no K split); 3 = 64x128 (2n x 2m x 2k, 32x64 wave tiles)
hipError_t gemm_f32t(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  switch (variant) {
    case 0: return launch_f32t_epi<FT<64, 64, 2, 2, 2>>(a, epi, st);
    case 1: return launch_f32t_epi<FT<128, 64, 2, 2, 2>>(a, epi, st);
    case 2: return launch_f32t_epi<FT<64, 64, 2, 2, 1>>(a, epi, st);
    case 3: return launch_f32t_epi<FT<64, 128, 2, 2, 2>>(a, epi, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t gemm_t(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  if (!a.a_bf16) return hipErrorInvalidValue;
  switch (variant) {
    case 0: return launch_t_epi<TT<256, 256, 2, 4>>(a, epi, st);
    case 1: return launch_t_epi<TT<128, 256, 2, 4>>(a, epi, st);
    case 2: return launch_t_epi<TT<256, 128, 2, 4>>(a, epi, st);
    case 3: return launch_t_epi<TT<128, 128, 2, 4>>(a, epi, st);
    case 4: return launch_t2_epi<TT<256, 128, 2, 2>>(a, epi, st);   // 2 workgroups per CU
    case 5: return launch_t2_epi<TT<128, 128, 2, 2>>(a, epi, st);
    default: return hipErrorInvalidValue;
  }
}

// fp32-by-split variants (LDS per workgroup): 0 = 64x64, 8 waves (2n x 2m x 2k), 3 stages (120 KiB);
// 1 = 128x64, 8 waves, 2 stages (128 KiB, paired epilogues); 2 = 64x128, 8 waves, 2 stages
// (112 KiB); 3 = 128x128, 4 waves (no K split), 3 stages (120 KiB); 4 = 64x64, 4 waves, 3 stages
// (60 KiB, 2 workgroups per CU); 5 = 128x64, 4 waves, 3 stages (96 KiB, paired epilogues)
hipError_t gemm_x3(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  switch (variant) {
    case 0: return launch_x3_epi<XT<64, 64, 2, 2, 2, 3>>(a, epi, st);
    case 1: return launch_x3_epi<XT<128, 64, 2, 2, 2, 2>>(a, epi, st);
    case 2: return launch_x3_epi<XT<64, 128, 2, 2, 2, 2>>(a, epi, st);
    case 3: return launch_x3_epi<XT<128, 128, 2, 2, 1, 3>>(a, epi, st);
    case 4: return launch_x3_epi<XT<64, 64, 2, 2, 1, 3>>(a, epi, st);
    case 5: return launch_x3_epi<XT<128, 64, 2, 2, 1, 3>>(a, epi, st);
    // two waves per SIMD (one wave issues its LDS-DMA pieces while the other runs MFMAs)
    case 6: return launch_x3_epi<XT<128, 128, 2, 4, 1, 3>>(a, epi, st);   // 8 waves, 120 KiB
    case 7: return launch_x3_epi<XT<256, 128, 4, 2, 1, 2>>(a, epi, st);   // 8 waves, 128 KiB
    case 8: return launch_x3_epi<XT<128, 256, 2, 4, 1, 2>>(a, epi, st);   // 8 waves, 112 KiB
    // narrow tiles, four-way in-workgroup K split: twice the workgroups for the N = 384 projections
    case 9: return launch_x3_epi<XT<64, 32, 2, 1, 4, 2>>(a, epi, st);     // 8 waves, 128 KiB
    case 10: return launch_x3_epi<XT<32, 64, 1, 2, 4, 2>>(a, epi, st);    // 8 waves, 112 KiB
    case 11: return launch_x3_epi<XT<64, 32, 2, 1, 2, 3>>(a, epi, st);    // 4 waves, 96 KiB
    default: return hipErrorInvalidValue;
  }
}

// fp32-by-split, fp32 W and X through a K-tile ring (gemm_r3_kernel).  RT<BN, BM, WN, WM, R, NB>:
// tile BN W rows x BM X rows, WN x WM waves, R K-tiles of (BN + BM) x 128 B, bias for N <= NB.
hipError_t gemm_r3(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  switch (variant) {
    case 0: return launch_r3_epi<RT<256, 128, 4, 2, 3, kBiasMax>>(a, epi, st);   // 8 waves, 156 KiB
    case 1: return launch_r3_epi<RT<128, 128, 2, 4, 4, kBiasMax>>(a, epi, st);   // 8 waves, 140 KiB
    case 2: return launch_r3_epi<RT<64, 64, 2, 2, 6, 1536>>(a, epi, st);         // 4 waves, 102 KiB
    case 3: return launch_r3_epi<RT<64, 32, 2, 1, 6, 1536>>(a, epi, st);         // 2 waves, 78 KiB
    case 4: return launch_r3_epi<RT<32, 64, 1, 2, 6, 1536>>(a, epi, st);         // 2 waves, 78 KiB
    case 5: return launch_r3_epi<RT<128, 64, 2, 2, 5, 1536>>(a, epi, st);        // 4 waves, 126 KiB (paired)
    case 6: return launch_r3_epi<RT<64, 64, 1, 2, 6, 1536>>(a, epi, st);         // 2 waves, 102 KiB (paired)
    case 7: return launch_r3_epi<RT<128, 128, 4, 2, 4, kBiasMax>>(a, epi, st);   // 8 waves, 140 KiB
    case 8: return launch_r3_epi<RT<256, 128, 2, 4, 3, kBiasMax>>(a, epi, st);   // 8 waves, 156 KiB
    case 9: return launch_r3_epi<RT<64, 64, 2, 2, 4, 1536>>(a, epi, st);         // 4 waves, 70 KiB
    default: return hipErrorInvalidValue;
  }
}


}  // namespace tone
