// X-stationary bf16 GEMM for the K = 384 encoder projections at large batch (FFN up + SwiGLU, pw1 + GLU,
// q|k|v), computed in the transposed orientation D[n][m] = W[n][:] . X[m][:] like gemm_t.
//
// Why: with K = 384 a 256 x 256 output tile does only 2 * 256 * 256 * 384 FLOP per (256 + 256) x 384 x 2 bytes
// staged through LDS (128 FLOP/B), and gemm_t's loop is bound by that LDS-DMA fill (~32 GB/s per CU) plus a
// SwiGLU epilogue during which every wave of the CU idles the matrix pipe.  Here
//   * eight waves, two per SIMD (256 registers each); each wave keeps ITS OWN 32 X rows x 384 K in registers
//     for a whole work item (96 VGPRs of bf16 fragments, kXsMB = 2 m-blocks of 16 rows, loaded once from L2 /
//     HBM, with the folded-RMSNorm row sums taken from them), so only W streams through LDS: 64 W rows x 384 K
//     (48 KiB) per tile for 2 x 64 x 256 x 384 FLOP = 262 FLOP/B per workgroup (256 X rows), twice gemm_t's;
//   * the W tiles go through a 3-deep LDS ring by global_load_lds_dwordx4, tile t + 2 issued as soon as tile t
//     starts (its slot held tile t - 1, whose reads every wave finished before the barrier), so a tile has two
//     tiles of MFMAs to land; every lane issues a fixed number of stores per tile, which keeps the counted
//     vmcnt exact;
//     16-byte chunk c of W row r sits at LDS slot c ^ (r & 15) of its 768-byte row, which makes every
//     ds_read_b128 of the 16x16x32 fragment map conflict-free;
//   * the accumulators are small (2 m-blocks x 4 n-blocks x 4 per lane), so they are double-buffered: the
//     epilogue of tile t - 1 (bias, SwiGLU / GLU, bf16 pack, stores) is interleaved with the MFMAs of tile
//     t in the same wave instead of running with the matrix pipe idle.
// Work item = (256 X rows, a run of nc W tiles); items are dealt so the items of one X row block share an
// XCD (its X rows are fetched into one L2).  Epilogues (gemm.hip): SWIGLU / GLU on W rows interleaved in
// 32-row blocks (one 64-row W tile = one g | u block pair -> 32 output columns), STORE (+bias, bf16 out).
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

#include <type_traits>

namespace tone {
namespace {

constexpr int kXsK = 384;                 // K (d_model)
constexpr int kXsKS = kXsK / 32;          // 16x16x32 K-steps
constexpr int kXsWaves = 8;               // two waves per SIMD: 256 registers each
constexpr int kXsMB = 2;                  // 16-row m-blocks per wave
constexpr int kXsBM = kXsWaves * 16 * kXsMB;   // X rows per work item (256)
constexpr int kXsBN = 64;                 // W rows per tile
constexpr int kXsRowB = kXsK * 2;         // bytes per W row (768)
constexpr int kXsTile = kXsBN * kXsRowB;  // 48 KiB
constexpr int kXsR = 3;                   // W ring depth
constexpr int kXsPieces = kXsTile / 1024 / kXsWaves;   // 1 KiB DMA pieces per wave per tile (6)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t2 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pkb(float a, float b) {
  const __bf16 ha = (__bf16)a, hb = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

// DBG (XS_ABLATE microbenchmark builds only): 1 no epilogue in the loop, 2 no MFMA, 4 W DMA in the prologue only,
// 8 explicit K-step schedule, 16 no W reads from LDS, 32 no X loads
template <int EPI, bool RS, bool OBF, int DBG = 0>
__global__ void __launch_bounds__(kXsWaves * 64) gemm_xs_kernel(GemmArgs p, int nc) {
  static_assert(EPI == EPI_SWIGLU || EPI == EPI_GLU || EPI == EPI_STORE, "SWIGLU / GLU / STORE");
  constexpr bool PAIRED = (EPI != EPI_STORE);
  constexpr int kStores = 2 * kXsMB * (PAIRED ? 1 : 2);           // vector stores per tile epilogue (per lane)
  __shared__ __attribute__((aligned(16))) uint8_t lds[kXsR * kXsTile + 4 * kBiasMax];
  float* sbias = reinterpret_cast<float*>(lds + kXsR * kXsTile);

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lg = lane >> 4;
  const int nwt = p.N / kXsBN, ntm = (p.M + kXsBM - 1) / kXsBM, nch = (nwt + nc - 1) / nc;
  const int items = ntm * nch;
  // items of one X row block are consecutive; deal contiguous item ranges to XCDs (blocks b, b + 8, ... share one)
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (items + 7) >> 3, ibeg = xcd * q, iend = min(items, ibeg + q);
  if (ibeg + jb >= iend) return;                                  // workgroup-uniform

  for (int i = tid; i < p.N; i += kXsWaves * 64) sbias[i] = p.bias ? p.bias[i] : 0.f;
  __syncthreads();                                                // no DMA in flight yet

  const uint16_t* __restrict__ X = static_cast<const uint16_t*>(p.A);
  const uint8_t* __restrict__ Wb = static_cast<const uint8_t*>(p.W);

  // DMA of W tile t (global rows 64 t ..) into ring slot t % R: wave w moves pieces 6 w .. 6 w + 5; lane i of
  // piece pc lands at linear 16-byte slot 64 pc + i of the tile = (row, slot) with 48 slots per row and
  // fetches the chunk slot ^ (row & 15) of that row
  auto dma = [&](int t) {
    uint8_t* base = lds + (t % kXsR) * kXsTile;
    (void)base;
#pragma unroll
    for (int i = 0; i < kXsPieces; ++i) {
      const int pc = wid * kXsPieces + i, lin = pc * 64 + lane, row = lin / 48, slot = lin % 48;
      const uint8_t* src = Wb + ((int64_t)(t * kXsBN + row) * kXsK) * 2 + ((slot ^ (row & 15)) << 4);
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_global_load_lds(src, base + pc * 1024, 16, 0, 0);
#else
      (void)src;
#endif
    }
  };

  for (int item = ibeg + jb; item < iend; item += nxb) {
    const int mt = item / nch, ch = item % nch;
    const int t0 = ch * nc, t1 = min(nwt, t0 + nc), n = t1 - t0;
    const int mbase = mt * kXsBM + wid * 16 * kXsMB;              // this wave's 32 X rows

    // this wave's X fragments: m-block mb, K-step ks -> lane holds row mbase + 16 mb + l15, k 32 ks + 8 lg ..
    bf16x8_t xf[kXsMB][kXsKS];
    float inv[kXsMB];
#pragma unroll
    for (int mb = 0; mb < kXsMB; ++mb) {
      const int64_t row = min(mbase + 16 * mb + l15, p.M - 1);
      const uint16_t* xr = X + row * p.lda + 8 * lg;
      float ss = 0.f;
#pragma unroll
      for (int ks = 0; ks < kXsKS; ++ks) {
        if constexpr (DBG & 32) xf[mb][ks] = bf16x8_t{} + (__bf16)(float)(lane + ks + item);
        else xf[mb][ks] = *reinterpret_cast<const bf16x8_t*>(xr + 32 * ks);
        if constexpr (RS) ss = sumsq8(xf[mb][ks], ss);
      }
      if constexpr (RS) {
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        inv[mb] = 1.0f / (sqrtf(ss) * p.inv_sqrt_k + kRmsEps);
      } else {
        inv[mb] = 1.0f;
      }
    }

    f32x4_t2 acc[2][kXsMB][4];   // [buffer][mb][nb]
    // epilogue of W tile t from accumulator buffer b (one eighth at a time: part = mb * 2 + half)
    auto epi_part = [&](int b, int t, int part) __attribute__((always_inline)) {
      const int mb = part >> 1, hh = part & 1;
      // every lane stores (the counted vmcnt below relies on a fixed number of stores per tile): a row past M
      // holds row M - 1's values (its X fragments were clamped to that row), so it rewrites them unchanged
      const int64_t mrow = min(mbase + 16 * mb + l15, p.M - 1);
      if constexpr (PAIRED) {
        // g rows 16 nb + 4 lg + r (nb = hh), u rows 32 + 16 nb + 4 lg + r -> output column 32 t + 16 hh + 4 lg + r
        const int ng = kXsBN * t + 16 * hh + 4 * lg;
        // value pairs as two-float vectors: the fused multiply-adds and products issue as v_pk_* with the same
        // per-element roundings as the scalar form
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        float o[4];
        const f32x2 inv2 = {inv[mb], inv[mb]};
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const f32x2 g = __builtin_elementwise_fma(f32x2{acc[b][mb][hh][r], acc[b][mb][hh][r + 1]}, inv2,
                                                    f32x2{sbias[ng + r], sbias[ng + r + 1]});
          const f32x2 u = __builtin_elementwise_fma(f32x2{acc[b][mb][2 + hh][r], acc[b][mb][2 + hh][r + 1]}, inv2,
                                                    f32x2{sbias[ng + 32 + r], sbias[ng + 33 + r]});
          const f32x2 z = (EPI == EPI_SWIGLU) ? g : u;              // the sigmoid's argument
          const f32x2 t = z * -1.4426950408889634f;
          const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
          const f32x2 sg = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
          const f32x2 y = (EPI == EPI_SWIGLU) ? g * sg * u : g * sg;
          o[r] = y.x;
          o[r + 1] = y.y;
        }
        const int col = 32 * t + 16 * hh + 4 * lg;
        if constexpr (OBF) {
          const u32x2_t w = {pkb(o[0], o[1]), pkb(o[2], o[3])};
          *reinterpret_cast<u32x2_t*>(static_cast<uint16_t*>(p.C) + mrow * p.ldc + col) = w;
        } else {
          const f32x4_t2 w = {o[0], o[1], o[2], o[3]};
          *reinterpret_cast<f32x4_t2*>(static_cast<float*>(p.C) + mrow * p.ldc + col) = w;
        }
      } else {
#pragma unroll
        for (int nb2 = 0; nb2 < 2; ++nb2) {
          const int nb = 2 * hh + nb2, col = kXsBN * t + 16 * nb + 4 * lg;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = fmaf(acc[b][mb][nb][r], inv[mb], sbias[col + r]);
          const u32x2_t w = {pkb(o[0], o[1]), pkb(o[2], o[3])};
          *reinterpret_cast<u32x2_t*>(static_cast<uint16_t*>(p.C) + mrow * p.ldc + col) = w;
        }
      }
    };

    // ring prologue
    dma(t0);
    if (n > 1) dma(t0 + 1);
    // one W tile; the accumulator buffer is a compile-time index (B), so the tile loop is unrolled by two
    // (the first tile of an item, F = true, has no previous epilogue: peeled so no branch splits the K-steps)
    auto tile = [&](auto Bc, auto Fc, int j) __attribute__((always_inline)) {
      constexpr int b = decltype(Bc)::value;
      constexpr bool first = decltype(Fc)::value;
      const int t = t0 + j;
      // tile t landed (ring_younger: the ops issued after its DMA -- later DMAs and the fixed-count stores)
      ring_wait<kXsR, kXsPieces, kStores>(j, n);
      barrier_lds();                                              // ... for every wave; slot (t - 1) % R free
      if (j + 2 < n && !(DBG & 4)) dma(t + 2);                   // two tiles of lead
      const uint8_t* base = lds + (t % kXsR) * kXsTile;
#pragma unroll
      for (int mb = 0; mb < kXsMB; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[b][mb][nb] = f32x4_t2{0.f, 0.f, 0.f, 0.f};
      // W fragments one K-step ahead of the MFMAs that use them (two register sets), so the LDS latency of step
      // ks + 1 hides under step ks's MFMAs
      auto rdw = [&](int ks, bf16x8_t (&wf)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int row = 16 * nb + l15, c = 4 * ks + lg;
          wf[nb] = *reinterpret_cast<const bf16x8_t*>(base + row * kXsRowB + ((c ^ l15) << 4));
        }
      };
      bf16x8_t wa[4], wb[4];
      if constexpr (DBG & 16) {   // no LDS reads: fragments from X (the operands still feed the keep-alive)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) wa[nb] = wb[nb] = xf[0][nb];
      } else {
        rdw(0, wa);
      }
#pragma unroll
      for (int ks = 0; ks < kXsKS; ++ks) {
        bf16x8_t(&cur)[4] = (ks & 1) ? wb : wa;
        bf16x8_t(&nxt)[4] = (ks & 1) ? wa : wb;
        if (ks + 1 < kXsKS && !(DBG & 16)) rdw(ks + 1, nxt);
#pragma unroll
        for (int mb = 0; mb < kXsMB; ++mb)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
            if constexpr (DBG & 2) asm volatile("" ::"v"(cur[nb]), "v"(xf[mb][ks]));
            else acc[b][mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[nb], xf[mb][ks], acc[b][mb][nb], 0, 0, 0);
        // previous tile's epilogue, one part every other K-step, under these MFMAs
        if (!first && ks % 2 == 1 && ks / 2 < 2 * kXsMB && !(DBG & 1)) epi_part(b ^ 1, t - 1, ks / 2);
        if constexpr (DBG & 8) {   // the next step's W reads first, then the MFMAs with the epilogue's VALU between
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
          for (int i = 0; i < 2 * kXsMB * 2; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    tile(I0{}, std::true_type{}, 0);
    for (int j = 1; j < n; j += 2) {
      tile(I1{}, std::false_type{}, j);
      if (j + 1 < n) tile(I0{}, std::false_type{}, j + 1);
    }
    if ((n - 1) & 1) {
#pragma unroll
      for (int part = 0; part < 2 * kXsMB; ++part) epi_part(1, t1 - 1, part);
    } else {
#pragma unroll
      for (int part = 0; part < 2 * kXsMB; ++part) epi_part(0, t1 - 1, part);
    }
    __syncthreads();                                              // the ring is reused by the next item
  }
}

template <int EPI>
hipError_t launch_xs(const GemmArgs& a, int nc, hipStream_t st) {
  const int items = ((a.M + kXsBM - 1) / kXsBM) * ((a.N / kXsBN + nc - 1) / nc);
  int grid = 256;
  const int need = (items + 7) / 8 * 8;
  if (grid > need) grid = need;
#ifdef XS_ABLATE
  if constexpr (EPI == EPI_SWIGLU) {
    switch (a.rowscale ? a.dbg : 0) {
#define XS_D(d) case d: hipLaunchKernelGGL((gemm_xs_kernel<EPI, true, true, d>), dim3(grid), dim3(kXsWaves * 64), 0, st, a, nc); return hipGetLastError();
      XS_D(1) XS_D(2) XS_D(3) XS_D(4) XS_D(5) XS_D(6) XS_D(7) XS_D(8) XS_D(9) XS_D(23) XS_D(17) XS_D(55) XS_D(32) XS_D(39)
#undef XS_D
      default: break;
    }
  }
#endif
  constexpr bool kF32 = (EPI != EPI_STORE);   // fp32 output only for the paired epilogues (pw1 GLU -> dwconv)
  if (a.c_bf16) {
    if (a.rowscale) hipLaunchKernelGGL((gemm_xs_kernel<EPI, true, true>), dim3(grid), dim3(kXsWaves * 64), 0, st, a, nc);
    else hipLaunchKernelGGL((gemm_xs_kernel<EPI, false, true>), dim3(grid), dim3(kXsWaves * 64), 0, st, a, nc);
  } else if constexpr (kF32) {
    if (a.rowscale) hipLaunchKernelGGL((gemm_xs_kernel<EPI, true, false>), dim3(grid), dim3(kXsWaves * 64), 0, st, a, nc);
    else hipLaunchKernelGGL((gemm_xs_kernel<EPI, false, false>), dim3(grid), dim3(kXsWaves * 64), 0, st, a, nc);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

// nc = W tiles per work item (0: chosen so the items fill the 256 CUs in whole rounds)
hipError_t gemm_xs(const GemmArgs& a, int epi, int nc, hipStream_t st) {
  if (!a.a_bf16 || a.K != kXsK || a.N % kXsBN || a.N > kBiasMax || a.M <= 0 || a.rpg || a.lda % 8 || a.ldc % 8 ||
      a.k_split || a.C2)
    return hipErrorInvalidValue;
  if (epi == EPI_STORE && !a.c_bf16) return hipErrorInvalidValue;
  const int nwt = a.N / kXsBN, ntm = (a.M + kXsBM - 1) / kXsBM;
  if (nc <= 0) nc = xs_run_length(ntm, nwt);
  switch (epi) {
    case EPI_SWIGLU: return launch_xs<EPI_SWIGLU>(a, nc, st);
    case EPI_GLU: return launch_xs<EPI_GLU>(a, nc, st);
    case EPI_STORE: return launch_xs<EPI_STORE>(a, nc, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
