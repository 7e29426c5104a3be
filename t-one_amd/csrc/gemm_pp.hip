// fp32 projections by exact bf16 splitting on a ping-pong schedule (gemm_pp_kernel).
#include "gemm_common.h"

#include <cstdlib>

namespace tone {

// ---------------------------------------------------------------------------------------------
// fp32 projections by exact splitting, ping-pong schedule ("pp").
//
// The arithmetic of gemm_x3 (W and X as three bf16 terms each, the six products with i + j <= 2 on
// v_mfma_f32_32x32x16_bf16, fp32 accumulate).  What changes is the schedule.  gemm_x3's eight waves
// all run the same phases at the same time (DMA issue, fragment reads, the X split, MFMAs, one
// barrier per K-step), so the matrix pipe idles while every wave reads and splits: measured, the
// kernel costs the SUM of its MFMA, read/split and fill times.  Here the eight waves form two groups
// (waves 0-3 and 4-7: the two waves of each SIMD are in different groups) that alternate two kinds
// of segment, one barrier apart, the second group one segment behind the first:
//   L(j): issue this wave's LDS-DMA pieces of K-segment j + R - 1, read the W / X fragments of
//         segment j from LDS, split X into its three bf16 terms (and the folded-RMSNorm row sums of
//         squares), wait until this wave's pieces of segment j + 1 have landed;
//   C(j): the 6 x TI x TJ x KS MFMAs of segment j, nothing else.
// So on every SIMD one wave is in C while its partner is in L: the matrix pipe stays busy while
// LDS, VALU and the DMA issue run beside it.  Ring of R K-segments (KS x 16 deep); RAW: a segment's
// pieces are confirmed by their issuing waves' counted vmcnt at the end of an L two segments before
// any wave reads them, then a barrier; WAR: segment j + R - 1 goes into the buffer of j - 1, whose
// last reader (group 1's L(j - 1)) finished one barrier earlier.
// W comes K16-blocked, [3][K/16][N][16] (GemmArgs::W3b, written at upload), so every 1 KiB DMA piece
// is 32 whole rows of 32 B (contiguous in HBM); X stays fp32 [M][lda], pieces of 16 rows x 64 B.
// LDS per K16 sub-stage: W [3][BNW][32 B] (16-byte slot ^= (row >> 2) & 1), X [BMX][64 B]
// (slot ^= (row >> 1) & 3); both swizzles are applied to the per-lane DMA source address.
// The row factor of the folded RMSNorm stays in registers: every wave accumulates the sums of squares
// of its own X rows.
template <int BNW_, int BMX_, int WN_, int WM_, int KS_, int R_>
struct PT {
  static constexpr int BNW = BNW_, BMX = BMX_, WN = WN_, WM = WM_, KS = KS_, R = R_;
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// RG: the pieces go global -> VGPR -> ds_write_b128 instead of LDS-DMA: loaded in L(j) for segment j + R - 1,
// written in L(j + 1), read from L(j + R - 1) on (two register sets, the K loop unrolled by two; nk even).
template <class TL, int EPI, bool RS, bool RG = false>
__global__ void __launch_bounds__(512) gemm_pp_kernel(GemmArgs p) {
  constexpr int BNW = TL::BNW, BMX = TL::BMX, WN = TL::WN, WM = TL::WM, KS = TL::KS, R = TL::R;
  static_assert(WN * WM == 8, "8 waves");
  static_assert(R >= 3 && R <= 4, "ring of 3 or 4 K-segments");
  constexpr int WTN = BNW / WN, WTM = BMX / WM, TI = WTN / 32, TJ = WTM / 32;
  static_assert(TI >= 1 && TJ >= 1 && WTN % 32 == 0 && WTM % 32 == 0, "wave tile");
  constexpr int WSL = BNW * 32, XSL = BMX * 64;      // bytes of one K16 W plane slice / X slice
  constexpr int KSB = 3 * WSL + XSL, STAGE = KS * KSB;
  constexpr int WPC = 3 * BNW / 32, XPC = BMX / 16, PCS = KS * (WPC + XPC), IPW = PCS / 8;
  static_assert(PCS % 8 == 0 && BNW % 32 == 0 && BMX % 16 == 0, "DMA pieces per wave");
  __shared__ __attribute__((aligned(16))) uint8_t lds[R * STAGE + BNW * 4];
  float* sbias = reinterpret_cast<float*>(lds + R * STAGE);

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // SIMD partners (w, w + 4) are in different groups; dbg 32 (A/B): group by parity instead
  const int grp = (p.dbg & 32) ? (wid & 1) : (wid >> 2);
  const int wn = wid % WN, wm = wid / WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int ntn = p.N / BNW;
  int m0, n0;
  if (p.xcd_a) {
    const int a = p.xcd_a, xcd = blockIdx.x & 7, li = blockIdx.x >> 3;
    const int npg = ntn / a, mpg = ((p.M + BMX - 1) / BMX) / (8 / a);
    n0 = ((xcd % a) * npg + li % npg) * BNW;
    m0 = ((xcd / a) * mpg + li / npg) * BMX;
  } else {
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (blockIdx.x >> 3);
    m0 = (wgid / ntn) * BMX;
    n0 = (wgid % ntn) * BNW;
  }
  const int nk = p.K / (16 * KS);
  const float* __restrict__ X = static_cast<const float*>(p.A);
  const uint16_t* __restrict__ Wb = p.W3b;
  const int64_t plane = (int64_t)p.N * p.K;
  const bool no_mfma = p.dbg & 1, no_dma = p.dbg & 4;

  for (int i = tid; i < BNW; i += 512) sbias[i] = p.bias ? p.bias[n0 + i] : 0.f;

  // per-lane DMA source of each of this wave's pieces for K-segment 0, its advance per segment (bytes,
  // wave-uniform) and its LDS offset within a stage
  const uint8_t* src0[IPW];
  int64_t sstep[IPW];
  int doff[IPW];
  bool isw[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int piece = wid + 8 * i;                    // wave-uniform
    const int ks = piece / (WPC + XPC), pr = piece % (WPC + XPC);
    if (pr < WPC) {                                   // 32 W rows x 32 B of plane pl
      const int pl = pr / (BNW / 32), rb = (pr % (BNW / 32)) * 32, row = rb + (lane >> 1);
      const int slot = (lane & 1) ^ ((row >> 2) & 1);
      src0[i] = reinterpret_cast<const uint8_t*>(Wb + pl * plane + ((int64_t)ks * p.N + n0 + row) * 16 + slot * 8);
      sstep[i] = (int64_t)KS * p.N * 32;
      isw[i] = true;
      doff[i] = ks * KSB + pl * WSL + rb * 32;
    } else {                                          // 16 X rows x 64 B
      const int rb = (pr - WPC) * 16, row = rb + (lane >> 2);
      const int slot = (lane & 3) ^ ((row >> 1) & 3);
      src0[i] = reinterpret_cast<const uint8_t*>(X + (int64_t)min(m0 + row, p.M - 1) * p.lda + ks * 16 + slot * 4);
      sstep[i] = KS * 64;
      isw[i] = false;
      doff[i] = ks * KSB + 3 * WSL + rb * 64;
    }
  }
  auto stage = [&](int kt) {   // this wave's pieces of K-segment kt into buffer kt % R
    uint8_t* base = lds + (kt % R) * STAGE;
    if (no_dma) return;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if ((p.dbg & 128) && isw[i]) continue;          // A/B: X pieces only
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_global_load_lds(src0[i] + kt * sstep[i], base + doff[i], 16, 0, 0);
#else
      (void)base;
#endif
    }
  };
  // wait until at most c K-segments of this wave's pieces are in flight
  auto wait_segs = [&](int c) {
    if constexpr (R == 4) {
      if (c >= 2) vm_wait<2 * IPW>();
      else if (c == 1) vm_wait<IPW>();
      else vm_wait<0>();
    } else {
      if (c >= 1) vm_wait<IPW>();
      else vm_wait<0>();
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float ss[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) ss[j] = 0.f;
  bf16x8 w[KS][3][TI], xs[KS][3][TJ];

  u32x4 rg0[IPW], rg1[IPW];
  auto gload = [&](int seg, u32x4(&r)[IPW]) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) r[i] = *reinterpret_cast<const u32x4*>(src0[i] + seg * sstep[i]);
  };
  auto swrite = [&](int seg, const u32x4(&r)[IPW]) {
    uint8_t* base = lds + (seg % R) * STAGE;
#pragma unroll
    for (int i = 0; i < IPW; ++i) *reinterpret_cast<u32x4*>(base + doff[i] + lane * 16) = r[i];
  };
  auto seg_load = [&](int kt, u32x4(&rw)[IPW], u32x4(&rl)[IPW]) {
    if constexpr (RG) {
      if (kt + R - 2 < nk) swrite(kt + R - 2, rw);
      if (kt + R - 1 < nk) gload(kt + R - 1, rl);
    } else {
      if (kt + R - 1 < nk) stage(kt + R - 1);
    }
    const uint8_t* base = lds + (kt % R) * STAGE;
    f32x4 xv[KS][TJ][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wm * WTM + 32 * j + lr, cs = (row >> 1) & 3;
        const uint8_t* xr = base + ks * KSB + 3 * WSL + row * 64;
        xv[ks][j][0] = *reinterpret_cast<const f32x4*>(xr + (((2 * lh) ^ cs) << 4));
        xv[ks][j][1] = *reinterpret_cast<const f32x4*>(xr + (((2 * lh + 1) ^ cs) << 4));
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = wn * WTN + 32 * i + lr;
        const uint8_t* wr = base + ks * KSB + row * 32 + ((lh ^ ((row >> 2) & 1)) << 4);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) w[ks][pl][i] = *reinterpret_cast<const bf16x8*>(wr + pl * WSL);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        split3(xv[ks][j][0], xv[ks][j][1], xs[ks][0][j], xs[ks][1][j], xs[ks][2][j]);
        if constexpr (RS) {
          const f32x4 a = xv[ks][j][0], b = xv[ks][j][1];
          float t = ss[j];
          t = fmaf(a.x, a.x, t); t = fmaf(a.y, a.y, t); t = fmaf(a.z, a.z, t); t = fmaf(a.w, a.w, t);
          t = fmaf(b.x, b.x, t); t = fmaf(b.y, b.y, t); t = fmaf(b.z, b.z, t); t = fmaf(b.w, b.w, t);
          ss[j] = t;
        }
      }
    // pin the split here: without a use hipcc sinks it below the barrier into the MFMA segment
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) asm volatile("" : "+v"(xs[ks][pl][j]));
#pragma unroll
        for (int i = 0; i < TI; ++i) asm volatile("" : "+v"(w[ks][pl][i]));
      }
    if (!RG && !(p.dbg & 256)) wait_segs(min(kt + R, nk) - (kt + 2));   // this wave's pieces of segment kt + 1 landed
  };
  auto seg_mfma = [&]() {
    if (no_mfma) return;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // small terms first; the four (i, j) accumulators interleaved between dependent products
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        constexpr int wt[6] = {2, 1, 0, 1, 0, 0}, xt[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[ks][wt[t]][i], xs[ks][xt[t]][j], acc[i][j], 0, 0, 0);
      }
    }
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    barrier_lds();
    __builtin_amdgcn_sched_barrier(0);
  };

  const bool lock = p.dbg & 64;                       // A/B: both groups in lockstep (no ping-pong)
  if constexpr (RG) {
    for (int s = 0; s < R - 2 && s < nk; ++s) {
      gload(s, rg0);
      swrite(s, rg0);
    }
    if (R - 2 < nk) gload(R - 2, rg0);
    bar();
    if (grp == 1 && !lock) bar();
    for (int kt = 0; kt < nk; kt += 2) {              // nk even (launcher)
      seg_load(kt, rg0, rg1);
      bar();
      seg_mfma();
      bar();
      seg_load(kt + 1, rg1, rg0);
      bar();
      seg_mfma();
      if (kt + 2 < nk || grp == 0 || lock) bar();
    }
  } else {
    const int pro = min(R - 1, nk);
    for (int s = 0; s < pro; ++s) stage(s);
    wait_segs(pro - 1);                               // segment 0 landed (this wave's pieces)
    bar();                                            // ... and every wave's; sbias visible
    if (grp == 1 && !lock) bar();                     // group 1 runs one segment behind
    for (int kt = 0; kt < nk; ++kt) {
      seg_load(kt, rg0, rg1);
      bar();
      seg_mfma();
      if (kt + 1 < nk || grp == 0 || lock) bar();
    }
  }

  float invj[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const float t = ss[j] + __shfl_xor(ss[j], 32, 64);
    invj[j] = RS ? 1.0f / (sqrtf(t) * p.inv_sqrt_k + kRmsEps) : 1.0f;
  }
  if (p.dbg & 8) return;
  tile_epilogue_inv<EPI, RS, TI, TJ, WTN, WTM>(p, acc, invj, sbias, m0, n0, wn, wm, lr, lh);
}

template <class TL, int EPI, bool RG = false>
hipError_t launch_pp(const GemmArgs& a0, hipStream_t st) {
  GemmArgs a = a0;
  a.xcd_a = 0;
  const int ntn = a.N / TL::BNW, ntm = (a.M + TL::BMX - 1) / TL::BMX;
  if (a.dbg & 16) {   // 2D XCD blocks (microbenchmark): the smallest per-XCD compulsory fill, as x3_xcd_split
    const double wb = 6.0 * a.N * a.K, xb = 4.0 * a.M * a.K;
    double cost = wb + xb / 8;
    for (int s = 2; s <= 8; s *= 2) {
      if (ntn % s || ntm % (8 / s) || a.M % TL::BMX) continue;
      const double c = wb / s + xb / (8 / s);
      if (c < 0.8 * cost) { cost = c; a.xcd_a = s; }
    }
  }
  const dim3 tiles(ntn * ntm), block(512);
  if (RG && (a.K / (16 * TL::KS)) % 2) return hipErrorInvalidValue;
  if (a.rowscale) hipLaunchKernelGGL((gemm_pp_kernel<TL, EPI, true, RG>), tiles, block, 0, st, a);
  else hipLaunchKernelGGL((gemm_pp_kernel<TL, EPI, false, RG>), tiles, block, 0, st, a);
  return hipGetLastError();
}

template <class TL, bool RG = false>
hipError_t launch_pp_epi(const GemmArgs& a, int epi, hipStream_t st) {
  if (!a.W3b || a.a_bf16 || a.c_bf16 || a.rpg || a.a_plane || a.k_split || a.M <= 0 || a.N % TL::BNW ||
      a.K % (16 * TL::KS) || a.K / (16 * TL::KS) < 1 || a.lda % 4 || a.ldc % 8 ||
      (a.c_plane && (a.c_plane % 8 || (epi != EPI_SWIGLU && epi != EPI_GLU))) || a.c2_plane % 8)
    return hipErrorInvalidValue;
  constexpr bool pairable = (TL::BNW / TL::WN / 32) % 2 == 0;
  switch (epi) {
    case EPI_STORE: return launch_pp<TL, EPI_STORE, RG>(a, st);
    case EPI_RESID: return launch_pp<TL, EPI_RESID, RG>(a, st);
    case EPI_SWIGLU: if constexpr (pairable) return launch_pp<TL, EPI_SWIGLU, RG>(a, st); else return hipErrorInvalidValue;
    case EPI_GLU: if constexpr (pairable) return launch_pp<TL, EPI_GLU, RG>(a, st); else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// PT<BNW, BMX, WN, WM, KS, R>: tile BNW W rows x BMX X rows, 8 waves WN x WM, K-segments of 16 KS,
// a ring of R segments (LDS = R * KS * (96 BNW + 64 BMX) bytes)
hipError_t gemm_pp(const GemmArgs& a, int epi, int variant, hipStream_t st) {
  switch (variant) {
    case 0: return launch_pp_epi<PT<256, 128, 4, 2, 1, 4>>(a, epi, st);   // 128 KiB
    case 1: return launch_pp_epi<PT<256, 128, 4, 2, 1, 3>>(a, epi, st);   // 96 KiB
    case 2: return launch_pp_epi<PT<128, 128, 2, 4, 2, 3>>(a, epi, st);   // 120 KiB
    case 4: return launch_pp_epi<PT<128, 128, 4, 2, 2, 3>>(a, epi, st);   // 120 KiB, 32-row W wave tiles
    case 5: return launch_pp_epi<PT<128, 64, 4, 2, 2, 3>>(a, epi, st);    // 96 KiB
    // register-staged (global -> VGPR -> ds_write) instead of LDS-DMA
    case 6: return launch_pp_epi<PT<256, 128, 4, 2, 1, 4>, true>(a, epi, st);
    case 7: return launch_pp_epi<PT<256, 128, 4, 2, 1, 3>, true>(a, epi, st);
    case 8: return launch_pp_epi<PT<128, 128, 2, 4, 2, 3>, true>(a, epi, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
