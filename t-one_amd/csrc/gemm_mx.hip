// MXFP8 projections for TONE_PRECISION_FP8 (BASELINE config 5: fp8 MFMA on the q/k/v and FFN weights).
//
// Format: OCP MX -- every 32 consecutive values along K share one E8M0 scale (a power of two), the
// values are e4m3 (OCP e4m3fn, max 448).  A block with max |v| = a gets the exponent
// E = floor(log2 a) - 8, so v / 2^E lies below 512 and e4m3's 448 clamps the top of the binade
// (the OCP MX conversion rule).  Weights are quantized once at finalize (session.hip), activations
// by quant_mx_kernel below or, for the FFN intermediate, directly by the up-projection's epilogue.
//
// GEMM: v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, E8M0 scales): twice the bf16 MFMA rate per
// clock (MI355X_MICROARCH.md, Matrix cores).  Operand map, measured on the MI355X (tools/mx_probe.hip):
// lane l holds row (l & 15) and the k-values 16 g .. 16 g + 15 and 64 + 16 g .. 64 + 16 g + 15 of the
// 128-deep K-tile (g = l >> 4), and passes the scale of block g (k 32 g .. 32 g + 31) of its row.
// Structure as gemm_p_kernel (gemm_t.hip): transposed orientation D[n][m] = W[n] . X[m], persistent
// XCD-contiguous tiles, BNW (256 | 128) W rows x 256 X rows, K-tile = 128 fp8 = one 128-byte line per
// row, 16 KiB quarters staged by LDS-DMA into a two-stage ring, every fragment of a K-tile read in
// its first two MFMA phases so the stage is free after the first barrier, the whole of K-tile t+2 issued
// right after that barrier and kept in flight across the end-of-step wait (counted vmcnt).  The tile's
// scales, bias and row factors go to LDS at the tile's start; tile positions advance once per K-tile.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace tone {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void barrier_lds() {   // keeps LDS-DMA in flight (no vmcnt(0) fence)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ float fsig(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}

// 8 floats -> 8 e4m3 bytes of the block with biased exponent e (common.h mx_exp / mx_cvt2: the scaled conversion, no
// saturation needed with the exponent's headroom; a NaN stays a NaN)
__device__ __forceinline__ u32x2 quant8(const float (&v)[8], int e) {
  const float sc = mx_scale(e);
  uint32_t w0 = mx_cvt2<false>(v[0], v[1], sc, 0u);
  w0 = mx_cvt2<true>(v[2], v[3], sc, w0);
  uint32_t w1 = mx_cvt2<false>(v[4], v[5], sc, 0u);
  w1 = mx_cvt2<true>(v[6], v[7], sc, w1);
  return u32x2{w0, w1};
}

}  // namespace

// ---- activation quantization: bf16 [M][K] -> e4m3 [M][K] + E8M0 [M][K/32] (+ 1/(rms + eps)) -------
// one wave per row, 8 values per lane per pass; the four lanes of a 32-block reduce their max with two
// xor shuffles.  inv (optional): 1 / (||x||_2 / sqrt(K) + 1e-8), the folded RMSNorm row factor.
__global__ void __launch_bounds__(256) quant_mx_kernel(const uint16_t* __restrict__ X, int64_t ldx, int M, int K,
                                                       uint8_t* __restrict__ Q, uint8_t* __restrict__ S,
                                                       float* __restrict__ ss8) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;                                    // wave-uniform
  const uint16_t* x = X + (int64_t)row * ldx;
  float ss = 0.f;
  for (int c0 = 0; c0 < K / 8; c0 += 64) {
    const int c = c0 + lane;
    const bool on = c < K / 8;
    u32x4 u = {0u, 0u, 0u, 0u};
    if (on) u = *reinterpret_cast<const u32x4*>(x + 8 * c);
    float v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      am = fmaxf(am, fabsf(v[i]));
      ss = fmaf(v[i], v[i], ss);
    }
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    const int e = mx_exp(am);
    const u32x2 q = quant8(v, e);
    if (on) {
      *reinterpret_cast<u32x2*>(Q + (int64_t)row * K + 8 * c) = q;
      if ((c & 3) == 0) S[(int64_t)row * (K / 32) + c / 4] = (uint8_t)e;
    }
  }
  if (ss8) {   // the whole row's sum in slot 0, zeros in the others (common.h kSsSlots)
    ss = wave_sum(ss);
    if (lane < kSsSlots) ss8[(int64_t)row * kSsSlots + lane] = lane == 0 ? ss : 0.f;
  }
}

hipError_t launch_quant_mx(const uint16_t* X, int64_t ldx, int M, int K, uint8_t* Q, uint8_t* S, float* ss8,
                           hipStream_t st) {
  if (K % 32 || M <= 0 || ldx % 8 || (ss8 && K != 32 * kSsSlots)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(quant_mx_kernel, dim3((M + 3) / 4), dim3(256), 0, st, X, ldx, M, K, Q, S, ss8);
  return hipGetLastError();
}

namespace {

constexpr int kMxKB = kDff / 32;   // largest K / 32 (FFN down: 48 scale bytes per row)

// the fragment of row r is 16-byte chunks (l >> 4) and 4 + (l >> 4) of its 128-byte line: the bf16
// kernels' slot ^= (r >> 1) & 7 makes both ds_read_b128 conflict-free
__device__ __forceinline__ int mx_swz(int r) { return (r >> 1) & 7; }

// DBG (microbenchmark ablations only): bit 0 no epilogue, bit 1 side data (scales, bias, row factors)
// loaded for the first tile only, bit 2 no MFMA; every accumulator stays live
// BMX: X rows per tile (256, or 128 for STORE / RESID when the 256-row tiles would leave the CUs one tile each:
// two tiles per CU overlap one tile's HBM-bound epilogue with the next one's K loop); waves WNW (W) x WMW (X)
template <int BNW, int EPI, bool RS, int DBG = 0, int BMX = 256, bool R16 = false>
__global__ void __launch_bounds__(512) gemm_mx_kernel(MxArgs p) {
  constexpr int BK = 128, QB = 128 * BK, NQW = BNW / 128, XQ = BMX / 128, STG = (NQW + XQ) * QB;
  constexpr int WMW = BMX / 64, WNW = 8 / WMW, RW = BNW / WNW;   // waves along X / W, W rows per wave
  constexpr int TI = RW / 16, TH = TI / 2;                   // n-tiles per wave, per phase half
  static_assert(TH >= 1 && (EPI != EPI_SWIGLU || TI % 4 == 0), "wave tile");
  constexpr bool PAIRED = (EPI == EPI_SWIGLU);
  static_assert(EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_SWIGLU, "STORE/RESID/SWIGLU");
  // ONE LDS object: ring | W scales [BNW][48] | X scales [BMX][48] | bias [BNW] | row factors [BMX]
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STG + (BNW + BMX) * kMxKB + 4 * (BNW + BMX)];
  uint8_t* sW = lds + 2 * STG;
  uint8_t* sX = sW + BNW * kMxKB;
  float* sb = reinterpret_cast<float*>(sX + BMX * kMxKB);
  float* sr = sb + BNW;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / WMW, wm = wid % WMW, l15 = lane & 15, lg = lane >> 4, g = mx_swz(l15);
  const int ntn = p.N / BNW, ntm = (p.M + BMX - 1) / BMX, ntiles = ntn * ntm;
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (ntiles + 7) >> 3, tbeg = xcd * q, tend = min(ntiles, tbeg + q);
  const int nmine = (tbeg + jb < tend) ? (tend - tbeg - jb + nxb - 1) / nxb : 0;
  if (nmine <= 0) return;                                       // workgroup-uniform
  const int nk = p.K / BK, KB = p.K / 32, G = nmine * nk;

  // running position of a K-step (uniform scalars): K-tile kt of the workgroup's ti-th tile at (m0, n0).  The
  // loop carries the positions of steps t, t + 1, t + 2 and advances the last once per step, so the tile
  // index divisions run once per tile instead of once per DMA quarter (they were ~130 SALU per K-step)
  struct Pos {
    int kt, ti, m0, n0;
  };
  auto pos_tile = [&](Pos& s) {
    const int t = tbeg + jb + s.ti * nxb;
    s.m0 = (t / ntn) * BMX;
    s.n0 = (t % ntn) * BNW;
  };
  auto advance = [&](Pos& s) {
    if (++s.kt == nk) {
      s.kt = 0;
      ++s.ti;
      pos_tile(s);
    }
  };
  // quarter j of K-step u (position s): W rows 128 j.. (j < NQW) or X rows 128 (j - NQW)..; pieces of 8 rows x 128 B
  auto issue = [&](int u, const Pos& s, int j) {
    if constexpr ((DBG & 16) != 0)   // no DMA after the first two K-steps (timing only)
      if (u >= 2) return;
    const int m0 = s.m0, n0 = s.n0, k0 = s.kt * BK;
    uint8_t* dst = lds + (u & 1) * STG + j * QB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int piece = 2 * wid + h, row = piece * 8 + (lane >> 3);
      const int c = (lane & 7) ^ mx_swz(row);
      const uint8_t* src = (j < NQW) ? p.W + (int64_t)(n0 + 128 * j + row) * p.K + k0 + 16 * c
                                     : p.A + (int64_t)min(m0 + 128 * (j - NQW) + row, p.M - 1) * p.lda + k0 + 16 * c;
      lds_dma16(src, dst + piece * 8 * BK);
    }
  };
  auto issue_kt = [&](int u, const Pos& s, int from, int to) {   // quarters [from, to) of K-step u (NQW + XQ each)
    for (int j = from; j < to; ++j) issue(u, s, j);
  };
  // per-tile side data: scales, bias, row factors (at tile boundaries only).  Fetched into registers as dwords,
  // every load issued before any LDS store, the next tile's fetch ahead of this tile's epilogue: the byte-wise
  // load/store loop it replaces cost ~5 us per tile boundary at M = 40960 (profiles/r03_mx_resid_ablate3.jsonl)
  constexpr int XD = BMX * (kMxKB / 4) / 512, WD = (BNW * (kMxKB / 4) + 511) / 512;
  struct Side {
    uint32_t x[XD], w[WD];
    float b, r;
  };
  auto side_fetch = [&](const Pos& s) {
    const int m0 = s.m0, n0 = s.n0, nd = KB >> 2;   // dwords of scales per row
    Side v;
#pragma unroll
    for (int q = 0; q < XD; ++q) {
      const int i = tid + 512 * q, r = i / nd, c = i - r * nd;
      v.x[q] = r < BMX ? *reinterpret_cast<const uint32_t*>(p.As + (int64_t)min(m0 + r, p.M - 1) * p.ldas + 4 * c) : 0u;
    }
#pragma unroll
    for (int q = 0; q < WD; ++q) {
      const int i = tid + 512 * q, r = i / nd, c = i - r * nd;
      v.w[q] = r < BNW ? *reinterpret_cast<const uint32_t*>(p.Ws + (int64_t)(n0 + r) * KB + 4 * c) : 0u;
    }
    v.b = (tid < BNW && p.bias) ? p.bias[n0 + tid] : 0.f;
    v.r = (RS && tid < BMX) ? mx_row_inv(p.rs_ss + (int64_t)min(m0 + tid, p.M - 1) * kSsSlots) : 1.f;
    return v;
  };
  auto side_store = [&](const Side& v) {
    const int nd = KB >> 2;
#pragma unroll
    for (int q = 0; q < XD; ++q) {
      const int i = tid + 512 * q, r = i / nd, c = i - r * nd;
      if (r < BMX) *reinterpret_cast<uint32_t*>(sX + r * kMxKB + 4 * c) = v.x[q];
    }
#pragma unroll
    for (int q = 0; q < WD; ++q) {
      const int i = tid + 512 * q, r = i / nd, c = i - r * nd;
      if (r < BNW) *reinterpret_cast<uint32_t*>(sW + r * kMxKB + 4 * c) = v.w[q];
    }
    if (tid < BNW) sb[tid] = v.b;
    if (RS && tid < BMX) sr[tid] = v.r;
  };

  const uint8_t* wq = lds + (wn * RW / 128) * QB + ((wn * RW) % 128) * BK;   // wave's W rows
  const uint8_t* xq = lds + (NQW + (wm >> 1)) * QB + (wm & 1) * 64 * BK;
  const int wrow0 = wn * RW, xrow0 = wm * 64;
  auto rd = [&](const uint8_t* qb, int buf, int tile) {
    if constexpr ((DBG & 8) != 0) {   // no fragment reads from LDS (timing only)
      const int v = (int)(intptr_t)qb ^ (buf << 4) ^ tile;
      return i32x8{v, v, v, v, v, v, v, v};
    }
    const uint8_t* r = qb + buf * STG + (16 * tile + l15) * BK;
    const u32x4 a = *reinterpret_cast<const u32x4*>(r + 16 * (lg ^ g));
    const u32x4 b = *reinterpret_cast<const u32x4*>(r + 16 * ((4 + lg) ^ g));
    return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
  };

  f32x4 acc[TI][4];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto epilogue = [&](const Pos& s) {
    const int m0 = s.m0, n0 = s.n0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ml = xrow0 + 16 * j + l15, m = m0 + ml;
      const bool ok = m < p.M;
      const int64_t mrow = min(m, p.M - 1);
      const float inv = RS ? sr[ml] : 1.0f;
      if constexpr (PAIRED) {
        // W rows interleaved in 32-row blocks (g | u); tiles ig, ig + 1 (g) pair with ig + 2, ig + 3 (u)
#pragma unroll
        for (int pb = 0; pb < TI / 4; ++pb) {
          float o[2][4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int ig = 4 * pb + h, nl = wrow0 + 16 * ig + 4 * lg;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gg = fmaf(acc[ig][j][r], inv, sb[nl + r]);
              const float uu = fmaf(acc[ig + 2][j][r], inv, sb[nl + 32 + r]);
              o[h][r] = gg * fsig(gg) * uu;
            }
          }
          // lanes lg = 0..3 of this row hold the 32-column MX block: swap so each holds 8 contiguous
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(o[0][r]), __float_as_uint(o[1][r]), false, false);
            v[r] = __uint_as_float(sw[0]);
            v[4 + r] = __uint_as_float(sw[1]);
          }
          float am = 0.f;
#pragma unroll
          for (int r = 0; r < 8; ++r) am = fmaxf(am, fabsf(v[r]));
          am = lg_max(am);
          const int e = mx_exp(am);
          const u32x2 qv = quant8(v, e);
          const int blk = (n0 >> 1) + (wrow0 >> 1) + 32 * pb;     // first output column of the block
          if (ok) {
            *reinterpret_cast<u32x2*>(p.C8 + mrow * p.ldc + blk + 16 * (lg & 1) + 8 * (lg >> 1)) = qv;
            if (lg == 0) p.C8s[mrow * p.ldc8s + blk / 32] = (uint8_t)e;
          }
        }
      } else {
        float vq[TI][4];   // RESID with Q8: the shadow's bf16 values, for its MXFP8 form
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int nl = wrow0 + 16 * i + 4 * lg;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaf(acc[i][j][r], inv, sb[nl + r]);
          if constexpr (EPI == EPI_RESID) {
            const f32x4 rr = load_res4(p.R, mrow * p.ldr + n0 + nl, R16);   // fp32 or the fp16 residual stream
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rr[r] + p.alpha * v[r];
          }
          if (EPI == EPI_RESID || !p.c_bf16) {
            const f32x4 w = {v[0], v[1], v[2], v[3]};
            if (ok) store_res4(p.C, mrow * p.ldc + n0 + nl, w, EPI == EPI_RESID && R16);
          }
          if ((EPI == EPI_STORE && p.c_bf16) || p.C2) {
            uint16_t* dst = (EPI == EPI_STORE && p.c_bf16) ? static_cast<uint16_t*>(p.C) : p.C2;
            const __bf16 b0 = (__bf16)v[0], b1 = (__bf16)v[1], b2 = (__bf16)v[2], b3 = (__bf16)v[3];
            const u32x2 w = {(uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16),
                             (uint32_t)__builtin_bit_cast(uint16_t, b2) | ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16)};
            if (ok) *reinterpret_cast<u32x2*>(dst + mrow * p.ldc + n0 + nl) = w;
            vq[i][0] = (float)b0;
            vq[i][1] = (float)b1;
            vq[i][2] = (float)b2;
            vq[i][3] = (float)b3;
          }
        }
        if constexpr (EPI == EPI_RESID) {
          if (p.Q8) {
            // the MXFP8 form of this row's shadow values, as quant_mx would make it: a 32-column block is tiles
            // 2k, 2k + 1 across the row's four lanes lg; the wave's partial sum of squares over its RW columns goes
            // to the first of its RW / 32 slots of the row's sum-of-squares slab (zeros in the others)
            float ssq = 0.f;
#pragma unroll
            for (int k = 0; k < TI / 2; ++k) {
              float am = 0.f;
#pragma unroll
              for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  am = fmaxf(am, fabsf(vq[2 * k + h][r]));
                  ssq = fmaf(vq[2 * k + h][r], vq[2 * k + h][r], ssq);
                }
              am = lg_max(am);
              const int e = mx_exp(am);
              const int col = n0 + wrow0 + 32 * k + 4 * lg;
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const uint32_t q4 = quant4(vq[2 * k + h][0], vq[2 * k + h][1], vq[2 * k + h][2], vq[2 * k + h][3], e);
                if (ok) *reinterpret_cast<uint32_t*>(p.Q8 + mrow * p.ldc + col + 16 * h) = q4;
              }
              if (ok && lg == 0) p.Q8s[mrow * (p.ldc / 32) + (n0 + wrow0) / 32 + k] = (uint8_t)e;
            }
            ssq = lg_sum(ssq);
            if (ok && lg == 0) {
#pragma unroll
              for (int k = 0; k < RW / 32; ++k) p.ss8[mrow * kSsSlots + (n0 + wrow0) / 32 + k] = k == 0 ? ssq : 0.f;
            }
          }
        }
      }
    }
  };

  Pos s0{0, 0, 0, 0};
  pos_tile(s0);
  Pos s1 = s0;
  advance(s1);
  Pos s2 = s1;
  advance(s2);
  zero();
  constexpr int QPT = NQW + XQ;                                 // quarters per K-tile
  // prologue: K-tile 0 whole, the first half of K-tile 1's quarters
  // E quarters of K-step t + 2 go out after the stage-freeing barrier of step t, the other QPT - E in the first
  // two phases of step t + 1.  All of them (E = QPT): the X quarters, the ones that miss L2, get 1.5 steps of
  // cover instead of one (FFN down M = 40960: 62.0 -> 60.3 us; profiles/r03_mx_resid_early.jsonl); DBG bit 64
  // restores E = QPT / 2 for the A/B
  constexpr int E = (DBG & 64) ? QPT / 2 : QPT;
  issue_kt(0, s0, 0, QPT);
  if (G > 1) issue_kt(1, s1, 0, E);
  // the first tile's side data behind the prologue DMA (its latency overlaps the ring fill; the region is disjoint)
  side_store(side_fetch(s0));
  __syncthreads();                                              // side data visible
  if (G > 1) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * E) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier_lds();
  for (int t = 0; t < G; ++t) {
    const int buf = t & 1, kt = s0.kt;
    i32x8 xf[4], wa[TH], wb[TH];
    int xs[4], wsa[TH], wsb[TH];
    // phase 0: every X fragment + the first half of the W tiles
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xf[j] = rd(xq, buf, j);
      xs[j] = sX[(xrow0 + 16 * j + l15) * kMxKB + 4 * kt + lg];
    }
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      wa[i] = rd(wq, buf, i);
      wsa[i] = sW[(wrow0 + 16 * i + l15) * kMxKB + 4 * kt + lg];
    }
    if (t + 1 < G) issue_kt(t + 1, s1, E, E + (QPT - E + 1) / 2);
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = (DBG & 4) ? acc[i][j] + (float)(wa[i][0] ^ xf[j][1] ^ wsa[i] ^ xs[j])
                              : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wa[i], xf[j], acc[i][j], 0, 0, 0, wsa[i], 0, xs[j]);
    // phase 1: the second half of the W tiles (the stage's last reads)
#pragma unroll
    for (int i = 0; i < TH; ++i) {
      wb[i] = rd(wq, buf, TH + i);
      wsb[i] = sW[(wrow0 + 16 * (TH + i) + l15) * kMxKB + 4 * kt + lg];
    }
    if (t + 1 < G) issue_kt(t + 1, s1, E + (QPT - E + 1) / 2, QPT);
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int j = 2; j < 4; ++j)
        acc[i][j] = (DBG & 4) ? acc[i][j] + (float)(wa[i][2] ^ xf[j][3] ^ wsa[i] ^ xs[j])
                              : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wa[i], xf[j], acc[i][j], 0, 0, 0, wsa[i], 0, xs[j]);
    if constexpr (!(DBG & 128)) barrier_lds();                  // every wave's reads of stage buf done (128: timing only)
    // phase 2
    if (t + 2 < G) issue_kt(t + 2, s2, 0, (E + 1) / 2);
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int j = 2; j < 4; ++j)
        acc[TH + i][j] = (DBG & 4) ? acc[TH + i][j] + (float)(wb[i][4] ^ xf[j][5] ^ wsb[i] ^ xs[j])
                                   : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wb[i], xf[j], acc[TH + i][j], 0, 0, 0, wsb[i], 0, xs[j]);
    // phase 3
    if (t + 2 < G) issue_kt(t + 2, s2, (E + 1) / 2, E);
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[TH + i][j] = (DBG & 4) ? acc[TH + i][j] + (float)(wb[i][6] ^ xf[j][7] ^ wsb[i] ^ xs[j])
                                   : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wb[i], xf[j], acc[TH + i][j], 0, 0, 0, wsb[i], 0, xs[j]);
    // K-tile t+1 landed; the E quarters of K-tile t+2 (2 pieces each) stay in flight
    if (t + 2 < G) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * E) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_lds();
    if (kt == nk - 1) {
      const bool more = t + 1 < G && !(DBG & 2);
      Side nxt;
      if (more) nxt = side_fetch(s1);                           // in flight under the epilogue
      if constexpr ((DBG & 1) != 0) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)   // never true (alpha is finite): keeps every accumulator live
            if (p.alpha == -1.2345e30f) *reinterpret_cast<f32x4*>(static_cast<float*>(p.C) + 4 * (64 * (i * 4 + j) + lane)) = acc[i][j];
      } else {
        epilogue(s0);
      }
      zero();
      if (more) {
        __syncthreads();                                        // every epilogue done with the side data
        side_store(nxt);
        __syncthreads();
      }
    }
    s0 = s1;
    s1 = s2;
    advance(s2);
  }
}

template <int BNW, int EPI, int BMX = 256>
hipError_t launch_mx(const MxArgs& a, hipStream_t st) {
  const int ntiles = (a.N / BNW) * ((a.M + BMX - 1) / BMX);
  int grid = 256;
  const int need = ((ntiles + 7) / 8) * 8;
  if (grid > need) grid = need;
#ifdef XS8_ABLATE
  if (getenv("MXGRID")) grid = std::min(grid, atoi(getenv("MXGRID")));   // persistent-grid size sweep
  if constexpr (EPI == EPI_SWIGLU) {   // microbenchmark ablations (tools/gemm_bench MXDBG)
    switch (a.dbg) {
      case 0: break;
      case 1: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 1>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
      case 2: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 2>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
      case 3: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 3>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
      case 4: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 4>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
      case 7: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 7>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
      default: return hipErrorInvalidValue;
    }
  }
  if constexpr (EPI == EPI_RESID) {   // K-loop / epilogue split of the fp8 FFN down (no epilogue; no MFMA; neither)
    // MXDBG = 256 x (kernel DBG bits): 1 no epilogue, 2 side data for the first tile only, 4 no MFMA, 8 no LDS fragment reads, 16 no DMA, 64 E = QPT / 2, 128 no mid-step barrier (races: timing only)
#define TONE_MXA(d) \
  case d: hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, false, d, BMX>), dim3(grid), dim3(512), 0, st, a); return hipGetLastError();
    switch (a.dbg >> 8) {
      case 0: break;
      TONE_MXA(1) TONE_MXA(3) TONE_MXA(4) TONE_MXA(5) TONE_MXA(13) TONE_MXA(21) TONE_MXA(29) TONE_MXA(31) TONE_MXA(64) TONE_MXA(65) TONE_MXA(129) TONE_MXA(159)
      default: return hipErrorInvalidValue;
    }
#undef TONE_MXA
  }
#endif
  if constexpr (EPI == EPI_RESID) {   // the residual stream fp16 (R16, the fp8 mode's) or fp32
    if (a.rs_ss) return hipErrorInvalidValue;
    if (a.res16) hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, false, 0, BMX, true>), dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, false, 0, BMX>), dim3(grid), dim3(512), 0, st, a);
    return hipGetLastError();
  }
  if (a.res16) return hipErrorInvalidValue;
  if (a.rs_ss) hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, true, 0, BMX>), dim3(grid), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm_mx_kernel<BNW, EPI, false, 0, BMX>), dim3(grid), dim3(512), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// X-stationary MXFP8 GEMM for K = 384 (FFN up + SwiGLU -> MXFP8 h, q|k|v STORE), the fp8 form of round 3's bf16
// gemm_xs (now gemm_xw.hip): each wave keeps its 32 X rows x 384 e4m3 in registers (48 VGPRs) with their E8M0 scales and
// row factors, W tiles of 64 rows x 384 B (24 KiB) stream through a 4-deep LDS ring (chunk c of row r at slot
// c ^ ((r >> 1) & 7), the mx_swz map on 384-byte rows: conflict-free for both ds_read_b128 of a fragment), the
// W scales of the whole matrix sit in LDS for the launch, and the accumulators are double-buffered so tile
// t - 1's epilogue (SwiGLU + the MXFP8 quantization of h: one 64-row W tile = one 32-column MX block of h)
// runs under tile t's MFMAs.  2 x 64 x 256 x 384 FLOP per 24 KiB of W: 524 FLOP per staged byte.
constexpr int kX8K = 384, kX8KS = kX8K / 128, kX8BM = 256, kX8BN = 64, kX8Tile = kX8BN * kX8K, kX8R = 4;
constexpr int kX8Pieces = kX8Tile / 1024 / 8;   // 3
constexpr int kX8MaxN = 3072;

// DBG (XS8_ABLATE microbenchmark builds only): 1 no epilogue, 2 no MFMA, 4 no W DMA after the prologue, 8 SwiGLU
// without the MX quantization (raw bits stored), 16 no workgroup barrier per W tile (wrong results: timing only),
// 32 static priority for waves 4-7, 256 no W fragment reads, 512 no X loads, 1024 no epilogue stores, 2048 no bias
// reads (timing only)
template <int EPI, bool RS, int DBG = 0>
__global__ void __launch_bounds__(512) gemm_xs8_kernel(MxArgs p, int nc) {
  static_assert(EPI == EPI_SWIGLU || EPI == EPI_STORE, "SWIGLU / STORE");
  constexpr int kStores8 = EPI == EPI_SWIGLU ? 2 * 3 : 4 * 2;      // vector stores per tile epilogue (per lane)
  // W scales [N][12] and bias first, the ring after them: every per-tile scale read is then a per-tile base plus an
  // immediate below 64 KiB (behind a 96 KiB ring each of the 12 scale reads of a tile took its own address add)
  constexpr int kRingOff = kX8MaxN * (kX8K / 32) + 4 * kX8MaxN;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRingOff + kX8R * kX8Tile];
  uint8_t* sWs = lds;
  float* sb = reinterpret_cast<float*>(sWs + kX8MaxN * (kX8K / 32));
  uint8_t* ring = lds + kRingOff;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lg = lane >> 4, swz = (l15 >> 1) & 7;
  if constexpr ((DBG & 32) != 0) {
    if (wid >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int nwt = p.N / kX8BN, ntm = (p.M + kX8BM - 1) / kX8BM, nch = (nwt + nc - 1) / nc;
  const int items = ntm * nch;
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (items + 7) >> 3, ibeg = xcd * q, iend = min(items, ibeg + q);
  if (ibeg + jb >= iend) return;                                  // workgroup-uniform

  // W scales and bias for the launch: 16-byte pieces, every load ahead of the LDS stores (a byte-wise
  // load/store loop here was 72 dependent round trips per thread at N = 3072)
  if ((((uintptr_t)p.Ws | (uintptr_t)p.bias) & 15) == 0) {
    constexpr int kSq = (kX8MaxN * (kX8K / 32) / 16 + 511) / 512, kBq = (kX8MaxN / 4 + 511) / 512;
    const int nsq = p.N * (kX8K / 32) / 16, nbq = p.N / 4;
    u32x4 vs[kSq];
    f32x4 vb[kBq];
#pragma unroll
    for (int q = 0; q < kSq; ++q)
      if (tid + 512 * q < nsq) vs[q] = reinterpret_cast<const u32x4*>(p.Ws)[tid + 512 * q];
#pragma unroll
    for (int q = 0; q < kSq; ++q)
      if (tid + 512 * q < nsq) reinterpret_cast<u32x4*>(sWs)[tid + 512 * q] = vs[q];
#pragma unroll
    for (int q = 0; q < kBq; ++q)
      if (tid + 512 * q < nbq) vb[q] = p.bias ? reinterpret_cast<const f32x4*>(p.bias)[tid + 512 * q] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < kBq; ++q)
      if (tid + 512 * q < nbq) reinterpret_cast<f32x4*>(sb)[tid + 512 * q] = vb[q];
  } else {
    for (int i = tid; i < p.N * (kX8K / 32); i += 512) sWs[i] = p.Ws[i];
    for (int i = tid; i < p.N; i += 512) sb[i] = p.bias ? p.bias[i] : 0.f;
  }
  __syncthreads();                                                // no DMA in flight yet

  // the lane's byte offset in a W tile for each of its DMA pieces, computed once (32-bit: three VGPRs; recomputed per
  // tile the division by 24 and its multiplies were ~35 VALU of the tile's VALU-bound epilogue budget)
  uint32_t doff[kX8Pieces];
#pragma unroll
  for (int i = 0; i < kX8Pieces; ++i) {
    const int pc = wid * kX8Pieces + i, lin = pc * 64 + lane, row = lin / 24, slot = lin % 24;
    doff[i] = (uint32_t)(row * kX8K + ((slot ^ ((row >> 1) & 7)) << 4));
  }
  auto dma = [&](int t) {
    uint8_t* base = ring + (t % kX8R) * kX8Tile;
    (void)base;
    const uint8_t* wt = p.W + (int64_t)t * kX8Tile;               // uniform: the tile's first W row
#pragma unroll
    for (int i = 0; i < kX8Pieces; ++i) {
      const uint8_t* src = wt + doff[i];
      lds_dma16(src, base + (wid * kX8Pieces + i) * 1024);
    }
  };

  for (int item = ibeg + jb; item < iend; item += nxb) {
    const int mt = item / nch, ch = item % nch;
    const int t0 = ch * nc, t1 = min(nwt, t0 + nc), n = t1 - t0;
    const int mbase = mt * kX8BM + wid * 32;

    i32x8 xf[2][kX8KS];
    int xs[2][kX8KS];
    float inv[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int64_t row = min(mbase + 16 * mb + l15, p.M - 1);
      const uint8_t* xr = p.A + row * p.lda;
#pragma unroll
      for (int ks = 0; ks < kX8KS; ++ks) {
        if constexpr ((DBG & 512) != 0) {   // no X loads (timing only)
          xf[mb][ks] = i32x8{} + (int)(lane * 0x01010101u + ks + item);
          xs[mb][ks] = 127;
        } else {
          const u32x4 a = *reinterpret_cast<const u32x4*>(xr + 128 * ks + 16 * lg);
          const u32x4 b = *reinterpret_cast<const u32x4*>(xr + 128 * ks + 64 + 16 * lg);
          xf[mb][ks] = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
          xs[mb][ks] = p.As[row * p.ldas + 4 * ks + lg];
        }
      }
      inv[mb] = RS && !(DBG & 512) ? mx_row_inv(p.rs_ss + row * kSsSlots) : 1.0f;
    }

    f32x4 acc[2][2][4];   // [buffer][mb][nb]
    // output row offsets of this lane's two rows (32-bit, from the uniform bases; every lane stores -- fixed count
    // per tile for the counted vmcnt -- and a row past M rewrites row M - 1's values)
    uint32_t orow[2], srow[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const uint32_t mrow = (uint32_t)min(mbase + 16 * mb + l15, p.M - 1);
      orow[mb] = mrow * (uint32_t)p.ldc;
      srow[mb] = mrow * (uint32_t)p.ldc8s;
    }
    // SwiGLU bias of the tile whose epilogue runs next: its 16 values per lane (g and u, columns 16 h2 + 4 lg + r) are
    // read at the top of the tile, ahead of the fragment reads, so the epilogue's first use waits on these four reads
    // only (read inside the epilogue, their lgkmcnt wait also drained the K-step's fragment reads issued before them)
    f32x4 bias4[4];
    auto fetch_bias = [&](int t) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) bias4[q] = *reinterpret_cast<const f32x4*>(sb + kX8BN * t + 16 * (q & 1) + 32 * (q >> 1) + 4 * lg);
    };
    auto epi_part = [&](int b, int t, int part) __attribute__((always_inline)) {
      const int mb = part >> 1, hh = part & 1;
      if constexpr (EPI == EPI_SWIGLU) {
        if (hh) return;                       // one MX block (32 h columns) per row and tile: both halves here
        // scalar fp32 (packed f32 VALU beside MFMAs costs more issue time than two plain ops, MI355X_MICROARCH.md
        // constants table; the file is built with -fno-slp-vectorize so these stay scalar)
        float v[8];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float bg = bias4[h2][r], bu = bias4[2 + h2][r];
            if constexpr ((DBG & 2048) != 0) { bg = 0.f; bu = 0.f; }   // no bias (timing only)
            const float g = fmaf(acc[b][mb][h2][r], inv[mb], bg);
            const float u = fmaf(acc[b][mb][2 + h2][r], inv[mb], bu);
            const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g * -1.4426950408889634f));
            v[4 * h2 + r] = g * sg * u;
          }
        }
        int e = 0;
        u32x2 qv;
        if constexpr (DBG & 8) {
          qv = u32x2{__float_as_uint(v[0] + v[1] + v[2] + v[3]), __float_as_uint(v[4] + v[5] + v[6] + v[7])};
        } else {
          e = mx_exp(__uint_as_float(lg_max_abs_bits(v)));
          qv = quant8(v, e);
        }
        const int col = 32 * t;                                   // first h column of the block
        uint8_t* c8 = p.C8 + orow[mb] + (col + 4 * lg);
        if constexpr ((DBG & 1024) != 0) {   // no stores (timing only; the ring wait then counts ops that do not exist)
          asm volatile("" ::"v"(qv[0]), "v"(qv[1]), "v"(e), "v"(c8));
        } else {
          *reinterpret_cast<uint32_t*>(c8) = qv[0];
          *reinterpret_cast<uint32_t*>(c8 + 16) = qv[1];
          p.C8s[srow[mb] + t] = (uint8_t)e;                       // the 4 lanes of the block write the same byte
        }
      } else {
#pragma unroll
        for (int nb2 = 0; nb2 < 2; ++nb2) {
          const int nb = 2 * hh + nb2, col = kX8BN * t + 16 * nb + 4 * lg;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = fmaf(acc[b][mb][nb][r], inv[mb], sb[col + r]);
          const __bf16 b0 = (__bf16)o[0], b1 = (__bf16)o[1], b2 = (__bf16)o[2], b3 = (__bf16)o[3];
          const u32x2 w = {(uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16),
                           (uint32_t)__builtin_bit_cast(uint16_t, b2) | ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16)};
          *reinterpret_cast<u32x2*>(static_cast<uint16_t*>(p.C) + orow[mb] + col) = w;
        }
      }
    };

    // ring: tiles t0 .. t0 + R - 2 in flight before the loop; tile t + R - 1 issued at the start of tile t
#pragma unroll
    for (int s0 = 0; s0 < kX8R - 1; ++s0)
      if (s0 < n) dma(t0 + s0);
    // lane-constant parts of the W fragment / scale addresses (row l15 of each 16-row n-block, chunk lg / 4 + lg)
    const int xa0 = l15 * kX8K + 16 * (lg ^ swz), xa1 = l15 * kX8K + 16 * ((4 + lg) ^ swz);
    const int xas = l15 * (kX8K / 32) + lg;
    // W fragments of tile t, K-step ks (two register slots, wf / ws)
    auto rdw = [&](int t, int ks, i32x8 (&wf)[4], int (&ws)[4]) __attribute__((always_inline)) {
      if constexpr ((DBG & 256) != 0) {   // no W fragment reads from LDS (timing only)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) { wf[nb] = xf[nb & 1][ks]; ws[nb] = xs[nb & 1][ks]; }
        return;
      }
      // (8 ks + c) ^ swz = 8 ks + (c ^ swz) for swz < 8: one lane-constant address per half plus compile-time offsets
      // (n-block, K-step) that fold into the ds_read immediates; the ring slot and the tile's scale rows are uniform
      const uint8_t* b0 = ring + (t % kX8R) * kX8Tile + xa0;
      const uint8_t* b1 = ring + (t % kX8R) * kX8Tile + xa1;
      const uint8_t* bs = sWs + t * kX8BN * (kX8K / 32) + xas;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(b0 + nb * 16 * kX8K + 128 * ks);
        const u32x4 c = *reinterpret_cast<const u32x4*>(b1 + nb * 16 * kX8K + 128 * ks);
        wf[nb] = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)c[0], (int)c[1], (int)c[2], (int)c[3]};
        ws[nb] = bs[nb * 16 * (kX8K / 32) + 4 * ks];
      }
    };
    // the 8 MFMAs of K-step ks into accumulator buffer BB
    auto mstep = [&](auto Bc, int ks, const i32x8 (&wf)[4], const int (&ws)[4]) __attribute__((always_inline)) {
      constexpr int bb = decltype(Bc)::value;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          if constexpr (DBG & 2) {
            const i32x8 wv = wf[nb], xv = xf[mb][ks];
            const int wsv = ws[nb], xsv = xs[mb][ks];
            asm volatile("" ::"v"(wv), "v"(xv), "v"(wsv), "v"(xsv));
          } else {
            acc[bb][mb][nb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[nb], xf[mb][ks], acc[bb][mb][nb],
                                                                               0, 0, 0, ws[nb], 0, xs[mb][ks]);
          }
    };
    // Tile t in buffer b: its K-step 2 is deferred into the next tile's iteration, so the first LDS reads after
    // each barrier (tile t's K-step 0 fragments) are in flight under the previous tile's last eight MFMAs instead of
    // in front of an idle matrix pipe.  Fragment slots: tile t's K-step 0 / 2 in slot b, K-step 1 in slot b ^ 1 (which
    // held the previous tile's deferred K-step 2 until its MFMAs were issued).  The stores per iteration (the
    // previous tile's epilogue) are unchanged, so ring_younger's count holds.
    i32x8 wslot[2][4];
    int sslot[2][4];
    // The first tile of a run is its own instantiation (FIRST: no deferred K-step, no epilogue): with a run-time
    // `j > 0` around them the compiler sank this tile's K-step 0/1 MFMAs below the branch, i.e. after the whole
    // epilogue, and the epilogue ran serially (SwiGLU M = 40960: 97 us with it, 53 us without, MFMA at 16 %).
    auto tile = [&](auto Bc, auto Fc, int j) __attribute__((always_inline)) {
      constexpr int b = decltype(Bc)::value;
      constexpr bool first = decltype(Fc)::value;
      using PB = std::integral_constant<int, b ^ 1>;
      const int t = t0 + j;
      ring_wait<kX8R, kX8Pieces, kStores8>(j, n);                   // tile t landed
      if constexpr (!(DBG & 16)) barrier_lds();                   // ... for every wave; slot (t - 1) % R free
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (j + kX8R - 1 < n && !(DBG & 4)) dma(t + kX8R - 1);
      if constexpr (!first) mstep(PB{}, 2, wslot[b ^ 1], sslot[b ^ 1]);   // the previous tile's deferred K-step
      if constexpr (EPI == EPI_SWIGLU && !first) fetch_bias(t - 1);
      rdw(t, 0, wslot[b], sslot[b]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[b][mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      rdw(t, 1, wslot[b ^ 1], sslot[b ^ 1]);
      mstep(Bc, 0, wslot[b], sslot[b]);
      if constexpr (!first && !(DBG & 1)) epi_part(b ^ 1, t - 1, 0);   // previous tile, under these MFMAs
      __builtin_amdgcn_sched_barrier(0);
      rdw(t, 2, wslot[b], sslot[b]);
      mstep(Bc, 1, wslot[b ^ 1], sslot[b ^ 1]);
      if constexpr (!first && !(DBG & 1)) {
        epi_part(b ^ 1, t - 1, 2);
        epi_part(b ^ 1, t - 1, 1);
        epi_part(b ^ 1, t - 1, 3);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    tile(I0{}, std::true_type{}, 0);
    for (int j = 1; j < n; j += 2) {
      tile(I1{}, std::false_type{}, j);
      if (j + 1 < n) tile(I0{}, std::false_type{}, j + 1);
    }
    // the last tile: its deferred K-step, then its epilogue
    auto drain = [&](auto Bc) __attribute__((always_inline)) {
      constexpr int b = decltype(Bc)::value;
      mstep(Bc, 2, wslot[b], sslot[b]);
      if constexpr (DBG & 1) {   // keep the accumulators alive
        float k = 0.f;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) k += acc[0][mb][nb][0] + acc[1][mb][nb][1];
        if (k == 1234.5f) p.C8[mbase] = 1;
      } else {
        if constexpr (EPI == EPI_SWIGLU) fetch_bias(t1 - 1);
#pragma unroll
        for (int part = 0; part < 4; ++part) epi_part(b, t1 - 1, part);
      }
    };
    if ((n - 1) & 1) drain(std::integral_constant<int, 1>{});
    else drain(std::integral_constant<int, 0>{});
    __syncthreads();
  }
}

template <int EPI>
hipError_t launch_xs8(const MxArgs& a, int nc, hipStream_t st) {
  const int items = ((a.M + kX8BM - 1) / kX8BM) * ((a.N / kX8BN + nc - 1) / nc);
  int grid = 256;
  const int need = (items + 7) / 8 * 8;
  if (grid > need) grid = need;
#ifdef XS8_ABLATE
  if constexpr (EPI == EPI_SWIGLU) {
    switch (a.rs_ss ? a.dbg : 0) {
#define X8_D(d) case d: hipLaunchKernelGGL((gemm_xs8_kernel<EPI, true, d>), dim3(grid), dim3(512), 0, st, a, nc); return hipGetLastError();
      X8_D(1) X8_D(2) X8_D(3) X8_D(4) X8_D(5) X8_D(8) X8_D(7) X8_D(16) X8_D(17) X8_D(32) X8_D(20) X8_D(259) X8_D(515) X8_D(771) X8_D(263) X8_D(19) X8_D(256) X8_D(512)
      X8_D(1024) X8_D(2048) X8_D(3072) X8_D(1032) X8_D(1026)
#undef X8_D
      default: break;
    }
  }
#endif
  if (a.rs_ss) hipLaunchKernelGGL((gemm_xs8_kernel<EPI, true>), dim3(grid), dim3(512), 0, st, a, nc);
  else hipLaunchKernelGGL((gemm_xs8_kernel<EPI, false>), dim3(grid), dim3(512), 0, st, a, nc);
  return hipGetLastError();
}

}  // namespace

// X-stationary MXFP8 GEMM for K = 384 (gemm_xs8_kernel); nc = W tiles per work item (0: auto)
hipError_t gemm_xs8(const MxArgs& a, int epi, int nc, hipStream_t st) {
  if (a.K != kX8K || a.N % kX8BN || a.N > kX8MaxN || a.M <= 0 || a.lda % 16 || a.ldas != kX8K / 32 || a.C2)
    return hipErrorInvalidValue;
  if (epi == EPI_SWIGLU && (!a.C8 || !a.C8s || a.ldc % 16)) return hipErrorInvalidValue;
  if ((int64_t)a.M * a.ldc >= (1ll << 32) || (int64_t)a.M * a.ldc8s >= (1ll << 32)) return hipErrorInvalidValue;   // 32-bit row offsets
  if (epi == EPI_STORE && (!a.c_bf16 || a.ldc % 8)) return hipErrorInvalidValue;
  const int nwt = a.N / kX8BN, ntm = (a.M + kX8BM - 1) / kX8BM;
  if (nc <= 0) nc = xs_run_length(ntm, nwt);
  switch (epi) {
    case EPI_SWIGLU: return launch_xs8<EPI_SWIGLU>(a, nc, st);
    case EPI_STORE: return launch_xs8<EPI_STORE>(a, nc, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t gemm_mx(const MxArgs& a0, int epi, hipStream_t st) {
  const MxArgs& a = a0;
  // 128 W rows per tile: the 256-row tile needs 96 fragment VGPRs per wave at 32 bytes per lane and
  // spills at two waves per SIMD
  if (a.K % 128 || a.K / 32 > kMxKB || a.M <= 0 || a.lda % 16 || a.ldas % 4 || (a.ldc % 8) || a.N % 128)
    return hipErrorInvalidValue;
  // the fused MXFP8 operand (Q8) quantizes the bf16 shadow's registers and indexes the sum-of-squares slab by
  // 32-column block: RESID with a shadow, every output, and whole rows of 384 only (as gemm.hip checks C8)
  if (a.Q8 && (epi != EPI_RESID || !a.C2 || !a.Q8s || !a.ss8 || a.N != 32 * kSsSlots || a.ldc != a.N))
    return hipErrorInvalidValue;
  switch (epi) {
    case EPI_SWIGLU: return (!a.C8 || !a.C8s) ? hipErrorInvalidValue : launch_mx<128, EPI_SWIGLU>(a, st);
    // 128 X rows per tile while there are few 256-row tiles (FFN down at M = 10240: 22.0 vs 31.7 us, M = 2560-5120:
    // 18-19 vs 28-30; at M = 20480 the 256-row tile wins 34.4 vs 40.1; q|k|v only below ~128 tiles;
    // profiles/r02_mx_x128.jsonl).  MXDBG = 16 / 32 force 256 / 128 (tools/gemm_bench)
    case EPI_STORE:
    case EPI_RESID: {
      const int64_t t256 = (int64_t)(a.N / 128) * ((a.M + 255) / 256);
      const bool x128 = (a.dbg & 32) || (!(a.dbg & 16) && t256 < (epi == EPI_RESID ? 200 : 128));
      if (epi == EPI_STORE) return x128 ? launch_mx<128, EPI_STORE, 128>(a, st) : launch_mx<128, EPI_STORE>(a, st);
      return x128 ? launch_mx<128, EPI_RESID, 128>(a, st) : launch_mx<128, EPI_RESID>(a, st);
    }
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
