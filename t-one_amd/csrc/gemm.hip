// Dense contractions of the acoustic path on CDNA4 MFMA, with fused epilogues.
//
//   C[M][N] = epilogue( rowscale(A)[M][K] . W[N][K]^T )
//
// W is row-major [N][K] exactly like torch Linear / 1x1 Conv1d weights, so the B operand is read
// K-contiguous like A.  Two arithmetic modes share one tiling:
//   fp32: v_mfma_f32_32x32x2_f32   (exact fp32 products, fp32 accumulate; BASELINE config 2), BK = 32
//   bf16: v_mfma_f32_32x32x16_bf16 (A rounded to bf16 while staging or already stored bf16, W bf16,
//         fp32 accumulate; BASELINE config 3), BK = 64
// A K-step always moves 128-byte rows of W into LDS.
//
// A rows are addressed as  row r -> (r / rpg) * gstride + (r % rpg) * lda  (rpg = 0: r * lda), which
// covers plain activations and overlapping mel windows (hop 80 inside a 2480-sample stream), or are
// gathered per (kt, kf) tap for the conv2 implicit GEMM.
//
// Fused epilogues (the reference ops they absorb):
//   rowscale  RMSNorm folded into the GEMM: the gain is pre-multiplied into W's columns and the
//             row's 1/(||a||/sqrt(K) + 1e-8) is computed from the staged fp32 A tile
//             (submodules.py:34-54 feeding Linear/Conv1d with K = d_model = 384)
//   STORE     + bias                                       (nn.Linear)
//   RESID     R + alpha*(acc + bias)                       (residual adds, conformer_blocks.py:814-834)
//   SWIGLU    silu(g + b1) * (v + bv) on interleaved 32-row W1/Wv blocks (conformer_blocks.py:479-482)
//   GLU       (a + ba) * sigmoid(g + bg) on interleaved pw1 halves     (conformer_blocks.py:419-422)
//   CONV2     SiLU(acc * bn_scale + bn_shift) scattered to the subsampling Linear's input
//   POWER     re^2 + im^2 of interleaved 32-bin re/im blocks            (feats.py:98)
//   LOGMEL    fp16(log(acc + 2^-24)) for the first 64 columns           (feats.py:99-102)
//
// Pipeline: A/W tiles of the next K-step are fetched into registers while the MFMAs run on the
// current LDS buffer (two LDS buffers, one barrier per K-step).  When M*N gives too few tiles to
// fill 256 CUs (small batches, N = 384) the K range is split over blocks (blockIdx.y); the fp32
// partials go to a workspace and a second kernel sums them in a fixed order (deterministic) and
// applies the epilogue.
#include "common.h"

#include <cstdlib>
#include "kernels.h"

#include <string>

#include <type_traits>

namespace tone {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  __bf16 ha = (__bf16)a, hb = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ uint16_t bf16_bits(float a) {
  __bf16 h = (__bf16)a;
  return __builtin_bit_cast(uint16_t, h);
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float sumsq_bf16x8(bf16x8 v, float acc) {
  const bf16x2 p0 = __builtin_shufflevector(v, v, 0, 1), p1 = __builtin_shufflevector(v, v, 2, 3);
  const bf16x2 p2 = __builtin_shufflevector(v, v, 4, 5), p3 = __builtin_shufflevector(v, v, 6, 7);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p0, p0, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p1, p1, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(p2, p2, acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(p3, p3, acc, false);
}

template <class T>
__device__ __forceinline__ void st_out(T* ptr, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, ptr);
  else *ptr = v;
}

template <int BM_, int BN_, int WM_, int WN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
};

// Shared epilogue.  C/D map of v_mfma_*_32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
// Every operand the epilogue reads (bias, BN scale/shift, residual rows) is loaded into registers
// before the first store: C may alias R, so a load placed after a store could not be hoisted and
// each one would pay a full memory latency in series.
// R16: the residual stream R / C (RESID, and a STORE that starts it) is fp16 (bf16 / fp8 modes), a compile-time choice so
// the residual loads stay straight-line (a per-launch branch makes the compiler drain them one at a time)
template <class TL, int EPI, bool CBF, bool SPLIT, bool R16 = false, int TM = TL::BM / TL::WM / 32,
          int TN = TL::BN / TL::WN / 32>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& p, f32x16 (&acc)[TM][TN], const float* rden, int m0, int n0,
                                              int wm, int wn, int lane) {
  constexpr int WTM = TL::BM / TL::WM, WTN = TL::BN / TL::WN;
  constexpr bool CONV2 = (EPI == EPI_CONV2);
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU || EPI == EPI_POWER);
  const int lr = lane & 31, lh = lane >> 5;
  const int cbase = n0 + wn * WTN + lr;          // column of n-tile j: cbase + 32 j
  const bool nt = p.nt_store;
  float bcol[TN], scol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    bcol[j] = 0.f;
    scol[j] = 1.f;
    if constexpr (!SPLIT && EPI != EPI_POWER && EPI != EPI_LOGMEL) {
      if (p.bias) bcol[j] = p.bias[cbase + j * 32];
      if constexpr (CONV2) scol[j] = p.scale[cbase + j * 32];
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float rres[16][TN];
    if constexpr (EPI == EPI_RESID && !SPLIT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = min(m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh, p.M - 1);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t o = (int64_t)row * p.ldr + cbase + j * 32;
          rres[r][j] = R16 ? __half2float(reinterpret_cast<const __half*>(p.R)[o]) : p.R[o];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lrow = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int row = m0 + lrow;
      if (row >= p.M) continue;
      if constexpr (SPLIT) {
        float* dst = p.ws + ((int64_t)blockIdx.y * p.M + row) * p.N;
#pragma unroll
        for (int j = 0; j < TN; ++j) dst[cbase + j * 32] = acc[i][j][r];
      } else if constexpr (CONV2) {
        const int64_t o = (int64_t)row * kSub2C;   // flat [B*T][34*64]: row (b, t, f) -> ((b T + t) 34 + f) 64
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int c = cbase + j * 32;
          const float y = silu_f(fmaf(acc[i][j][r], scol[j], bcol[j]));
          if constexpr (CBF) static_cast<uint16_t*>(p.C)[o + c] = bf16_bits(y);
          else static_cast<float*>(p.C)[o + c] = y;
        }
      } else if constexpr (EPI == EPI_LOGMEL) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = cbase + j * 32;
          if (col < p.n_out)
            static_cast<float*>(p.C)[(int64_t)row * p.ldc + col] = round_h(logf(acc[i][j][r] + 5.9604644775390625e-08f));
        }
      } else if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
        const float den = p.rowscale ? rden[lrow] : 1.0f;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = cbase + j * 32;
          float v = acc[i][j][r];
          if (p.rowscale) v = v / den;
          v += bcol[j];
          if constexpr (EPI == EPI_RESID) v = rres[r][j] + p.alpha * v;
          if constexpr (CBF) st_out(static_cast<uint16_t*>(p.C) + (int64_t)row * p.ldc + col, bf16_bits(v), nt);
          else if (R16) static_cast<__half*>(p.C)[(int64_t)row * p.ldc + col] = __float2half_rn(v);   // fp16 residual
          else st_out(static_cast<float*>(p.C) + (int64_t)row * p.ldc + col, v, nt);
          if (p.C2) st_out(p.C2 + (int64_t)row * p.ldc + col, bf16_bits(v), nt);   // bf16 shadow of the residual
        }
      } else {
        static_assert(PAIRED, "unhandled epilogue");
        const float den = p.rowscale ? rden[lrow] : 1.0f;
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
          const int oc = (n0 + wn * WTN) / 2 + jp * 32 + lr;
          float o;
          if constexpr (EPI == EPI_POWER) {
            o = g * g + u * u;
          } else {
            if (p.rowscale) { g = g / den; u = u / den; }
            g += bcol[2 * jp];
            u += bcol[2 * jp + 1];
            if constexpr (EPI == EPI_SWIGLU) o = silu_f(g) * u;   // linear1 -> SiLU, times linearv
            else o = g * sigmoid_f(u);                            // GLU: first half * sigmoid(second)
          }
          if constexpr (CBF) st_out(static_cast<uint16_t*>(p.C) + (int64_t)row * p.ldc + oc, bf16_bits(o), nt);
          else st_out(static_cast<float*>(p.C) + (int64_t)row * p.ldc + oc, o, nt);
        }
      }
    }
  }
}

// Workgroup barrier that leaves LDS-DMA (vmcnt) in flight: __syncthreads() fences with vmcnt(0).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-staged epilogue (LDS-DMA kernel): the wave tiles go to LDS as fp32 in the MFMA layout (the
// stage buffers are free after the K loop), then the block writes whole output rows with 16-byte
// fp32 / 8-byte bf16 vectors, so each 128-byte line leaves in one instruction instead of as 64-byte
// halves from two waves, and residual rows are read as vectors (all before the first store).
// PRE (RESID): the residual rows were loaded by the caller before its K loop (rin, in the order below), so their
// latency hides under the MFMAs instead of stalling the epilogue
template <class TL, int EPI, bool CBF, bool SPLIT, bool R16, bool PRE = false, int TM, int TN, int NVR = 1>
__device__ __forceinline__ void gemm_epilogue_lds(const GemmArgs& p, f32x16 (&acc)[TM][TN], const float* rden, float* Cs,
                                                  int m0, int n0, int wm, int wn, int tid, const f32x4 (&rin)[NVR] = {}) {
  constexpr int NT = TL::WM * TL::WN * 64;
  constexpr int WTM = TL::BM / TL::WM, WTN = TL::BN / TL::WN;
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU);
  static_assert(PAIRED || EPI == EPI_STORE || EPI == EPI_RESID, "LDS epilogue: STORE/RESID/SWIGLU/GLU");
  constexpr int BNO = PAIRED ? TL::BN / 2 : TL::BN;
  const int lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bcol[j] = (!SPLIT && p.bias) ? p.bias[n0 + wn * WTN + j * 32 + lr] : 0.f;
  float inv[TM][16];                           // folded RMSNorm: 1 / (||a|| / sqrt(K) + eps) per row
  const bool rs = !SPLIT && p.rowscale;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      inv[i][r] = rs ? 1.0f / rden[wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] : 1.0f;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lrow = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if constexpr (PAIRED) {
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          float g = acc[i][2 * jp][r] * inv[i][r], u = acc[i][2 * jp + 1][r] * inv[i][r];
          g += bcol[2 * jp];
          u += bcol[2 * jp + 1];
          const float o = (EPI == EPI_SWIGLU) ? silu_f(g) * u : g * sigmoid_f(u);
          Cs[lrow * BNO + (wn * WTN) / 2 + jp * 32 + lr] = o;
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v = acc[i][j][r];
          if constexpr (!SPLIT) v = fmaf(v, inv[i][r], bcol[j]);
          Cs[lrow * BNO + wn * WTN + j * 32 + lr] = v;
        }
      }
    }
  }
  lds_barrier();
  constexpr int RV = BNO / 4;                 // 4-float vectors per row
  constexpr int NV = TL::BM * RV / NT;        // vectors per thread
  static_assert(NV >= 1 && (TL::BM * RV) % NT == 0, "tile/thread mismatch");
  const int ocol0 = PAIRED ? n0 / 2 : n0;
  f32x4 val[NV], res[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = tid + k * NT, row = q / RV, c = (q % RV) * 4;
    val[k] = *reinterpret_cast<const f32x4*>(Cs + row * BNO + c);
    if constexpr (EPI == EPI_RESID && !SPLIT) {
      if constexpr (PRE) {
        static_assert(NVR == NV, "prefetched residual vectors");
        res[k] = rin[k];
      } else {
        const int grow = min(m0 + row, p.M - 1);
        res[k] = load_res4(p.R, (int64_t)grow * p.ldr + ocol0 + c, R16);
      }
    }
  }
  const bool nt = p.nt_store;
  const bool full = m0 + TL::BM <= p.M;        // block-uniform: no row guards
  if constexpr (EPI == EPI_RESID && !SPLIT && RV == 32) {
    if (p.C8) {
      // fp8 mode: the shadow's MXFP8 form, as quant_mx would make it from the shadow (a 32-column block = 8 lanes),
      // and the row's sum of squares over the tile's 128 columns into the first of its 4 slots of the slab
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int q = tid + k * NT, row = q / RV, c = (q % RV) * 4;
        const int grow = m0 + row;
        const bool ok = full || grow < p.M;
        const f32x4 v = res[k] + p.alpha * val[k];
        const int64_t o = (int64_t)grow * p.ldc + ocol0 + c;
        u32x2 h;
        h.x = pack_bf16x2(v.x, v.y);
        h.y = pack_bf16x2(v.z, v.w);
        if (ok) {
          store_res4(p.C, o, v, R16, nt);
          if (p.C2) st_out(reinterpret_cast<u32x2*>(p.C2 + o), h, nt);
        }
        const float b0 = __uint_as_float(h.x << 16), b1 = __uint_as_float(h.x & 0xffff0000u);
        const float b2 = __uint_as_float(h.y << 16), b3 = __uint_as_float(h.y & 0xffff0000u);
        float am = fmaxf(fmaxf(fabsf(b0), fabsf(b1)), fmaxf(fabsf(b2), fabsf(b3)));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        am = fmaxf(am, __shfl_xor(am, 2, 64));
        am = fmaxf(am, __shfl_xor(am, 4, 64));
        const int e = mx_exp(am);
        const uint32_t q4 = quant4(b0, b1, b2, b3, e);
        float ssq = fmaf(b3, b3, fmaf(b2, b2, fmaf(b1, b1, b0 * b0)));
#pragma unroll
        for (int w = 1; w < 32; w <<= 1) ssq += __shfl_xor(ssq, w, 64);
        if (ok) {
          *reinterpret_cast<uint32_t*>(p.C8 + o) = q4;
          if ((q & 7) == 0) p.C8s[grow * (p.ldc / 32) + (ocol0 + c) / 32] = (uint8_t)e;
          if ((q & 31) < 4) p.ss8[grow * kSsSlots + ocol0 / 32 + (q & 31)] = (q & 31) == 0 ? ssq : 0.f;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = tid + k * NT, row = q / RV, c = (q % RV) * 4;
    const int grow = m0 + row;
    if (!full && grow >= p.M) continue;
    f32x4 v = val[k];
    if constexpr (SPLIT) {
      st_out(reinterpret_cast<f32x4*>(p.ws + ((int64_t)blockIdx.y * p.M + grow) * p.N + n0 + c), v, nt);
      continue;
    }
    if constexpr (EPI == EPI_RESID) v = res[k] + p.alpha * v;
    const int64_t o = (int64_t)grow * p.ldc + ocol0 + c;
    u32x2 h;
    h.x = pack_bf16x2(v.x, v.y);
    h.y = pack_bf16x2(v.z, v.w);
    if constexpr (CBF) st_out(reinterpret_cast<u32x2*>(static_cast<uint16_t*>(p.C) + o), h, nt);
    else store_res4(p.C, o, v, R16, nt);   // fp32, or the fp16 residual stream (R16)
    if (p.C2) st_out(reinterpret_cast<u32x2*>(p.C2 + o), h, nt);
  }
}

// MMA16: bf16 MFMA (W bf16); ABF: A stored bf16; CBF: C stored bf16 (STORE/SWIGLU/GLU/CONV2)
template <class TL, int EPI, bool MMA16, bool ABF, bool CBF, bool SPLIT>
__global__ void __launch_bounds__(TL::WM * TL::WN * 64) gemm_kernel(GemmArgs p) {
  constexpr int BM = TL::BM, BN = TL::BN, WM = TL::WM, WN = TL::WN;
  constexpr int NT = WM * WN * 64;
  constexpr int BK = MMA16 ? 64 : 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU || EPI == EPI_POWER);
  constexpr bool CONV2 = (EPI == EPI_CONV2);
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  static_assert(!PAIRED || (TN % 2 == 0), "paired epilogues pair n-tiles");
  static_assert(!SPLIT || EPI == EPI_STORE || EPI == EPI_RESID, "split-K only for STORE/RESID");
  static_assert(MMA16 || !ABF, "bf16 A needs the bf16 MFMA");
  constexpr int LDS_ROW = BK + (MMA16 ? 8 : 4);          // elements; conflict-free ds_read_b128 rows
  using ST = typename std::conditional<MMA16, uint16_t, float>::type;   // LDS / W element
  using AT = typename std::conditional<ABF, uint16_t, float>::type;     // A element in memory
  constexpr int AVE = 16 / sizeof(AT);                   // A elements per 16-byte vector
  constexpr int A_V = BM * BK / AVE / NT;                // A vectors per thread per K-step
  constexpr int WVE = 16 / sizeof(ST);
  constexpr int W_V = BN * BK / WVE / NT;
  constexpr int A_RV = BK / AVE;                         // vectors per A row per K-step
  static_assert(A_V >= 1 && W_V >= 1 && (NT % A_RV) == 0, "tile too small for the thread count");

  __shared__ __attribute__((aligned(16))) ST lds_all[2 * (BM + BN) * LDS_ROW];   // A and W stages; C tile after
  ST(*As)[BM * LDS_ROW] = reinterpret_cast<ST(*)[BM * LDS_ROW]>(lds_all);
  ST(*Bs)[BN * LDS_ROW] = reinterpret_cast<ST(*)[BN * LDS_ROW]>(lds_all + 2 * BM * LDS_ROW);
  __shared__ float rden[BM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = p.N / BN;
  // XCD-aware order (blocks are dealt round-robin over the 8 XCDs): consecutive logical tiles,
  // which share the same A rows, land on one XCD so the A tile is fetched into one L2 only.
  int wgid = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = wgid & 7, q = nwg >> 3, rr = nwg & 7;
    wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (wgid >> 3);
  }
  const int bm = wgid / ntn, bn = wgid % ntn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int kb = SPLIT ? blockIdx.y * p.k_split : 0;
  const int nk = (SPLIT ? p.k_split : p.K) / BK;
  const AT* __restrict__ A = static_cast<const AT*>(p.A);

  // per-thread A row offsets (rows are fixed for the whole K loop)
  int64_t rowoff[A_V];
  bool rvalid[A_V];
#pragma unroll
  for (int i = 0; i < A_V; ++i) {
    const int r = (tid + i * NT) / A_RV;
    const int gm = min(m0 + r, p.M - 1);
    rvalid[i] = (m0 + r) < p.M;
    if constexpr (CONV2) {   // chunk geometry from the launcher (conv_t frames, conv_in input rows)
      const int b = gm / (p.conv_t * kSub2F), rem = gm % (p.conv_t * kSub2F);
      const int t = rem / kSub2F, f = rem % kSub2F;
      rowoff[i] = (((int64_t)b * p.conv_in + kSub2Stride * t) * kSub1F + f) * kSub1C;
    } else {
      rowoff[i] = p.rpg ? (int64_t)(gm / p.rpg) * p.gstride + (int64_t)(gm % p.rpg) * p.lda : (int64_t)gm * p.lda;
    }
  }

  u32x4 ra[A_V];
  u32x4 rw[W_V];
  float ss[A_V];
#pragma unroll
  for (int i = 0; i < A_V; ++i) ss[i] = 0.f;

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int c = (tid + i * NT) % A_RV;
      int64_t off;
      if constexpr (CONV2) {
        const int k = k0 + c * AVE, tap = k >> 5, ci = k & 31;
        const int kt = tap / kSub2Kf, kf = tap % kSub2Kf;
        off = tap < kSub2Kt * kSub2Kf ? rowoff[i] + (kt * kSub1F + kf) * kSub1C + ci : rowoff[i];
      } else {
        off = rowoff[i] + k0 + c * AVE;
      }
      const u32x4 v = *reinterpret_cast<const u32x4*>(A + off);
      ra[i] = rvalid[i] ? v : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / WVE), c = idx % (BK / WVE);
      const ST* base = static_cast<const ST*>(p.W) + (int64_t)(n0 + r) * p.K + k0 + c * WVE;
      rw[i] = *reinterpret_cast<const u32x4*>(base);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int idx = tid + i * NT, r = idx / A_RV, c = idx % A_RV;
      if constexpr (ABF) {
        *reinterpret_cast<u32x4*>(&As[buf][r * LDS_ROW + c * AVE]) = ra[i];
      } else {
        const f32x4 v = __builtin_bit_cast(f32x4, ra[i]);
        if (p.rowscale) ss[i] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        if constexpr (MMA16) {
          u32x2 u;
          u.x = pack_bf16x2(v.x, v.y);
          u.y = pack_bf16x2(v.z, v.w);
          *reinterpret_cast<u32x2*>(&As[buf][r * LDS_ROW + c * 4]) = u;
        } else {
          *reinterpret_cast<f32x4*>(&As[buf][r * LDS_ROW + c * 4]) = v;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / WVE), c = idx % (BK / WVE);
      *reinterpret_cast<u32x4*>(&Bs[buf][r * LDS_ROW + c * WVE]) = rw[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    if constexpr (MMA16) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(&As[buf][(wm * WTM + i * 32 + lr) * LDS_ROW + ks * 16 + lh * 8]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(&Bs[buf][(wn * WTN + j * 32 + lr) * LDS_ROW + ks * 16 + lh * 8]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // lane half h owns k in [16h, 16h+16) of the tile; both operands use the same k map
#pragma unroll
      for (int kq = 0; kq < BK / 8; ++kq) {
        f32x4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const f32x4*>(&As[buf][(wm * WTM + i * 32 + lr) * LDS_ROW + lh * 16 + kq * 4]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const f32x4*>(&Bs[buf][(wn * WTN + j * 32 + lr) * LDS_ROW + lh * 16 + kq * 4]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
      }
    }
  };

  load(kb);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // branch-free prefetch (the last step re-reads its own tile into the idle buffer) keeps the
    // staging registers in VGPRs instead of scratch
    const int knext = kb + ((kt + 1 < nk) ? kt + 1 : kt) * BK;
    load(knext);
    compute(cur);
    if (kt + 1 >= nk) {
#pragma unroll
      for (int i = 0; i < A_V; ++i) ra[i] = u32x4{0u, 0u, 0u, 0u};   // no double count in ss
    }
    store(cur ^ 1);
    __syncthreads();
  }

  if constexpr (!ABF) {
    if (p.rowscale) {
#pragma unroll
      for (int i = 0; i < A_V; ++i) {
        float v = ss[i];
#pragma unroll
        for (int o = 1; o < A_RV; o <<= 1) v += __shfl_xor(v, o, 64);
        const int idx = tid + i * NT, r = idx / A_RV;
        if ((idx % A_RV) == 0) {
          if constexpr (SPLIT) {
            if (bn == 0 && m0 + r < p.M) p.ws_ss[(int64_t)blockIdx.y * p.M + m0 + r] = v;
          } else {
            rden[r] = sqrtf(v) * p.inv_sqrt_k + kRmsEps;
          }
        }
      }
      if constexpr (!SPLIT) __syncthreads();
    }
  }

  constexpr bool kLdsEpi = (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_SWIGLU || EPI == EPI_GLU) &&
                           BM * BN * 4 <= (int)sizeof(lds_all);
  if constexpr (kLdsEpi) {
    gemm_epilogue_lds<TL, EPI, CBF, SPLIT, false>(p, acc, rden, reinterpret_cast<float*>(lds_all), m0, n0, wm, wn, tid);
  } else {
    gemm_epilogue<TL, EPI, CBF, SPLIT>(p, acc, rden, m0, n0, wm, wn, lane);
  }
}


// ---------------------------------------------------------------------------------------------
// bf16 GEMM with LDS-DMA staging.  Both operands are bf16 in memory; each K-step (64) moves
// 128-byte rows of A and W straight into LDS with global_load_lds_dwordx4 (one wave instruction =
// 8 rows x 128 B), the next K-step's DMA in flight while the MFMAs run on the current buffer.
// LDS rows are lane-linear, so the ds_read_b128 bank spread comes from an XOR swizzle applied to
// the per-lane SOURCE address (16-byte slot ^= (row >> 1) & 7) and undone on the read (guide rule 21).  Two
// 128-byte rows share a 256-byte bank window, so a 16-lane ds_read_b128 group (rows {0-3, 12-15, 20-27} or
// {4-11, 16-19, 28-31} of the 32-row fragment) needs 8 distinct slots per row parity: (row >> 1) & 7 gives them;
// round 4's row & 7 repeated each slot twice (41-48 % of the kernel's LDS cycles were conflict cycles,
// profiles/r05_pmc_lds_bf16.txt).
// A rowscale GEMM reads the bf16 shadow of the residual and takes each row's sum of squares from
// its own A fragments (waves of the first N column only).
// Split-K is a runtime mode here (p.k_split > 0: K slice blockIdx.y, raw partials to p.ws).

template <class TL, int EPI, bool CBF, int S, bool R16 = false>
__global__ void __launch_bounds__(TL::WM * TL::WN * 64) gemm_glds_kernel(GemmArgs p) {
  constexpr int BM = TL::BM, BN = TL::BN, WM = TL::WM, WN = TL::WN;
  constexpr int kNWaves = WM * WN;
  constexpr int BK = 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr bool CONV2 = (EPI == EPI_CONV2);
  constexpr int A_I = BM / 8 / kNWaves, W_I = BN / 8 / kNWaves;     // DMA wave-instructions per K-step
  static_assert(A_I >= 1 && W_I >= 1 && BM % (8 * kNWaves) == 0 && BN % (8 * kNWaves) == 0, "tile/wave mismatch");
  static_assert(!(EPI == EPI_SWIGLU || EPI == EPI_GLU) || TN % 2 == 0, "paired epilogues pair n-tiles");
  constexpr int kStageElems = (BM + BN) * BK;                    // bf16 elements per buffer
  static_assert(S >= 2 && S <= 4, "2..4 LDS stages");
  constexpr int kIps = A_I + W_I;                                // DMA instructions per stage per thread
  __shared__ __attribute__((aligned(16))) uint16_t lds[S * kStageElems + 2 * BM];   // one LDS object (+ rden)
  float* rden = reinterpret_cast<float*>(lds + S * kStageElems);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = p.N / BN;
  int bm, bn;
  if (p.order_n && (ntn & 7) == 0) {
    // large W: each XCD keeps an eighth of W's rows hot in its L2 and walks every M-tile
    const int npx = ntn >> 3, li = blockIdx.x >> 3;
    bm = li / npx;
    bn = (blockIdx.x & 7) * npx + li % npx;
  } else {
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (blockIdx.x >> 3);
    bm = wgid / ntn;
    bn = wgid % ntn;
  }
  const int m0 = bm * BM, n0 = bn * BN;
  const bool split = p.k_split > 0;
  const int kb = split ? (int)blockIdx.y * p.k_split : 0;
  const int nk = (split ? p.k_split : p.K) / BK;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);

  const int lrow8 = lane >> 3, lslot = lane & 7;
  int64_t aoff[A_I];
  int aslot[A_I];
#pragma unroll
  for (int i = 0; i < A_I; ++i) {
    const int row = 8 * (wid + i * kNWaves) + lrow8;
    const int gm = min(m0 + row, p.M - 1);
    aslot[i] = lslot ^ ((row >> 1) & 7);
    if constexpr (CONV2) {
      const int b = gm / (p.conv_t * kSub2F), rem = gm % (p.conv_t * kSub2F);
      const int t = rem / kSub2F, f = rem % kSub2F;
      aoff[i] = (((int64_t)b * p.conv_in + kSub2Stride * t) * kSub1F + f) * kSub1C;
    } else {
      aoff[i] = (p.rpg ? (int64_t)(gm / p.rpg) * p.gstride + (int64_t)(gm % p.rpg) * p.lda : (int64_t)gm * p.lda) +
                aslot[i] * 8;
    }
  }
  int64_t woff[W_I];
#pragma unroll
  for (int i = 0; i < W_I; ++i) {
    const int row = 8 * (wid + i * kNWaves) + lrow8;
    woff[i] = (int64_t)(n0 + row) * p.K + (lslot ^ ((row >> 1) & 7)) * 8;
  }

  auto stage = [&](int buf, int k0) {
    uint16_t* base = lds + buf * kStageElems;
    (void)base;
    (void)W;
#pragma unroll
    for (int i = 0; i < A_I; ++i) {
      const uint16_t* src;
      if constexpr (CONV2) {
        const int k = k0 + aslot[i] * 8, tap = k >> 5, ci = k & 31;
        const int kt = tap / kSub2Kf, kf = tap % kSub2Kf;
        src = A + (tap < kSub2Kt * kSub2Kf ? aoff[i] + (kt * kSub1F + kf) * kSub1C + ci : aoff[i]);
      } else {
        src = A + aoff[i] + k0;
      }
      lds_dma16(src, base + (8 * (wid + i * kNWaves)) * BK);
    }
#pragma unroll
    for (int i = 0; i < W_I; ++i) {
      lds_dma16(W + woff[i] + k0, base + (BM + 8 * (wid + i * kNWaves)) * BK);
    }
  };

  // RESID through the LDS epilogue: this tile's residual rows (the epilogue's vector order) requested before the K
  // loop, in their stored type (converted after it), so their latency hides under the MFMAs (the epilogue would
  // otherwise wait a full memory round trip with the matrix pipe idle); C may alias R, and only this tile writes it
  constexpr bool kLdsEpiC = (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_SWIGLU || EPI == EPI_GLU) &&
                            BM * BN * 4 <= S * kStageElems * 2;
  constexpr bool kPre = kLdsEpiC && EPI == EPI_RESID;
  constexpr int kRV = BN / 4, kNVR = kPre ? BM * kRV / (kNWaves * 64) : 1;
  using RawT = typename std::conditional<R16, f16x4_t, f32x4>::type;
  RawT rraw[kNVR];
  if constexpr (kPre) {
#pragma unroll
    for (int k = 0; k < kNVR; ++k) {
      const int q = tid + k * kNWaves * 64, row = q / kRV, c = (q % kRV) * 4;
      const int grow = min(m0 + row, p.M - 1);
      rraw[k] = *reinterpret_cast<const RawT*>(static_cast<const char*>(static_cast<const void*>(p.R)) +
                                              ((int64_t)grow * p.ldr + n0 + c) * (R16 ? 2 : 4));
    }
  }
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float ss[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) ss[i] = 0.f;
  const bool want_ss = p.rowscale && wn == 0;

  const int lr = lane & 31, lh = lane >> 5;
  auto compute = [&](int buf) {
    const uint16_t* base = lds + buf * kStageElems;
    // all fragments of the K-step first (one counted LDS wait), then the MFMAs
    bf16x8 a[BK / 16][TM], b[BK / 16][TN];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int slot = ks * 2 + lh;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 32 + lr;
        a[ks][i] = *reinterpret_cast<const bf16x8*>(base + row * BK + ((slot ^ ((row >> 1) & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 32 + lr;
        b[ks][j] = *reinterpret_cast<const bf16x8*>(base + (BM + row) * BK + ((slot ^ ((row >> 1) & 7)) << 3));
      }
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][i], b[ks][j], acc[i][j], 0, 0, 0);
      // row sums of squares for a folded RMSNorm (v_dot2 on bf16 pairs, beside the MFMAs)
#pragma unroll
      for (int i = 0; i < TM; ++i) ss[i] = sumsq_bf16x8(a[ks][i], ss[i]);
    }
  };

  // S-deep ring: stages kt+1 .. kt+S-2 stay in flight while stage kt is consumed; one barrier per
  // K-step both publishes stage kt and frees buffer (kt-1) % S for the DMA of stage kt+S-1.
#pragma unroll
  for (int s0 = 0; s0 < S - 1; ++s0)
    if (s0 < nk) stage(s0, kb + s0 * BK);
  for (int kt = 0; kt < ((p.dbg & 4) ? 0 : nk); ++kt) {
    const int ahead = min(S - 2, nk - 1 - kt);      // younger stages allowed to remain in flight
    if (S >= 4 && ahead >= 2) wait_vmcnt<(S >= 4 ? 2 * kIps : 0)>();
    else if (S >= 3 && ahead >= 1) wait_vmcnt<(S >= 3 ? kIps : 0)>();
    else wait_vmcnt<0>();
    lds_barrier();   // not __syncthreads(): its vmcnt(0) fence would drain the DMAs kept in flight
    if (kt + S - 1 < nk) stage((kt + S - 1) % S, kb + (kt + S - 1) * BK);
    compute(kt % S);
  }
  __syncthreads();

  if (p.rowscale) {
    if (want_ss) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float v = ss[i] + __shfl_xor(ss[i], 32, 64);
        if (lh == 0) {
          const int r = wm * WTM + i * 32 + lr;
          if (split) {
            if (bn == 0 && m0 + r < p.M) p.ws_ss[(int64_t)blockIdx.y * p.M + m0 + r] = v;
          } else {
            rden[r] = sqrtf(v) * p.inv_sqrt_k + kRmsEps;
          }
        }
      }
    }
    __syncthreads();
  }
  if (p.dbg & 1) {
    if (acc[0][0][0] == 1234.5f) static_cast<float*>(p.C)[tid] = acc[TM - 1][TN - 1][15];
    return;
  }
  constexpr bool kLdsEpi = (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_SWIGLU || EPI == EPI_GLU) &&
                           BM * BN * 4 <= S * kStageElems * 2;
  if constexpr (kLdsEpi) {
    float* Cs = reinterpret_cast<float*>(lds);
    if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
      if (split) {
        gemm_epilogue_lds<TL, EPI_STORE, false, true, false>(p, acc, rden, Cs, m0, n0, wm, wn, tid);
        return;
      }
    }
    if constexpr (kPre) {
      f32x4 rin[kNVR];
#pragma unroll
      for (int k = 0; k < kNVR; ++k) {
        if constexpr (R16) rin[k] = __builtin_convertvector(rraw[k], f32x4);
        else rin[k] = rraw[k];
      }
      gemm_epilogue_lds<TL, EPI, CBF, false, R16, true>(p, acc, rden, Cs, m0, n0, wm, wn, tid, rin);
    } else {
      gemm_epilogue_lds<TL, EPI, CBF, false, R16>(p, acc, rden, Cs, m0, n0, wm, wn, tid);
    }
    return;
  }
  if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
    if (split) {
      gemm_epilogue<TL, EPI_STORE, false, true>(p, acc, rden, m0, n0, wm, wn, lane);
      return;
    }
  }
  gemm_epilogue<TL, EPI, CBF, false, R16>(p, acc, rden, m0, n0, wm, wn, lane);
}

// Split-K combine: fixed-order sum of the partials, then the STORE/RESID epilogue.
template <int EPI, bool CBF>
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(GemmArgs p, int nsplit) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;     // one float4 of C
  const int64_t n4 = (int64_t)p.M * (p.N / 4);
  if (idx >= n4) return;
  const int row = (int)(idx / (p.N / 4)), col = (int)(idx % (p.N / 4)) * 4;
  f32x4 v = *reinterpret_cast<const f32x4*>(p.ws + (int64_t)row * p.N + col);
  for (int s = 1; s < nsplit; ++s) v += *reinterpret_cast<const f32x4*>(p.ws + ((int64_t)s * p.M + row) * p.N + col);
  if (p.rowscale) {
    float ss = 0.f;
    for (int s = 0; s < nsplit; ++s) ss += p.ws_ss[(int64_t)s * p.M + row];
    const float den = sqrtf(ss) * p.inv_sqrt_k + kRmsEps;
    v.x /= den; v.y /= den; v.z /= den; v.w /= den;
  }
  if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + col);
  if constexpr (EPI == EPI_RESID) {
    if (p.res16) {
      const __half* r = reinterpret_cast<const __half*>(p.R) + (int64_t)row * p.ldr + col;
      v.x = __half2float(r[0]) + p.alpha * v.x; v.y = __half2float(r[1]) + p.alpha * v.y;
      v.z = __half2float(r[2]) + p.alpha * v.z; v.w = __half2float(r[3]) + p.alpha * v.w;
    } else {
      const float* r = p.R + (int64_t)row * p.ldr + col;
      v.x = r[0] + p.alpha * v.x; v.y = r[1] + p.alpha * v.y; v.z = r[2] + p.alpha * v.z; v.w = r[3] + p.alpha * v.w;
    }
  }
  if constexpr (CBF) {
    uint16_t* d = static_cast<uint16_t*>(p.C) + (int64_t)row * p.ldc + col;
    d[0] = bf16_bits(v.x); d[1] = bf16_bits(v.y); d[2] = bf16_bits(v.z); d[3] = bf16_bits(v.w);
  } else if (p.res16) {
    __half* d = static_cast<__half*>(p.C) + (int64_t)row * p.ldc + col;
    d[0] = __float2half_rn(v.x); d[1] = __float2half_rn(v.y); d[2] = __float2half_rn(v.z); d[3] = __float2half_rn(v.w);
  } else {
    float* d = static_cast<float*>(p.C) + (int64_t)row * p.ldc + col;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  if (p.C2) {
    uint16_t* d = p.C2 + (int64_t)row * p.ldc + col;
    d[0] = bf16_bits(v.x); d[1] = bf16_bits(v.y); d[2] = bf16_bits(v.z); d[3] = bf16_bits(v.w);
  }
}

// ---------------------------------------------------------------------------------------------
template <class TL, int EPI, bool MMA16, bool ABF, bool CBF>
static hipError_t launch_one(const GemmArgs& a, int nsplit, hipStream_t st) {
  const int tiles = ((a.M + TL::BM - 1) / TL::BM) * (a.N / TL::BN);
  const dim3 block(TL::WM * TL::WN * 64);
  if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
    if (nsplit > 1) {
      GemmArgs b = a;
      b.k_split = a.K / nsplit;
      hipLaunchKernelGGL((gemm_kernel<TL, EPI_STORE, MMA16, ABF, false, true>), dim3(tiles, nsplit), block, 0, st, b);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      const int64_t n4 = (int64_t)a.M * (a.N / 4);
      hipLaunchKernelGGL((splitk_epilogue_kernel<EPI, CBF>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, b,
                         nsplit);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_kernel<TL, EPI, MMA16, ABF, CBF, false>), dim3(tiles), block, 0, st, a);
  return hipGetLastError();
}

template <class TL, bool MMA16, bool ABF, bool CBF>
static hipError_t launch_epi(const GemmArgs& a, int epi, int nsplit, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_one<TL, EPI_STORE, MMA16, ABF, CBF>(a, nsplit, st);
    case EPI_RESID: return launch_one<TL, EPI_RESID, MMA16, ABF, false>(a, nsplit, st);
    case EPI_SWIGLU: return launch_one<TL, EPI_SWIGLU, MMA16, ABF, CBF>(a, 1, st);
    case EPI_GLU: return launch_one<TL, EPI_GLU, MMA16, ABF, CBF>(a, 1, st);
    default: return hipErrorInvalidValue;
  }
}

template <class TL>
static hipError_t launch_prec(const GemmArgs& a, int epi, bool bf16, int nsplit, hipStream_t st) {
  if (!bf16) return launch_epi<TL, false, false, false>(a, epi, nsplit, st);
  if (a.a_bf16)
    return a.c_bf16 ? launch_epi<TL, true, true, true>(a, epi, nsplit, st) : launch_epi<TL, true, true, false>(a, epi, nsplit, st);
  return a.c_bf16 ? launch_epi<TL, true, false, true>(a, epi, nsplit, st) : launch_epi<TL, true, false, false>(a, epi, nsplit, st);
}

template <class TL, int EPI, bool CBF, int S = 2>
static hipError_t launch_glds(const GemmArgs& a, int nsplit, hipStream_t st) {
  if (a.N % TL::BN || (nsplit > 1 && (a.K % (nsplit * 64)))) return hipErrorInvalidValue;
  const int tiles = ((a.M + TL::BM - 1) / TL::BM) * (a.N / TL::BN);
  const dim3 block(TL::WM * TL::WN * 64);
  if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
    if (nsplit > 1) {
      GemmArgs b = a;
      b.k_split = a.K / nsplit;
      hipLaunchKernelGGL((gemm_glds_kernel<TL, EPI_STORE, false, S>), dim3(tiles, nsplit), block, 0, st, b);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      const int64_t n4 = (int64_t)a.M * (a.N / 4);
      hipLaunchKernelGGL((splitk_epilogue_kernel<EPI, CBF>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, b,
                         nsplit);
      return hipGetLastError();
    }
  }
  GemmArgs c = a;
  c.k_split = 0;
  if constexpr ((EPI == EPI_STORE || EPI == EPI_RESID) && !CBF) {
    if (c.res16) {
      hipLaunchKernelGGL((gemm_glds_kernel<TL, EPI, CBF, S, true>), dim3(tiles), block, 0, st, c);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_glds_kernel<TL, EPI, CBF, S>), dim3(tiles), block, 0, st, c);
  return hipGetLastError();
}

template <class TL, int S = 2>
static hipError_t launch_glds_epi(const GemmArgs& a, int epi, int nsplit, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return a.c_bf16 ? launch_glds<TL, EPI_STORE, true, S>(a, nsplit, st) : launch_glds<TL, EPI_STORE, false, S>(a, nsplit, st);
    case EPI_RESID: return launch_glds<TL, EPI_RESID, false, S>(a, nsplit, st);
    case EPI_SWIGLU: return a.c_bf16 ? launch_glds<TL, EPI_SWIGLU, true, S>(a, 1, st) : launch_glds<TL, EPI_SWIGLU, false, S>(a, 1, st);
    case EPI_GLU: return a.c_bf16 ? launch_glds<TL, EPI_GLU, true, S>(a, 1, st) : launch_glds<TL, EPI_GLU, false, S>(a, 1, st);
    default: return hipErrorInvalidValue;
  }
}

// bf16 operands already in memory: LDS-DMA kernels
// c8_done: set when the launched kernel also wrote a RESID's MXFP8 outputs (a.C8; the LDS-DMA kernels without K split)
static hipError_t gemm_bf16(const GemmArgs& a, int epi, hipStream_t st, bool* c8_done) {
  constexpr int kTarget = 512;
  *c8_done = false;
  // large batches: the persistent transposed-orientation kernels (gemm_t.hip, tools/gemm_bench sweep)
  // the residual-output projections (N = 384) at large M: whole rows per workgroup (gemm_rp.hip)
  // (an argument set it does not implement falls through to the tiled kernels)
  if (epi == EPI_RESID && gemm_rp_routed(a.M, a.K) && gemm_rp_accepts(a)) {
    *c8_done = true;
    return gemm_rp(a, st);
  }
  const int64_t t256 = (int64_t)((a.M + 255) / 256) * (a.N / 256);
  // K = 384 paired projections from 40 (SwiGLU) / 60 (GLU) blocks of 256 rows up: the X-stationary kernel
  // (round 3's gemm_xs: FFN up M = 40960: 114 vs 165 us for gemm_t, M = 10240: 37 vs 41; pw1 M = 40960: 42 vs 47,
  // profiles/r03_xs_route_sweep.jsonl; round 4's gemm_xw 1.8 % / 3 % below gemm_xs in the bf16 B = 4096 step,
  // profiles/r04_xw_step_ab.json)
  const int xblocks = (a.M + 255) / 256;
  // ... and the K = 384 bf16-output STOREs of N >= 768 (q|k|v of layers 0 / 7, k|v of layers 14 / 15) from 80 blocks:
  // M = 40960, N = 1152: 56 vs 74 us; N = 384 stays on the LDS-DMA tiles (29 vs 27 us; profiles/r04_xw_store.jsonl)
  if (a.K == 384 && ((epi == EPI_SWIGLU && xblocks >= 40) || (epi == EPI_GLU && xblocks >= 60) ||
                     (epi == EPI_STORE && a.c_bf16 && !a.C2 && a.N >= 768 && xblocks >= 80))) {
    const hipError_t e = gemm_xw(a, epi, 0, st);
    if (e != hipErrorInvalidValue) return e;   // shape outside gemm_xw's contract: the routes below
  }
  // FFN up: 256 x 256 tiles once there are ~180 of them (M >= 3840 at N = 3072), 256 W x 128 X rows below that
  // down to ~200 tiles (M = 2560: 14.5 vs 20.2 us; tools/gemm_bench, profiles/r02_ffnup_route.jsonl)
  if (epi == EPI_SWIGLU && a.N % 256 == 0 && t256 >= 180) return gemm_t(a, epi, 0, st);
  if (epi == EPI_SWIGLU && a.N % 256 == 0 && (int64_t)((a.M + 127) / 128) * (a.N / 256) >= 200) return gemm_t(a, epi, 2, st);
  if (epi == EPI_GLU && a.N % 128 == 0 && (int64_t)((a.M + 127) / 128) * (a.N / 128) >= 512) return gemm_t(a, epi, 5, st);
  const int64_t t128 = (int64_t)((a.M + 127) / 128) * (a.N / 128);
  const int64_t t64 = (int64_t)((a.M + 63) / 64) * (a.N / 128);
  // 8 waves of 32x64 per 128x128 tile once there is a tile per CU (tools/gemm_bench sweep)
  if (t128 >= kTarget / 2) return *c8_done = true, launch_glds_epi<Tile<128, 128, 4, 2>>(a, epi, 1, st);
  // pw1 (GLU, N = 768) at config 4's per-GPU batch of 512 (M = 5120: 10.3 vs 11.1 us; M = 2560 on 64x128 tiles:
  // 8.5 vs 9.7; profiles/r02_b512_sweep.jsonl)
  if (epi == EPI_GLU && t128 >= 200) return launch_glds_epi<Tile<128, 128, 4, 2>>(a, epi, 1, st);
  if (epi == EPI_GLU && t64 >= 200) return launch_glds_epi<Tile<64, 128, 2, 2>, 2>(a, epi, 1, st);
  // half-chip M (the reduced layers at B = 2048): 64x128 LDS-DMA tiles (scripts/bf16_resid_sweep.sh)
  if ((epi == EPI_STORE || epi == EPI_RESID) && t64 >= kTarget / 2)
    return *c8_done = true, launch_glds_epi<Tile<64, 128, 2, 2>, 2>(a, epi, 1, st);
  if ((epi == EPI_STORE || epi == EPI_RESID) && t64 < kTarget && a.N % 64 == 0 && a.ldc % 8 == 0 && a.lda % 8 == 0 &&
      !a.rpg)
    return gemm_f32t(a, epi, 2, st);   // 64x64 tiles (bf16 operands) instead of a split-K workspace round trip
  int nsplit = 1;
  if ((epi == EPI_STORE || epi == EPI_RESID) && a.ws && t64 < kTarget) {
    const int ksteps = a.K / 64;
    for (int s = 2; s <= 16; ++s) {
      if (ksteps % s || ksteps / s < 3) continue;
      if ((int64_t)s * a.M * a.N > a.ws_cap) break;
      nsplit = s;
      if (t64 * s >= kTarget) break;
    }
  }
  *c8_done = nsplit == 1;
  if (nsplit > 1 || t64 >= kTarget / 2) return launch_glds_epi<Tile<64, 128, 2, 2>>(a, epi, nsplit, st);
  return launch_glds_epi<Tile<32, 128, 1, 2>>(a, epi, 1, st);
}

// Fixed bf16 tile/stage variants (tools/gemm_bench.hip), bypassing the size heuristics.
hipError_t gemm_bf16_variant(const GemmArgs& a, int epi, int variant, int nsplit, hipStream_t st) {
  switch (variant) {
    case 0: return launch_glds_epi<Tile<128, 128, 2, 2>, 2>(a, epi, nsplit, st);
    case 1: return launch_glds_epi<Tile<128, 128, 2, 2>, 3>(a, epi, nsplit, st);
    case 2: return launch_glds_epi<Tile<128, 128, 2, 2>, 4>(a, epi, nsplit, st);
    case 3: return launch_glds_epi<Tile<256, 128, 4, 2>, 2>(a, epi, nsplit, st);
    case 4: return launch_glds_epi<Tile<256, 128, 4, 2>, 3>(a, epi, nsplit, st);
    case 5: return launch_glds_epi<Tile<128, 256, 2, 4>, 2>(a, epi, nsplit, st);
    case 6: return launch_glds_epi<Tile<256, 256, 2, 4>, 2>(a, epi, nsplit, st);
    case 7: return launch_glds_epi<Tile<64, 128, 2, 2>, 2>(a, epi, nsplit, st);
    case 8: return launch_glds_epi<Tile<64, 128, 2, 2>, 3>(a, epi, nsplit, st);
    case 9: return launch_glds_epi<Tile<64, 128, 2, 2>, 4>(a, epi, nsplit, st);
    case 14: return launch_glds_epi<Tile<128, 128, 4, 2>, 2>(a, epi, nsplit, st);
    default: return hipErrorInvalidValue;
  }
}

// Split fp32 (gemm_x3) with the K range split over nsplit workgroups: raw partials into a.ws, then
// the fixed-order combine + epilogue (bias, residual, alpha) -- for the small-M, large-K projections
// (FFN down at B = 256: 60 tiles of 128 x 128 would leave most CUs idle).
hipError_t gemm_x3_splitk(const GemmArgs& a, int epi, int variant, int nsplit, hipStream_t st) {
  if ((epi != EPI_STORE && epi != EPI_RESID) || nsplit < 2 || !a.ws || a.rowscale || a.c_plane || a.c2_plane ||
      a.K % nsplit || (int64_t)nsplit * a.M * a.N > a.ws_cap || a.N % 4)
    return hipErrorInvalidValue;
  GemmArgs b = a;
  b.k_split = a.K / nsplit;
  b.C = a.ws;
  b.ldc = a.N;
  b.bias = nullptr;
  b.R = nullptr;
  b.C2 = nullptr;
  hipError_t e = gemm_x3(b, EPI_STORE, variant, st);
  if (e != hipSuccess) return e;
  GemmArgs c = a;
  c.k_split = a.K / nsplit;
  const int64_t n4 = (int64_t)a.M * (a.N / 4);
  if (epi == EPI_RESID)
    hipLaunchKernelGGL((splitk_epilogue_kernel<EPI_RESID, false>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, c, nsplit);
  else
    hipLaunchKernelGGL((splitk_epilogue_kernel<EPI_STORE, false>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, c, nsplit);
  return hipGetLastError();
}

hipError_t gemm(const GemmArgs& a, int epi, bool bf16, hipStream_t st) {
  const int bk = bf16 ? 64 : 32;
  // the depthwise conv in the GLU epilogue exists on gemm_sm only (fp32 mode, M <= 64): no other route
  if (a.dw.w) return (!bf16 && epi == EPI_GLU && a.M <= 64) ? gemm_sm(a, epi, st) : hipErrorInvalidValue;
  if (a.att.probs) return (!bf16 && epi == EPI_RESID && a.M <= 64) ? gemm_sm(a, epi, st) : hipErrorInvalidValue;
  // the blocked FFN hidden (common.h hblk_off) exists between gemm_xw (SwiGLU out) and gemm_rp (RESID in) only
  if (a.h_blocked) {
    if (!bf16 || !a.a_bf16) return hipErrorInvalidValue;
    if (epi == EPI_SWIGLU) return gemm_xw(a, epi, 0, st);
    return (epi == EPI_RESID && gemm_rp_accepts(a)) ? gemm_rp(a, st) : hipErrorInvalidValue;
  }
  // a fused row norm exists on the row-panel kernel only
  if (a.norm_w)
    return (bf16 && epi == EPI_RESID && gemm_rp_routed(a.M, a.K) && gemm_rp_accepts(a)) ? gemm_rp(a, st)
                                                                                       : hipErrorInvalidValue;
  // the fp16 residual stream exists in the bf16 / fp8 modes only (the LDS-DMA and f32t kernels of gemm_bf16)
  if (a.res16 && (!bf16 || !a.a_bf16 || a.c_bf16 || (epi != EPI_STORE && epi != EPI_RESID))) return hipErrorInvalidValue;
  if (bf16 && a.a_bf16) {
    if (a.K % 64 != 0 || a.N % 128 != 0 || a.M <= 0 || (epi == EPI_RESID && a.c_bf16)) return hipErrorInvalidValue;
    if (a.C8 && (epi != EPI_RESID || !a.C2 || a.N != 32 * kSsSlots || a.ldc != a.N)) return hipErrorInvalidValue;
    bool c8 = false;
    const hipError_t e = gemm_bf16(a, epi, st, &c8);
    // a route without the MXFP8 epilogue (K split, gemm_f32t): quantize the shadow it wrote
    if (e == hipSuccess && a.C8 && !c8) return launch_quant_mx(a.C2, a.ldc, a.M, a.N, a.C8, a.C8s, a.ss8, st);
    return e;
  }
  // fp32 split mode, fragment-packed operands (common.h xpk_off): the consumer is gemm_d3, the producer the fp32 SwiGLU
  // epilogue of gemm_x3 -- nothing else reads or writes that layout
  if (a.a_packed) {
    if (bf16) return hipErrorInvalidValue;
    // the rowscale projections (FFN up, pw1, q|k|v) on the wide form, the N = 384 RESID / STORE ones on gemm_d3
    if (a.rowscale || epi == EPI_SWIGLU || epi == EPI_GLU || a.N != kD) return gemm_d3n(a, epi, -1, st);
    return gemm_d3(a, epi, -1, st);
  }
  if (a.CP) return hipErrorInvalidValue;   // the packed copy of C: written by the direct-load kernels only
  if (a.c_packed && (bf16 || epi != EPI_SWIGLU || !a.W3 || a.a_bf16 || a.c_bf16 || a.c_plane || a.M <= 64 ||
                     a.ldc % 32 != 0))
    return hipErrorInvalidValue;
  if (!bf16 && a.W3 && !a.a_bf16 && !a.c_bf16 && !a.rpg && a.K % 64 == 0 && a.lda % 4 == 0 && a.ldc % 4 == 0) {
    // fp32 by exact bf16 splitting (gemm_t.hip gemm_x3); tile per shape from tools/gemm_bench
    // (scripts/x3_sweep.sh, profiles/r01_x3_sweep_b256.jsonl)
    // (scripts/x3_sweep.sh, scripts/x3w_sweep.sh; profiles/r01_x3_*.jsonl)
    // k|v of layers 14 / 15 (M = B (S + T) >= 5120 at B = 256, N = 768): fp32 W and X through the K-tile
    // ring (gemm_r3) -- 48.8 vs 77.5 us at M = 10240, 33.5 vs 39.8 at 5120; on every other shape of the
    // step the ring kernel is slower (profiles/r02_r3_sweep.jsonl)
    if (epi == EPI_STORE && a.N == 768 && a.M >= 4096 && a.W && !a.rowscale)
      return gemm_r3(a, epi, a.M >= 8192 ? 0 : 1, st);
    // a few rows (B <= 6 streams: the drop-in's per-call batch): the launch is bound by streaming W through the
    // few workgroups' LDS, so spread W over more of them (profiles/r03_b1_sweep.jsonl, M = 10 / 5): FFN up on
    // 128x64 four-wave tiles (16.6 vs 20.7 us), FFN down / the reduction 1x1 split four ways on 64x32 tiles (9.6 vs
    // 15.0), the subsampling Linear (K = 2176) split four ways on 64x64 four-wave tiles (16.9 vs 19.1), the other
    // N = 384 / 1152 projections on 64x32 tiles (6.5 vs 6.8, 7.2 vs 18.6)
    if (a.M <= 64) {
      // B <= 6 streams: fp32 W streamed straight into registers on the exact fp32 MFMA (gemm_sm.hip)
      const hipError_t es = gemm_sm(a, epi, st);
      if (es != hipErrorInvalidValue) return es;
      if (epi == EPI_SWIGLU && a.N % 128 == 0) return gemm_x3(a, epi, 5, st);
      if ((epi == EPI_STORE || epi == EPI_RESID) && a.N % 64 == 0) {
        if (a.K >= 1024 && !a.rowscale && a.ws && a.K % 4 == 0 && (int64_t)4 * a.M * a.N <= a.ws_cap &&
            !a.c_plane && !a.c2_plane) {
          const hipError_t e = gemm_x3_splitk(a, epi, a.K >= 2048 ? 4 : 9, 4, st);
          if (e != hipErrorInvalidValue) return e;
        }
        return gemm_x3(a, epi, 9, st);
      }
    }
    // FFN up: 128 W x 256 X tiles while they fill the CUs at most once (M = 1536 / 2560: 38.1 / 45.2 vs 45.5 / 47.8 us
    // for the previous 256 x 128 / 128 x 128 routes), 128 x 128 tiles otherwise (M = 3328, the 400 ms full layers: 70.5
    // vs 82.4; M = 1280: 25.5) (scripts/r05_x3_sweep2.sh, profiles/r05_x3_sweep2.jsonl, three interleaved runs)
    if (epi == EPI_SWIGLU && a.N % 256 == 0) {
      const int64_t t8 = (int64_t)((a.M + 255) / 256) * (a.N / 128);
      return gemm_x3(a, epi, (t8 > 128 && t8 <= 256) ? 8 : 6, st);
    }
    if (epi == EPI_SWIGLU && a.N % 128 == 0) return gemm_x3(a, epi, 6, st);
    // pw1: 128 W x 64 X tiles, or 128 x 128 once those overflow one round of the CUs (M = 3328, the 400 ms full layers:
    // 312 vs 156 workgroups, 22.1 vs 26.4 us; scripts/r05_x3_400.sh, profiles/r05_x3_400.jsonl)
    if (epi == EPI_GLU && a.N % 128 == 0)
      return gemm_x3(a, epi, ((int64_t)((a.M + 63) / 64) * (a.N / 128) > 256 && a.M <= 4096) ? 6 : 1, st);
    // q|k|v (N = 1152): 128 W x 64 X tiles below ~128 tiles of 128 x 128 (M = 1280 / 1536: 15.5 / 16.3 vs 22.7 / 23.1 us)
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N >= 1024 && a.N % 128 == 0)
      return gemm_x3(a, epi, (int64_t)((a.M + 127) / 128) * (a.N / 128) < 128 ? 1 : 6, st);
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N % 64 == 0 && a.K % 128 == 0 &&
        (int64_t)((a.M + 63) / 64) * (a.N / 32) <= 256)
      // up to one 32x64 tile per CU (the reduced layers at B = 256, M = 1280): 32x64 tiles with a four-way in-WG
      // K split fill twice the CUs; beats split-K on FFN down (19.1 vs 22.2 us) and the 64x64 tile on the
      // K = 384 projections (8.1 vs 11.1 us) (scripts/x3n_sweep.sh, profiles/r01_x3n_sweep_b256.jsonl); past one per
      // CU the 64x64 tile (M = 1536, the 400 ms reduced layers: FFN down 28.4 vs 34.3 us, K = 384 10.9 vs 13.8)
      return gemm_x3(a, epi, 10, st);
    // N = 384, K = 1536 (FFN down) where the 64x64 tiles miss one full round of the CUs -- 312 of them at M = 3328 (the
    // 400 ms full layers: 1.22 rounds), 144 at M = 1536 (the 400 ms reduced layers) -- a 3-way K split on 128x128 /
    // 64W x 128X tiles (234 / 216 workgroups, partials reduced in a fixed order by splitk_epilogue): 36.4 vs 54.5 us and
    // 23.8 vs 28.2; at M = 2560 (240 tiles) the split is no faster (scripts/r05_x3_splitk.sh,
    // profiles/r05_x3_splitk.jsonl)
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N == 384 && a.K == 1536 && !a.rowscale && a.ws && !a.c_plane &&
        !a.c2_plane && (int64_t)3 * a.M * a.N <= a.ws_cap) {
      const int64_t t0 = (int64_t)((a.M + 63) / 64) * (a.N / 64);
      if ((t0 > 256 || t0 < 192) && a.M <= 4096) {   // measured up to M = 3328
        const hipError_t e = gemm_x3_splitk(a, epi, a.M >= 2048 ? 6 : 2, 3, st);
        if (e != hipErrorInvalidValue) return e;
      }
    }
    // K = 384 at M = 3328 (attn-out / pw2 of the 400 ms full layers): the 64x64 tiles make 1.22 rounds, 128 W x 64 X
    // tiles one (15.8 vs 20.8 us, profiles/r05_x3_400.jsonl)
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N % 128 == 0 && a.K == 384 && a.M <= 4096 &&
        (int64_t)((a.M + 63) / 64) * (a.N / 64) > 256)
      return gemm_x3(a, epi, 1, st);
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N % 64 == 0) return gemm_x3(a, epi, 0, st);
  }
  if (!bf16 && !a.a_bf16 && !a.c_bf16 && !a.rpg && a.K % 64 == 0 && a.lda % 4 == 0 && a.ldc % 4 == 0) {
    // exact-fp32 projections other than the FFN up-projection: in-workgroup K split (gemm_t.hip)
    if ((epi == EPI_STORE || epi == EPI_RESID) && a.N % 64 == 0) return gemm_f32t(a, epi, 0, st);
    if (epi == EPI_GLU && a.N % 128 == 0) return gemm_f32t(a, epi, 1, st);
  }
  if (a.K % bk != 0 || a.N % 128 != 0 || a.M <= 0) return hipErrorInvalidValue;
  if (!bf16 && (a.a_bf16 || a.c_bf16)) return hipErrorInvalidValue;
  if (epi == EPI_RESID && a.c_bf16) return hipErrorInvalidValue;
  constexpr int kTarget = 512;     // >= 2 tiles per CU on 256 CUs
  const int64_t t128 = (int64_t)((a.M + 127) / 128) * (a.N / 128);
  const int64_t t64 = (int64_t)((a.M + 63) / 64) * (a.N / 128);
  if (t128 >= kTarget) return launch_prec<Tile<128, 128, 2, 2>>(a, epi, bf16, 1, st);
  int nsplit = 1;
  if ((epi == EPI_STORE || epi == EPI_RESID) && a.ws && t64 < kTarget) {
    // smallest split of the K-steps that reaches the target, keeping >= 3 K-steps per split
    const int ksteps = a.K / bk;
    for (int s = 2; s <= 16; ++s) {
      if (ksteps % s || ksteps / s < 3) continue;
      if ((int64_t)s * a.M * a.N > a.ws_cap) break;
      nsplit = s;
      if (t64 * s >= kTarget) break;
    }
  }
  if (nsplit > 1 || t64 >= kTarget / 2) return launch_prec<Tile<64, 128, 2, 2>>(a, epi, bf16, nsplit, st);
  return launch_prec<Tile<32, 128, 1, 2>>(a, epi, bf16, 1, st);
}

hipError_t conv2_gemm(const void* x2, const void* w, const float* scale, const float* shift, void* flat, int B,
                      bool bf16, hipStream_t st, int chunk, const void* w2p) {
  const Geom geo = make_geom(chunk);
  // per-stream LDS slab kernel (frontend.hip): the 300 ms slab (38 rows, 107 KB) fits, 400 ms (48) does not
  if (bf16 && geo.T == kT) return launch_conv2_bf16(x2, w, scale, shift, flat, B, st);
  // fp32 split mode (frontend.hip): input rows split once per kernel row (conv2_p3)
  // (B <= 8 streams: conv2_sm, the taps spread over 120 workgroups per stream on the exact fp32 MFMA)
  if (w2p) return B <= 8 ? launch_conv2_sm(x2, w, scale, shift, flat, B, geo.T, st)
                         : launch_conv2_p3(x2, w2p, scale, shift, flat, B, geo.T, st);
  GemmArgs a{};
  a.A = x2;
  a.W = w;
  a.C = flat;
  a.bias = shift;
  a.scale = scale;
  a.M = B * geo.T * kSub2F;
  a.N = kSub2C;
  a.K = bf16 ? kConv2KPad : kSub2Kt * kSub2Kf * kSub1C;
  a.conv_t = geo.T;
  a.conv_in = geo.sub2In;
  const dim3 grid((a.M + 127) / 128), block(256);
  if (bf16) hipLaunchKernelGGL((gemm_glds_kernel<Tile<128, 64, 4, 1>, EPI_CONV2, true, 2>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((gemm_kernel<Tile<128, 64, 4, 1>, EPI_CONV2, false, false, false, false>), grid, block, 0, st, a);
  return hipGetLastError();
}

// Log-mel as two fp32-MFMA GEMMs over all B*30 frames (feats.py:95-102):
//   power[(b,t)][f] = |sum_k basis_f[k] wave[b][80t + k]|^2      K = 160, N = 256 (re/im blocks)
//   feats[(b,t)][m] = fp16(log(sum_f fbank[m][f] power[f] + 2^-24))  K = 128, N = 128 (64 used)
hipError_t mel_gemms(const float* wave, const float* basis_p, const float* fbank_p, float* power, float* feats, int B,
                     int chunk, hipStream_t st) {
  const Geom geo = make_geom(chunk);
  GemmArgs a{};
  a.A = wave;
  a.lda = kHop;
  a.rpg = geo.melT;
  a.gstride = geo.wave;
  a.W = basis_p;
  a.C = power;
  a.ldc = kMelPowCols;
  a.M = B * geo.melT;
  a.K = kWin;
  const dim3 block(256);
  if (a.M >= 16384) {
    // large batch: bins 0..95 only (the 81 real bins in three 32-bin Re | Im blocks; the fourth block of the packed
    // basis is all zero and its power columns keep the buffer's zero fill), 64 x 64 tiles, one Re | Im pair per wave:
    // 103 -> 89 us at M = 122880; at M = 7680 the 128-thread tiles are slower (15.2 vs 11.8 us), so the 64 x 128 tiles
    // over all four blocks stay there (profiles/r04_power_bins96_ab.jsonl, r04_power_bins96_*_step_breakdown.txt)
    static_assert(kBins <= 96 && kMelPowCols >= 96, "three 32-bin blocks cover the spectrum");
    a.N = 2 * 96;
    hipLaunchKernelGGL((gemm_kernel<Tile<64, 64, 2, 1>, EPI_POWER, false, false, false, false>),
                       dim3(((a.M + 63) / 64) * (a.N / 64)), dim3(128), 0, st, a);
  } else {
    a.N = 2 * kMelPowCols;
    hipLaunchKernelGGL((gemm_kernel<Tile<64, 128, 2, 2>, EPI_POWER, false, false, false, false>),
                       dim3(((a.M + 63) / 64) * (a.N / 128)), block, 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  GemmArgs m{};
  m.A = power;
  m.lda = kMelPowCols;
  m.W = fbank_p;
  m.C = feats;
  m.ldc = kMels;
  m.n_out = kMels;
  m.M = B * geo.melT;
  m.N = kMels;   // the 64 filter rows of the zero-padded [128][128] fbank (a 128-wide tile computed 64 zero columns)
  m.K = kMelPowCols;
  hipLaunchKernelGGL((gemm_kernel<Tile<64, 64, 2, 2>, EPI_LOGMEL, false, false, false, false>),
                     dim3((m.M + 63) / 64), block, 0, st, m);
  return hipGetLastError();
}

}  // namespace tone
