// Small-M exact-fp32 projections (fp32 mode, M <= 64): the drop-in's per-call batch, B = 1 .. 6 streams
// (tone/pipeline.py:146 calls the model one chunk at a time).
//
// At M = 10 (one stream, T = 10) a projection is a weight stream: FFN up reads 4.7 MB of W for 24 MFLOP.  The split
// kernels (gemm_x3) stage W as three bf16 planes (6 B per weight) through the LDS of a few dozen workgroups and
// reached ~0.3 TB/s (profiles/r03_fp32_b1_step_breakdown.txt).  Here W is read once in fp32
// (4 B per weight) straight into registers -- no LDS staging, every lane's 16-byte load is one MFMA operand -- and
// multiplied on v_mfma_f32_16x16x4_f32, whose result is bit for bit a k-ordered fp32 fma chain (exact fp32: the
// MFMA rate is irrelevant at these M):
//   * a workgroup owns 16 output columns (one 16-row W block; SWIGLU / GLU: the g and u blocks of 16 hidden units)
//     and all M rows (MB 16-row blocks, rows past M clamped), its KS waves split K and reduce through LDS;
//   * lane l of a 16-deep K step loads W[n0 + (l & 15)][k0 + 4 (l >> 4) .. + 3] and X[m0 + (l & 15)][same k]: MFMA j
//     of the step takes element j, i.e. the k set {k0 + 4 g + j : g = 0..3} -- the four MFMAs cover the step's 16 k
//     with both operands in the same order;
//   * D[n][m] has m on the lane (l & 15) and four consecutive n in the registers: the epilogue (bias, folded-RMSNorm
//     row factor, residual, SwiGLU / GLU with the IEEE exp and division of the fp32 epilogues) stores 16 bytes per
//     lane and row.
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

namespace tone {
namespace {

//   * DWT > 0 (EPI_GLU, the conv module's pointwise-1 at T = DWT frames per stream): the 16 GLU output channels of
//     all M rows go through LDS to one lane per (stream, channel), which runs dwconv_kernel's depthwise conv over
//     [conv state ; the stream's T rows] (same taps, same fma order, IEEE SiLU) and writes the next state: the
//     separate dwconv launch (5 us at B = 1) is gone.  Its taps and state are loaded before the K loop.
//   * ATT > 0 (EPI_RESID, K = 384: the attn-out projection of a shared-probability layer at T = ATT frames): the A
//     operand is ctx = P V, computed per 4-column fragment in the K loop (attention_kernel's j-ordered fma chain, so
//     the same values) from the probabilities and V; the separate attention launch is gone.
template <int EPI, int MB, int KS, int STEPS, bool RS, int DWT = 0, int ATT = 0>
__global__ void __launch_bounds__(KS * 64) gemm_sm_kernel(GemmArgs p) {
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU);
  constexpr int NB = PAIRED ? 2 : 1;
  constexpr int RED = (KS - 1) * NB * MB * 4 * 64;                 // K-split partial sums (floats)
  constexpr int REDS = RS ? (KS - 1) * MB * 64 : 0;                // ... and row sums of squares
  static_assert(DWT == 0 || (EPI == EPI_GLU && RED >= MB * 16 * 16), "dwconv fusion: GLU, the tile fits in LDS");
  __shared__ __attribute__((aligned(16))) float lds[(RED > 0 ? RED : 1) + (REDS > 0 ? REDS : 1)];

  const int tid = threadIdx.x, lane = tid & 63, wk = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lg = lane >> 4;
  int n0[NB];
  int c0;                                                          // first output column of this workgroup
  if constexpr (PAIRED) {
    const int qb = blockIdx.x >> 1, hh = blockIdx.x & 1;          // W rows 64 qb + 16 hh (g) and + 32 (u)
    n0[0] = 64 * qb + 16 * hh;
    n0[NB - 1] = 64 * qb + 32 + 16 * hh;
    c0 = 32 * qb + 16 * hh;
  } else {
    n0[0] = 16 * blockIdx.x;
    c0 = n0[0];
  }
  const float* __restrict__ W = static_cast<const float*>(p.W);
  const float* __restrict__ X = static_cast<const float*>(p.A);
  const int kb = wk * STEPS * 16;                                 // this wave's K range: STEPS 16-deep steps

  f32x4 acc[NB][MB];
  float ss[MB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[i][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) ss[mb] = 0.f;
  const float* wr[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) wr[i] = W + (int64_t)(n0[i] + l16) * p.K + kb + 4 * lg;
  const float* xr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xr[mb] = X + (int64_t)min(16 * mb + l16, p.M - 1) * p.lda + kb + 4 * lg;

  // dwconv operands of the lane's first (stream, channel) pair, loaded under the W stream
  constexpr int DT = DWT > 0 ? DWT : 1;
  float dwk[DWT > 0 ? kConvK : 1], dwx[DWT > 0 ? kConvS : 1], dwb = 0.f;
  if constexpr (DWT > 0) {
    const int ch = c0 + (lane & 15), b = min(lane >> 4, p.M / DT - 1);
#pragma unroll
    for (int k = 0; k < kConvK; ++k) dwk[k] = p.dw.w[k * kD + ch];
    dwb = p.dw.b[ch];
    const __half* st = p.dw.s.in + p.dw.s.row_in(b) + kOffConv + (int64_t)p.dw.layer * kD * kConvS + ch * kConvS;
#pragma unroll
    for (int i = 0; i < kConvS; ++i) dwx[i] = __half2float(st[i]);
  }

#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    f32x4 w[NB], x[MB];
#pragma unroll
    for (int i = 0; i < NB; ++i) w[i] = *reinterpret_cast<const f32x4*>(wr[i] + 16 * s);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      if constexpr (ATT > 0) {
        const int m = min(16 * mb + l16, p.M - 1), sb = m / ATT, i = m - sb * ATT;
        const int k0 = kb + 16 * s + 4 * lg, h = k0 / kDk;
        const float* pr = p.att.probs + (((int64_t)sb * kHeads + h) * ATT + i) * ATT;
        const float* vr = p.att.v + (int64_t)sb * ATT * p.att.ldv + k0;
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < ATT; ++j) {
          const float pj = pr[j];
          const f32x4 vj = *reinterpret_cast<const f32x4*>(vr + (int64_t)j * p.att.ldv);
          c.x = fmaf(pj, vj.x, c.x);
          c.y = fmaf(pj, vj.y, c.y);
          c.z = fmaf(pj, vj.z, c.z);
          c.w = fmaf(pj, vj.w, c.w);
        }
        x[mb] = c;
      } else {
        x[mb] = *reinterpret_cast<const f32x4*>(xr[mb] + 16 * s);
      }
    }
    if constexpr (RS) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        ss[mb] = fmaf(x[mb].x, x[mb].x, ss[mb]);
        ss[mb] = fmaf(x[mb].y, x[mb].y, ss[mb]);
        ss[mb] = fmaf(x[mb].z, x[mb].z, ss[mb]);
        ss[mb] = fmaf(x[mb].w, x[mb].w, ss[mb]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[i][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[i][j], x[mb][j], acc[i][mb], 0, 0, 0);
  }

  // K-split reduction: waves 1.. park their partials in LDS, wave 0 adds them in a fixed order
  if constexpr (KS > 1) {
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          *reinterpret_cast<f32x4*>(lds + ((((wk - 1) * NB + i) * MB + mb) * 64 + lane) * 4) = acc[i][mb];
      if constexpr (RS) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) lds[RED + ((wk - 1) * MB + mb) * 64 + lane] = ss[mb];
      }
    }
    __syncthreads();
    if constexpr (DWT == 0) {
      if (wk > 0) return;
    }
  }
  // reduction + epilogue: wave 0 (with DWT the other waves wait for the GLU tile, then share the depthwise conv)
  if (DWT == 0 || wk == 0) {
    if constexpr (KS > 1) {
#pragma unroll
      for (int g = 1; g < KS; ++g) {
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(lds + ((((g - 1) * NB + i) * MB + mb) * 64 + lane) * 4);
            acc[i][mb] += v;
          }
        if constexpr (RS) {
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) ss[mb] += lds[RED + ((g - 1) * MB + mb) * 64 + lane];
        }
      }
    }

    // epilogue (wave 0): lane holds row m = 16 mb + l16, columns c0 + 4 lg .. + 3
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float inv = 1.0f;
      if constexpr (RS) {
        const float t = lg_sum(ss[mb]);   // v_permlane16/32_swap (the xor-16 / xor-32 shuffles' association)
        inv = 1.0f / (sqrtf(t) * p.inv_sqrt_k + kRmsEps);
      }
      const int m = 16 * mb + l16;
      if (m >= p.M) continue;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0[0] + 4 * lg + r;
        const float bg = p.bias ? p.bias[n] : 0.f;
        const float g = fmaf(acc[0][mb][r], inv, bg);
        if constexpr (PAIRED) {
          const float bu = p.bias ? p.bias[n0[NB - 1] + 4 * lg + r] : 0.f;
          const float u = fmaf(acc[NB - 1][mb][r], inv, bu);
          o[r] = (EPI == EPI_SWIGLU) ? silu_f(g) * u : g * sigmoid_f(u);
        } else {
          o[r] = g;
        }
      }
      if constexpr (DWT > 0) {   // the GLU tile -> LDS (the partial sums there are consumed)
        *reinterpret_cast<f32x4*>(lds + m * 16 + 4 * lg) = f32x4{o[0], o[1], o[2], o[3]};
        continue;
      }
      float* crow = static_cast<float*>(p.C) + (int64_t)m * p.ldc + c0 + 4 * lg;
      if constexpr (EPI == EPI_RESID) {
        const f32x4 rr = *reinterpret_cast<const f32x4*>(p.R + (int64_t)m * p.ldr + c0 + 4 * lg);
        *reinterpret_cast<f32x4*>(crow) = f32x4{rr.x + p.alpha * o[0], rr.y + p.alpha * o[1], rr.z + p.alpha * o[2],
                                                rr.w + p.alpha * o[3]};
      } else {
        *reinterpret_cast<f32x4*>(crow) = f32x4{o[0], o[1], o[2], o[3]};
      }
    }
  }
  if constexpr (DWT > 0) {
    __syncthreads();                                     // the GLU tile is in LDS
    const int nb = p.M / DT;
    // uniform trip count over the waves (the barrier below): every wave handles the same (stream, channel) pairs
    for (int base = 0; base < nb * 16; base += 64) {
      const int pr = base + lane;
      if (base > 0) {   // streams 4 and up (B > 4): their state now, read by every wave before any wave writes
        if (pr < nb * 16) {
          const __half* st = p.dw.s.in + p.dw.s.row_in(pr >> 4) + kOffConv + (int64_t)p.dw.layer * kD * kConvS +
                             (c0 + (pr & 15)) * kConvS;
#pragma unroll
          for (int i = 0; i < kConvS; ++i) dwx[i] = __half2float(st[i]);
        }
        __syncthreads();   // the state rows may be written in place (slots_out == slots)
      }
      if (pr >= nb * 16) continue;
      const int b = pr >> 4, cl = pr & 15, ch = c0 + cl;
      const int64_t sec = kOffConv + (int64_t)p.dw.layer * kD * kConvS + ch * kConvS;
      float x[kConvS + DT];
#pragma unroll
      for (int i = 0; i < kConvS; ++i) x[i] = dwx[i];
#pragma unroll
      for (int t = 0; t < DT; ++t) x[kConvS + t] = lds[(b * DT + t) * 16 + cl];
#pragma unroll
      for (int t = 0; t < DT; ++t) {                     // the KS waves take every KS-th output frame
        if (t % KS != wk) continue;
        float acc = dwb;
#pragma unroll
        for (int k = 0; k < kConvK; ++k) acc = fmaf(dwk[k], x[t + k], acc);
        p.dw.out[((int64_t)b * DT + t) * kD + ch] = silu_f(acc);
      }
      __half* so = p.dw.s.out + p.dw.s.row_out(b) + sec;
#pragma unroll
      for (int i = 0; i < kConvS; ++i)
        if (i % KS == wk) so[i] = __float2half_rn(x[DT + i]);
    }
  }
}

template <int EPI, int KS, int STEPS, bool RS, int DWT = 0, int ATT = 0>
hipError_t launch_sm_mb(const GemmArgs& a, hipStream_t st) {
  constexpr bool PAIRED = (EPI == EPI_SWIGLU || EPI == EPI_GLU);
  const dim3 grid(PAIRED ? a.N / 32 : a.N / 16), block(KS * 64);
  switch ((a.M + 15) / 16) {
    case 1: hipLaunchKernelGGL((gemm_sm_kernel<EPI, 1, KS, STEPS, RS, DWT, ATT>), grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL((gemm_sm_kernel<EPI, 2, KS, STEPS, RS, DWT, ATT>), grid, block, 0, st, a); break;
    case 3: hipLaunchKernelGGL((gemm_sm_kernel<EPI, 3, KS, STEPS, RS, DWT, ATT>), grid, block, 0, st, a); break;
    case 4: hipLaunchKernelGGL((gemm_sm_kernel<EPI, 4, KS, STEPS, RS, DWT, ATT>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// pointwise-1 (GLU, rowscale, K = 384) with the depthwise conv in the epilogue: frames per stream as a template
// argument (the dwconv registers stay registers)
template <int DWT>
hipError_t launch_sm_dw(const GemmArgs& a, hipStream_t st) {
  if (a.M % DWT || a.N != 2 * kD) return hipErrorInvalidValue;
  return launch_sm_mb<EPI_GLU, 4, 6, true, DWT>(a, st);
}

}  // namespace

// K split over KS waves with ~6 16-deep steps each: K = 384 -> 4 waves, 1536 -> 16, 2176 -> 8; the rowscale
// (folded RMSNorm) GEMMs are the K = 384 ones
hipError_t gemm_sm(const GemmArgs& a, int epi, hipStream_t st) {
  if (!a.W || a.a_bf16 || a.c_bf16 || a.C2 || a.rpg || a.k_split || a.a_plane || a.c_plane || a.M <= 0 || a.M > 64 ||
      a.lda % 4 || a.ldc % 4 || (epi == EPI_RESID && a.ldr % 4))
    return hipErrorInvalidValue;
  const bool paired = (epi == EPI_SWIGLU || epi == EPI_GLU);
  if (a.N % (paired ? 64 : 16)) return hipErrorInvalidValue;
  const bool rs = a.rowscale != 0;
  if (a.dw.w) {
    if (epi != EPI_GLU || a.K != 384 || !rs || !a.dw.out) return hipErrorInvalidValue;
    switch (a.dw.T) {
      case 10: return launch_sm_dw<10>(a, st);
      case 5: return launch_sm_dw<5>(a, st);
      case 13: return launch_sm_dw<13>(a, st);
      case 6: return launch_sm_dw<6>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if (a.att.probs) {   // attn-out of a shared-probability layer, ctx computed in the operand loads
    if (epi != EPI_RESID || a.K != kD || rs || !a.att.v || a.att.ldv % 4 || a.M % a.att.T) return hipErrorInvalidValue;
    switch (a.att.T) {
      case 10: return launch_sm_mb<EPI_RESID, 4, 6, false, 0, 10>(a, st);
      case 5: return launch_sm_mb<EPI_RESID, 4, 6, false, 0, 5>(a, st);
      case 13: return launch_sm_mb<EPI_RESID, 4, 6, false, 0, 13>(a, st);
      case 6: return launch_sm_mb<EPI_RESID, 4, 6, false, 0, 6>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if (a.K == 384) {
    switch (epi) {
      case EPI_STORE: return rs ? launch_sm_mb<EPI_STORE, 4, 6, true>(a, st) : launch_sm_mb<EPI_STORE, 4, 6, false>(a, st);
      case EPI_RESID: return rs ? launch_sm_mb<EPI_RESID, 4, 6, true>(a, st) : launch_sm_mb<EPI_RESID, 4, 6, false>(a, st);
      case EPI_SWIGLU: return rs ? launch_sm_mb<EPI_SWIGLU, 4, 6, true>(a, st) : launch_sm_mb<EPI_SWIGLU, 4, 6, false>(a, st);
      case EPI_GLU: return rs ? launch_sm_mb<EPI_GLU, 4, 6, true>(a, st) : launch_sm_mb<EPI_GLU, 4, 6, false>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if (rs || (epi != EPI_STORE && epi != EPI_RESID)) return hipErrorInvalidValue;
  if (a.K == 1536) return epi == EPI_STORE ? launch_sm_mb<EPI_STORE, 16, 6, false>(a, st) : launch_sm_mb<EPI_RESID, 16, 6, false>(a, st);
  if (a.K == 2176) return epi == EPI_STORE ? launch_sm_mb<EPI_STORE, 8, 17, false>(a, st) : launch_sm_mb<EPI_RESID, 8, 17, false>(a, st);
  return hipErrorInvalidValue;
}

}  // namespace tone
