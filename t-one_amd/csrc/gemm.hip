// Dense contractions of the acoustic path on CDNA4 MFMA, with fused epilogues.
//
//   C[M][N] = epilogue( rowscale(A)[M][K] . W[N][K]^T )
//
// W is row-major [N][K] exactly like torch Linear / 1x1 Conv1d weights, so the B operand is read
// K-contiguous like A.  Two arithmetic modes share one tiling:
//   fp32: v_mfma_f32_32x32x2_f32  (exact fp32 products, fp32 accumulate; BASELINE config 2)
//   bf16: v_mfma_f32_32x32x16_bf16 (A converted to bf16 while staging, fp32 accumulate; config 3)
//
// Fused epilogues (the reference ops they absorb):
//   rowscale  RMSNorm folded into the GEMM: the gain is pre-multiplied into W's columns and the
//             row's 1/(||a||/sqrt(K) + 1e-8) is computed from the staged A tile
//             (submodules.py:34-54 feeding Linear/Conv1d with K = d_model = 384)
//   STORE     + bias                                       (nn.Linear)
//   RESID     R + alpha*(acc + bias)                       (residual adds, conformer_blocks.py:814-834)
//   SWIGLU    silu(g + b1) * (v + bv) on interleaved 32-row W1/Wv blocks (conformer_blocks.py:479-482)
//   GLU       (a + ba) * sigmoid(g + bg) on interleaved pw1 halves     (conformer_blocks.py:419-422)
//
// Pipeline: A/W tiles of the next K-step are fetched into registers while the MFMAs run on the
// current LDS buffer (two LDS buffers, one barrier per K-step).  When M*N gives too few tiles to
// fill 256 CUs (small batches, N = 384) the K range is split over blocks (blockIdx.y); the fp32
// partials go to a workspace and a second kernel sums them in a fixed order (deterministic) and
// applies the epilogue.
#include "common.h"
#include "kernels.h"

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

template <int BM, int BN, int WM, int WN, int EPI, bool BF16, bool SPLIT>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(GemmArgs p) {
  constexpr int NT = WM * WN * 64;
  constexpr int BK = 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  static_assert(EPI < EPI_SWIGLU || (TN % 2 == 0), "gated epilogues pair n-tiles");
  static_assert(!SPLIT || EPI < EPI_SWIGLU, "split-K only for STORE/RESID");
  constexpr bool CONV2 = (EPI == EPI_CONV2);
  constexpr int LDS_ROW = BF16 ? (BK + 8) : (BK + 4);  // elements; keeps ds_read_b128 conflict-free
  using ST = typename std::conditional<BF16, uint16_t, float>::type;
  constexpr int A_V = BM * BK / 4 / NT;                 // float4 of A per thread per k-tile
  constexpr int W_VE = BF16 ? 8 : 4;                    // W elements per 16-byte vector
  constexpr int W_V = BN * BK / W_VE / NT;              // 16-byte W vectors per thread
  static_assert(A_V >= 1 && W_V >= 1, "tile too small for the thread count");

  __shared__ __attribute__((aligned(16))) ST As[2][BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) ST Bs[2][BN * LDS_ROW];
  __shared__ float rden[BM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = p.N / BN;
  const int bm = blockIdx.x / ntn, bn = blockIdx.x % ntn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int kb = SPLIT ? blockIdx.y * p.k_split : 0;
  const int nk = (SPLIT ? p.k_split : p.K) / BK;
  const float* __restrict__ A = p.A;

  f32x4 ra[A_V];
  u32x4 rw[W_V];
  float ss[A_V];
  int64_t rowbase[CONV2 ? A_V : 1];
#pragma unroll
  for (int i = 0; i < A_V; ++i) ss[i] = 0.f;
  if constexpr (CONV2) {
    // output position (b, t, f) of A row r -> base of its receptive field in x2[b][38][44][32]
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int r = (tid + i * NT) / (BK / 4);
      const int pos = min(m0 + r, p.M - 1);
      const int b = pos / (kT * kSub2F), rem = pos % (kT * kSub2F);
      const int t = rem / kSub2F, f = rem % kSub2F;
      rowbase[i] = (((int64_t)b * kSub2In + kSub2Stride * t) * kSub1F + f) * kSub1C;
    }
  }

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / 4), c = idx % (BK / 4);
      const int gm = m0 + r;
      const int gmc = gm < p.M ? gm : p.M - 1;        // clamped row; zeroed below (no branch)
      int64_t off;
      if constexpr (CONV2) {
        const int tap = k0 / BK, kt = tap / kSub2Kf, kf = tap % kSub2Kf;
        off = rowbase[i] + (kt * kSub1F + kf) * kSub1C + c * 4;
      } else {
        off = (int64_t)gmc * p.lda + k0 + c * 4;
      }
      f32x4 v = *reinterpret_cast<const f32x4*>(A + off);
      ra[i] = gm < p.M ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / W_VE), c = idx % (BK / W_VE);
      const ST* base = static_cast<const ST*>(p.W) + (int64_t)(n0 + r) * p.K + k0 + c * W_VE;
      rw[i] = *reinterpret_cast<const u32x4*>(base);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / 4), c = idx % (BK / 4);
      const f32x4 v = ra[i];
      if (p.rowscale) ss[i] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      if constexpr (BF16) {
        u32x2 u;
        u.x = pack_bf16x2(v.x, v.y);
        u.y = pack_bf16x2(v.z, v.w);
        *reinterpret_cast<u32x2*>(&As[buf][r * LDS_ROW + c * 4]) = u;
      } else {
        *reinterpret_cast<f32x4*>(&As[buf][r * LDS_ROW + c * 4]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / W_VE), c = idx % (BK / W_VE);
      *reinterpret_cast<u32x4*>(&Bs[buf][r * LDS_ROW + c * W_VE]) = rw[i];
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
    if constexpr (BF16) {
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
      for (int i = 0; i < A_V; ++i) ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};   // no double count in ss
    }
    store(cur ^ 1);
    __syncthreads();
  }

  if (p.rowscale) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      const int idx = tid + i * NT, r = idx / (BK / 4);
      if ((idx % (BK / 4)) == 0) {
        if constexpr (SPLIT) {
          if (bn == 0 && m0 + r < p.M) p.ws_ss[(int64_t)blockIdx.y * p.M + m0 + r] = v;
        } else {
          rden[r] = sqrtf(v) * p.inv_sqrt_k + kRmsEps;
        }
      }
    }
    if constexpr (!SPLIT) __syncthreads();
  }

  // ---- epilogue: C/D map of v_mfma_*_32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lrow = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int row = m0 + lrow;
      if (row >= p.M) continue;
      if constexpr (SPLIT) {
        float* dst = p.ws + ((int64_t)blockIdx.y * p.M + row) * p.N;
#pragma unroll
        for (int j = 0; j < TN; ++j) dst[n0 + wn * WTN + j * 32 + lr] = acc[i][j][r];
        continue;
      } else if constexpr (CONV2) {
        const int b = row / (kT * kSub2F), rem = row % (kT * kSub2F);
        const int t = rem / kSub2F, f = rem % kSub2F;
        float* dst = p.C + ((int64_t)b * kT + t) * kSubOut + f * kSub2C;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int c = n0 + wn * WTN + j * 32 + lr;
          dst[c] = silu_f(fmaf(acc[i][j][r], p.scale[c], p.bias[c]));
        }
        continue;
      } else {
        const float den = p.rowscale ? rden[lrow] : 1.0f;
        if constexpr (EPI == EPI_STORE || EPI == EPI_RESID) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * WTN + j * 32 + lr;
            float v = acc[i][j][r];
            if (p.rowscale) v = v / den;
            if (p.bias) v += p.bias[col];
            if constexpr (EPI == EPI_RESID) v = p.R[(int64_t)row * p.ldr + col] + p.alpha * v;
            p.C[(int64_t)row * p.ldc + col] = v;
          }
        } else {
#pragma unroll
          for (int jp = 0; jp < TN / 2; ++jp) {
            const int cg = n0 + wn * WTN + 2 * jp * 32 + lr;   // packed column of the gate/first half
            float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
            if (p.rowscale) { g = g / den; u = u / den; }
            g += p.bias[cg];
            u += p.bias[cg + 32];
            const int oc = (n0 + wn * WTN) / 2 + jp * 32 + lr;
            float o;
            if constexpr (EPI == EPI_SWIGLU) o = silu_f(g) * u;   // linear1 -> SiLU, times linearv
            else o = g * sigmoid_f(u);                            // GLU: first half * sigmoid(second)
            p.C[(int64_t)row * p.ldc + oc] = o;
          }
        }
      }
    }
  }
}

// Split-K combine: fixed-order sum of the partials, then the STORE/RESID epilogue.
template <int EPI>
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(GemmArgs p, int nsplit) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;     // one float4 of C
  const int64_t n4 = (int64_t)p.M * (p.N / 4);
  if (idx >= n4) return;
  const int row = (int)(idx / (p.N / 4)), col = (int)(idx % (p.N / 4)) * 4;
  float4 v = *reinterpret_cast<const float4*>(p.ws + (int64_t)row * p.N + col);
  for (int s = 1; s < nsplit; ++s) {
    const float4 w = *reinterpret_cast<const float4*>(p.ws + ((int64_t)s * p.M + row) * p.N + col);
    v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
  }
  if (p.rowscale) {
    float ss = 0.f;
    for (int s = 0; s < nsplit; ++s) ss += p.ws_ss[(int64_t)s * p.M + row];
    const float den = sqrtf(ss) * p.inv_sqrt_k + kRmsEps;
    v.x /= den; v.y /= den; v.z /= den; v.w /= den;
  }
  if (p.bias) {
    v.x += p.bias[col]; v.y += p.bias[col + 1]; v.z += p.bias[col + 2]; v.w += p.bias[col + 3];
  }
  float* dst = p.C + (int64_t)row * p.ldc + col;
  if constexpr (EPI == EPI_RESID) {
    const float* r = p.R + (int64_t)row * p.ldr + col;
    v.x = r[0] + p.alpha * v.x; v.y = r[1] + p.alpha * v.y; v.z = r[2] + p.alpha * v.z; v.w = r[3] + p.alpha * v.w;
  }
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
}

// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool BF16>
static hipError_t launch_cfg(const GemmArgs& a, int epi, int nsplit, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
  const dim3 block(WM * WN * 64);
  if (nsplit > 1) {
    GemmArgs b = a;
    b.k_split = a.K / nsplit;
    const dim3 grid(tiles, nsplit);
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_STORE, BF16, true>), grid, block, 0, st, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t n4 = (int64_t)a.M * (a.N / 4);
    const dim3 g2((unsigned)((n4 + 255) / 256));
    if (epi == EPI_RESID) hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_RESID>, g2, dim3(256), 0, st, b, nsplit);
    else hipLaunchKernelGGL(splitk_epilogue_kernel<EPI_STORE>, g2, dim3(256), 0, st, b, nsplit);
    return hipGetLastError();
  }
  const dim3 grid(tiles);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_STORE, BF16, false>), grid, block, 0, st, a); break;
    case EPI_RESID: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_RESID, BF16, false>), grid, block, 0, st, a); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_SWIGLU, BF16, false>), grid, block, 0, st, a); break;
    case EPI_GLU: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_GLU, BF16, false>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t conv2_gemm(const float* x2, const void* w, const float* scale, const float* shift, float* flat, int B,
                      bool bf16, hipStream_t st) {
  GemmArgs a{};
  a.A = x2;
  a.W = w;
  a.C = flat;
  a.bias = shift;
  a.scale = scale;
  a.M = B * kT * kSub2F;
  a.N = kSub2C;
  a.K = kSub2Kt * kSub2Kf * kSub1C;
  const dim3 grid((a.M + 127) / 128), block(256);
  if (bf16) hipLaunchKernelGGL((gemm_kernel<128, 64, 4, 1, EPI_CONV2, true, false>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((gemm_kernel<128, 64, 4, 1, EPI_CONV2, false, false>), grid, block, 0, st, a);
  return hipGetLastError();
}

hipError_t gemm(const GemmArgs& a, int epi, bool bf16, hipStream_t st) {
  if (a.K % 32 != 0 || a.N % 128 != 0 || a.M <= 0) return hipErrorInvalidValue;
  constexpr int kTarget = 512;     // >= 2 tiles per CU on 256 CUs
  const int64_t t128 = (int64_t)((a.M + 127) / 128) * (a.N / 128);
  const int64_t t64 = (int64_t)((a.M + 63) / 64) * (a.N / 128);
  if (t128 >= kTarget) return bf16 ? launch_cfg<128, 128, 2, 2, true>(a, epi, 1, st) : launch_cfg<128, 128, 2, 2, false>(a, epi, 1, st);
  int nsplit = 1;
  if ((epi == EPI_STORE || epi == EPI_RESID) && a.ws && t64 < kTarget) {
    // smallest split of the K-steps that reaches the target, keeping >= 3 K-steps per split
    const int ksteps = a.K / 32;
    for (int s = 2; s <= 16; ++s) {
      if (ksteps % s || ksteps / s < 3) continue;
      if ((int64_t)s * a.M * a.N > a.ws_cap) break;
      nsplit = s;
      if (t64 * s >= kTarget) break;
    }
  }
  if (nsplit > 1 || t64 >= kTarget / 2)
    return bf16 ? launch_cfg<64, 128, 2, 2, true>(a, epi, nsplit, st) : launch_cfg<64, 128, 2, 2, false>(a, epi, nsplit, st);
  return bf16 ? launch_cfg<32, 128, 1, 2, true>(a, epi, 1, st) : launch_cfg<32, 128, 1, 2, false>(a, epi, 1, st);
}

}  // namespace tone
