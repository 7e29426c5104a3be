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
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace tone {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  __bf16 ha = (__bf16)a, hb = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

template <int BM, int BN, int WM, int WN, int EPI, bool BF16>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(GemmArgs p) {
  constexpr int NT = WM * WN * 64;
  constexpr int BK = 32;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  static_assert(EPI < EPI_SWIGLU || (TN % 2 == 0), "gated epilogues pair n-tiles");
  constexpr int LDS_ROW = BF16 ? (BK + 8) : (BK + 4);  // elements; keeps ds_read_b128 conflict-free
  using ST = typename std::conditional<BF16, uint16_t, float>::type;
  constexpr int A_V = BM * BK / 4 / NT;                 // float4 of A per thread per k-tile
  constexpr int W_VE = BF16 ? 8 : 4;                    // W elements per 16-byte vector
  constexpr int W_V = BN * BK / W_VE / NT;              // 16-byte W vectors per thread
  static_assert(A_V >= 1 && W_V >= 1, "tile too small for the thread count");

  __shared__ __attribute__((aligned(16))) ST As[BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) ST Bs[BN * LDS_ROW];
  __shared__ float rden[BM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = p.N / BN;
  const int bm = blockIdx.x / ntn, bn = blockIdx.x % ntn;
  const int m0 = bm * BM, n0 = bn * BN;
  const float* __restrict__ A = p.A;

  float4 ra[A_V];
  uint4 rw[W_V];
  float ss[A_V];
#pragma unroll
  for (int i = 0; i < A_V; ++i) ss[i] = 0.f;

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / 4), c = idx % (BK / 4);
      const int gm = m0 + r;
      ra[i] = gm < p.M ? *reinterpret_cast<const float4*>(A + (int64_t)gm * p.lda + k0 + c * 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / W_VE), c = idx % (BK / W_VE);
      const char* base = static_cast<const char*>(p.W) + ((int64_t)(n0 + r) * p.K + k0 + c * W_VE) * sizeof(ST);
      rw[i] = *reinterpret_cast<const uint4*>(base);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / 4), c = idx % (BK / 4);
      const float4 v = ra[i];
      if (p.rowscale) ss[i] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      if constexpr (BF16) {
        uint2 u;
        u.x = pack_bf16x2(v.x, v.y);
        u.y = pack_bf16x2(v.z, v.w);
        *reinterpret_cast<uint2*>(&As[r * LDS_ROW + c * 4]) = u;
      } else {
        *reinterpret_cast<float4*>(&As[r * LDS_ROW + c * 4]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < W_V; ++i) {
      const int idx = tid + i * NT, r = idx / (BK / W_VE), c = idx % (BK / W_VE);
      *reinterpret_cast<uint4*>(&Bs[r * LDS_ROW + c * W_VE]) = rw[i];
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
  load(0);
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    __syncthreads();
    store();
    __syncthreads();
    if (k0 + BK < p.K) load(k0 + BK);
    if constexpr (BF16) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 32 + lr) * LDS_ROW + ks * 16 + lh * 8]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 32 + lr) * LDS_ROW + ks * 16 + lh * 8]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // lane half h owns k in [16h, 16h+16) of the tile; both operands use the same k map
#pragma unroll
      for (int kq = 0; kq < BK / 8; ++kq) {
        float4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const float4*>(&As[(wm * WTM + i * 32 + lr) * LDS_ROW + lh * 16 + kq * 4]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const float4*>(&Bs[(wn * WTN + j * 32 + lr) * LDS_ROW + lh * 16 + kq * 4]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
      }
    }
  }

  if (p.rowscale) {
#pragma unroll
    for (int i = 0; i < A_V; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      const int idx = tid + i * NT, r = idx / (BK / 4);
      if ((idx % (BK / 4)) == 0) rden[r] = sqrtf(v) * p.inv_sqrt_k + kRmsEps;
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map of v_mfma_*_32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lrow = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int row = m0 + lrow;
      if (row >= p.M) continue;
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

// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool BF16>
static hipError_t launch_cfg(const GemmArgs& a, int epi, hipStream_t st) {
  const int blocks = ((a.M + BM - 1) / BM) * (a.N / BN);
  dim3 grid(blocks), block(WM * WN * 64);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_STORE, BF16>), grid, block, 0, st, a); break;
    case EPI_RESID: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_RESID, BF16>), grid, block, 0, st, a); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_SWIGLU, BF16>), grid, block, 0, st, a); break;
    case EPI_GLU: hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI_GLU, BF16>), grid, block, 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t gemm(const GemmArgs& a, int epi, bool bf16, hipStream_t st) {
  if (a.K % 32 != 0 || a.N % 128 != 0 || a.M <= 0) return hipErrorInvalidValue;
  // Tile choice: the largest tile that still gives >= ~2 blocks per CU (256 CUs).
  const int64_t big = (int64_t)((a.M + 127) / 128) * (a.N / 128);
  const int64_t mid = (int64_t)((a.M + 63) / 64) * (a.N / 128);
  if (big >= 512) return bf16 ? launch_cfg<128, 128, 2, 2, true>(a, epi, st) : launch_cfg<128, 128, 2, 2, false>(a, epi, st);
  if (mid >= 256) return bf16 ? launch_cfg<64, 128, 2, 2, true>(a, epi, st) : launch_cfg<64, 128, 2, 2, false>(a, epi, st);
  return bf16 ? launch_cfg<32, 128, 1, 2, true>(a, epi, st) : launch_cfg<32, 128, 1, 2, false>(a, epi, st);
}

}  // namespace tone
