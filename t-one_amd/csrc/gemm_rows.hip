// Full-row bf16 GEMM for the encoder's N = 384 residual projections (FFN down K = 1536, attention out and pw2
// K = 384): C = R + alpha (A W^T + bias), fp32 C plus its bf16 shadow C2, optionally followed by the RMSNorm of
// each output row (norm_out, conformer_blocks.py:836, submodules.py:34-54) in the same epilogue.
//
// Why: the 128 x 128 LDS-DMA tiles (gemm.hip) stream A three times (N / 128) and W once per 128 rows; a
// workgroup that owns whole 384-column rows reads A exactly once, and owning whole rows is also what lets the
// epilogue normalise them.  Layout (computed as D[n][m] = W[n][:] . X[m][:], like gemm_t / gemm_xs, so a lane holds
// 4 consecutive columns of one row for vector stores):
//   * a work tile = TM = 16 MB rows x all 384 columns; 8 waves, wave w owns columns [48 w, 48 w + 48) (three
//     16-column n-blocks) of all MB 16-row m-blocks: MB x 3 x 4 fp32 accumulators per lane;
//   * K goes in 32-wide stages through a 4-slot LDS ring by global_load_lds_dwordx4 (stage = TM + 384 rows of
//     64 bytes), stage s + 3 issued right after the barrier of stage s (its slot held stage s - 1, which every wave
//     finished before that barrier); 16-byte chunk c of row r sits at slot c ^ ((r >> 1) & 3), which makes the
//     16x16x32 fragment reads (lane: row l & 15, chunk l >> 4) conflict-free;
//   * per stage a wave reads its 3 W fragments once and streams the MB X fragments: 3 + MB ds_read_b128 per
//     3 MB MFMAs.
// TM is chosen per M so the tiles fill the 256 CUs in whole rounds (gemm_rows_mb below).
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

namespace tone {
namespace {

constexpr int kRwN = 384;              // output columns (d_model)
constexpr int kRwWaves = 8;
constexpr int kRwR = 4;                // ring slots
constexpr int kRwMaxMB = 8;            // TM <= 128 (MB = 10 spills)
constexpr int kRowsMinM = 10240;       // routed from here up (profiles/r03_rows_sweep.jsonl)
constexpr float kRwInvSqrtD = 0.05103103630798288f;   // 384^-0.5, as rmsnorm_kernel (encoder.hip)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int MB, bool NORM>
__global__ void __launch_bounds__(kRwWaves * 64) gemm_rows_kernel(GemmArgs p, const float* __restrict__ norm_w) {
  constexpr int TM = 16 * MB;
  constexpr int kA = TM * 64, kW = kRwN * 64, kStage = kA + kW;   // bytes per stage
  constexpr int kPa = kA / 1024, kP = kPa + kW / 1024;            // 1 KiB DMA pieces per stage
  constexpr int kPi = (kP + kRwWaves - 1) / kRwWaves;             // piece slots per wave
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRwR * kStage];
  __shared__ float red[NORM ? kRwWaves * TM : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lg = lane >> 4;
  const int nk = p.K / 32, ntiles = (p.M + TM - 1) / TM;
  const int npw = (kP - wid + kRwWaves - 1) / kRwWaves;           // pieces this wave issues per stage
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);

  // DMA lane geometry: lane i of a 1 KiB piece covers row 16 piece + (i >> 2), LDS slot i & 3, and fetches chunk
  // (i & 3) ^ ((row >> 1) & 3) = (i & 3) ^ ((i >> 3) & 3) of that row (the piece's row base is a multiple of 16)
  const uint32_t ch_lane = 16u * ((lane & 3) ^ ((lane >> 3) & 3));                  // bytes
  const uint32_t a_lane = (uint32_t)(lane >> 2) * (uint32_t)p.lda * 2u + ch_lane;
  const uint32_t w_lane = (uint32_t)(lane >> 2) * (uint32_t)p.K * 2u + ch_lane;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int m0 = tile * TM;
    // stage s (K columns 32 s ..) into slot s % R: piece pc = wid + 8 i (A rows, then W rows, 16 per piece)
    auto dma = [&](int s) {
      uint8_t* base = lds + (s % kRwR) * kStage;
      const int k0 = 32 * s;
#pragma unroll
      for (int i = 0; i < kPi; ++i) {
        const int pc = wid + kRwWaves * i;
        if (pc < kP) {                                            // wave-uniform
          // a uniform (scalar) row base plus the lane's 32-bit byte offset: the saddr form of the load
          const char* src;
          if (pc < kPa) {
            const int row0 = m0 + 16 * pc;                        // rows past M re-read row M - 1
            if (row0 + 15 < p.M) {
              src = reinterpret_cast<const char*>(A + ((int64_t)row0 * p.lda + k0)) + a_lane;
            } else {
              const int row = min(row0 + (lane >> 2), p.M - 1);
              src = reinterpret_cast<const char*>(A + ((int64_t)row * p.lda + k0)) + ch_lane;
            }
          } else {
            src = reinterpret_cast<const char*>(W + ((int64_t)(16 * (pc - kPa)) * p.K + k0)) + w_lane;
          }
#if defined(__HIP_DEVICE_COMPILE__)
          __builtin_amdgcn_global_load_lds(src, base + pc * 1024, 16, 0, 0);
#else
          (void)src;
          (void)base;
#endif
        }
      }
    };
    dma(0);
    if (nk > 1) dma(1);
    if (nk > 2) dma(2);

    f32x4_t acc[MB][3];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) acc[mb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < nk; ++s) {
      // stage s landed: this wave's younger DMA ops are stages s + 1, s + 2 (the loads the epilogue of the
      // previous tile issued are older and so covered as well)
      vmcnt_dyn(min(2, nk - 1 - s) * npw);
      barrier_lds();                                              // ... for every wave; slot (s - 1) % R free
      if (s + 3 < nk) dma(s + 3);
      const uint8_t* base = lds + (s % kRwR) * kStage;
      bf16x8_t wf[3];
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) {
        const int row = 48 * wid + 16 * nb + l15;
        wf[nb] = *reinterpret_cast<const bf16x8_t*>(base + kA + row * 64 + ((lg ^ ((row >> 1) & 3)) << 4));
      }
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int row = 16 * mb + l15;
        const bf16x8_t xf = *reinterpret_cast<const bf16x8_t*>(base + row * 64 + ((lg ^ ((row >> 1) & 3)) << 4));
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nb], xf, acc[mb][nb], 0, 0, 0);
        if (MB > 6 && mb == MB / 2 - 1) __builtin_amdgcn_sched_barrier(0);   // X reads in two halves (registers)
      }
    }

    // epilogue: y = R + alpha (acc + bias) for rows m0 + 16 mb + l15, columns 48 w + 16 nb + 4 lg ..
    float* __restrict__ C = static_cast<float*>(p.C);
    f32x4_t bl[3];                                                // the lane's 12 columns' bias (L2-resident)
#pragma unroll
    for (int nb = 0; nb < 3; ++nb)
      bl[nb] = p.bias ? *reinterpret_cast<const f32x4_t*>(p.bias + 48 * wid + 16 * nb + 4 * lg) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    float ss[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int64_t row = min(m0 + 16 * mb + l15, p.M - 1);
      f32x4_t rr[3];
#pragma unroll
      for (int nb = 0; nb < 3; ++nb)
        rr[nb] = *reinterpret_cast<const f32x4_t*>(p.R + row * p.ldr + 48 * wid + 16 * nb + 4 * lg);
      ss[mb] = 0.f;
#pragma unroll
      for (int nb = 0; nb < 3; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = rr[nb][r] + p.alpha * (acc[mb][nb][r] + bl[nb][r]);
          acc[mb][nb][r] = y;
          if constexpr (NORM) ss[mb] = fmaf(y, y, ss[mb]);
        }
      __builtin_amdgcn_sched_barrier(0);                          // R loads one m-block at a time (registers)
    }
    if constexpr (NORM) {
      // row sums of squares: the lane's 12 columns, then the 4 lanes of the row (lg), then the 8 waves (LDS)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        ss[mb] += __shfl_xor(ss[mb], 16, 64);
        ss[mb] += __shfl_xor(ss[mb], 32, 64);
        if (lg == 0) red[wid * TM + 16 * mb + l15] = ss[mb];
      }
      __syncthreads();
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kRwWaves; ++w) t += red[w * TM + 16 * mb + l15];
        const float inv = 1.0f / (sqrtf(t) * kRwInvSqrtD + kRmsEps);   // one division per row, not per element
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) {
          const f32x4_t nw = *reinterpret_cast<const f32x4_t*>(norm_w + 48 * wid + 16 * nb + 4 * lg);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mb][nb][r] = nw[r] * (acc[mb][nb][r] * inv);
        }
      }
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int row = m0 + 16 * mb + l15;
      if (row < p.M) {
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) {
          const int col = 48 * wid + 16 * nb + 4 * lg;
          *reinterpret_cast<f32x4_t*>(C + (int64_t)row * p.ldc + col) = acc[mb][nb];
          if (p.C2) {
            const uint2 h = make_uint2(pk2(acc[mb][nb][0], acc[mb][nb][1]), pk2(acc[mb][nb][2], acc[mb][nb][3]));
            *reinterpret_cast<uint2*>(p.C2 + (int64_t)row * p.ldc + col) = h;
          }
        }
      }
    }
    __syncthreads();                                              // the ring (and red) are reused by the next tile
  }
}

template <bool NORM>
hipError_t launch_rows(const GemmArgs& a, const float* norm_w, int mb, hipStream_t st) {
  const int ntiles = (a.M + 16 * mb - 1) / (16 * mb);
  const dim3 grid(std::min(ntiles, 256)), block(kRwWaves * 64);
  switch (mb) {
#define TONE_RW(k) case k: hipLaunchKernelGGL((gemm_rows_kernel<k, NORM>), grid, block, 0, st, a, norm_w); break;
    TONE_RW(1) TONE_RW(2) TONE_RW(3) TONE_RW(4) TONE_RW(5) TONE_RW(6) TONE_RW(8)
#undef TONE_RW
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

// m-blocks per tile: the MB in {1..6, 8} minimising rounds x (MB + 2) over 256 CUs (2 m-blocks being the
// per-tile prologue / epilogue cost); ties to the larger MB (fewer W passes)
int gemm_rows_mb(int M) {
  static const int kMbs[] = {8, 6, 5, 4, 3, 2, 1};
  int best = 1;
  int64_t best_cost = INT64_MAX;
  for (int mb : kMbs) {
    const int64_t tiles = (M + 16 * mb - 1) / (16 * mb), rounds = (tiles + 255) / 256;
    const int64_t cost = rounds * (mb + 2);
    if (cost < best_cost) { best_cost = cost; best = mb; }
  }
  return best;
}

bool gemm_rows_route(int M, int K) {
  (void)K;
  return M >= kRowsMinM;
}

hipError_t gemm_rows(const GemmArgs& a, const float* norm_w, int mb, hipStream_t st) {
  if (!a.a_bf16 || a.c_bf16 || a.N != kRwN || a.K % 32 || a.K < 32 || a.M <= 0 || !a.R || a.lda % 8 || a.ldc % 4 ||
      a.ldr % 4 || a.rowscale || a.k_split || a.rpg || a.W3 || a.a_plane || a.c_plane || a.c2_plane)
    return hipErrorInvalidValue;
  if (mb <= 0) mb = gemm_rows_mb(a.M);
  if (mb > kRwMaxMB) return hipErrorInvalidValue;
  return norm_w ? launch_rows<true>(a, norm_w, mb, st) : launch_rows<false>(a, norm_w, mb, st);
}

}  // namespace tone
