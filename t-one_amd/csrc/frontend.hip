// Front end of one streaming step: PCM -> log-mel (a1/a2) and the Conv2d subsampling (a3).
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace tone {

// ---------------------------------------------------------------------------------------------
// a1.  Tone.forward_for_export raw branch (tone/nn/model.py:164-165) and the streaming concat of
// FilterbankFeatures.forward_streaming (tone/nn/modules/feats.py:128-133):
//   wav = fp16(pcm / 32767); x = [state(80) ; wav] (2480 samples); next state = x[-80:]
// x is stored as fp32 values for the spectrum GEMM (mel_gemms, gemm.hip).  Also writes
// mhsa_len' = min(mhsa_len + 10, 30) (EncoderState.next, conformer_blocks.py:191).
__global__ void __launch_bounds__(256) mel_prep_kernel(const int32_t* __restrict__ pcm, StateRef s,
                                                       float* __restrict__ wave, int B) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)B * kWave) return;
  const int b = (int)(idx / kWave), i = (int)(idx % kWave);
  const int64_t srow = s.row(b);
  __half hv;
  if (i < kPreState) hv = s.in[srow + kOffPre + i];
  else hv = __float2half_rn((float)pcm[(int64_t)b * kChunk + (i - kPreState)] / 32767.0f);
  wave[idx] = __half2float(hv);
  if (i >= kChunk) s.out[srow + kOffPre + (i - kChunk)] = hv;
  if (i == 0) {
    const float ml = __half2float(s.in[srow + kOffMhsaLen]);
    s.out[srow + kOffMhsaLen] = __float2half_rn(fminf(ml + (float)kT, (float)kMhsaS));
  }
}

hipError_t launch_mel_prep(const int32_t* pcm, StateRef s, float* wave, int B, hipStream_t st) {
  const int64_t n = (int64_t)B * kWave;
  hipLaunchKernelGGL(mel_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pcm, s, wave, B);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// a3 part 1.  ConvSubsamplingPreEncode.forward (conformer_blocks.py:631-641), first conv:
//   xn = RMSNorm_64(feats); x1 = [sub1 state (10 rows) ; xn] (40 x 64); next sub1 = x1[-10:]
//   c1[c][t][f] = SiLU(BN(bias + sum_{kt<11,kf<21} w[c][kt][kf] x1[t+kt][f+kf])), t<30, f<44
//   x2 = [sub2 state (8 rows) ; c1] written channels-last [38][44][32] for the conv2 implicit GEMM;
//   next sub2 = c1[:, 22:30, :].
// One workgroup per stream.  The conv is an implicit GEMM on the MFMA (fp32, or bf16 in bf16 mode):
// M = 1320 positions (32-row tiles per wave), N = 32 channels, K = 231 taps padded to 256, A gathered
// from x1 in LDS.
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int kK1 = kSub1Kt * kSub1Kf;      // 231
constexpr int kK1P = 256;                   // padded K
constexpr int kPos1 = kMelT * kSub1F;       // 1320

template <bool OBF>   // x2 stored as bf16 bits (bf16 mode) or fp32
__global__ void __launch_bounds__(256) sub1_kernel(const float* __restrict__ feats, StateRef s,
                                                   const float* __restrict__ pre_norm_w, const float* __restrict__ w1,
                                                   const float* __restrict__ scale1, const float* __restrict__ shift1,
                                                   void* __restrict__ x2) {
  using XT = typename std::conditional<OBF, __bf16, float>::type;
  __shared__ float x1[(kSub1S + kMelT) * kMels];
  __shared__ float wk[kSub1C][kK1P + 1];
  __shared__ int koff[kK1P];
  __shared__ float sc[kSub1C], sh[kSub1C];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t srow = s.row(b);
  for (int i = tid; i < kSub1C * kK1P; i += 256) {
    const int c = i / kK1P, k = i % kK1P;
    wk[c][k] = k < kK1 ? w1[c * kK1 + k] : 0.f;
  }
  for (int k = tid; k < kK1P; k += 256) koff[k] = k < kK1 ? (k / kSub1Kf) * kMels + k % kSub1Kf : 0;
  if (tid < kSub1C) { sc[tid] = scale1[tid]; sh[tid] = shift1[tid]; }
  for (int i = tid; i < kSub1S * kMels; i += 256) x1[i] = __half2float(s.in[srow + kOffSub1 + i]);
  // RMSNorm over 64 features: one wave per frame, one lane per feature
  for (int t = wid; t < kMelT; t += 4) {
    const float v = feats[((int64_t)b * kMelT + t) * kMels + lane];
    const float ssq = wave_sum(v * v);
    const float rms = sqrtf(ssq) * 0.125f;          // * 64^-0.5
    const float y = pre_norm_w[lane] * (v / (rms + kRmsEps));
    x1[(kSub1S + t) * kMels + lane] = y;
    if (t >= kMelT - kSub1S) s.out[srow + kOffSub1 + (t - (kMelT - kSub1S)) * kMels + lane] = __float2half_rn(y);
  }
  // carried conv2 input rows -> x2 rows 0..7 (channels-last)
  XT* xb = static_cast<XT*>(x2) + (int64_t)b * kSub2In * kSub1F * kSub1C;
  for (int i = tid; i < kSub1C * kSub2S * kSub1F; i += 256) {
    const int c = i / (kSub2S * kSub1F), r = (i / kSub1F) % kSub2S, f = i % kSub1F;
    xb[(r * kSub1F + f) * kSub1C + c] = (XT)__half2float(s.in[srow + kOffSub2 + i]);
  }
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  for (int tile = wid; tile * 32 < kPos1; tile += 4) {
    const int pos = min(tile * 32 + li, kPos1 - 1);
    const int base = (pos / kSub1F) * kMels + pos % kSub1F;
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (OBF) {
      // bf16 mode: v_mfma_f32_32x32x16_bf16, lane (i, h) holds A[pos_i][16s + 8h + e] (gathered)
#pragma unroll 4
      for (int st = 0; st < kK1P / 16; ++st) {
        bf16x8_t av, bv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = 16 * st + 8 * lh + e;
          av[e] = (__bf16)x1[base + koff[k]];
          bv[e] = (__bf16)wk[li][k];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      }
    } else {
#pragma unroll 8
      for (int st = 0; st < kK1P / 2; ++st) {
        const int k = 2 * st + lh;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[base + koff[k]], wk[li][k], acc, 0, 0, 0);
      }
    }
    const int c = li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (p >= kPos1) continue;
      const int t = p / kSub1F, f = p % kSub1F;
      const float y = silu_f(fmaf(acc[r], sc[c], sh[c]));
      xb[((kSub2S + t) * kSub1F + f) * kSub1C + c] = (XT)y;
      if (t >= kMelT - kSub2S)
        s.out[srow + kOffSub2 + (c * kSub2S + (t - (kMelT - kSub2S))) * kSub1F + f] = __float2half_rn(y);
    }
  }
}

hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const float* scale1,
                       const float* shift1, void* x2, bool x2_bf16, int B, hipStream_t st) {
  if (x2_bf16) hipLaunchKernelGGL(sub1_kernel<true>, dim3(B), dim3(256), 0, st, feats, s, pre_norm_w, w1, scale1, shift1, x2);
  else hipLaunchKernelGGL(sub1_kernel<false>, dim3(B), dim3(256), 0, st, feats, s, pre_norm_w, w1, scale1, shift1, x2);
  return hipGetLastError();
}

}  // namespace tone
