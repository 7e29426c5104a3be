// Front end of one streaming step: PCM -> log-mel (a1/a2) and the Conv2d subsampling (a3).
#include "common.h"
#include "kernels.h"

namespace tone {

// ---------------------------------------------------------------------------------------------
// a1/a2.  Tone.forward_for_export raw branch (tone/nn/model.py:164-169) and
// FilterbankFeatures.forward_streaming/_forward (tone/nn/modules/feats.py:95-102,118-133):
//   wav = fp16(pcm / 32767); x = [state(80) ; wav] (2480); next state = x[-80:]
//   spec[t][r] = sum_k basis[r][k] * x[80t + k]      (162 x 160 basis: DFT * Hann * pre-emphasis)
//   power = re^2 + im^2 (81 bins); mel = fbank(64x81) . power; feats = fp16(log(mel + 2^-24))
// One workgroup per stream; the 2480 samples and the 30x162 spectrum stay in LDS.
// Also writes mhsa_len' = min(mhsa_len + 10, 30) (EncoderState.next, conformer_blocks.py:191).
__global__ void __launch_bounds__(256) mel_kernel(const int32_t* __restrict__ pcm, StateRef s,
                                                  const float* __restrict__ basis, const float* __restrict__ fbank,
                                                  float* __restrict__ feats) {
  __shared__ __attribute__((aligned(16))) float x[kWave];
  __shared__ float spec[kMelT][kBasisRows + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t srow = s.row(b);
  for (int i = tid; i < kWave; i += 256) {
    __half hv;
    if (i < kPreState) hv = s.in[srow + kOffPre + i];
    else hv = __float2half_rn((float)pcm[(int64_t)b * kChunk + (i - kPreState)] / 32767.0f);
    x[i] = __half2float(hv);
    if (i >= kChunk) s.out[srow + kOffPre + (i - kChunk)] = hv;
  }
  if (tid == 0) {
    const float ml = __half2float(s.in[srow + kOffMhsaLen]);
    s.out[srow + kOffMhsaLen] = __float2half_rn(fminf(ml + (float)kT, (float)kMhsaS));
  }
  __syncthreads();
  for (int p = tid; p < kMelT * kBasisRows; p += 256) {
    const int t = p / kBasisRows, r = p % kBasisRows;
    const float4* bw = reinterpret_cast<const float4*>(basis + r * kWin);
    const float4* xw = reinterpret_cast<const float4*>(x + t * kHop);
    float acc = 0.f;
#pragma unroll 8
    for (int k = 0; k < kWin / 4; ++k) {
      const float4 w = bw[k], v = xw[k];
      acc = fmaf(w.x, v.x, acc);
      acc = fmaf(w.y, v.y, acc);
      acc = fmaf(w.z, v.z, acc);
      acc = fmaf(w.w, v.w, acc);
    }
    spec[t][r] = acc;
  }
  __syncthreads();
  for (int p = tid; p < kMelT * kMels; p += 256) {
    const int t = p / kMels, m = p % kMels;
    float acc = 0.f;
    for (int f = 0; f < kBins; ++f) {
      const float re = spec[t][f], im = spec[t][kBins + f];
      acc = fmaf(fbank[m * kBins + f], re * re + im * im, acc);
    }
    feats[((int64_t)b * kMelT + t) * kMels + m] = round_h(logf(acc + 5.9604644775390625e-08f));
  }
}

hipError_t launch_mel(const int32_t* pcm, StateRef s, const float* basis, const float* fbank, float* feats, int B,
                      hipStream_t st) {
  hipLaunchKernelGGL(mel_kernel, dim3(B), dim3(256), 0, st, pcm, s, basis, fbank, feats);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// a3 part 1.  ConvSubsamplingPreEncode.forward (conformer_blocks.py:631-641), first conv:
//   xn = RMSNorm_64(feats); x1 = [sub1 state (10 rows) ; xn] (40 x 64); next sub1 = x1[-10:]
//   c1[c][t][f] = SiLU(BN(bias + sum_{kt<11,kf<21} w[c][kt][kf] x1[t+kt][f+kf])), t<30, f<44
//   x2 = [sub2 state (8 rows) ; c1] written channels-last [38][44][32] for the conv2 implicit GEMM;
//   next sub2 = c1[:, 22:30, :].
// One workgroup per stream.  The conv is an implicit GEMM on the fp32 MFMA: M = 1320 positions
// (32-row tiles per wave), N = 32 channels, K = 231 taps padded to 256, A gathered from x1 in LDS.
typedef float f32x16_t __attribute__((ext_vector_type(16)));
constexpr int kK1 = kSub1Kt * kSub1Kf;      // 231
constexpr int kK1P = 256;                   // padded K
constexpr int kPos1 = kMelT * kSub1F;       // 1320

__global__ void __launch_bounds__(256) sub1_kernel(const float* __restrict__ feats, StateRef s,
                                                   const float* __restrict__ pre_norm_w, const float* __restrict__ w1,
                                                   const float* __restrict__ scale1, const float* __restrict__ shift1,
                                                   float* __restrict__ x2) {
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
  float* xb = x2 + (int64_t)b * kSub2In * kSub1F * kSub1C;
  for (int i = tid; i < kSub1C * kSub2S * kSub1F; i += 256) {
    const int c = i / (kSub2S * kSub1F), r = (i / kSub1F) % kSub2S, f = i % kSub1F;
    xb[(r * kSub1F + f) * kSub1C + c] = __half2float(s.in[srow + kOffSub2 + i]);
  }
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  for (int tile = wid; tile * 32 < kPos1; tile += 4) {
    const int pos = min(tile * 32 + li, kPos1 - 1);
    const int base = (pos / kSub1F) * kMels + pos % kSub1F;
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 8
    for (int st = 0; st < kK1P / 2; ++st) {
      const int k = 2 * st + lh;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[base + koff[k]], wk[li][k], acc, 0, 0, 0);
    }
    const int c = li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (p >= kPos1) continue;
      const int t = p / kSub1F, f = p % kSub1F;
      const float y = silu_f(fmaf(acc[r], sc[c], sh[c]));
      xb[((kSub2S + t) * kSub1F + f) * kSub1C + c] = y;
      if (t >= kMelT - kSub2S)
        s.out[srow + kOffSub2 + (c * kSub2S + (t - (kMelT - kSub2S))) * kSub1F + f] = __float2half_rn(y);
    }
  }
}

hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const float* scale1,
                       const float* shift1, float* x2, int B, hipStream_t st) {
  hipLaunchKernelGGL(sub1_kernel, dim3(B), dim3(256), 0, st, feats, s, pre_norm_w, w1, scale1, shift1, x2);
  return hipGetLastError();
}

}  // namespace tone
