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
//   next sub2 = c1[:, 22:30, :] (the last 8 rows of [sub2 ; c1])
// One workgroup per stream; each thread owns (t, f) positions and all 32 channels.
__global__ void __launch_bounds__(256) sub1_kernel(const float* __restrict__ feats, StateRef s,
                                                   const float* __restrict__ pre_norm_w, const float* __restrict__ w1t,
                                                   const float* __restrict__ scale1, const float* __restrict__ shift1,
                                                   float* __restrict__ c1) {
  constexpr int KT = kSub1Kt * kSub1Kf;  // 231
  __shared__ float xn[kSub1S + kMelT][kMels];
  __shared__ __attribute__((aligned(16))) float wt[KT][kSub1C];
  __shared__ float sc[kSub1C], sh[kSub1C];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t srow = s.row(b);
  for (int i = tid; i < KT * kSub1C; i += 256) (&wt[0][0])[i] = w1t[i];
  if (tid < kSub1C) { sc[tid] = scale1[tid]; sh[tid] = shift1[tid]; }
  for (int i = tid; i < kSub1S * kMels; i += 256) xn[i / kMels][i % kMels] = __half2float(s.in[srow + kOffSub1 + i]);
  // RMSNorm over 64 features: one wave per frame, one lane per feature
  for (int t = wid; t < kMelT; t += 4) {
    const float v = feats[((int64_t)b * kMelT + t) * kMels + lane];
    const float ssq = wave_sum(v * v);
    const float rms = sqrtf(ssq) * 0.125f;          // * 64^-0.5
    const float y = pre_norm_w[lane] * (v / (rms + kRmsEps));
    xn[kSub1S + t][lane] = y;
    if (t >= kMelT - kSub1S) s.out[srow + kOffSub1 + (t - (kMelT - kSub1S)) * kMels + lane] = __float2half_rn(y);
  }
  __syncthreads();
  for (int pos = tid; pos < kMelT * kSub1F; pos += 256) {
    const int t = pos / kSub1F, f = pos % kSub1F;
    float acc[kSub1C];
#pragma unroll
    for (int c = 0; c < kSub1C; ++c) acc[c] = 0.f;
    for (int kt = 0; kt < kSub1Kt; ++kt) {
      for (int kf = 0; kf < kSub1Kf; ++kf) {
        const float xv = xn[t + kt][f + kf];
        const float4* w4 = reinterpret_cast<const float4*>(&wt[kt * kSub1Kf + kf][0]);
#pragma unroll
        for (int c4 = 0; c4 < kSub1C / 4; ++c4) {
          const float4 w = w4[c4];
          acc[c4 * 4 + 0] = fmaf(w.x, xv, acc[c4 * 4 + 0]);
          acc[c4 * 4 + 1] = fmaf(w.y, xv, acc[c4 * 4 + 1]);
          acc[c4 * 4 + 2] = fmaf(w.z, xv, acc[c4 * 4 + 2]);
          acc[c4 * 4 + 3] = fmaf(w.w, xv, acc[c4 * 4 + 3]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < kSub1C; ++c) {
      const float y = silu_f(fmaf(acc[c], sc[c], sh[c]));
      c1[(((int64_t)b * kSub1C + c) * kMelT + t) * kSub1F + f] = y;
      if (t >= kMelT - kSub2S)
        s.out[srow + kOffSub2 + (c * kSub2S + (t - (kMelT - kSub2S))) * kSub1F + f] = __float2half_rn(y);
    }
  }
}

hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1t, const float* scale1,
                       const float* shift1, float* c1, int B, hipStream_t st) {
  hipLaunchKernelGGL(sub1_kernel, dim3(B), dim3(256), 0, st, feats, s, pre_norm_w, w1t, scale1, shift1, c1);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// a3 part 2.  Second conv (conformer_blocks.py:637-641) and the flatten feeding `out`
// (conformer_blocks.py:649):
//   x2 = [sub2 state (8 rows) ; c1 (30 rows)] per input channel (38 x 44)
//   y[c][t][f] = SiLU(BN(bias + sum_{ci<32,kt<11,kf<11} w[c][ci][kt][kf] x2[ci][3t+kt][f+kf])), t<10, f<34
//   flat[b][t][c*34 + f] = y[c][t][f]
// Workgroup = (stream, group of 16 output channels); thread = one of the 340 (t, f) positions.
constexpr int kS2G = 16;   // output channels per workgroup
constexpr int kS2CI = 8;   // input channels staged per LDS pass
__global__ void __launch_bounds__(384) sub2_kernel(const float* __restrict__ c1, StateRef s, const float* __restrict__ w2,
                                                   const float* __restrict__ scale2, const float* __restrict__ shift2,
                                                   float* __restrict__ flat) {
  constexpr int KK = kSub2Kt * kSub2Kf;  // 121
  __shared__ float xin[kS2CI][kSub2In][kSub1F];
  __shared__ __attribute__((aligned(16))) float wt[kS2CI][KK][kS2G];
  const int b = blockIdx.x / (kSub2C / kS2G), cg = blockIdx.x % (kSub2C / kS2G), tid = threadIdx.x;
  const int64_t srow = s.row(b);
  const bool active = tid < kT * kSub2F;
  const int t = tid / kSub2F, f = tid % kSub2F;
  float acc[kS2G];
#pragma unroll
  for (int c = 0; c < kS2G; ++c) acc[c] = 0.f;
  for (int ci0 = 0; ci0 < kSub1C; ci0 += kS2CI) {
    __syncthreads();
    for (int i = tid; i < kS2CI * kSub2In * kSub1F; i += 384) {
      const int ci = i / (kSub2In * kSub1F), r = (i / kSub1F) % kSub2In, ff = i % kSub1F;
      float v;
      if (r < kSub2S) v = __half2float(s.in[srow + kOffSub2 + ((ci0 + ci) * kSub2S + r) * kSub1F + ff]);
      else v = c1[(((int64_t)b * kSub1C + ci0 + ci) * kMelT + (r - kSub2S)) * kSub1F + ff];
      xin[ci][r][ff] = v;
    }
    for (int i = tid; i < kS2CI * KK * kS2G; i += 384) {
      const int ci = i / (KK * kS2G), kk = (i / kS2G) % KK, c = i % kS2G;
      wt[ci][kk][c] = w2[((int64_t)(cg * kS2G + c) * kSub1C + ci0 + ci) * KK + kk];
    }
    __syncthreads();
    if (active) {
      for (int ci = 0; ci < kS2CI; ++ci) {
        for (int kt = 0; kt < kSub2Kt; ++kt) {
#pragma unroll
          for (int kf = 0; kf < kSub2Kf; ++kf) {
            const float xv = xin[ci][kSub2Stride * t + kt][f + kf];
            const float4* w4 = reinterpret_cast<const float4*>(&wt[ci][kt * kSub2Kf + kf][0]);
#pragma unroll
            for (int c4 = 0; c4 < kS2G / 4; ++c4) {
              const float4 w = w4[c4];
              acc[c4 * 4 + 0] = fmaf(w.x, xv, acc[c4 * 4 + 0]);
              acc[c4 * 4 + 1] = fmaf(w.y, xv, acc[c4 * 4 + 1]);
              acc[c4 * 4 + 2] = fmaf(w.z, xv, acc[c4 * 4 + 2]);
              acc[c4 * 4 + 3] = fmaf(w.w, xv, acc[c4 * 4 + 3]);
            }
          }
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int c = 0; c < kS2G; ++c) {
      const int co = cg * kS2G + c;
      flat[((int64_t)b * kT + t) * kSubOut + co * kSub2F + f] = silu_f(fmaf(acc[c], scale2[co], shift2[co]));
    }
  }
}

hipError_t launch_sub2(const float* c1, StateRef s, const float* w2, const float* scale2, const float* shift2,
                       float* flat, int B, hipStream_t st) {
  hipLaunchKernelGGL(sub2_kernel, dim3(B * (kSub2C / kS2G)), dim3(384), 0, st, c1, s, w2, scale2, shift2, flat);
  return hipGetLastError();
}

}  // namespace tone
