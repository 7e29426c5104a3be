// Front end of one streaming step: PCM -> log-mel (a1/a2) and the Conv2d subsampling (a3).
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace tone {

__device__ __forceinline__ void barrier_lds_c2() {   // keeps LDS-DMA in flight (no vmcnt(0) fence)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// ---------------------------------------------------------------------------------------------
// a1.  Tone.forward_for_export raw branch (tone/nn/model.py:164-165) and the streaming concat of
// FilterbankFeatures.forward_streaming (tone/nn/modules/feats.py:128-133):
//   wav = fp16(pcm / 32767); x = [state(80) ; wav] (2480 samples); next state = x[-80:]
// x is stored as fp32 values for the spectrum GEMM (mel_gemms, gemm.hip).  Also writes
// mhsa_len' = min(mhsa_len + 10, 30) (EncoderState.next, conformer_blocks.py:191).
__global__ void __launch_bounds__(256) mel_prep_kernel(const int32_t* __restrict__ pcm, StateRef s,
                                                       float* __restrict__ wave, int B, int chunk, int T) {
  const int wv = chunk + kPreState;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)B * wv) return;
  const int b = (int)(idx / wv), i = (int)(idx % wv);
  const int64_t srow = s.row_in(b), orow = s.row_out(b);
  __half hv;
  if (i < kPreState) hv = s.in[srow + kOffPre + i];
  else hv = __float2half_rn((float)pcm[(int64_t)b * chunk + (i - kPreState)] / 32767.0f);
  wave[idx] = __half2float(hv);
  if (i >= chunk) s.out[orow + kOffPre + (i - chunk)] = hv;
  if (i == 0) {   // mhsa_len + T: EncoderState.state_keep_size = the chunk's frame count (conformer_blocks.py:206)
    const float ml = __half2float(s.in[srow + kOffMhsaLen]);
    s.out[orow + kOffMhsaLen] = __float2half_rn(fminf(ml + (float)T, (float)kMhsaS));
    // resident form: the chunk counter (mod 30) that sets the conv rings' phases (common.h StateRef)
    if (s.ring) s.out[orow + kOffConv] = __float2half_rn((float)((s.chunk_counter(b) + 1) % kConvS));
  }
}

hipError_t launch_mel_prep(const int32_t* pcm, StateRef s, float* wave, int B, int chunk, hipStream_t st) {
  const Geom g = make_geom(chunk);
  const int64_t n = (int64_t)B * g.wave;
  hipLaunchKernelGGL(mel_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pcm, s, wave, B, chunk, g.T);
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

// ---- fp32 (exact-fp32 MFMA v_mfma_f32_32x32x2_f32): 8 waves per stream, 32-position tiles; the tap
// loop runs kt (11) x kf pairs (11, the 22nd tap zero-weighted), so the gathered x1 address is plain
// arithmetic (no tap table).
constexpr int kKfP = 22;                    // kf padded to an even count (fp32 path)

template <int MT>   // mel frames per chunk: 30 (300 ms) | 40 (400 ms)
__global__ void __launch_bounds__(512) sub1_f32_kernel(const float* __restrict__ feats, StateRef s,
                                                       const float* __restrict__ pre_norm_w,
                                                       const float* __restrict__ w1, const float* __restrict__ scale1,
                                                       const float* __restrict__ shift1, float* __restrict__ x2) {
  constexpr int kMelT = MT, kSub2In = kSub2S + MT, kPos1 = MT * kSub1F;   // 1320 positions at 300 ms
  __shared__ float x1[(kSub1S + kMelT) * kMels + 32];   // +32: taps past column 63 read zeros
  __shared__ float wk[kSub1C][kSub1Kt * kKfP + 1];
  __shared__ float sc[kSub1C], sh[kSub1C];
  __shared__ __half st2[kSub1C * kSub2S * kSub1F];      // sub2 state [c][8][44]: carried in, then next
  __shared__ __attribute__((aligned(16))) float tbuf[8][32 * kSub1C];   // per-wave output tile (32 pos x 32 ch)
  // gridDim.y parts of one stream (small batches, the drop-in's B = 1 call pattern): part y computes the position
  // tiles y * 8 + wave, + 8 * parts ...; part 0 also writes the sub1 state and the carried x2 rows; with parts > 1
  // the next sub2 state goes straight to global memory instead of through the LDS image
  const int b = blockIdx.x, part = blockIdx.y, parts = gridDim.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t srow = s.row_in(b), orow = s.row_out(b);
  if (part == 0)
    for (int i = tid; i < kSub1C * kSub2S * kSub1F; i += 512) st2[i] = s.in[srow + kOffSub2 + i];
  for (int i = tid; i < kSub1C * kSub1Kt * kKfP; i += 512) {
    const int c = i / (kSub1Kt * kKfP), k = i % (kSub1Kt * kKfP), kt = k / kKfP, kf = k % kKfP;
    wk[c][k] = kf < kSub1Kf ? w1[(c * kSub1Kt + kt) * kSub1Kf + kf] : 0.f;
  }
  if (tid < kSub1C) { sc[tid] = scale1[tid]; sh[tid] = shift1[tid]; }
  for (int i = tid; i < kSub1S * kMels; i += 512) x1[i] = __half2float(s.in[srow + kOffSub1 + i]);
  if (tid < 32) x1[(kSub1S + kMelT) * kMels + tid] = 0.f;
  for (int t = wid; t < kMelT; t += 8) {   // RMSNorm over 64 features: one wave per frame
    const float v = feats[((int64_t)b * kMelT + t) * kMels + lane];
    const float ssq = wave_sum(v * v);
    const float rms = sqrtf(ssq) * 0.125f;          // * 64^-0.5
    const float y = pre_norm_w[lane] * (v / (rms + kRmsEps));
    x1[(kSub1S + t) * kMels + lane] = y;
    if (part == 0 && t >= kMelT - kSub1S) s.out[orow + kOffSub1 + (t - (kMelT - kSub1S)) * kMels + lane] = __float2half_rn(y);
  }
  float* xb = x2 + (int64_t)b * kSub2In * kSub1F * kSub1C;
  __syncthreads();
  for (int i = part == 0 ? tid : 1 << 30; i < kSub1C * kSub2S * kSub1F / 4; i += 512) {   // carried rows -> x2 rows 0..7
    const int c = (4 * i) % kSub1C, rf = (4 * i) / kSub1C;            // 4 channels per thread, 16-byte stores
    const int e = c * kSub2S * kSub1F + rf;
    *reinterpret_cast<float4*>(xb + 4 * i) =
        make_float4(__half2float(st2[e]), __half2float(st2[e + kSub2S * kSub1F]), __half2float(st2[e + 2 * kSub2S * kSub1F]),
                    __half2float(st2[e + 3 * kSub2S * kSub1F]));
  }
  __syncthreads();                                              // st2 is reused for the next state below
  const int li = lane & 31, lh = lane >> 5;
  for (int tile = part * 8 + wid; tile * 32 < kPos1; tile += 8 * parts) {
    const int pos = min(tile * 32 + li, kPos1 - 1);
    const float* xa = x1 + (pos / kSub1F) * kMels + pos % kSub1F + lh;
    const float* wb = &wk[li][lh];
    f32x16_t acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int kt = 0; kt < kSub1Kt; ++kt) {
#pragma unroll
      for (int k2 = 0; k2 < kKfP / 2; ++k2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[kt * kMels + 2 * k2], wb[kt * kKfP + 2 * k2], acc, 0, 0, 0);
    }
    const int c = li;
    float* tw = tbuf[wid];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int pl = (r & 3) + 8 * (r >> 2) + 4 * lh, p = tile * 32 + pl;
      const float y = silu_f(fmaf(acc[r], sc[c], sh[c]));
      tw[pl * kSub1C + c] = y;
      if (p >= kPos1) continue;
      const int t = p / kSub1F, f = p % kSub1F;
      if (t >= kMelT - kSub2S) {
        const int e = (c * kSub2S + (t - (kMelT - kSub2S))) * kSub1F + f;
        if (parts == 1) st2[e] = __float2half_rn(y);
        else s.out[orow + kOffSub2 + e] = __float2half_rn(y);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the tile's 32 positions are consecutive in the flattened (t, f) order: one contiguous 4 KB run
    float* dst = xb + (int64_t)(kSub2S * kSub1F + tile * 32) * kSub1C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int v = lane + 64 * q, pl = v >> 3;
      if (tile * 32 + pl < kPos1) *reinterpret_cast<float4*>(dst + v * 4) = *reinterpret_cast<const float4*>(tw + v * 4);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (parts > 1) return;
  __syncthreads();
  for (int i = tid; i < kSub1C * kSub2S * kSub1F; i += 512) s.out[orow + kOffSub2 + i] = st2[i];
}

// ---- bf16 (v_mfma_f32_16x16x32_bf16): conv1 as a Toeplitz GEMM.  For output row t and kernel row
// kt the 21 kf taps are padded to 32, so one MFMA's K = one kernel row; lane (position f, group g)
// needs x1[t + kt][f + 8g .. f + 8g + 7], which is 16-byte aligned in one of 8 shifted bf16 copies of
// x1 kept in LDS (copy s holds row[j + s]).  The weights ([kt][c][32] bf16, 22 fragments) stay in
// registers for the whole workgroup.  Tiles: 16 positions (f0 = 0, 16, 32 of one row t) x 32
// channels (2 MFMA column tiles); 90 tiles per stream over 8 waves.
constexpr int kX1Cols = 80;                 // shifted-copy row length (taps reach column 43 + 31)

template <int MT>
__global__ void __launch_bounds__(512) sub1_bf16_kernel(const float* __restrict__ feats, StateRef s,
                                                        const float* __restrict__ pre_norm_w,
                                                        const uint16_t* __restrict__ w1t, const float* __restrict__ scale1,
                                                        const float* __restrict__ shift1, uint16_t* __restrict__ x2) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int kMelT = MT, kSub2In = kSub2S + MT;
  constexpr int kRows = kSub1S + kMelT;     // 40 (300 ms) | 50 (400 ms)
  // 8 shifted copies, each padded by 32 B so the copies start 8 banks apart (a wave's A reads hit
  // all 8 copies at the same in-copy offset)
  constexpr int kCopy = kRows * kX1Cols + 16;
  // LDS kept under 80 KiB so two streams share a CU: the sub2 state goes HBM -> x2 and tile -> HBM
  // directly (no [c][8][44] staging copy), and x1 is dead once the shifted copies exist
  __shared__ __attribute__((aligned(16))) uint16_t xc[8 * kCopy];
  __shared__ __attribute__((aligned(16))) float x1[kRows * kMels];   // later: per-wave output tiles
  __shared__ float sc[kSub1C], sh[kSub1C];
  uint16_t(*tbuf)[16 * kSub1C] = reinterpret_cast<uint16_t(*)[16 * kSub1C]>(x1);   // 8 x 1 KiB <= 10 KiB
  static_assert(8 * 16 * kSub1C * 2 <= kRows * kMels * 4, "tbuf fits in x1");
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t srow = s.row_in(b), orow = s.row_out(b);
  // weight fragments: B operand lane (n = lane & 15, k group g = lane >> 4): w1t[kt][16 nt + n][8 g .. 8 g + 7]
  const int g = lane >> 4, n = lane & 15;
  bf16x8 wf[kSub1Kt][2];
#pragma unroll
  for (int kt = 0; kt < kSub1Kt; ++kt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      wf[kt][nt] = *reinterpret_cast<const bf16x8*>(w1t + ((kt * kSub1C + 16 * nt + n) * 32 + 8 * g));
  if (tid < kSub1C) { sc[tid] = scale1[tid]; sh[tid] = shift1[tid]; }
  for (int i = tid; i < kSub1S * kMels; i += 512) x1[i] = __half2float(s.in[srow + kOffSub1 + i]);
  for (int t = wid; t < kMelT; t += 8) {
    const float v = feats[((int64_t)b * kMelT + t) * kMels + lane];
    const float ssq = wave_sum(v * v);
    const float rms = sqrtf(ssq) * 0.125f;
    const float y = pre_norm_w[lane] * (v / (rms + kRmsEps));
    x1[(kSub1S + t) * kMels + lane] = y;
    if (t >= kMelT - kSub1S) s.out[orow + kOffSub1 + (t - (kMelT - kSub1S)) * kMels + lane] = __float2half_rn(y);
  }
  uint16_t* xb = x2 + (int64_t)b * kSub2In * kSub1F * kSub1C;
  __syncthreads();
  const __half* st2in = s.in + srow + kOffSub2;          // sub2 state [c][8][44]
  for (int i = tid; i < kSub1C * kSub2S * kSub1F / 8; i += 512) {   // carried rows -> x2 rows 0..7 (channels-last)
    const int c = (8 * i) % kSub1C, rf = (8 * i) / kSub1C;            // 8 channels per thread, 16-byte stores
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const __bf16 lo = (__bf16)__half2float(st2in[(c + 2 * q) * kSub2S * kSub1F + rf]);
      const __bf16 hi = (__bf16)__half2float(st2in[(c + 2 * q + 1) * kSub2S * kSub1F + rf]);
      w[q] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    *reinterpret_cast<uint4*>(xb + 8 * i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  // shifted bf16 copies, 8 elements (one 16-byte LDS store) per item: 6-7 items per thread instead of 50 one-element
  // ones with two integer divisions each
  constexpr int kChunks = kX1Cols / 8;
  static_assert(kX1Cols % 8 == 0 && kCopy % 8 == 0, "16-byte aligned copy rows");
  for (int i = tid; i < 8 * kRows * kChunks; i += 512) {
    const int sh8 = i / (kRows * kChunks), rem = i - sh8 * (kRows * kChunks), r = rem / kChunks;
    const int j0 = (rem - r * kChunks) * 8;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e0 = j0 + 2 * q + sh8;
      const float v0 = e0 < kMels ? x1[r * kMels + e0] : 0.f;
      const float v1 = e0 + 1 < kMels ? x1[r * kMels + e0 + 1] : 0.f;
      const __bf16 h0 = (__bf16)v0, h1 = (__bf16)v1;
      w[q] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    }
    *reinterpret_cast<uint4*>(xc + sh8 * kCopy + r * kX1Cols + j0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  __syncthreads();                                        // x1 is dead from here: its space holds tbuf
  __half* st2out = s.out + orow + kOffSub2;
  for (int tile = wid; tile < kMelT * 3; tile += 8) {
    const int t = tile / 3, f0 = (tile % 3) * 16;
    const int a = f0 + n + 8 * g, sh8 = a & 7;                 // A operand: position f0 + n, k group g
    const uint16_t* arow = xc + sh8 * kCopy + t * kX1Cols + (a - sh8);
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kt = 0; kt < kSub1Kt; ++kt) {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(arow + kt * kX1Cols);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, wf[kt][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, wf[kt][1], acc[1], 0, 0, 0);
    }
    // D layout 16x16: lane holds column (channel) n + 16 nt, rows (positions) f0 + 4 g + r; the tile
    // goes through the wave's LDS slice so the 16 positions x 64 B (contiguous in x2) leave as one
    // 16-byte store per lane
    uint16_t* tw = tbuf[wid];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int c = 16 * nt + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = f0 + 4 * g + r;
        const float z = fmaf(acc[nt][r], sc[c], sh[c]);   // SiLU via v_exp_f32 / v_rcp_f32 (bf16 output)
        const float y = z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
        const __bf16 hy = (__bf16)y;
        tw[(4 * g + r) * kSub1C + c] = __builtin_bit_cast(uint16_t, hy);
        if (f < kSub1F && t >= kMelT - kSub2S) st2out[(c * kSub2S + (t - (kMelT - kSub2S))) * kSub1F + f] = __float2half_rn(y);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (f0 + (lane >> 2) < kSub1F)
      *reinterpret_cast<uint4*>(xb + ((int64_t)(kSub2S + t) * kSub1F + f0) * kSub1C + lane * 8) =
          *reinterpret_cast<const uint4*>(tw + lane * 8);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MT>
static hipError_t launch_sub1_t(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const void* w1t,
                                const float* scale1, const float* shift1, void* x2, bool x2_bf16, int B, hipStream_t st) {
  if (x2_bf16) {
    if (!w1t) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sub1_bf16_kernel<MT>, dim3(B), dim3(512), 0, st, feats, s, pre_norm_w,
                       static_cast<const uint16_t*>(w1t), scale1, shift1, static_cast<uint16_t*>(x2));
  } else {
    // a few streams: split each stream's position tiles over parts workgroups (one tile per wave)
    const int parts = B <= 16 ? (MT * kSub1F / 32 + 1 + 7) / 8 : 1;
    hipLaunchKernelGGL(sub1_f32_kernel<MT>, dim3(B, parts), dim3(512), 0, st, feats, s, pre_norm_w, w1, scale1, shift1,
                       static_cast<float*>(x2));
  }
  return hipGetLastError();
}

hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const void* w1t,
                       const float* scale1, const float* shift1, void* x2, bool x2_bf16, int B, int chunk,
                       hipStream_t st) {
  const int mt = make_geom(chunk).melT;
  if (mt == 30) return launch_sub1_t<30>(feats, s, pre_norm_w, w1, w1t, scale1, shift1, x2, x2_bf16, B, st);
  if (mt == 40) return launch_sub1_t<40>(feats, s, pre_norm_w, w1, w1t, scale1, shift1, x2, x2_bf16, B, st);
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// a3 conv2 (Conv2d 32->64, k 11x11, stride (3,1)) + BN + SiLU in bf16 mode, one workgroup per stream.
// The stream's whole channels-last input [38][44][32] (107 KB bf16) is staged in LDS once by LDS-DMA
// and every one of the 121 taps reads it from there (the implicit GEMM over all streams gathers each
// input row from L2 once per tap instead).  The 64 x 32 weights of the taps (4 KB each) stream
// through a 3-slot LDS ring of 4 taps per slot, two slots ahead (one barrier per 4 taps).  MFMA 16x16x32: A = the tap's weights (rows = output channels),
// B = the slab (columns = output positions p = 34 t + f, input position (3t + kt) * 44 + f + kf), so
// a lane ends up with 4 consecutive channels of one position: 8-byte bf16 stores into the flat
// [B*10][34*64] output the subsampling Linear reads.  8 waves: wave w owns position tiles
// {w, w + 8, w + 16} (22 tiles of 16 cover the 340 positions) x the 4 channel tiles.
// LDS 16-byte slots are swizzled slot ^ ((q >> 2) & 1) << 1 on the 64-byte rows of both images
// (q = slab position or weight row), which makes the 16x16x32 fragment reads conflict-free
// (ds_read_b128 lane groups {0-3,12-15,20-27}, ...): applied to the DMA source, undone on the read.
constexpr int kC2Pos = kT * kSub2F;                       // 340 output positions per stream
constexpr int kC2In = kSub2In * kSub1F;                   // 1672 input positions (64 B each)
constexpr int kC2SlabPieces = (kC2In * 64 + 1023) / 1024; // 105 one-KiB DMA pieces
constexpr int kC2Taps = kSub2Kt * kSub2Kf;                // 121
constexpr int kC2Slab = kC2SlabPieces * 1024 / 4;         // floats of the slab image
constexpr int kC2TP = 4;                                  // taps per ring slot (one barrier per 4 taps)
constexpr int kC2Ring = 1024 * kC2TP;                     // floats per weight-ring slot (16 KB)
constexpr int kC2Stages = (kC2Taps + kC2TP - 1) / kC2TP;  // 31

__host__ __device__ __forceinline__ int c2_swz(int q) { return ((q >> 2) & 1) << 1; }

// The 121-tap loop + BatchNorm/SiLU epilogue of conv2 over a slab already in LDS (ring first, then the slab, as
// conv2_bf16_kernel lays them out); stage_taps(sg) issues stage sg's weight DMA; stages 0 and 1 are in flight.
template <typename StageFn>
__device__ __forceinline__ void conv2_taps(const float* lds, const float* sc, const float* sh, StageFn&& stage_taps,
                                           uint16_t* __restrict__ flat, int b, int wid, int lane) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const char* lb = reinterpret_cast<const char*>(lds);
  // Per-lane byte offsets, computed once.  Slab position q = qb + toff (qb: the lane's output position's first input
  // position, toff = kt * 44 + kf: the tap) is read at q * 64 B + 16 B * (g ^ swz(q)); swz depends on bit 2 of q only,
  // i.e. on (qb + (toff & 7)) & 4, so xa[i][c] holds the offset for toff & 7 == c and the tap adds toff * 64 B as an
  // immediate.  Waves 6-7 own 2 of the 22 position tiles: their third tile repeats position 339 (its MFMAs keep
  // every SIMD at 6 tiles, which the other SIMDs need anyway, and keep the unrolled loop free of branches).
  const int n = lane & 15, g = lane >> 4;
  uint32_t xa[3][8], wa[4];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int p = min((wid + 8 * i) * 16 + n, kC2Pos - 1);
    const int qb = (kSub2Stride * (p / kSub2F)) * kSub1F + p % kSub2F;
#pragma unroll
    for (int c = 0; c < 8; ++c) xa[i][c] = (uint32_t)((3 * kC2Ring + qb * 16 + ((g ^ c2_swz(qb + c)) << 2)) * 4);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int row = 16 * c + n;
    wa[c] = (uint32_t)((row * 16 + ((g ^ c2_swz(row)) << 2)) * 4);
  }
  f32x4 acc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // every stage is its own instantiation (a 31-stage loop is past the unroller's size limit, and a runtime stage
  // index would turn xa[i][toff & 7] into a scratch-memory lookup).  Reading the next tap's fragments ahead of
  // this tap's MFMAs by hand measured no faster: the scheduler already interleaves them.
  static_for<kC2Stages>([&](auto sgc) {
    constexpr int sg = decltype(sgc)::value;
    if constexpr (sg + 1 < kC2Stages) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier_lds_c2();                                      // stage sg (and the slab) landed; slot (sg+2)%3 free
    if constexpr (sg + 2 < kC2Stages) stage_taps(sg + 2);
#pragma unroll
    for (int u = 0; u < kC2TP; ++u) {
      const int j = sg * kC2TP + u;
      if (j >= kC2Taps) break;
      const int toff = (j / kSub2Kf) * kSub1F + j % kSub2Kf;
      const int woff = ((sg % 3) * kC2Ring + u * 1024) * 4;
      bf16x8 wf[4], xf[3];
#pragma unroll
      for (int c = 0; c < 4; ++c) wf[c] = *reinterpret_cast<const bf16x8*>(lb + wa[c] + woff);
#pragma unroll
      for (int i = 0; i < 3; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(lb + xa[i][toff & 7] + toff * 64);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[i], acc[i][c], 0, 0, 0);
    }
  });
  // epilogue: D[channel][position]; lane: position 16 tile + n, channels 16 c + 4 g + r
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int p = (wid + 8 * i) * 16 + n;
    if (p >= kC2Pos) continue;
    uint16_t* dst = flat + ((int64_t)b * kC2Pos + p) * kSub2C;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ch = 16 * c + 4 * g + r;
        const float z = fmaf(acc[i][c][r], sc[ch], sh[ch]);   // SiLU via v_exp_f32 / v_rcp_f32 (bf16 output)
        y[r] = z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
      }
      const __bf16 h0 = (__bf16)y[0], h1 = (__bf16)y[1], h2 = (__bf16)y[2], h3 = (__bf16)y[3];
      const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
      const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, h2) | ((uint32_t)__builtin_bit_cast(uint16_t, h3) << 16);
      *reinterpret_cast<uint2*>(dst + 16 * c + 4 * g) = make_uint2(lo, hi);
    }
  }
}

__global__ void __launch_bounds__(512) conv2_bf16_kernel(const uint16_t* __restrict__ x2, const uint16_t* __restrict__ w2c,
                                                         const float* __restrict__ scale, const float* __restrict__ shift,
                                                         uint16_t* __restrict__ flat) {
  // ONE LDS object: 3 ring slots | slab | scale | shift.  The ring comes first so that every fragment read of the
  // unrolled tap loop is a per-lane VGPR base plus a compile-time immediate below 64 KiB: the ring slot and tap
  // (slot * 16 KiB + u * 4 KiB) for the weights, the tap's input offset toff * 64 B for the slab.
  __shared__ __attribute__((aligned(16))) float lds[3 * kC2Ring + kC2Slab + 2 * kSub2C];
  float* ring = lds;
  float* slab = lds + 3 * kC2Ring;
  float* sc = slab + kC2Slab;
  float* sh = sc + kSub2C;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint16_t* xb = x2 + (int64_t)b * kC2In * kSub1C;
  if (tid < kSub2C) {
    sc[tid] = scale[tid];
    sh[tid] = shift[tid];
  }
  __syncthreads();                                        // before any LDS-DMA is in flight

  auto stage_taps = [&](int sg) {                         // taps 4 sg .. 4 sg + 3: 16 pieces, 2 per wave
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pc = wid * 2 + h, tap = min(sg * kC2TP + (pc >> 2), kC2Taps);   // past the end: the zero tap
      const int L = (pc & 3) * 64 + lane, c = L >> 2, s = L & 3;
      const uint16_t* src = w2c + (int64_t)c * kConv2KPad + tap * kSub1C + ((s ^ c2_swz(c)) << 3);
      lds_dma16(src, ring + (sg % 3) * kC2Ring + pc * 256);
    }
  };
  for (int pc = wid; pc < kC2SlabPieces; pc += 8) {       // the stream's input, once
    const int L = pc * 64 + lane, q = min(L >> 2, kC2In - 1), s = L & 3;
    const uint16_t* src = xb + q * kSub1C + ((s ^ c2_swz(q)) << 3);
    lds_dma16(src, slab + pc * 256);
  }
  stage_taps(0);
  stage_taps(1);

  conv2_taps(lds, sc, sh, stage_taps, flat, b, wid, lane);
}

// a3 in bf16 mode at 300 ms, fused: the pre-encode RMSNorm + conv1 (sub1_bf16_kernel's arithmetic) write the
// conv2 input rows straight into this workgroup's LDS slab, so the 107 KB per stream of x2 is never written to HBM and
// read back (sub1_bf16 + conv2_bf16: 287 + 598 us at B = 4096).  Phases of one workgroup (one stream):
//   1. conv2 stage 0's weights DMA'd into ring slot 0 (in flight throughout);
//   2. x1 = [sub1 state (10 rows) ; RMSNorm(feats) (30 rows)] (a wave per row, a lane per mel; the new sub1 state
//      rows go out as fp16) -> four shifted bf16 copies in ring slots 1-2 (copy s holds x1[r][j + s], so an A fragment
//      of 8 columns starting at any a is two 8-byte reads at column a - (a & 3));
//   3. the sub2 state (fp16 [c][8][44]) -> slab rows 0..7 as 16-byte channel chunks;
//   4. conv1 as sub1_bf16_kernel's Toeplitz MFMA (90 tiles of 16 positions x 32 channels over 8 waves, the weight
//      fragments in registers), BN + SiLU, bf16 into slab rows 8..37 (the swizzled layout conv2 reads) and fp16 into
//      the new sub2 state (rows 22..29);
//   5. ring slots 1-2 are free again: stage 1's DMA, then conv2_taps as in conv2_bf16_kernel.
constexpr int kF1Rows = kSub1S + 30;                 // x1 rows at 300 ms: 10 carried + 30 new
constexpr int kF1Copy = kF1Rows * kX1Cols + 16;      // halves per shifted copy
static_assert(4 * kF1Copy * 2 <= 2 * kC2Ring * 4, "four shifted copies fit in ring slots 1-2");

__global__ void __launch_bounds__(512) sub_conv_bf16_kernel(const float* __restrict__ feats, StateRef s,
                                                            const float* __restrict__ pre_norm_w,
                                                            const uint16_t* __restrict__ w1t,
                                                            const float* __restrict__ scale1,
                                                            const float* __restrict__ shift1,
                                                            const uint16_t* __restrict__ w2c,
                                                            const float* __restrict__ scale2,
                                                            const float* __restrict__ shift2,
                                                            uint16_t* __restrict__ flat) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int kMT = 30;                            // mel frames (300 ms)
  __shared__ __attribute__((aligned(16))) float lds[3 * kC2Ring + kC2Slab + 2 * kSub2C + 2 * kSub1C];
  float* ring = lds;
  float* slab = lds + 3 * kC2Ring;
  float* sc = slab + kC2Slab;
  float* sh = sc + kSub2C;
  float* sc1 = sh + kSub2C;
  float* sh1 = sc1 + kSub1C;
  uint16_t* xc = reinterpret_cast<uint16_t*>(ring + kC2Ring);
  uint16_t* slab16 = reinterpret_cast<uint16_t*>(slab);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t srow = s.row_in(b), orow = s.row_out(b);
  if (tid < kSub2C) {
    sc[tid] = scale2[tid];
    sh[tid] = shift2[tid];
  }
  if (tid < kSub1C) {
    sc1[tid] = scale1[tid];
    sh1[tid] = shift1[tid];
  }
  __syncthreads();                                        // before any LDS-DMA is in flight

  auto stage_taps = [&](int sg) {                         // taps 4 sg .. 4 sg + 3: 16 pieces, 2 per wave
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pc = wid * 2 + h, tap = min(sg * kC2TP + (pc >> 2), kC2Taps);   // past the end: the zero tap
      const int L = (pc & 3) * 64 + lane, c = L >> 2, q = L & 3;
      const uint16_t* src = w2c + (int64_t)c * kConv2KPad + tap * kSub1C + ((q ^ c2_swz(c)) << 3);
      lds_dma16(src, ring + (sg % 3) * kC2Ring + pc * 256);
    }
  };
  stage_taps(0);

  // conv1 weight fragments: B operand lane (n = lane & 15, k group g = lane >> 4): w1t[kt][16 nt + n][8 g .. 8 g + 7]
  const int g = lane >> 4, n = lane & 15;
  bf16x8 wf[kSub1Kt][2];
#pragma unroll
  for (int kt = 0; kt < kSub1Kt; ++kt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      wf[kt][nt] = *reinterpret_cast<const bf16x8*>(w1t + ((kt * kSub1C + 16 * nt + n) * 32 + 8 * g));

  // every global load of phases 2-3 is issued before any of their arithmetic (one memory round trip, not one per
  // row: the first version, a loop of dependent row loads, spent as long in this phase as the separate sub1 launch)
  constexpr int kRowsPerWave = kF1Rows / 8;               // 5
  constexpr int kStItems = kSub2S * kSub1F * 4;           // 1408 (position, 8-channel chunk) items
  constexpr int kStPerThread = (kStItems + 511) / 512;    // 3
  static_assert(kF1Rows % 8 == 0, "x1 rows over 8 waves");
  float xs[kRowsPerWave], xf[kRowsPerWave];
#pragma unroll
  for (int k = 0; k < kRowsPerWave; ++k) {
    const int r = wid + 8 * k;
    xs[k] = __half2float(s.in[srow + kOffSub1 + min(r, kSub1S - 1) * kMels + lane]);
    xf[k] = feats[((int64_t)b * kMT + max(r - kSub1S, 0)) * kMels + lane];
  }
  const float pw = pre_norm_w[lane];
  const __half* st2in = s.in + srow + kOffSub2;
  __half sv[kStPerThread][8];
#pragma unroll
  for (int k = 0; k < kStPerThread; ++k) {
    const int i = min(tid + 512 * k, kStItems - 1), q = i >> 2, ck = i & 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) sv[k][e] = st2in[(8 * ck + e) * kSub2S * kSub1F + q];
  }
  // x1 rows -> the four shifted bf16 copies (copy q, row r, column j: x1[r][j + q], zero past the row)
#pragma unroll
  for (int k = 0; k < kRowsPerWave; ++k) {
    const int r = wid + 8 * k;
    float y;
    if (r < kSub1S) {
      y = xs[k];
    } else {
      const int t = r - kSub1S;
      const float v = xf[k];
      const float ssq = wave_sum(v * v);
      const float rms = sqrtf(ssq) * 0.125f;
      y = pw * (v / (rms + kRmsEps));
      if (t >= kMT - kSub1S) s.out[orow + kOffSub1 + (t - (kMT - kSub1S)) * kMels + lane] = __float2half_rn(y);
    }
    const __bf16 hy = (__bf16)y;
    const uint16_t hb = __builtin_bit_cast(uint16_t, hy);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint16_t* row = xc + q * kF1Copy + r * kX1Cols;
      if (lane >= q) row[lane - q] = hb;
      if (lane < 16 + q) row[kMels - q + lane] = 0;
    }
  }
  // carried conv2-input rows (sub2 state [c][8][44], fp16) -> slab rows 0..7: 16-byte chunks of 8 channels
#pragma unroll
  for (int k = 0; k < kStPerThread; ++k) {
    const int i = tid + 512 * k, q = i >> 2, ck = i & 3;
    if (i < kStItems) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 lo = (__bf16)__half2float(sv[k][2 * e]);
        const __bf16 hi = (__bf16)__half2float(sv[k][2 * e + 1]);
        w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
      }
      *reinterpret_cast<uint4*>(slab16 + q * kSub1C + ((ck ^ c2_swz(q)) << 3)) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  __syncthreads();

  // conv1 tiles -> slab rows 8..37 (and the new sub2 state).  Software-pipelined: tile i + 1's fragment reads and
  // MFMAs are issued before tile i's BN + SiLU epilogue, so the epilogue's VALU runs under the next tile's matrix work.
  // Every wave runs 12 steps (90 tiles over 8 waves: waves 2-7 have 11, their 12th repeats tile 89 and writes the same
  // values wave 1 writes there), so the loop has no tile-count branch for the compiler to sink the MFMAs under.
  __half* st2out = s.out + orow + kOffSub2;
  constexpr int kC1Tiles = kMT * 3, kC1Steps = (kC1Tiles + 7) / 8;
  auto c1_mma = [&](int tile, f32x4 (&acc)[2]) __attribute__((always_inline)) {
    const int t = tile / 3, f0 = (tile % 3) * 16;
    const int a = f0 + n + 8 * g, q = a & 3;                 // A operand: position f0 + n, k group g
    const uint16_t* arow = xc + q * kF1Copy + t * kX1Cols + (a - q);
    // every A fragment of the tile requested before its first MFMA (read one K-step ahead, each pair of MFMAs waited
    // on its own read)
    bf16x8 av[kSub1Kt];
#pragma unroll
    for (int kt = 0; kt < kSub1Kt; ++kt) {
      const uint2 lo = *reinterpret_cast<const uint2*>(arow + kt * kX1Cols);
      const uint2 hi = *reinterpret_cast<const uint2*>(arow + kt * kX1Cols + 4);
      av[kt] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
    __builtin_amdgcn_sched_barrier(0);
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < kSub1Kt; ++kt) {
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[kt], wf[kt][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[kt], wf[kt][1], acc[1], 0, 0, 0);
    }
  };
  // D 16x16: lane holds channel 16 nt + n of positions f0 + 4 g + r.  A lane's four positions are all valid or all
  // past the 44 columns (f0 = 32, g = 3), so one lane predicate covers its eight stores; with a test per element the
  // compiler sank each value's BN + SiLU chain under its own branch and ran the eight chains one after another
  // (profiles/r05_subconv_ablate.txt)
  auto c1_epi = [&](int tile, const f32x4 (&acc)[2]) __attribute__((always_inline)) {
    const int t = tile / 3, f0 = (tile % 3) * 16;
    if (f0 + 4 * g < kSub1F) {
      float y[2][4];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int c = 16 * nt + n;
        const float s1 = sc1[c], h1 = sh1[c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = fmaf(acc[nt][r], s1, h1);           // SiLU via v_exp_f32 / v_rcp_f32 (bf16 output)
          y[nt][r] = z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -1.4426950408889634f));
        }
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int c = 16 * nt + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = (kSub2S + t) * kSub1F + f0 + 4 * g + r;
          const __bf16 hy = (__bf16)y[nt][r];
          slab16[p * kSub1C + (((c >> 3) ^ c2_swz(p)) << 3) + (c & 7)] = __builtin_bit_cast(uint16_t, hy);
        }
      }
      if (t >= kMT - kSub2S) {                                // the new sub2 state rows (tile-uniform)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st2out[((16 * nt + n) * kSub2S + (t - (kMT - kSub2S))) * kSub1F + f0 + 4 * g + r] = __float2half_rn(y[nt][r]);
      }
    }
  };
  {
    f32x4 accA[2], accB[2];
    c1_mma(wid, accA);
#pragma unroll 1
    for (int i = 0; i < kC1Steps; i += 2) {
      const int t0 = min(wid + 8 * i, kC1Tiles - 1), t1 = min(wid + 8 * (i + 1), kC1Tiles - 1);
      const int t2 = min(wid + 8 * (i + 2), kC1Tiles - 1);
      c1_mma(t1, accB);
      c1_epi(t0, accA);
      if (i + 2 < kC1Steps) c1_mma(t2, accA);
      c1_epi(t1, accB);
    }
  }
#ifndef SUBCONV_DROP_BARRIER   // test-only build (Makefile kernel_check_nobar): shows tests/test_gpu_kernels.py sees the race
  __syncthreads();                                        // the slab is complete; ring slots 1-2 are free
#endif
  stage_taps(1);
  conv2_taps(lds, sc, sh, stage_taps, flat, b, wid, lane);
}

hipError_t launch_sub_conv_bf16(const float* feats, StateRef s, const float* pre_norm_w, const void* w1t,
                                const float* scale1, const float* shift1, const void* w2c, const float* scale2,
                                const float* shift2, void* flat, int B, hipStream_t st) {
  if (!w1t) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sub_conv_bf16_kernel, dim3(B), dim3(512), 0, st, feats, s, pre_norm_w,
                     static_cast<const uint16_t*>(w1t), scale1, shift1, static_cast<const uint16_t*>(w2c), scale2,
                     shift2, static_cast<uint16_t*>(flat));
  return hipGetLastError();
}

hipError_t launch_conv2_bf16(const void* x2, const void* w2c, const float* scale, const float* shift, void* flat, int B,
                             hipStream_t st) {
  hipLaunchKernelGGL(conv2_bf16_kernel, dim3(B), dim3(512), 0, st, static_cast<const uint16_t*>(x2),
                     static_cast<const uint16_t*>(w2c), scale, shift, static_cast<uint16_t*>(flat));
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// a3 conv2 in fp32 (split) mode, input split once per kernel row ("p3").  The round-1 kernel (conv2_x3, since
// removed) split every slab fragment again for each of the 121 taps (21x redundant VALU,
// profiles/r02_conv2_x3_ablate.txt: the split cost ~58 us of 283 at B = 256).  Here the loop runs kernel row kt
// outer, kernel column kf inner: the 5 input rows that kt reads (3 r + kt for output rows r) are split ONCE into three bf16
// planes in LDS, and the 11 taps of that row read their X fragments from the planes directly (three
// ds_read_b128, no VALU).  Per workgroup (stream, part of 5 output rows), 8 waves:
//   * W taps (pre-split, natural channel order) stream through a 3-slot ring, issued by waves 0-3
//     (3 x 1 KiB each), two taps ahead: one counted wait + one barrier per tap;
//   * the fp32 rows of kernel row kt + 1 are fetched by waves 4-7 into an fp32 staging area (28 KiB)
//     during the taps of kt, and split into the idle plane buffer by all waves at tap kf = 3;
//   * 16-byte chunk swizzle g ^ s((row >> 2) & 3), s(q) = q ^ ((q & 1) << 1), on 64-byte rows (channel
//     rows of W, position rows of X): the four 16-lane groups of a ds_read_b128 hit distinct banks for
//     16 aligned rows.
// Arithmetic: the six products of gemm_x3 (fp32-accurate), D[channel][position] on 16x16x32 MFMA.
constexpr int kP3Rows = 5;                                        // output rows per workgroup
constexpr int kP3Plane = kP3Rows * kSub1F * kSub1C;               // bf16 of one plane (5 rows x 44 x 32)
constexpr int kP3Stage = kP3Rows * kSub1F * kSub1C;               // fp32 staged per kernel row (7040)
constexpr int kP3StagePieces = (kP3Stage * 4 + 1023) / 1024;      // 28
constexpr int kP3Tap = 3 * kSub2C * kSub1C;                       // bf16 of one tap (12 KiB)
constexpr int kP3LdsBytes = 2 * 3 * kP3Plane * 2 + 3 * kP3Tap * 2 + kP3StagePieces * 1024 + 2 * kSub2C * 4;
static_assert(kP3LdsBytes <= 160 * 1024, "conv2_p3 LDS");
static_assert(kP3StagePieces % 4 == 0, "staging pieces over waves 4-7");

__host__ __device__ __forceinline__ int p3_swz(int row) {   // 16-byte chunk XOR for 64-byte rows
  const int q = (row >> 2) & 3;
  return q ^ ((q & 1) << 1);
}

template <int T>
__global__ void __launch_bounds__(512) conv2_p3_kernel(const float* __restrict__ x2, const uint16_t* __restrict__ w2p,
                                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                                     float* __restrict__ flat) {
  constexpr int NWV = 8;
  constexpr int kParts = (T + kP3Rows - 1) / kP3Rows;
  constexpr int kIn = (T == make_geom(3200).T ? make_geom(3200) : make_geom(2400)).sub2In;   // input rows per stream
  constexpr int kC2PosT = T * kSub2F;
  constexpr int kTiles = (kP3Rows * kSub2F + 15) / 16;            // 11
  constexpr int KT = (kTiles + NWV - 1) / NWV, KU = kTiles / NWV; // position tiles per wave: max, unconditional
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) uint8_t lds[kP3LdsBytes];
  uint16_t* xpl = reinterpret_cast<uint16_t*>(lds);                               // [2][3][5][44][32] bf16
  uint16_t* ring = xpl + 2 * 3 * kP3Plane;                                         // [3][3][64][32] bf16
  float* stg = reinterpret_cast<float*>(ring + 3 * kP3Tap);                        // [5][44][32] fp32
  float* sc = stg + kP3StagePieces * 256;
  float* sh = sc + kSub2C;
  const int b = blockIdx.x / kParts, part = blockIdx.x % kParts;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rows = min(kP3Rows, T - part * kP3Rows), posT = rows * kSub2F;
  const float* xb = x2 + (int64_t)b * kIn * kSub1F * kSub1C;
  if (tid < kSub2C) {
    sc[tid] = scale[tid];
    sh[tid] = shift[tid];
  }
  __syncthreads();                                                // before any LDS-DMA is in flight

  // waves 0-3: tap j (clamped to the last) into ring slot j % 3, 3 pieces each
  auto stage_tap = [&](int j) {
    j = min(j, kC2Taps - 1);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int pc = wid * 3 + i;
      const uint16_t* src = w2p + (int64_t)j * kP3Tap + pc * 512 + lane * 8;
      lds_dma16(src, ring + (j % 3) * kP3Tap + pc * 512);
    }
  };
  // waves 4-7: the fp32 input rows 3 r + kt (r < 5, row past the stream clamped) into the staging area
  auto stage_rows = [&](int kt) {
#pragma unroll
    for (int i = 0; i < kP3StagePieces / 4; ++i) {
      const int pc = (wid - 4) + 4 * i;
      const int e = min(pc * 256 + lane * 4, kP3Stage - 4);       // staged float index
      const int rr = e / (kSub1F * kSub1C), o = e - rr * (kSub1F * kSub1C);
      const int row = min(kSub2Stride * (part * kP3Rows + rr) + kt, kIn - 1);
      const float* src = xb + (int64_t)row * kSub1F * kSub1C + o;
      lds_dma16(src, stg + pc * 256);
    }
  };
  // all waves: staging -> the three planes of buffer `buf` (each thread a few 4-channel groups)
  auto split_rows = [&](int buf) {
    uint16_t* dst = xpl + buf * 3 * kP3Plane;
    for (int i = tid; i < kP3Stage / 4; i += NWV * 64) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(stg + 4 * i);
      const int pos = (4 * i) / kSub1C, ch = (4 * i) % kSub1C;   // pos = r * 44 + f
      const int f = pos % kSub1F;
      const int off = pos * kSub1C + ((((ch >> 3) ^ p3_swz(f)) << 3) | (ch & 4));
      uint32_t w[3][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float t0[2], t1[2], t2[2];
        split3_f(v[2 * h], t0[0], t1[0], t2[0]);
        split3_f(v[2 * h + 1], t0[1], t1[1], t2[1]);
        w[0][h] = (__float_as_uint(t0[0]) >> 16) | (__float_as_uint(t0[1]) & 0xffff0000u);
        w[1][h] = (__float_as_uint(t1[0]) >> 16) | (__float_as_uint(t1[1]) & 0xffff0000u);
        w[2][h] = (__float_as_uint(t2[0]) >> 16) | (__float_as_uint(t2[1]) & 0xffff0000u);
      }
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x2*>(dst + pl * kP3Plane + off) = u32x2{w[pl][0], w[pl][1]};
    }
  };

  // prologue: taps 0, 1; the rows of kt = 0 staged and split into buffer 0
  if (wid < 4) {
    stage_tap(0);
    stage_tap(1);
  } else {
    stage_rows(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier_lds_c2();
  split_rows(0);

  const int n = lane & 15, g = lane >> 4;
  // wave-uniform; from this part's own rows, so the short last part at 400 ms (T = 13: 5 + 5 + 3 rows, 7 position tiles)
  // runs one tile per wave instead of repeating clamped positions
  const int ntile = wid + NWV * (KT - 1) < (posT + 15) / 16 ? KT : KT - 1;
  int xr[KT], xf[KT];                                              // output row / column of this lane's position
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int p = min((wid + NWV * k) * 16 + n, posT - 1);
    xr[k] = p / kSub2F;
    xf[k] = p % kSub2F;
  }
  int wofs[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int c = 16 * ct + n;
    wofs[ct] = c * kSub1C + ((g ^ p3_swz(c)) << 3);
  }
  f32x4 acc[KT][4];
#pragma unroll
  for (int k = 0; k < KT; ++k)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[k][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kt = 0; kt < kSub2Kt; ++kt) {
    const uint16_t* xp = xpl + (kt & 1) * 3 * kP3Plane;
    for (int kf = 0; kf < kSub2Kf; ++kf) {
      const int j = kt * kSub2Kf + kf;
      if (wid < 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // tap j landed, tap j + 1 in flight
      else if (kf == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // rows of kt + 1 staged
      barrier_lds_c2();                                           // ... for every wave; slot (j + 2) % 3 free
      if (wid < 4) stage_tap(j + 2);
      else if (kf == 0 && kt + 1 < kSub2Kt) stage_rows(kt + 1);  // staging free: its split was at kt - 1, kf 3
      if (kf == 3 && kt + 1 < kSub2Kt) split_rows((kt + 1) & 1); // that buffer was last read in kt - 1
      const uint16_t* wr = ring + (j % 3) * kP3Tap;
      bf16x8 w[3][4];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) w[pl][ct] = *reinterpret_cast<const bf16x8*>(wr + pl * kSub2C * kSub1C + wofs[ct]);
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k < KU || k < ntile) {
          const int f = xf[k] + kf;
          const int off = (xr[k] * kSub1F + f) * kSub1C + ((g ^ p3_swz(f)) << 3);
          const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(xp + off);
          const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(xp + kP3Plane + off);
          const bf16x8 x2v = *reinterpret_cast<const bf16x8*>(xp + 2 * kP3Plane + off);
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) {
            f32x4 t = acc[k][ct];
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2][ct], x0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1][ct], x1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0][ct], x2v, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1][ct], x0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0][ct], x1, t, 0, 0, 0);
            acc[k][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0][ct], x0, t, 0, 0, 0);
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");               // the clamped tap DMAs
  // epilogue: D[channel][position]; lane: position tile 16 + n, channels 16 ct + 4 g + r
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (k >= ntile) break;
    const int p = (wid + NWV * k) * 16 + n;
    if (p >= posT) continue;
    float* dst = flat + ((int64_t)b * kC2PosT + part * kP3Rows * kSub2F + p) * kSub2C;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int ch = 16 * ct + 4 * g;
      float4 y;
      y.x = silu_f(fmaf(acc[k][ct][0], sc[ch], sh[ch]));
      y.y = silu_f(fmaf(acc[k][ct][1], sc[ch + 1], sh[ch + 1]));
      y.z = silu_f(fmaf(acc[k][ct][2], sc[ch + 2], sh[ch + 2]));
      y.w = silu_f(fmaf(acc[k][ct][3], sc[ch + 3], sh[ch + 3]));
      *reinterpret_cast<float4*>(dst + ch) = y;
    }
  }
}

// a3 conv2 for a few streams in fp32 mode (the drop-in's B = 1 call pattern): conv2_p3 runs 2-3 workgroups per
// stream, each bound by its own CU's split-MFMA rate (117 us at B = 1, profiles/r03_fp32_b1_step_breakdown.txt).
// Here a workgroup owns one output row t, 16 output channels and 16 positions f of one stream, its 11 waves take one
// kernel row kt each (K = 11 kf x 32 channels = 22 steps of 16) on the exact fp32 MFMA v_mfma_f32_16x16x4_f32 (the
// lane / k map of gemm_sm.hip: lane l loads W[c][k0 + 4 (l >> 4) ..] and x2[row][f + kf][same channels]), and the 11
// partial sums are added in kt order through LDS before the BatchNorm + SiLU epilogue: 10 x 4 x 3 = 120 workgroups
// per stream.
template <int T>
__global__ void __launch_bounds__(kSub2Kt * 64) conv2_sm_kernel(const float* __restrict__ x2, const float* __restrict__ w2,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, float* __restrict__ flat) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int kIn = (T == make_geom(3200).T ? make_geom(3200) : make_geom(2400)).sub2In;   // input rows per stream
  __shared__ __attribute__((aligned(16))) float red[(kSub2Kt - 1) * 64 * 4];
  const int t = blockIdx.x, cb = blockIdx.y, b = blockIdx.z / 3, mbk = blockIdx.z % 3;
  const int tid = threadIdx.x, lane = tid & 63, kt = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, lg = lane >> 4;
  const int c = 16 * cb + l16;                                   // A-operand row: output channel
  const int f = min(16 * mbk + l16, kSub2F - 1);                 // B-operand column: output position (clamped)
  const float* wr = w2 + (int64_t)c * kConv2K + kt * kSub2Kf * kSub1C + 4 * lg;
  const float* xr = x2 + (((int64_t)b * kIn + kSub2Stride * t + kt) * kSub1F + f) * kSub1C + 4 * lg;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < 2 * kSub2Kf; ++st) {                     // step = (kf, channel half)
    const int kf = st >> 1, ch = 16 * (st & 1);
    const f32x4 w = *reinterpret_cast<const f32x4*>(wr + kf * kSub1C + ch);
    const f32x4 x = *reinterpret_cast<const f32x4*>(xr + kf * kSub1C + ch);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w[j], x[j], acc, 0, 0, 0);
  }
  if (kt > 0) *reinterpret_cast<f32x4*>(red + ((kt - 1) * 64 + lane) * 4) = acc;
  __syncthreads();
  if (kt > 0) return;
#pragma unroll
  for (int g = 1; g < kSub2Kt; ++g) acc += *reinterpret_cast<const f32x4*>(red + ((g - 1) * 64 + lane) * 4);
  const int fo = 16 * mbk + l16;                                 // lane: position fo, channels 16 cb + 4 lg .. + 3
  if (fo >= kSub2F) return;
  const int c0 = 16 * cb + 4 * lg;
  f32x4 y;
#pragma unroll
  for (int r = 0; r < 4; ++r) y[r] = silu_f(fmaf(acc[r], scale[c0 + r], shift[c0 + r]));
  *reinterpret_cast<f32x4*>(flat + ((int64_t)b * T + t) * (kSub2F * kSub2C) + fo * kSub2C + c0) = y;
}

hipError_t launch_conv2_sm(const void* x2, const void* w2, const float* scale, const float* shift, void* flat, int B,
                           int T, hipStream_t st) {
  const float* xs = static_cast<const float*>(x2);
  const float* ws = static_cast<const float*>(w2);
  float* fl = static_cast<float*>(flat);
  if (T == 13) hipLaunchKernelGGL((conv2_sm_kernel<13>), dim3(13, 4, 3 * B), dim3(kSub2Kt * 64), 0, st, xs, ws, scale, shift, fl);
  else if (T == kT) hipLaunchKernelGGL((conv2_sm_kernel<kT>), dim3(kT, 4, 3 * B), dim3(kSub2Kt * 64), 0, st, xs, ws, scale, shift, fl);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_conv2_p3(const void* x2, const void* w2p, const float* scale, const float* shift, void* flat, int B,
                           int T, hipStream_t st) {
  const float* xs = static_cast<const float*>(x2);
  const uint16_t* ws = static_cast<const uint16_t*>(w2p);
  float* fl = static_cast<float*>(flat);
  if (T == 13) hipLaunchKernelGGL((conv2_p3_kernel<13>), dim3(3 * B), dim3(512), 0, st, xs, ws, scale, shift, fl);
  else if (T == kT) hipLaunchKernelGGL((conv2_p3_kernel<kT>), dim3(2 * B), dim3(512), 0, st, xs, ws, scale, shift, fl);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Host-side layout of w2p: [tap][plane][c 64][32 bf16], natural channel order, 16-byte chunk g of row c
// stored at g ^ p3_swz(c).  planes[pl][c][tap][ci] are the three bf16 split terms.
void conv2_p3_pack(const uint16_t* planes, uint16_t* w2p) {
  for (int tap = 0; tap < kC2Taps; ++tap)
    for (int pl = 0; pl < 3; ++pl)
      for (int c = 0; c < kSub2C; ++c)
        for (int ci = 0; ci < kSub1C; ++ci)
          w2p[(((int64_t)tap * 3 + pl) * kSub2C + c) * kSub1C + (((ci >> 3) ^ p3_swz(c)) << 3) + (ci & 7)] =
              planes[(((int64_t)pl * kSub2C + c) * kC2Taps + tap) * kSub1C + ci];
}

}  // namespace tone
