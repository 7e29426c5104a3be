// Non-GEMM encoder kernels: row norms, the MHSA input cache, RoPE attention, the stateful
// depthwise conv, temporal reduction / upsampling and the CTC log-softmax head.
#include "common.h"
#include "kernels.h"

namespace tone {

constexpr float kInvSqrtD = 0.05103103630798288f;   // 384^-0.5 (submodules.py:51)

// ---------------------------------------------------------------------------------------------
// RMSNorm (submodules.py:34-54) in place over rows of 384: one wave per row, 6 elements per lane.
__global__ void __launch_bounds__(256) rmsnorm_kernel(float* __restrict__ x, const float* __restrict__ w, int rows,
                                                      uint16_t* __restrict__ shadow) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* xr = x + (int64_t)row * kD;
  float v[6];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v[i] = xr[lane + 64 * i];
    ss += v[i] * v[i];
  }
  ss = wave_sum(ss);
  const float den = sqrtf(ss) * kInvSqrtD + kRmsEps;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float y = w[lane + 64 * i] * (v[i] / den);
    xr[lane + 64 * i] = y;
    if (shadow) store_bf16(shadow, (int64_t)row * kD + lane + 64 * i, y);
  }
}

hipError_t launch_rmsnorm(float* x, const float* w, int rows, uint16_t* shadow, hipStream_t st) {
  hipLaunchKernelGGL(rmsnorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, rows, shadow);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Layers 14/15 MHSA input cache.  EncoderState.update_before_layer slices the stored 30-row cache
// to its last S rows (conformer_blocks.py:147-148); MultiHeadAttention.update_state attends over
// kv = [cache_S ; xn] and keeps [cache_S[T:] ; xn] (submodules.py:295-302); update_after_layer
// left-pads it with zeros to 30 rows (conformer_blocks.py:161-163).  xn = norm_self_att(r).
template <bool OBF>
__global__ void __launch_bounds__(256) kv_assemble_kernel(const float* __restrict__ r, const float* __restrict__ norm_w,
                                                          StateRef s, int layer_slot, int T, int S,
                                                          void* __restrict__ xn, void* __restrict__ kv) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t cache = s.row(b) + kOffMhsa + (int64_t)layer_slot * kMhsaS * kD;
  const int TK = S + T;
  // normalized current rows
  for (int i = wid; i < T; i += 4) {
    const float* xr = r + ((int64_t)b * T + i) * kD;
    float v[6], ss = 0.f;
#pragma unroll
    for (int e = 0; e < 6; ++e) { v[e] = xr[lane + 64 * e]; ss += v[e] * v[e]; }
    ss = wave_sum(ss);
    const float den = sqrtf(ss) * kInvSqrtD + kRmsEps;
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int c = lane + 64 * e;
      const float y = norm_w[c] * (v[e] / den);
      store_act<OBF>(xn, ((int64_t)b * T + i) * kD + c, y);
      store_act<OBF>(kv, ((int64_t)b * TK + S + i) * kD + c, y);
      // new cache row (30 - S) + (S - T + i) = 30 - T + i holds xn[i]
      s.out[cache + (int64_t)(kMhsaS - T + i) * kD + c] = __float2half_rn(y);
    }
  }
  // cached rows: stored rows 30-S .. 29
  for (int i = tid; i < S * kD; i += 256) {
    const int j = i / kD, c = i % kD;
    store_act<OBF>(kv, ((int64_t)b * TK + j) * kD + c, __half2float(s.in[cache + (int64_t)(kMhsaS - S + j) * kD + c]));
  }
  // new cache rows 0 .. 30-T-1: zero padding below 30-S, then cache_S[T:]
  for (int i = tid; i < (kMhsaS - T) * kD; i += 256) {
    const int rr = i / kD, c = i % kD;
    __half h = __float2half_rn(0.f);
    if (rr >= kMhsaS - S) h = s.in[cache + (int64_t)(rr + T) * kD + c];
    s.out[cache + (int64_t)rr * kD + c] = h;
  }
}

hipError_t launch_kv_assemble(const float* r, const float* norm_w, StateRef s, int layer_slot, int T, int S, void* xn,
                              void* kv, bool obf, int B, hipStream_t st) {
  if (obf) hipLaunchKernelGGL(kv_assemble_kernel<true>, dim3(B), dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
  else hipLaunchKernelGGL(kv_assemble_kernel<false>, dim3(B), dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// RotaryMultiHeadAttention.forward (conformer_blocks.py:688-726) + forward_qkv/forward_attention
// (submodules.py:204-271).  One wave per (stream, head):
//   recompute: q,k -> per-head LayerNorm(48) -> RoPE on dims [0,32) (q at positions 0..T-1, k at
//              -S..T-1) -> scores = q.k^T / sqrt(48) -> mask (layers 14/15) -> softmax
//   shared   : probabilities of the last recomputing layer (scores are shared and no mask applies
//              to layers 1-6 / 8-13, so softmax(shared scores) = shared probabilities)
//   ctx = P . V
constexpr int kMaxT = 10, kMaxTK = 40;
template <bool OBF>
__global__ void __launch_bounds__(64) attention_kernel(AttnArgs a) {
  __shared__ float qs[kMaxT][kDk + 1];
  __shared__ float ks[kMaxTK][kDk + 1];
  __shared__ float vs[kMaxTK][kDk + 1];
  __shared__ float ps[kMaxT][kMaxTK + 1];
  const int b = blockIdx.x / kHeads, h = blockIdx.x % kHeads, lane = threadIdx.x;
  const int T = a.T, S = a.S, TK = S + T;
  for (int i = lane; i < TK * kDk; i += 64) {
    const int j = i / kDk, d = i % kDk;
    vs[j][d] = a.v[((int64_t)b * TK + j) * a.ldv + h * kDk + d];
  }
  if (a.recompute) {
    for (int i = lane; i < T * kDk; i += 64) {
      const int j = i / kDk, d = i % kDk;
      qs[j][d] = a.q[((int64_t)b * T + j) * a.ldq + h * kDk + d];
    }
    for (int i = lane; i < TK * kDk; i += 64) {
      const int j = i / kDk, d = i % kDk;
      ks[j][d] = a.k[((int64_t)b * TK + j) * a.ldk + h * kDk + d];
    }
    __syncthreads();
    // LayerNorm + RoPE, one lane per row (rows: T query rows then TK key rows)
    if (lane < T + TK) {
      const bool isq = lane < T;
      float* row = isq ? qs[lane] : ks[lane - T];
      const float* lw = isq ? a.qln_w : a.kln_w;
      const float* lb = isq ? a.qln_b : a.kln_b;
      const int pos = isq ? lane : (lane - T) - S;
      float mu = 0.f;
      for (int d = 0; d < kDk; ++d) mu += row[d];
      mu /= (float)kDk;
      float var = 0.f;
      for (int d = 0; d < kDk; ++d) { const float c = row[d] - mu; var += c * c; }
      var /= (float)kDk;
      const float rstd = 1.0f / sqrtf(var + kLnEps);
      for (int d = 0; d < kDk; ++d) row[d] = (row[d] - mu) * rstd * lw[d] + lb[d];
      const float* cs = a.rope_cos + (pos + kMhsaS) * (kRope / 2);
      const float* sn = a.rope_sin + (pos + kMhsaS) * (kRope / 2);
      for (int d = 0; d < kRope / 2; ++d) {
        const float x1 = row[d], x2 = row[d + kRope / 2];
        row[d] = x1 * cs[d] - x2 * sn[d];
        row[d + kRope / 2] = x2 * cs[d] + x1 * sn[d];
      }
    }
    __syncthreads();
    float off = -1e30f;
    if (S > 0) {
      off = (float)kMhsaS - __half2float(a.s.in[a.s.row(b) + kOffMhsaLen]);
      if (a.reduced) off = floorf(off / 2.0f);
    }
    for (int e = lane; e < T * TK; e += 64) {
      const int i = e / TK, j = e % TK;
      float acc = 0.f;
      for (int d = 0; d < kDk; ++d) acc = fmaf(qs[i][d], ks[j][d], acc);
      const float sc = acc / 6.928203230275509f;   // / math.sqrt(48) (submodules.py:185, conformer_blocks.py:725)
      const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
      ps[i][j] = masked ? -10000.0f : sc;
    }
    __syncthreads();
    if (lane < T) {
      const int i = lane;
      float m = -INFINITY;
      for (int j = 0; j < TK; ++j) m = fmaxf(m, ps[i][j]);
      float sum = 0.f;
      for (int j = 0; j < TK; ++j) { const float e = expf(ps[i][j] - m); ps[i][j] = e; sum += e; }
      for (int j = 0; j < TK; ++j) {
        const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
        ps[i][j] = masked ? 0.f : ps[i][j] / sum;
      }
    }
    __syncthreads();
    if (a.probs) {
      for (int e = lane; e < T * TK; e += 64)
        a.probs[(((int64_t)b * kHeads + h) * T + e / TK) * TK + e % TK] = ps[e / TK][e % TK];
    }
  } else {
    for (int e = lane; e < T * TK; e += 64)
      ps[e / TK][e % TK] = a.probs[(((int64_t)b * kHeads + h) * T + e / TK) * TK + e % TK];
    __syncthreads();
  }
  for (int e = lane; e < T * kDk; e += 64) {
    const int i = e / kDk, d = e % kDk;
    float acc = 0.f;
    for (int j = 0; j < TK; ++j) acc = fmaf(ps[i][j], vs[j][d], acc);
    store_act<OBF>(a.ctx, ((int64_t)b * T + i) * kD + h * kDk + d, acc);
  }
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t st) {
  if (a.T > kMaxT || a.S + a.T > kMaxTK) return hipErrorInvalidValue;
  if (a.ctx_bf16) hipLaunchKernelGGL(attention_kernel<true>, dim3(a.B * kHeads), dim3(64), 0, st, a);
  else hipLaunchKernelGGL(attention_kernel<false>, dim3(a.B * kHeads), dim3(64), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ConformerConvolution depthwise part (conformer_blocks.py:427-433, submodules.py:364-402):
//   x = [conv state (30) ; g (T)] per channel; next state = x[-30:]
//   out[t] = SiLU(BN(bias + sum_k w[k] x[t+k]))  with BN folded into (w, b) on the host.
// One thread per (stream, channel).
template <int T, bool OBF>
__global__ void __launch_bounds__(256) dwconv_kernel(const float* __restrict__ g, StateRef s, int layer,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     void* __restrict__ out, int B) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * kD) return;
  const int b = idx / kD, c = idx % kD;
  const int64_t st = s.row(b) + kOffConv + ((int64_t)layer * kD + c) * kConvS;
  float x[kConvS + T];
#pragma unroll
  for (int i = 0; i < kConvS; ++i) x[i] = __half2float(s.in[st + i]);
#pragma unroll
  for (int t = 0; t < T; ++t) x[kConvS + t] = g[((int64_t)b * T + t) * kD + c];
  float wr[kConvK];
#pragma unroll
  for (int k = 0; k < kConvK; ++k) wr[k] = w[c * kConvK + k];
  const float bb = bias[c];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    float acc = bb;
#pragma unroll
    for (int k = 0; k < kConvK; ++k) acc = fmaf(wr[k], x[t + k], acc);
    store_act<OBF>(out, ((int64_t)b * T + t) * kD + c, silu_f(acc));
  }
#pragma unroll
  for (int i = 0; i < kConvS; ++i) s.out[st + i] = __float2half_rn(x[T + i]);
}

hipError_t launch_dwconv(const float* g, StateRef s, int layer, const float* w, const float* b, void* out, bool obf,
                         int T, int B, hipStream_t st) {
  const dim3 grid((B * kD + 255) / 256);
  if (T == kT && obf) hipLaunchKernelGGL((dwconv_kernel<kT, true>), grid, dim3(256), 0, st, g, s, layer, w, b, out, B);
  else if (T == kT) hipLaunchKernelGGL((dwconv_kernel<kT, false>), grid, dim3(256), 0, st, g, s, layer, w, b, out, B);
  else if (T == kT / 2 && obf) hipLaunchKernelGGL((dwconv_kernel<kT / 2, true>), grid, dim3(256), 0, st, g, s, layer, w, b, out, B);
  else if (T == kT / 2) hipLaunchKernelGGL((dwconv_kernel<kT / 2, false>), grid, dim3(256), 0, st, g, s, layer, w, b, out, B);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// CausalTemporalReduction.forward streaming branch (conformer_blocks.py:888-907), grouped part:
//   x = [state (1) ; x^T (10)] per channel; next state = x[:, -1:]
//   y[o][t] = bias[o] + sum_{k<3} w[o][k] x[o/4][2t+k], o < 1536, t < 5
template <bool OBF>
__global__ void __launch_bounds__(256) reduce_conv_kernel(const float* __restrict__ x, StateRef s,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          void* __restrict__ y, int B) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * kD) return;
  const int b = idx / kD, c = idx % kD;
  const int64_t srow = s.row(b);
  float xc[kT + 1];
  xc[0] = __half2float(s.in[srow + kOffRed + c]);
  for (int t = 0; t < kT; ++t) xc[t + 1] = x[((int64_t)b * kT + t) * kD + c];
  s.out[srow + kOffRed + c] = __float2half_rn(xc[kT]);
  for (int q = 0; q < 4; ++q) {
    const int o = 4 * c + q;
    const float w0 = w[o * 3], w1 = w[o * 3 + 1], w2 = w[o * 3 + 2], bo = bias[o];
    for (int t = 0; t < kT / 2; ++t)
      store_act<OBF>(y, ((int64_t)b * (kT / 2) + t) * (4 * kD) + o, bo + w0 * xc[2 * t] + w1 * xc[2 * t + 1] + w2 * xc[2 * t + 2]);
  }
}

hipError_t launch_reduce_conv(const float* x, StateRef s, const float* w, const float* b, void* y, bool obf, int B,
                              hipStream_t st) {
  if (obf) hipLaunchKernelGGL(reduce_conv_kernel<true>, dim3((B * kD + 255) / 256), dim3(256), 0, st, x, s, w, b, y, B);
  else hipLaunchKernelGGL(reduce_conv_kernel<false>, dim3((B * kD + 255) / 256), dim3(256), 0, st, x, s, w, b, y, B);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// TemporalUpsampling (conformer_blocks.py:955-988): repeat_interleave x2, trim to 10, + residual.
__global__ void __launch_bounds__(256) upsample_add_kernel(float* __restrict__ x10, const float* __restrict__ x5, int B,
                                                           uint16_t* __restrict__ shadow) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)B * kT * kD) return;
  const int64_t row = idx / kD;
  const int c = idx % kD;
  const int64_t b = row / kT, t = row % kT;
  const float v = x5[(b * (kT / 2) + t / 2) * kD + c] + x10[idx];
  x10[idx] = v;
  if (shadow) store_bf16(shadow, idx, v);
}

hipError_t launch_upsample_add(float* x10, const float* x5, int B, uint16_t* shadow, hipStream_t st) {
  const int64_t n = (int64_t)B * kT * kD;
  hipLaunchKernelGGL(upsample_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x10, x5, B, shadow);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ConvASRDecoder.forward (conformer.py:338-354): 1x1 conv 384 -> 35 and log_softmax, fp32.
// The 35 x 384 weight sits in LDS (rows padded to 385 floats: conflict-free per-lane rows);
// one wave per frame, lane o < 35 owns logit o.
__global__ void __launch_bounds__(256) head_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, float* __restrict__ logp, int rows) {
  __shared__ float ws[kVocab][kD + 1];
  __shared__ float xs[4][kD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < kVocab * kD; i += 256) ws[i / kD][i % kD] = w[i];
  __syncthreads();
  for (int base = blockIdx.x * 4; base < rows; base += gridDim.x * 4) {
    const int row = base + wid;
    const bool valid = row < rows;
    __syncthreads();
    if (valid)
      for (int c = lane; c < kD; c += 64) xs[wid][c] = x[(int64_t)row * kD + c];
    __syncthreads();
    float z = -INFINITY;
    if (lane < kVocab) {
      float acc = 0.f;
      for (int c = 0; c < kD; ++c) acc = fmaf(ws[lane][c], xs[wid][c], acc);
      z = acc + bias[lane];
    }
    const float m = wave_max(z);
    const float e = lane < kVocab ? expf(z - m) : 0.f;
    const float lse = logf(wave_sum(e));
    if (valid && lane < kVocab) logp[(int64_t)row * kVocab + lane] = z - m - lse;
  }
}

hipError_t launch_head(const float* x, const float* w, const float* b, float* logp, int rows, hipStream_t st) {
  int blocks = (rows + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(head_kernel, dim3(blocks), dim3(256), 0, st, x, w, b, logp, rows);
  return hipGetLastError();
}

}  // namespace tone
