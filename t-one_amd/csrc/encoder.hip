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
// (submodules.py:204-271).  One 256-thread workgroup per (stream, group of 2 heads):
//   recompute: q,k -> per-head LayerNorm(48) -> RoPE on dims [0,32) (q at positions 0..T-1, k at
//              -S..T-1) -> scores = q.k^T / sqrt(48) -> mask (layers 14/15) -> softmax
//   shared   : probabilities of the last recomputing layer (scores are shared and no mask applies
//              to layers 1-6 / 8-13, so softmax(shared scores) = shared probabilities)
//   ctx = P . V
// LayerNorm+RoPE use 16 lanes per (row, head): lane l owns dims l, l+16 (a RoPE pair) and 32+l.
constexpr int kMaxT = 10, kMaxTK = 40;
constexpr int kHG = 2;                       // heads per workgroup
constexpr int kHC = kHG * kDk;               // 96 columns per workgroup

template <bool OBF>
__global__ void __launch_bounds__(256) attention_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / (kHeads / kHG), hg = blockIdx.x % (kHeads / kHG);
  const int c0 = hg * kHC, tid = threadIdx.x;
  const int T = a.T, S = a.S, TK = S + T;
  float* qs = sm;                    // [T][96]
  float* ks = qs + T * kHC;          // [TK][96]
  float* vs = ks + TK * kHC;         // [TK][96]
  float* ps = vs + TK * kHC;         // [2][T][TK]
  constexpr int C4 = kHC / 4;
  for (int e = tid; e < TK * C4; e += 256) {
    const int j = e / C4, c4 = e % C4;
    *reinterpret_cast<float4*>(vs + j * kHC + 4 * c4) =
        *reinterpret_cast<const float4*>(a.v + ((int64_t)b * TK + j) * a.ldv + c0 + 4 * c4);
  }
  if (a.recompute) {
    for (int e = tid; e < T * C4; e += 256) {
      const int j = e / C4, c4 = e % C4;
      *reinterpret_cast<float4*>(qs + j * kHC + 4 * c4) =
          *reinterpret_cast<const float4*>(a.q + ((int64_t)b * T + j) * a.ldq + c0 + 4 * c4);
    }
    for (int e = tid; e < TK * C4; e += 256) {
      const int j = e / C4, c4 = e % C4;
      *reinterpret_cast<float4*>(ks + j * kHC + 4 * c4) =
          *reinterpret_cast<const float4*>(a.k + ((int64_t)b * TK + j) * a.ldk + c0 + 4 * c4);
    }
    __syncthreads();
    // per-head LayerNorm (eps 1e-5) + partial RoPE: 16 lanes per (row, head)
    const int l = tid & 15;
    const int npairs = (T + TK) * kHG;
    for (int pr = tid >> 4; pr < ((npairs + 15) & ~15); pr += 16) {
      const bool live = pr < npairs;
      const int r = live ? pr / kHG : 0, hl = pr % kHG;
      const bool isq = r < T;
      float* base = (isq ? qs + r * kHC : ks + (r - T) * kHC) + hl * kDk;
      const float* lw = isq ? a.qln_w : a.kln_w;
      const float* lb = isq ? a.qln_b : a.kln_b;
      const float x0 = base[l], x1 = base[l + 16], x2 = base[l + 32];
      float sum = x0 + x1 + x2;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
      const float mu = sum / (float)kDk;
      const float d0 = x0 - mu, d1 = x1 - mu, d2 = x2 - mu;
      float var = d0 * d0 + d1 * d1 + d2 * d2;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) var += __shfl_xor(var, o, 64);
      var /= (float)kDk;
      const float rstd = 1.0f / sqrtf(var + kLnEps);
      const float y0 = d0 * rstd * lw[l] + lb[l];
      const float y1 = d1 * rstd * lw[l + 16] + lb[l + 16];
      const float y2 = d2 * rstd * lw[l + 32] + lb[l + 32];
      const int pos = isq ? r : (r - T) - S;
      const float cs = a.rope_cos[(pos + kMhsaS) * (kRope / 2) + l];
      const float sn = a.rope_sin[(pos + kMhsaS) * (kRope / 2) + l];
      if (live) {
        base[l] = y0 * cs - y1 * sn;            // rotate_half pairs (l, l+16), submodules.py:142-157
        base[l + 16] = y1 * cs + y0 * sn;
        base[l + 32] = y2;
      }
    }
    __syncthreads();
    float off = -1e30f;
    if (S > 0) {
      off = (float)kMhsaS - __half2float(a.s.in[a.s.row(b) + kOffMhsaLen]);
      if (a.reduced) off = floorf(off / 2.0f);
    }
    const int nsc = kHG * T * TK;
    for (int e = tid; e < nsc; e += 256) {
      const int hl = e / (T * TK), i = (e / TK) % T, j = e % TK;
      const float4* q4 = reinterpret_cast<const float4*>(qs + i * kHC + hl * kDk);
      const float4* k4 = reinterpret_cast<const float4*>(ks + j * kHC + hl * kDk);
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < kDk / 4; ++d) {
        const float4 x = q4[d], y = k4[d];
        acc = fmaf(x.x, y.x, acc);
        acc = fmaf(x.y, y.y, acc);
        acc = fmaf(x.z, y.z, acc);
        acc = fmaf(x.w, y.w, acc);
      }
      const float sc = acc / 6.928203230275509f;   // / math.sqrt(48) (submodules.py:185, conformer_blocks.py:725)
      const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
      ps[e] = masked ? -10000.0f : sc;
    }
    __syncthreads();
    for (int rr = tid; rr < kHG * T; rr += 256) {
      float* row = ps + rr * TK;
      const int i = rr % T;
      float m = -INFINITY;
      for (int j = 0; j < TK; ++j) m = fmaxf(m, row[j]);
      float sum = 0.f;
      for (int j = 0; j < TK; ++j) {
        const float e = expf(row[j] - m);
        row[j] = e;
        sum += e;
      }
      for (int j = 0; j < TK; ++j) {
        const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
        row[j] = masked ? 0.f : row[j] / sum;
      }
    }
    __syncthreads();
    if (a.probs) {
      for (int e = tid; e < kHG * T * TK; e += 256) {
        const int hl = e / (T * TK), rem = e % (T * TK);
        a.probs[(((int64_t)b * kHeads + hg * kHG + hl) * T) * TK + rem] = ps[e];
      }
    }
  } else {
    for (int e = tid; e < kHG * T * TK; e += 256) {
      const int hl = e / (T * TK), rem = e % (T * TK);
      ps[e] = a.probs[(((int64_t)b * kHeads + hg * kHG + hl) * T) * TK + rem];
    }
    __syncthreads();
  }
  for (int e = tid; e < T * kHC; e += 256) {
    const int i = e / kHC, c = e % kHC, hl = c / kDk;
    const float* pr = ps + (hl * T + i) * TK;
    float acc = 0.f;
    for (int j = 0; j < TK; ++j) acc = fmaf(pr[j], vs[j * kHC + c], acc);
    store_act<OBF>(a.ctx, ((int64_t)b * T + i) * kD + c0 + c, acc);
  }
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t st) {
  if (a.T > kMaxT || a.S + a.T > kMaxTK) return hipErrorInvalidValue;
  const int tk = a.S + a.T;
  const size_t smem = (size_t)(a.T * kHC + 2 * tk * kHC + kHG * a.T * tk) * sizeof(float);
  const dim3 grid(a.B * (kHeads / kHG));
  if (a.ctx_bf16) hipLaunchKernelGGL(attention_kernel<true>, grid, dim3(256), smem, st, a);
  else hipLaunchKernelGGL(attention_kernel<false>, grid, dim3(256), smem, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ConformerConvolution depthwise part (conformer_blocks.py:427-433, submodules.py:364-402):
//   x = [conv state (30) ; g (T)] per channel; next state = x[-30:]
//   out[t] = SiLU(BN(bias + sum_k w[k] x[t+k]))  with BN folded into (w, b) on the host.
// One 384-thread workgroup (a thread per channel) handles kDwStreams streams with the channel's 31 taps
// (stored tap-major) in registers.  Each stream's 23 KB conv-state section is moved HBM<->LDS in 16-byte
// vectors: state rows are only 2-byte aligned, so the section is read from the enclosing 16-byte-aligned
// window (the section is interior to the row) and the two partial end vectors are written element-wise.
constexpr int kDwStreams = 2;
constexpr int kDwSec = kD * kConvS;          // 11520 halves per (stream, layer)
constexpr int kDwVec = kDwSec / 8 + 1;       // 16-byte vectors covering a misaligned section
template <int T, bool OBF>
__global__ void __launch_bounds__(kD) dwconv_kernel(const float* __restrict__ g, StateRef s, int layer,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    void* __restrict__ out, int B) {
  __shared__ uint4 lds[kDwStreams][kDwVec];
  const int c = threadIdx.x;
  int shift[kDwStreams], nvec[kDwStreams];
  int64_t base[kDwStreams];
#pragma unroll
  for (int si = 0; si < kDwStreams; ++si) {
    const int b = min(blockIdx.x * kDwStreams + si, B - 1);
    base[si] = s.row(b) + kOffConv + (int64_t)layer * kDwSec;
    const uintptr_t a = reinterpret_cast<uintptr_t>(s.in + base[si]);
    shift[si] = (int)((a & 15) >> 1);
    nvec[si] = (shift[si] + kDwSec + 7) >> 3;
    const uint4* q = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
    for (int v = c; v < nvec[si]; v += kD) lds[si][v] = q[v];
  }
  float wr[kConvK];
#pragma unroll
  for (int k = 0; k < kConvK; ++k) wr[k] = w[k * kD + c];
  const float bb = bias[c];
  __syncthreads();
#pragma unroll
  for (int si = 0; si < kDwStreams; ++si) {
    const int b = blockIdx.x * kDwStreams + si;
    if (b >= B) break;
    __half* h = reinterpret_cast<__half*>(lds[si]) + shift[si] + c * kConvS;
    float x[kConvS + T];
#pragma unroll
    for (int t = 0; t < T; ++t) x[kConvS + t] = g[((int64_t)b * T + t) * kD + c];
#pragma unroll
    for (int i = 0; i < kConvS; ++i) x[i] = __half2float(h[i]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float acc = bb;
#pragma unroll
      for (int k = 0; k < kConvK; ++k) acc = fmaf(wr[k], x[t + k], acc);
      store_act<OBF>(out, ((int64_t)b * T + t) * kD + c, silu_f(acc));
    }
#pragma unroll
    for (int i = 0; i < kConvS; ++i) h[i] = __float2half_rn(x[T + i]);
  }
  __syncthreads();
#pragma unroll
  for (int si = 0; si < kDwStreams; ++si) {
    const int b = blockIdx.x * kDwStreams + si;
    if (b >= B) break;
    const uintptr_t a = reinterpret_cast<uintptr_t>(s.out + base[si]);
    const int sh = (int)((a & 15) >> 1);
    __half* dst = s.out + base[si];
    const __half* src = reinterpret_cast<const __half*>(lds[si]) + shift[si];
    if (sh == shift[si]) {
      uint4* q = reinterpret_cast<uint4*>(a & ~uintptr_t(15));
      const int n = nvec[si];
      for (int v = c; v < n; v += kD) {
        if ((v == 0 && sh) || (v == n - 1 && ((sh + kDwSec) & 7))) {
          const int e0 = v * 8 - sh;
          for (int e = max(e0, 0); e < min(e0 + 8, kDwSec); ++e) dst[e] = src[e];
        } else {
          q[v] = lds[si][v];
        }
      }
    } else {  // output slab aligned differently from the input slab
      for (int e = c; e < kDwSec; e += kD) dst[e] = src[e];
    }
  }
}

hipError_t launch_dwconv(const float* g, StateRef s, int layer, const float* w, const float* b, void* out, bool obf,
                         int T, int B, hipStream_t st) {
  const dim3 grid((B + kDwStreams - 1) / kDwStreams), block(kD);
  if (T == kT && obf) hipLaunchKernelGGL((dwconv_kernel<kT, true>), grid, block, 0, st, g, s, layer, w, b, out, B);
  else if (T == kT) hipLaunchKernelGGL((dwconv_kernel<kT, false>), grid, block, 0, st, g, s, layer, w, b, out, B);
  else if (T == kT / 2 && obf) hipLaunchKernelGGL((dwconv_kernel<kT / 2, true>), grid, block, 0, st, g, s, layer, w, b, out, B);
  else if (T == kT / 2) hipLaunchKernelGGL((dwconv_kernel<kT / 2, false>), grid, block, 0, st, g, s, layer, w, b, out, B);
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
// One lane per frame row: the 35 vocabulary dot products accumulate in registers while x streams
// through in 8-float slices and the (broadcast) weight rows come from LDS; log-softmax, the greedy
// token and the splitter's speech flag are per-lane epilogues, and the wave's 64 x 35 logprob block
// (contiguous in memory) leaves through LDS as coalesced stores.
//   frame_info[row] = argmax_v logp[row][v] (first index on ties, decoder.py:57)
//                   | (exp(logp[33]) + exp(logp[34]) <= 0.9) << 8      (logprob_splitter.py:134)
constexpr float kSilenceThreshold = 0.9f;
__global__ void __launch_bounds__(64) head_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                  const float* __restrict__ bias, float* __restrict__ logp,
                                                  int32_t* __restrict__ frame_info, int rows) {
  __shared__ __attribute__((aligned(16))) float ws[kVocab * kD];
  __shared__ float lo[64 * kVocab];
  const int lane = threadIdx.x;
  for (int i = lane; i < kVocab * kD / 4; i += 64)
    reinterpret_cast<f32x4_t*>(ws)[i] = reinterpret_cast<const f32x4_t*>(w)[i];
  __syncthreads();
  const int row0 = blockIdx.x * 64, row = row0 + lane;
  const float* xr = x + (int64_t)min(row, rows - 1) * kD;
  float acc[kVocab];
#pragma unroll
  for (int v = 0; v < kVocab; ++v) acc[v] = 0.f;
  f32x4_t xa = reinterpret_cast<const f32x4_t*>(xr)[0], xb = reinterpret_cast<const f32x4_t*>(xr)[1];
  for (int k = 0; k < kD; k += 8) {
    const f32x4_t ca = xa, cb = xb;
    if (k + 8 < kD) {
      xa = reinterpret_cast<const f32x4_t*>(xr + k + 8)[0];
      xb = reinterpret_cast<const f32x4_t*>(xr + k + 8)[1];
    }
#pragma unroll
    for (int v = 0; v < kVocab; ++v) {
      const f32x4_t wa = *reinterpret_cast<const f32x4_t*>(ws + v * kD + k);
      const f32x4_t wb = *reinterpret_cast<const f32x4_t*>(ws + v * kD + k + 4);
      float a = acc[v];
      a = fmaf(wa.x, ca.x, a); a = fmaf(wa.y, ca.y, a); a = fmaf(wa.z, ca.z, a); a = fmaf(wa.w, ca.w, a);
      a = fmaf(wb.x, cb.x, a); a = fmaf(wb.y, cb.y, a); a = fmaf(wb.z, cb.z, a); a = fmaf(wb.w, cb.w, a);
      acc[v] = a;
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    acc[v] += bias[v];
    m = fmaxf(m, acc[v]);
  }
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) se += expf(acc[v] - m);
  const float lse = logf(se);
  float best = -INFINITY;
  int tok = 0;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    const float lp = acc[v] - m - lse;
    lo[lane * kVocab + v] = lp;
    if (lp > best) { best = lp; tok = v; }
  }
  if (frame_info && row < rows) {
    const float sil = expf(lo[lane * kVocab + kVocab - 2]) + expf(lo[lane * kVocab + kVocab - 1]);
    frame_info[row] = tok | ((sil <= kSilenceThreshold) ? 256 : 0);
  }
  __syncthreads();
  const int nrow = min(64, rows - row0);
  float* dst = logp + (int64_t)row0 * kVocab;
  for (int i = lane; i < nrow * kVocab; i += 64) dst[i] = lo[i];
}

hipError_t launch_head(const float* x, const float* w, const float* b, float* logp, int32_t* frame_info, int rows,
                       hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(head_kernel, dim3((rows + 63) / 64), dim3(64), 0, st, x, w, b, logp, frame_info, rows);
  return hipGetLastError();
}

}  // namespace tone
