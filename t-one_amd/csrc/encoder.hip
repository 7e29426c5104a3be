// Non-GEMM encoder kernels: row norms, the MHSA input cache, RoPE attention, the stateful
// depthwise conv, temporal reduction / upsampling and the CTC log-softmax head.
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace tone {

constexpr float kInvSqrtD = 0.05103103630798288f;   // 384^-0.5 (submodules.py:51)

// ---------------------------------------------------------------------------------------------
// RMSNorm (submodules.py:34-54) in place over rows of 384: one wave per row, 6 elements per lane; the residual
// stream x fp32, or fp16 in the bf16 / fp8 modes (R16).
template <bool R16>
__global__ void __launch_bounds__(256) rmsnorm_kernel(void* __restrict__ x, const float* __restrict__ w, int rows,
                                                      uint16_t* __restrict__ shadow, int64_t plane,
                                                      uint8_t* __restrict__ q8, uint8_t* __restrict__ s8,
                                                      float* __restrict__ ss8, float* __restrict__ xp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t xr = (int64_t)row * kD;
  float v[6];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    v[i] = load_res<R16>(x, xr + lane + 64 * i);
    ss += v[i] * v[i];
  }
  ss = wave_sum(ss);
  const float den = sqrtf(ss) * kInvSqrtD + kRmsEps;
  float ssq = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float y = w[lane + 64 * i] * (v[i] / den);
    store_res<R16>(x, xr + lane + 64 * i, y);
    if (!R16 && xp) xp[xpk_off(row, lane + 64 * i, kD)] = y;
    if (shadow) store_shadow(shadow, plane, (int64_t)row * kD + lane + 64 * i, y);
    if (q8) {
      // fp8 mode: the MXFP8 form of the bf16 shadow row for the next layer's FFN up-projection, as
      // quant_mx_kernel (gemm_mx.hip) makes it from the shadow: element lane + 64 i lies in 32-block
      // 2 i + (lane >> 5), whose max |v| is a reduction over its 32 lanes
      const float vb = (float)(__bf16)y;
      ssq = fmaf(vb, vb, ssq);
      float am = fabsf(vb);
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
      const int e = mx_exp(am);
      q8[(int64_t)row * kD + lane + 64 * i] = (uint8_t)(mx_cvt2<false>(vb, 0.f, mx_scale(e), 0u) & 0xff);
      if ((lane & 31) == 0) s8[(int64_t)row * (kD / 32) + 2 * i + (lane >> 5)] = (uint8_t)e;
    }
  }
  if (q8 && ss8) {   // the sum-of-squares slab as quant_mx writes it: {ss, 0, ...}
    ssq = wave_sum(ssq);
    if (lane < kSsSlots) ss8[(int64_t)row * kSsSlots + lane] = lane == 0 ? ssq : 0.f;
  }
}

hipError_t launch_rmsnorm(void* x, const float* w, int rows, uint16_t* shadow, int64_t plane, bool r16, hipStream_t st,
                          uint8_t* q8, uint8_t* s8, float* ss8, float* xp) {
  if (r16 && xp) return hipErrorInvalidValue;   // the packed copy is fp32 (gemm_d3n's A)
  if (r16)
    hipLaunchKernelGGL(rmsnorm_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, rows, shadow, plane, q8, s8, ss8,
                       xp);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, rows, shadow, plane, q8, s8, ss8,
                       xp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Layers 14/15 MHSA input cache.  EncoderState.update_before_layer slices the stored 30-row cache
// to its last S rows (conformer_blocks.py:147-148); MultiHeadAttention.update_state attends over
// kv = [cache_S ; xn] and keeps [cache_S[T:] ; xn] (submodules.py:295-302); update_after_layer
// left-pads it with zeros to 30 rows (conformer_blocks.py:161-163).  xn = norm_self_att(r).
// norm_self_att of one residual row held by a wave (6 values per lane): ss by an explicit fma chain, den = fma(sqrt(ss),
// 1/sqrt(384), eps), y = w (v / den) rounded to fp32 -- with contraction off, so that the flat and the resident kernels
// (and every store of y: fp32 / bf16 activations, the fp16 cache) see the same bits whatever the compiler fuses around
// them (left to itself it summed ss with an fma chain in one kernel and with paired products in the other, and fused
// the product into the fp16 conversion as a v_fma_mixlo for some rows only).
template <bool OBF>
__device__ __forceinline__ void mhsa_norm_row(const void* __restrict__ r, int64_t xr, const float* __restrict__ norm_w,
                                              int lane, float (&y)[6]) {
#pragma clang fp contract(off)
  float v[6], ss = 0.f;
#pragma unroll
  for (int e = 0; e < 6; ++e) { v[e] = load_res<OBF>(r, xr + lane + 64 * e); ss = fmaf(v[e], v[e], ss); }
  ss = wave_sum(ss);
  const float den = fmaf(sqrtf(ss), kInvSqrtD, kRmsEps);
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    y[e] = norm_w[lane + 64 * e] * (v[e] / den);
    asm("" : "+v"(y[e]));   // y is an fp32 value from here on: no fusing the product into a later conversion
  }
}

template <bool OBF>
__global__ void __launch_bounds__(256) kv_assemble_kernel(const void* __restrict__ r, const float* __restrict__ norm_w,
                                                          StateRef s, int layer_slot, int T, int S,
                                                          void* __restrict__ xn, void* __restrict__ kv) {
  // grid (B, ns): workgroup y takes rows 4y..4y+3 and every ns-th 256-element block of the state
  // copies; ns = 4 at small batch (four workgroups per stream: the copies are latency-bound there; at
  // B = 2048 one workgroup per stream is faster, 85 vs 104 us per step)
  const int b = blockIdx.x, y = blockIdx.y, ns = gridDim.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t sec = kOffMhsa + (int64_t)layer_slot * kMhsaS * kD;
  const int64_t cache = s.row_in(b) + sec, cache_out = s.row_out(b) + sec;
  const int TK = S + T;
  // normalized current rows
  for (int i = 4 * y + wid; i < T; i += 4 * ns) {
    const int64_t xr = ((int64_t)b * T + i) * kD;   // the residual stream: fp16 in the bf16 / fp8 modes (OBF)
    float v[6];
    mhsa_norm_row<OBF>(r, xr, norm_w, lane, v);
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int c = lane + 64 * e;
      const float y = v[e];
      store_act<OBF>(xn, ((int64_t)b * T + i) * kD + c, y);
      store_act<OBF>(kv, ((int64_t)b * TK + S + i) * kD + c, y);
      // new cache row (30 - S) + (S - T + i) = 30 - T + i holds xn[i]
      s.out[cache_out + (int64_t)(kMhsaS - T + i) * kD + c] = __float2half_rn(y);
    }
  }
  // cached rows: stored rows 30-S .. 29
  for (int i = tid + 256 * y; i < S * kD; i += 256 * ns) {
    const int j = i / kD, c = i % kD;
    store_act<OBF>(kv, ((int64_t)b * TK + j) * kD + c, __half2float(s.in[cache + (int64_t)(kMhsaS - S + j) * kD + c]));
  }
  // new cache rows 0 .. 30-T-1: zero padding below 30-S, then cache_S[T:]
  for (int i = tid + 256 * y; i < (kMhsaS - T) * kD; i += 256 * ns) {
    const int rr = i / kD, c = i % kD;
    __half h = __float2half_rn(0.f);
    if (rr >= kMhsaS - S) h = s.in[cache + (int64_t)(rr + T) * kD + c];
    s.out[cache_out + (int64_t)rr * kD + c] = h;
  }
}

// The same on the resident form (common.h StateRef): the layer's 30 cached frames in the stream's ring (frame i at row
// (ph + i) mod 30), one workgroup per stream.  kv's cached rows are the ring's frames 30 - S .. 29; after a workgroup
// barrier (those reads done) the T new xn rows go over the T oldest ring rows ph .. ph + T - 1 -- no rewrite of the
// S - T kept rows or of layer 14's zero padding.  Same arithmetic as kv_assemble_kernel.
template <bool OBF>
__global__ void __launch_bounds__(256) kv_assemble_ring_kernel(const void* __restrict__ r, const float* __restrict__ norm_w,
                                                               StateRef s, int layer_slot, int T, int S,
                                                               void* __restrict__ xn, void* __restrict__ kv) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ph = ring_phase(s.chunk_counter(b), T);
  __half* rg = s.ring + (int64_t)s.ring_ids[b] * kRingElems + kRingConv + (int64_t)layer_slot * kMhsaS * kD;
  const int TK = S + T;
  constexpr int kMaxRowsPerWave = (kTMax + 3) / 4;
  float y[kMaxRowsPerWave][6];
  // normalized current rows (wave w: rows w, w + 4, ...)
#pragma unroll
  for (int q = 0; q < kMaxRowsPerWave; ++q) {
    const int i = wid + 4 * q;
    if (i >= T) break;
    const int64_t xr = ((int64_t)b * T + i) * kD;
    mhsa_norm_row<OBF>(r, xr, norm_w, lane, y[q]);
#pragma unroll
    for (int e = 0; e < 6; ++e) {
      const int c = lane + 64 * e;
      store_act<OBF>(xn, ((int64_t)b * T + i) * kD + c, y[q][e]);
      store_act<OBF>(kv, ((int64_t)b * TK + S + i) * kD + c, y[q][e]);
    }
  }
  // cached rows: ring frames 30 - S .. 29, eight channels per thread (ring rows and kv rows are 16-byte aligned)
  for (int i = tid; i < S * (kD / 8); i += 256) {
    const int j = i / (kD / 8), c = (i % (kD / 8)) * 8;
    const int fr = (ph + kMhsaS - S + j) % kMhsaS;
    const uint4 h = *reinterpret_cast<const uint4*>(rg + (int64_t)fr * kD + c);
    const __half* hv = reinterpret_cast<const __half*>(&h);
    const int64_t o = ((int64_t)b * TK + j) * kD + c;
    if constexpr (OBF) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 lo = (__bf16)__half2float(hv[2 * e]), hi = (__bf16)__half2float(hv[2 * e + 1]);
        w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
      }
      *reinterpret_cast<uint4*>(static_cast<uint16_t*>(kv) + o) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      float* d = static_cast<float*>(kv) + o;
      *reinterpret_cast<float4*>(d) = make_float4(__half2float(hv[0]), __half2float(hv[1]), __half2float(hv[2]),
                                                  __half2float(hv[3]));
      *reinterpret_cast<float4*>(d + 4) = make_float4(__half2float(hv[4]), __half2float(hv[5]), __half2float(hv[6]),
                                                      __half2float(hv[7]));
    }
  }
  __syncthreads();   // every ring read of this stream is done before its oldest rows are overwritten
#pragma unroll
  for (int q = 0; q < kMaxRowsPerWave; ++q) {
    const int i = wid + 4 * q;
    if (i >= T) break;
    const int row = ph + i < kMhsaS ? ph + i : ph + i - kMhsaS;
#pragma unroll
    for (int e = 0; e < 6; ++e) rg[(int64_t)row * kD + lane + 64 * e] = __float2half_rn(y[q][e]);
  }
}

hipError_t launch_kv_assemble(const void* r, const float* norm_w, StateRef s, int layer_slot, int T, int S, void* xn,
                              void* kv, bool obf, int B, hipStream_t st) {
  if (s.ring) {
    if (obf) hipLaunchKernelGGL(kv_assemble_ring_kernel<true>, dim3(B), dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
    else hipLaunchKernelGGL(kv_assemble_ring_kernel<false>, dim3(B), dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
    return hipGetLastError();
  }
  const dim3 grid(B, B >= 1024 ? 1 : 4);
  if (obf) hipLaunchKernelGGL(kv_assemble_kernel<true>, grid, dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
  else hipLaunchKernelGGL(kv_assemble_kernel<false>, grid, dim3(256), 0, st, r, norm_w, s, layer_slot, T, S, xn, kv);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// RotaryMultiHeadAttention.forward (conformer_blocks.py:688-726) + forward_qkv/forward_attention
// (submodules.py:204-271).  One wave per (stream, head), four heads per 256-thread workgroup;
// every wave works in its own small LDS slice, so the kernel has no workgroup barrier.
//   shared layers (this kernel): probabilities of the last recomputing layer (no mask in layers 1-6 / 8-13, so
//   softmax(shared scores) = shared probabilities), read from the probs buffer; ctx = P . V: lane c < 48 owns output
//   column c, its T values of V are loaded straight into registers at kernel start (one coalesced row per load), P
//   rows are read from LDS as broadcast float4s, the T output rows accumulate independently.
//   recomputing layers: attention_rec_kernel below (LayerNorm + RoPE + scores + softmax + P . V).
template <int T, bool OBF>
__global__ void __launch_bounds__(256) attention_kernel(AttnArgs a) {
  constexpr int TK = T, TKP = (TK + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float sm[4][T * TKP];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int b = blockIdx.x >> 1, h = ((blockIdx.x & 1) << 2) + wid;
  float* ps = sm[wid];                        // [T][TKP]
  const int c0 = h * kDk;
  const int cl = min(lane, kDk - 1);
  float vr[TK];                               // V column cl, all keys (issued first: in flight meanwhile)
#pragma unroll
  for (int j = 0; j < TK; ++j) vr[j] = load_act<OBF>(a.v, ((int64_t)b * TK + j) * a.ldv + c0 + cl);
  const float* pp = a.probs + ((int64_t)b * kHeads + h) * T * TK;
  for (int e = lane; e < T * TK; e += 64) ps[(e / TK) * TKP + e % TK] = pp[e];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float acc[T];
#pragma unroll
  for (int i = 0; i < T; ++i) acc[i] = 0.f;
#pragma unroll
  for (int j4 = 0; j4 < TKP / 4; ++j4) {
#pragma unroll
    for (int i = 0; i < T; ++i) {
      const float4 p4 = *reinterpret_cast<const float4*>(ps + i * TKP + 4 * j4);
      acc[i] = fmaf(p4.x, vr[4 * j4], acc[i]);
      if (4 * j4 + 1 < TK) acc[i] = fmaf(p4.y, vr[4 * j4 + 1], acc[i]);
      if (4 * j4 + 2 < TK) acc[i] = fmaf(p4.z, vr[4 * j4 + 2], acc[i]);
      if (4 * j4 + 3 < TK) acc[i] = fmaf(p4.w, vr[4 * j4 + 3], acc[i]);
    }
  }
  if (lane < kDk) {
#pragma unroll
    for (int i = 0; i < T; ++i) store_act<OBF>(a.ctx, act_off((int64_t)b * T + i, c0 + lane, kD, !OBF && a.ctx_packed), acc[i]);
  }
}

// Recomputing layers (0, 7, 14, 15) on the matrix pipe.  One wave per (stream, head) as above, but the lanes are
// (row, dim group): lane l = 16 g + r holds the 12 dims {4g .. 4g+3, 16+4g .. 16+4g+3, 32+4g .. 32+4g+3} of row r of
// a 16-row tile (three 4-element vector loads), which is at once
//   * the LayerNorm layout: the row's sums closed by two lane exchanges (xor 16, xor 32); each RoPE pair (d, d + 16),
//     d < 16, sits in one lane (elements m and m + 4);
//   * the operand layout of v_mfma_f32_16x16x4_f32 (lane l: A[l & 15][l >> 4], B[l >> 4][l & 15]): step m's k slot g
//     is dim 16 (m >> 2) + 4 g + (m & 3) for both Q and K, so the 12 steps sum all 48 products (exact fp32 fmas; the
//     order of the dims differs from a d-ordered chain, within the fp32 tolerance of the parity tests).
// Scores are computed transposed, S^T = K Q^T (tile t: keys 16 t .. 16 t + 15), so a lane ends with keys
// 16 t + 4 g + rr of query r: the softmax over keys is an in-lane reduction plus xor 16 / xor 32, and the
// probabilities are already the A operand of ctx = P V (k slot g of step s <-> key 16 t + 4 g + s).  V goes to the
// wave's LDS slice by LDS-DMA (4-8 instructions) and is read back in that order.  Every operand load is a vector
// load: the texture-address unit processes a wave's 64 addresses per instruction, so 165 two-byte loads per wave cost
// more than the arithmetic they replaced (measured 260 us at S + T = 40).  The round-3 kernel ran the 48-dim
// LayerNorms and the dot products serially in T or S + T lanes of 64 (VALU-bound: 118-144 us per launch at B = 4096).
template <int T, int S, bool OBF>
__global__ void __launch_bounds__(256) attention_rec_kernel(AttnArgs a) {
  constexpr int TK = S + T, NJT = (TK + 15) / 16;
  constexpr int ES = OBF ? 2 : 4;                                   // bytes per activation element
  constexpr int VPC = kDk * ES / 16;                                // 16-byte pieces per V row (6 | 12)
  constexpr int VINS = (TK * VPC + 63) / 64;                        // LDS-DMA instructions per wave
  static_assert(T <= 16, "one query tile");
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t vs[4][VINS * 1024];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int b = blockIdx.x >> 1, h = ((blockIdx.x & 1) << 2) + wid;
  const int c0 = h * kDk, r16 = lane & 15, g = lane >> 4;
  // V rows -> LDS (row j at j * 48 * ES bytes)
#pragma unroll
  for (int in = 0; in < VINS; ++in) {
    const int pc = min(in * 64 + lane, TK * VPC - 1), j = pc / VPC, e = (pc % VPC) * (16 / ES);
    const uint8_t* src = static_cast<const uint8_t*>(a.v) + (((int64_t)b * TK + j) * a.ldv + c0 + e) * ES;
    lds_dma16(src, vs[wid] + in * 1024);
  }
  // Q and K rows, three 4-element loads per row
  auto load_row = [&](const void* base, int64_t row, float (&x)[12]) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float4 v = load_act4<OBF>(base, row + c0 + 16 * ch + 4 * g);
      x[4 * ch] = v.x; x[4 * ch + 1] = v.y; x[4 * ch + 2] = v.z; x[4 * ch + 3] = v.w;
    }
  };
  float q[12], kk[NJT][12];
  load_row(a.q, ((int64_t)b * T + min(r16, T - 1)) * a.ldq, q);
#pragma unroll
  for (int t = 0; t < NJT; ++t) load_row(a.k, ((int64_t)b * TK + min(16 * t + r16, TK - 1)) * a.ldk, kk[t]);
  auto load_w = [&](const float* w, float (&x)[12]) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float4 v = *reinterpret_cast<const float4*>(w + 16 * ch + 4 * g);
      x[4 * ch] = v.x; x[4 * ch + 1] = v.y; x[4 * ch + 2] = v.z; x[4 * ch + 3] = v.w;
    }
  };
  // LayerNorm(48, eps 1e-5) + RoPE on dims [0, 32) of the row this lane's 12 dims belong to (pos = RoPE position)
  auto ln_rope = [&](float (&x)[12], const float (&lw)[12], const float (&lb)[12], int pos) {
    float sum = 0.f;
#pragma unroll
    for (int m = 0; m < 12; ++m) sum += x[m];
    sum = lg_sum(sum);
    const float mu = sum * (1.0f / kDk);
    float var = 0.f;
#pragma unroll
    for (int m = 0; m < 12; ++m) {
      x[m] -= mu;
      var += x[m] * x[m];
    }
    var = lg_sum(var);
    const float rstd = 1.0f / sqrtf(var * (1.0f / kDk) + kLnEps);
#pragma unroll
    for (int m = 0; m < 12; ++m) x[m] = x[m] * rstd * lw[m] + lb[m];
    const float4 cs = *reinterpret_cast<const float4*>(a.rope_cos + (pos + kMhsaS) * (kRope / 2) + 4 * g);
    const float4 sn = *reinterpret_cast<const float4*>(a.rope_sin + (pos + kMhsaS) * (kRope / 2) + 4 * g);
#pragma unroll
    for (int m = 0; m < 4; ++m) {                       // rotate_half pairs (d, d + 16), submodules.py:142-157
      const float y0 = x[m], y1 = x[m + 4];
      x[m] = y0 * cs[m] - y1 * sn[m];
      x[m + 4] = y1 * cs[m] + y0 * sn[m];
    }
  };
  {
    float lw[12], lb[12];
    load_w(a.qln_w, lw);
    load_w(a.qln_b, lb);
    ln_rope(q, lw, lb, min(r16, T - 1));
  }
  f32x4 st[NJT];
  {
    float lw[12], lb[12];
    load_w(a.kln_w, lw);
    load_w(a.kln_b, lb);
#pragma unroll
    for (int t = 0; t < NJT; ++t) {
      ln_rope(kk[t], lw, lb, min(16 * t + r16, TK - 1) - S);
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 12; ++m) st[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(kk[t][m], q[m], st[t], 0, 0, 0);
    }
  }
  // softmax over the keys of query i = r16 (this lane: keys 16 t + 4 g + rr)
  float off = -1e30f;
  if constexpr (S > 0) {
    off = (float)kMhsaS - __half2float(a.s.in[a.s.row_in(b) + kOffMhsaLen]);
    if (a.reduced) off = floorf(off / 2.0f);
  }
  const int i = r16;
  float x[NJT][4];
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < NJT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int j = 16 * t + 4 * g + rr;
      const float sc = st[t][rr] * 0.14433756729740643f;  // / math.sqrt(48) (submodules.py:185), as a product
      const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
      x[t][rr] = j < TK ? (masked ? -10000.0f : sc) : -INFINITY;
      mx = fmaxf(mx, x[t][rr]);
    }
  mx = lg_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < NJT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int j = 16 * t + 4 * g + rr;
      x[t][rr] = j < TK ? expf(x[t][rr] - mx) : 0.f;
      sum += x[t][rr];
    }
  sum = lg_sum(sum);   // v_permlane16/32_swap, the same association as the two xor shuffles
  const float rsum = 1.0f / sum;                        // one division per lane, not one per probability
  float* pr = a.probs ? a.probs + (((int64_t)b * kHeads + h) * T + i) * TK : nullptr;
#pragma unroll
  for (int t = 0; t < NJT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int j = 16 * t + 4 * g + rr;
      const bool masked = (S > 0) && (((float)j < off) || ((float)(S + i) < off));
      x[t][rr] = masked ? 0.f : x[t][rr] * rsum;
      if (pr && i < T && j < TK) pr[j] = x[t][rr];
    }
  // ctx = P V: D[query][column], lane: queries 4 g + rr, column 16 ct + r16; V from the LDS slice
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                 // the V DMA (this wave's own)
  const uint8_t* vb = vs[wid];
  f32x4 cx[3];
#pragma unroll
  for (int ct = 0; ct < 3; ++ct) cx[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NJT; ++t)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int j = min(16 * t + 4 * g + s4, TK - 1);
#pragma unroll
      for (int ct = 0; ct < 3; ++ct) {
        const int e = j * kDk + 16 * ct + r16;
        float v;
        if constexpr (OBF) v = __builtin_bit_cast(float, (uint32_t)(*reinterpret_cast<const uint16_t*>(vb + 2 * e)) << 16);
        else v = *reinterpret_cast<const float*>(vb + 4 * e);
        cx[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[t][s4], v, cx[ct], 0, 0, 0);
      }
    }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int iq = 4 * g + rr;
    if (iq < T) {
#pragma unroll
      for (int ct = 0; ct < 3; ++ct)
        store_act<OBF>(a.ctx, act_off((int64_t)b * T + iq, c0 + 16 * ct + r16, kD, !OBF && a.ctx_packed), cx[ct][rr]);
    }
  }
}

template <bool OBF>
static hipError_t launch_attention_t(const AttnArgs& a, hipStream_t st) {
  const dim3 grid(a.B * 2), block(256);
  // (T, S) of the 300 ms chunk: (10 | 5, 0), layer 14 (5, 15), layer 15 (10, 30); 400 ms: T 13 | 6
  if (!a.recompute) {
    if (a.S != 0) return hipErrorInvalidValue;
    if (a.T == 10) hipLaunchKernelGGL((attention_kernel<10, OBF>), grid, block, 0, st, a);
    else if (a.T == 5) hipLaunchKernelGGL((attention_kernel<5, OBF>), grid, block, 0, st, a);
    else if (a.T == 13) hipLaunchKernelGGL((attention_kernel<13, OBF>), grid, block, 0, st, a);
    else if (a.T == 6) hipLaunchKernelGGL((attention_kernel<6, OBF>), grid, block, 0, st, a);
    else return hipErrorInvalidValue;
  } else if (a.T == 10 && a.S == 0) hipLaunchKernelGGL((attention_rec_kernel<10, 0, OBF>), grid, block, 0, st, a);
  else if (a.T == 5 && a.S == 0) hipLaunchKernelGGL((attention_rec_kernel<5, 0, OBF>), grid, block, 0, st, a);
  else if (a.T == 5 && a.S == 15) hipLaunchKernelGGL((attention_rec_kernel<5, 15, OBF>), grid, block, 0, st, a);
  else if (a.T == 10 && a.S == 30) hipLaunchKernelGGL((attention_rec_kernel<10, 30, OBF>), grid, block, 0, st, a);
  else if (a.T == 13 && a.S == 0) hipLaunchKernelGGL((attention_rec_kernel<13, 0, OBF>), grid, block, 0, st, a);
  else if (a.T == 6 && a.S == 0) hipLaunchKernelGGL((attention_rec_kernel<6, 0, OBF>), grid, block, 0, st, a);
  else if (a.T == 6 && a.S == 15) hipLaunchKernelGGL((attention_rec_kernel<6, 15, OBF>), grid, block, 0, st, a);
  else if (a.T == 13 && a.S == 30) hipLaunchKernelGGL((attention_rec_kernel<13, 30, OBF>), grid, block, 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_attention(const AttnArgs& a, hipStream_t st) {
  if (a.ctx_bf16 && a.ctx_packed) return hipErrorInvalidValue;   // the packed layout is fp32 (gemm_d3's A)
  return a.ctx_bf16 ? launch_attention_t<true>(a, st) : launch_attention_t<false>(a, st);
}

// ---------------------------------------------------------------------------------------------
// ConformerConvolution depthwise part (conformer_blocks.py:427-433, submodules.py:364-402):
//   x = [conv state (30) ; g (T)] per channel; next state = x[-30:]; g (the GLU output) and out are bf16 in the
//   bf16 / fp8 modes (OBF), fp32 in fp32 mode
//   out[t] = SiLU(BN(bias + sum_k w[k] x[t+k]))  with BN folded into (w, b) on the host.
// A workgroup of CPW threads (a thread per channel) handles NS streams x CPW channels, the channel's 31
// taps (stored tap-major) in registers: 192 x 1 stream at large batch, 128 x 1 at small batch (B = 256:
// 768 workgroups instead of 128); the shapes measure within 1.5 % of each other once the new frames
// are loaded ahead of the state barrier (profiles/r01_dwconv_sweep.txt).  Each stream's slice of the 23 KB conv-state section (CPW x 30 halves)
// is moved HBM<->LDS in 16-byte vectors: state rows are only 2-byte aligned, so the slice is read from
// the enclosing 16-byte-aligned window and the two partial end vectors are written element-wise.
constexpr int kDwSec = kD * kConvS;          // 11520 halves per (stream, layer)
template <int T, bool OBF, int CPW, int NS>
__global__ void __launch_bounds__(CPW) dwconv_kernel(const void* __restrict__ g, StateRef s, int layer,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     void* __restrict__ out, int B, int opk) {
  constexpr int kSec = CPW * kConvS;           // halves of this workgroup's slice
  constexpr int kVec = kSec / 8 + 1;           // 16-byte vectors covering a misaligned slice
  __shared__ uint4 lds[NS][kVec];
  const int c = threadIdx.x, ch0 = blockIdx.y * CPW, ch = ch0 + c;
  int shift[NS], nvec[NS];
  int64_t base[NS];
  const int64_t sec = kOffConv + (int64_t)layer * kDwSec + ch0 * kConvS;
#pragma unroll
  for (int si = 0; si < NS; ++si) {
    const int b = min(blockIdx.x * NS + si, B - 1);
    base[si] = s.row_in(b) + sec;
    const uintptr_t a = reinterpret_cast<uintptr_t>(s.in + base[si]);
    shift[si] = (int)((a & 15) >> 1);
    nvec[si] = (shift[si] + kSec + 7) >> 3;
    const uint4* q = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
    for (int v = c; v < nvec[si]; v += CPW) lds[si][v] = q[v];
  }
  float wr[kConvK];
#pragma unroll
  for (int k = 0; k < kConvK; ++k) wr[k] = w[k * kD + ch];
  const float bb = bias[ch];
  float gx[NS][T];   // the new frames, loaded under the state copy's latency
#pragma unroll
  for (int si = 0; si < NS; ++si) {
    const int b = min(blockIdx.x * NS + si, B - 1);
#pragma unroll
    for (int t = 0; t < T; ++t) gx[si][t] = load_act<OBF>(g, ((int64_t)b * T + t) * kD + ch);
  }
  __syncthreads();
#pragma unroll
  for (int si = 0; si < NS; ++si) {
    const int b = blockIdx.x * NS + si;
    if (b >= B) break;
    __half* h = reinterpret_cast<__half*>(lds[si]) + shift[si] + c * kConvS;
    float x[kConvS + T];
#pragma unroll
    for (int t = 0; t < T; ++t) x[kConvS + t] = gx[si][t];
#pragma unroll
    for (int i = 0; i < kConvS; ++i) x[i] = __half2float(h[i]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float acc = bb;
#pragma unroll
      for (int k = 0; k < kConvK; ++k) acc = fmaf(wr[k], x[t + k], acc);
      // bf16 output: SiLU on v_exp_f32 / v_rcp_f32 as the conv epilogues (a few ulp of fp32 before the bf16
      // rounding; the IEEE expf + division was a third of the kernel's VALU); fp32 output: IEEE exp / division
      float y;
      if constexpr (OBF) y = acc * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc * -1.4426950408889634f));
      else y = silu_f(acc);
      store_act<OBF>(out, act_off((int64_t)b * T + t, ch, kD, !OBF && opk), y);
    }
#pragma unroll
    for (int i = 0; i < kConvS; ++i) h[i] = __float2half_rn(x[T + i]);
  }
  __syncthreads();
#pragma unroll
  for (int si = 0; si < NS; ++si) {
    const int b = blockIdx.x * NS + si;
    if (b >= B) break;
    __half* dst = s.out + s.row_out(b) + sec;
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    const int sh = (int)((a & 15) >> 1);
    const __half* src = reinterpret_cast<const __half*>(lds[si]) + shift[si];
    if (sh == shift[si]) {
      uint4* q = reinterpret_cast<uint4*>(a & ~uintptr_t(15));
      const int n = nvec[si];
      for (int v = c; v < n; v += CPW) {
        if ((v == 0 && sh) || (v == n - 1 && ((sh + kSec) & 7))) {
          const int e0 = v * 8 - sh;
          for (int e = max(e0, 0); e < min(e0 + 8, kSec); ++e) dst[e] = src[e];
        } else {
          q[v] = lds[si][v];
        }
      }
    } else {  // output slab aligned differently from the input slab
      for (int e = c; e < kSec; e += CPW) dst[e] = src[e];
    }
  }
}

// The same op on the resident form (common.h StateRef: the layer's 30 cached frames in the stream's ring, time-major
// [30][384], frame i at ring row (ph + i) mod 30).  A thread takes a channel pair of one stream: every load and store is
// a coalesced row segment (the flat form's [384][30] channel-major section needs the LDS staging above), and only the
// T new frames are written back, over the T oldest (ring rows ph .. ph + T - 1), instead of the whole shifted window:
// 30 + 3 T frames of HBM traffic per stream and layer instead of 60 + 2 T.  Arithmetic identical to dwconv_kernel
// (same fma order, same SiLU forms): outputs and the exported state are bit-identical to the flat form's.
template <int T, bool OBF, bool NTH>
__global__ void __launch_bounds__(kD / 2) dwconv_ring_kernel(const void* __restrict__ g, StateRef s, int layer,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            void* __restrict__ out, int opk) {
  const int b = blockIdx.x, c = 2 * threadIdx.x;
  const int ph = ring_phase(s.chunk_counter(b), T);
  __half* rg = s.ring + (int64_t)s.ring_ids[b] * kRingElems + (int64_t)layer * kConvS * kD + c;
  float x[kConvS + T][2];
#pragma unroll
  for (int i = 0; i < kConvS; ++i) {
    const int r = ph + i < kConvS ? ph + i : ph + i - kConvS;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(rg + (int64_t)r * kD);
    const __half2 h = __builtin_bit_cast(__half2, NTH ? __builtin_nontemporal_load(src) : *src);
    x[i][0] = __low2float(h);
    x[i][1] = __high2float(h);
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int64_t gi = ((int64_t)b * T + t) * kD + c;
    x[kConvS + t][0] = load_act<OBF>(g, gi);
    x[kConvS + t][1] = load_act<OBF>(g, gi + 1);
  }
  float wr[kConvK][2];
#pragma unroll
  for (int k = 0; k < kConvK; ++k) {
    const float2 wv = *reinterpret_cast<const float2*>(w + k * kD + c);
    wr[k][0] = wv.x;
    wr[k][1] = wv.y;
  }
  const float2 bb = *reinterpret_cast<const float2*>(bias + c);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    float y[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float acc = e ? bb.y : bb.x;
#pragma unroll
      for (int k = 0; k < kConvK; ++k) acc = fmaf(wr[k][e], x[t + k][e], acc);
      if constexpr (OBF) y[e] = acc * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc * -1.4426950408889634f));
      else y[e] = silu_f(acc);
    }
    const int64_t oi = act_off((int64_t)b * T + t, c, kD, !OBF && opk);   // c even: c, c + 1 adjacent packed too
    store_act<OBF>(out, oi, y[0]);
    store_act<OBF>(out, oi + 1, y[1]);
  }
  // the T new frames over the T oldest: ring rows ph .. ph + T - 1 (mod 30)
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int r = ph + j < kConvS ? ph + j : ph + j - kConvS;
    const __half2 v = __floats2half2_rn(x[kConvS + j][0], x[kConvS + j][1]);
    uint32_t* dst = reinterpret_cast<uint32_t*>(rg + (int64_t)r * kD);
    if constexpr (NTH) __builtin_nontemporal_store(__builtin_bit_cast(uint32_t, v), dst);
    else *dst = __builtin_bit_cast(uint32_t, v);
  }
}

template <int T, bool OBF>
static hipError_t launch_dwconv_t(const void* g, StateRef s, int layer, const float* w, const float* b, void* out,
                                  int B, int opk, hipStream_t st) {
  if (s.ring) {
    // the ring's rows read / written non-temporally (each read once per step, 16 layers apart: nothing worth keeping in
    // L2 / MALL): bf16 B = 4096 dwconv 615 -> 586 us per step, the step 8615 -> 8500 (the other kernels' lines stay
    // cached; profiles/r06_ring_nt_ab.txt); TONE_RING_NT=0 turns it off
    if (knobs().ring_nt)
      hipLaunchKernelGGL((dwconv_ring_kernel<T, OBF, true>), dim3(B), dim3(kD / 2), 0, st, g, s, layer, w, b, out, opk);
    else
      hipLaunchKernelGGL((dwconv_ring_kernel<T, OBF, false>), dim3(B), dim3(kD / 2), 0, st, g, s, layer, w, b, out, opk);
    return hipGetLastError();
  }
  // block shape by batch: 192 channels x 1 stream from B = 1024, else 128 x 1 (profiles/r01_dwconv_sweep.txt,
  // r03_dwconv_sweep.txt)
  if (B >= 1024)
    hipLaunchKernelGGL((dwconv_kernel<T, OBF, 192, 1>), dim3(B, 2), dim3(192), 0, st, g, s, layer, w, b, out, B, opk);
  else
    hipLaunchKernelGGL((dwconv_kernel<T, OBF, 128, 1>), dim3(B, kD / 128), dim3(128), 0, st, g, s, layer, w, b, out, B,
                       opk);
  return hipGetLastError();
}

hipError_t launch_dwconv(const void* g, StateRef s, int layer, const float* w, const float* b, void* out, bool obf,
                         int T, int B, hipStream_t st, bool out_packed) {
  if (obf && out_packed) return hipErrorInvalidValue;   // the packed layout is fp32 (gemm_d3's A)
  const int pk = out_packed;
  if (T == kT) return obf ? launch_dwconv_t<kT, true>(g, s, layer, w, b, out, B, pk, st)
                          : launch_dwconv_t<kT, false>(g, s, layer, w, b, out, B, pk, st);
  if (T == kT / 2) return obf ? launch_dwconv_t<kT / 2, true>(g, s, layer, w, b, out, B, pk, st)
                              : launch_dwconv_t<kT / 2, false>(g, s, layer, w, b, out, B, pk, st);
  if (T == 13) return obf ? launch_dwconv_t<13, true>(g, s, layer, w, b, out, B, pk, st)     // 400 ms chunks
                          : launch_dwconv_t<13, false>(g, s, layer, w, b, out, B, pk, st);
  if (T == 6) return obf ? launch_dwconv_t<6, true>(g, s, layer, w, b, out, B, pk, st)
                         : launch_dwconv_t<6, false>(g, s, layer, w, b, out, B, pk, st);
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// CausalTemporalReduction.forward streaming branch (conformer_blocks.py:888-907), grouped part:
//   x = [state (1) ; x^T (T)] per channel; next state = x[:, -1:]
//   y[o][t] = bias[o] + sum_{k<3} w[o][k] x[o/4][2t+k], o < 1536, t < Tr = (T + 1 - 3) / 2 + 1
//   (no padding in the streaming branch: T = 13 gives Tr = 6 and leaves the last frame to the state)
template <bool OBF, int T>
__global__ void __launch_bounds__(256) reduce_conv_kernel(const void* __restrict__ x, StateRef s,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          void* __restrict__ y, int B, int ypk) {
  constexpr int TR = (T + 1 - 3) / 2 + 1;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * kD) return;
  const int b = idx / kD, c = idx % kD;
  float xc[T + 1];
  xc[0] = __half2float(s.in[s.row_in(b) + kOffRed + c]);
  for (int t = 0; t < T; ++t) xc[t + 1] = load_res<OBF>(x, ((int64_t)b * T + t) * kD + c);   // fp16 residual when OBF
  s.out[s.row_out(b) + kOffRed + c] = __float2half_rn(xc[T]);
  if (!OBF && ypk) {   // packed y (gemm_d3's A): the 4 outputs of this channel are one 16-byte run there too
    float wq[4][3], bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = 4 * c + q;
      wq[q][0] = w[o * 3]; wq[q][1] = w[o * 3 + 1]; wq[q][2] = w[o * 3 + 2]; bq[q] = bias[o];
    }
    for (int t = 0; t < TR; ++t) {
      f32x4_t v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = bq[q] + wq[q][0] * xc[2 * t] + wq[q][1] * xc[2 * t + 1] + wq[q][2] * xc[2 * t + 2];
      *reinterpret_cast<f32x4_t*>(static_cast<float*>(y) + xpk_off((int64_t)b * TR + t, 4 * c, 4 * kD)) = v;
    }
    return;
  }
  for (int q = 0; q < 4; ++q) {
    const int o = 4 * c + q;
    const float w0 = w[o * 3], w1 = w[o * 3 + 1], w2 = w[o * 3 + 2], bo = bias[o];
    for (int t = 0; t < TR; ++t)
      store_act<OBF>(y, ((int64_t)b * TR + t) * (4 * kD) + o, bo + w0 * xc[2 * t] + w1 * xc[2 * t + 1] + w2 * xc[2 * t + 2]);
  }
}

hipError_t launch_reduce_conv(const void* x, StateRef s, const float* w, const float* b, void* y, bool obf, int B,
                              int T, hipStream_t st, bool y_packed) {
  if (obf && y_packed) return hipErrorInvalidValue;   // the packed layout is fp32 (gemm_d3's A)
  const dim3 grid((B * kD + 255) / 256), block(256);
  const int pk = y_packed;
  if (T == kT && obf) hipLaunchKernelGGL((reduce_conv_kernel<true, kT>), grid, block, 0, st, x, s, w, b, y, B, pk);
  else if (T == kT) hipLaunchKernelGGL((reduce_conv_kernel<false, kT>), grid, block, 0, st, x, s, w, b, y, B, pk);
  else if (T == 13 && obf) hipLaunchKernelGGL((reduce_conv_kernel<true, 13>), grid, block, 0, st, x, s, w, b, y, B, pk);
  else if (T == 13) hipLaunchKernelGGL((reduce_conv_kernel<false, 13>), grid, block, 0, st, x, s, w, b, y, B, pk);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// TemporalUpsampling (conformer_blocks.py:955-988): repeat_interleave x2, right-pad 1, trim to T, + residual.
// Frames t < 2 Tr take x5[t / 2]; a frame past 2 Tr (t = 12 of a 400 ms chunk: 2 x 6 < 13) is the zero pad,
// so it keeps the residual alone.
template <bool R16>
__global__ void __launch_bounds__(256) upsample_add_kernel(void* __restrict__ x10, const void* __restrict__ x5, int B,
                                                           int T, int Tr, uint16_t* __restrict__ shadow, int64_t plane,
                                                           float* __restrict__ xp) {
  // four consecutive channels per thread (8-byte fp16 / 16-byte fp32 residual vectors, 8-byte bf16 shadow)
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (idx >= (int64_t)B * T * kD) return;
  const int64_t row = idx / kD;
  const int c = idx % kD;
  const int64_t b = row / T, t = row % T;
  f32x4_t v = load_res4(x10, idx, R16);
  if (t < 2 * Tr) v += load_res4(x5, (b * Tr + t / 2) * kD + c, R16);
  store_res4(x10, idx, v, R16);
  if (!R16 && xp) *reinterpret_cast<f32x4_t*>(xp + xpk_off(row, c, kD)) = v;   // c % 4 == 0: one 16-byte run packed too
  if (shadow) {
    if (!plane) {
      const __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
      *reinterpret_cast<uint2*>(shadow + idx) =
          make_uint2((uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16),
                     (uint32_t)__builtin_bit_cast(uint16_t, h2) | ((uint32_t)__builtin_bit_cast(uint16_t, h3) << 16));
    } else {
      store_shadow(shadow, plane, idx, v.x);
      store_shadow(shadow, plane, idx + 1, v.y);
      store_shadow(shadow, plane, idx + 2, v.z);
      store_shadow(shadow, plane, idx + 3, v.w);
    }
  }
}

hipError_t launch_upsample_add(void* x10, const void* x5, int B, int T, uint16_t* shadow, int64_t plane, bool r16,
                               hipStream_t st, float* xp) {
  if (r16 && xp) return hipErrorInvalidValue;
  const int64_t n4 = (int64_t)B * T * kD / 4;
  const int Tr = (T + 1 - 3) / 2 + 1;
  if (r16)
    hipLaunchKernelGGL(upsample_add_kernel<true>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, x10, x5, B, T, Tr,
                       shadow, plane, xp);
  else
    hipLaunchKernelGGL(upsample_add_kernel<false>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, x10, x5, B, T, Tr,
                       shadow, plane, xp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ConvASRDecoder.forward (conformer.py:338-354): 1x1 conv 384 -> 35 and log_softmax, fp32.
// Four lanes per frame row (16 rows per wave): lane l owns row l >> 2 and the k quarter l & 3
// (96 k), so each LDS read of W serves 4 distinct broadcast addresses and x rows stream through
// L1; the 35 partial sums are combined over the quarter lanes with two xor shuffles, then
// log-softmax, the greedy token and the splitter's speech flag are per-row epilogues.
//   frame_info[row] = argmax_v logp[row][v] (first index on ties, decoder.py:57)
//                   | (exp(logp[33]) + exp(logp[34]) <= 0.9) << 8      (logprob_splitter.py:134)
constexpr float kSilenceThreshold = 0.9f;
constexpr int kHeadQ = kD / 4;              // 96
constexpr int kHeadWs = kHeadQ + 4;         // padded LDS row of a W quarter (bank spread)
template <bool R16>
__global__ void __launch_bounds__(256) head_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ bias, float* __restrict__ logp,
                                                   int32_t* __restrict__ frame_info, int rows) {
  __shared__ __attribute__((aligned(16))) float ws[4 * kVocab * kHeadWs];   // [quarter][v][96 (+4)]
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < kVocab * kD / 4; i += 256) {
    const int v = (4 * i) / kD, k = (4 * i) % kD, q = k / kHeadQ, kk = k % kHeadQ;
    *reinterpret_cast<f32x4_t*>(ws + (q * kVocab + v) * kHeadWs + kk) = reinterpret_cast<const f32x4_t*>(w)[i];
  }
  __syncthreads();
  const int row = blockIdx.x * 64 + (tid >> 2), q = lane & 3;
  const int64_t xr = (int64_t)min(row, rows - 1) * kD + q * kHeadQ;   // the residual stream (fp16 when R16)
  const float* wq = ws + q * kVocab * kHeadWs;
  float acc[kVocab];
#pragma unroll
  for (int v = 0; v < kVocab; ++v) acc[v] = 0.f;
  for (int k = 0; k < kHeadQ; k += 4) {
    const f32x4_t xv = load_res4(x, xr + k, R16);
#pragma unroll
    for (int v = 0; v < kVocab; ++v) {
      const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(wq + v * kHeadWs + k);
      float a = acc[v];
      a = fmaf(wv.x, xv.x, a); a = fmaf(wv.y, xv.y, a); a = fmaf(wv.z, xv.z, a); a = fmaf(wv.w, xv.w, a);
      acc[v] = a;
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    acc[v] += __shfl_xor(acc[v], 1, 64);
    acc[v] += __shfl_xor(acc[v], 2, 64);
    acc[v] += bias[v];
    m = fmaxf(m, acc[v]);
  }
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) se += expf(acc[v] - m);
  const float lse = logf(se);
  float best = -INFINITY;
  int tok = 0;
  float lp[kVocab];
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    lp[v] = acc[v] - m - lse;
    if (lp[v] > best) { best = lp[v]; tok = v; }
  }
  if (row < rows) {
    float* dst = logp + (int64_t)row * kVocab;
#pragma unroll
    for (int v = 0; v < kVocab; ++v)
      if ((v & 3) == q) dst[v] = lp[v];                // the 4 quarter lanes split the row's stores
    if (frame_info && q == 0) {
      const float sil = expf(lp[kVocab - 2]) + expf(lp[kVocab - 1]);
      frame_info[row] = tok | ((sil <= kSilenceThreshold) ? 256 : 0);
    }
  }
}

// The same on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32): head_kernel above reads its W quarter from LDS with the 16
// row groups of a wave on the same four addresses, so the LDS pipe (1 KiB per wave-wide 16-byte read) bounds it at
// ~3400 FMAs per lane on 40 CUs at M = 2560.  Here a workgroup owns 32 rows, its four waves a quarter of K (96) each;
// lane (r = l & 31, h = l >> 5) loads row m0 + r and vocab rows r, r + 32 (zero past 34) at k = kq + 16 s + 8 h .. + 7
// straight from L2 (W is 53 KB), MFMA e of step s takes element e -- A and B over the same k.  The quarters are added
// through LDS in wave order, the 32 x 35 logit tile goes through LDS to one lane per row for the log-softmax / greedy /
// speech-flag epilogue (head_kernel's formulas), and the block's 32 contiguous logprob rows leave as one coalesced run.
typedef float f32x16h_t __attribute__((ext_vector_type(16)));
template <bool R16>
__global__ void __launch_bounds__(256) head_mfma_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ logp,
                                                        int32_t* __restrict__ frame_info, int rows) {
  __shared__ float red[3][2][16][64];                // quarters 1..3 of the two 32-column vocab tiles
  __shared__ float lg[32 * kVocab];                  // [row][v] logits, then logprobs (row stride 35: conflict-free)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 32, kq = wid * kHeadQ;
  const int64_t xr = (int64_t)min(m0 + r, rows - 1) * kD + kq + 8 * h;
  constexpr int kS = kHeadQ / 16;                    // 6 steps of 16 k
  f32x4_t xv[kS][2], wv[kS][2][2];
#pragma unroll
  for (int s = 0; s < kS; ++s) {
    xv[s][0] = load_res4(x, xr + 16 * s, R16);
    xv[s][1] = load_res4(x, xr + 16 * s + 4, R16);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int v = r + 32 * t;
      const f32x4_t* wp = reinterpret_cast<const f32x4_t*>(w + (int64_t)min(v, kVocab - 1) * kD + kq + 8 * h + 16 * s);
      const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
      wv[s][t][0] = v < kVocab ? wp[0] : z;
      wv[s][t][1] = v < kVocab ? wp[1] : z;
    }
  }
  f32x16h_t acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
  for (int s = 0; s < kS; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[s][e >> 2][e & 3], wv[s][t][e >> 2][e & 3], acc[t], 0, 0, 0);
  if (wid > 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[wid - 1][t][i][lane] = acc[t][i];
  }
  __syncthreads();
  if (wid > 0) return;
  // D tile (row, vocab): register i of lane l holds row 8 (i >> 2) + 4 h + (i & 3), column r (+ 32 t)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int v = r + 32 * t;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float a = acc[t][i];
      a += red[0][t][i][lane];
      a += red[1][t][i][lane];
      a += red[2][t][i][lane];
      if (v < kVocab) lg[(8 * (i >> 2) + 4 * h + (i & 3)) * kVocab + v] = a + bias[v];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < 32) {   // lane = row of the block
    float* z = lg + lane * kVocab;
    float m = -INFINITY;
#pragma unroll
    for (int v = 0; v < kVocab; ++v) m = fmaxf(m, z[v]);
    float se = 0.f;
#pragma unroll
    for (int v = 0; v < kVocab; ++v) se += expf(z[v] - m);
    const float lse = logf(se);
    float best = -INFINITY;
    int tok = 0;
#pragma unroll
    for (int v = 0; v < kVocab; ++v) {
      const float l = z[v] - m - lse;
      z[v] = l;
      if (l > best) { best = l; tok = v; }
    }
    if (frame_info && m0 + lane < rows) {
      const float sil = expf(z[kVocab - 2]) + expf(z[kVocab - 1]);
      frame_info[m0 + lane] = tok | ((sil <= kSilenceThreshold) ? 256 : 0);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int n = min(32, rows - m0) * kVocab;         // the block's rows are contiguous in logp
  float* dst = logp + (int64_t)m0 * kVocab;
  for (int i = lane; i < n; i += 64) dst[i] = lg[i];
}

// The same for a few rows (the drop-in's B = 1 .. 6 streams): one wave per row, lane l owns k = l + 64 i (six k), W
// read straight from L2 (no LDS staging, which the 256-row blocks amortise), the 35 partial sums combined by a
// six-step xor butterfly; then the same log-softmax / greedy / speech-flag epilogue.
template <bool R16>
__global__ void __launch_bounds__(256) head_rows_kernel(const void* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ logp,
                                                        int32_t* __restrict__ frame_info, int rows) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;                                       // wave-uniform
  const int64_t xr = (int64_t)row * kD;
  float xv[kD / 64];
#pragma unroll
  for (int i = 0; i < kD / 64; ++i) xv[i] = load_res<R16>(x, xr + lane + 64 * i);
  float acc[kVocab];
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < kD / 64; ++i) a = fmaf(w[v * kD + lane + 64 * i], xv[i], a);
    acc[v] = a;
  }
  float m = -INFINITY;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    acc[v] = wave_sum(acc[v]) + bias[v];
    m = fmaxf(m, acc[v]);
  }
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) se += expf(acc[v] - m);
  const float lse = logf(se);
  float best = -INFINITY, mine = 0.f;
  int tok = 0;
#pragma unroll
  for (int v = 0; v < kVocab; ++v) {
    const float lp = acc[v] - m - lse;
    if (lp > best) { best = lp; tok = v; }
    if (v == lane) mine = lp;
  }
  if (lane < kVocab) logp[(int64_t)row * kVocab + lane] = mine;
  if (frame_info && lane == 0) {
    const float sil = expf(acc[kVocab - 2] - m - lse) + expf(acc[kVocab - 1] - m - lse);
    frame_info[row] = tok | ((sil <= kSilenceThreshold) ? 256 : 0);
  }
}

// ---------------------------------------------------------------------------------------------
// Flat state <-> resident form (common.h StateRef).  Import: flat row i -> slab row rows[i] (every section but conv, whose
// first element becomes the chunk counter 0) and ring ring_ids[i] (phase 0: ring row i of layer l = cache frame i).
// Export: the inverse, with each layer's phase from the counter and the layer's frames per step (T, or Tr in 7-14).
// One workgroup per stream; plain copies (bit-exact).
__global__ void __launch_bounds__(256) ring_import_kernel(const __half* __restrict__ flat, int64_t fstride,
                                                          __half* __restrict__ slab, int64_t sstride,
                                                          const int* __restrict__ rows, __half* __restrict__ ring,
                                                          const int* __restrict__ ring_ids) {
  const int i = blockIdx.x;
  const __half* f = flat + (int64_t)i * fstride;
  __half* r = slab + (int64_t)rows[i] * sstride;
  __half* rg = ring + (int64_t)ring_ids[i] * kRingElems;
  // every section but conv and mhsa (the ring's); the conv section's first element = chunk counter 0
  for (int64_t e = threadIdx.x; e < kStateSize; e += 256) {
    const bool conv = e >= kOffConv && e < kOffConv + kRingConv, mhsa = e >= kOffMhsa && e < kOffMhsa + kRingMhsa;
    if (!conv && !mhsa) r[e] = f[e];
    else if (e == kOffConv) r[e] = __float2half_rn(0.f);
  }
  // conv: ring[l][t][c] = flat conv[l][c][t]; mhsa: ring[16 + ls][t][c] = flat mhsa[ls][t][c] (both time-major there)
  for (int64_t e = threadIdx.x; e < kRingConv; e += 256) {
    const int c = (int)(e % kD), t = (int)((e / kD) % kConvS), l = (int)(e / (kD * kConvS));
    rg[e] = f[kOffConv + ((int64_t)l * kD + c) * kConvS + t];
  }
  for (int64_t e = threadIdx.x; e < kRingMhsa; e += 256) rg[kRingConv + e] = f[kOffMhsa + e];
}

__global__ void __launch_bounds__(256) ring_export_kernel(const __half* __restrict__ slab, int64_t sstride,
                                                          const int* __restrict__ rows, const __half* __restrict__ ring,
                                                          const int* __restrict__ ring_ids, __half* __restrict__ flat,
                                                          int64_t fstride, int T, int Tr) {
  const int i = blockIdx.x;
  const __half* r = slab + (int64_t)rows[i] * sstride;
  __half* f = flat + (int64_t)i * fstride;
  const __half* rg = ring + (int64_t)ring_ids[i] * kRingElems;
  const int n = (int)__half2float(r[kOffConv]);
  for (int64_t e = threadIdx.x; e < kStateSize; e += 256) {
    const bool conv = e >= kOffConv && e < kOffConv + kRingConv, mhsa = e >= kOffMhsa && e < kOffMhsa + kRingMhsa;
    if (!conv && !mhsa) f[e] = r[e];
  }
  // flat conv[l][c][t] = ring[l][(ph_l + t) mod 30][c]
  for (int64_t e = threadIdx.x; e < kRingConv; e += 256) {
    const int t = (int)(e % kConvS), c = (int)((e / kConvS) % kD), l = (int)(e / (kD * kConvS));
    const int ph = ring_phase(n, (l > 6 && l <= 14) ? Tr : T);
    f[kOffConv + e] = rg[((int64_t)l * kConvS + (ph + t) % kConvS) * kD + c];
  }
  // flat mhsa[ls][t][c] = ring[16 + ls][(ph + t) mod 30][c] for the layer's last S frames, zero below (the flat form's
  // left padding: layer 14 (ls 0) in the reduced block, S = 15, T_l = Tr; layer 15, S = 30, T_l = T)
  for (int64_t e = threadIdx.x; e < kRingMhsa; e += 256) {
    const int c = (int)(e % kD), t = (int)((e / kD) % kMhsaS), ls = (int)(e / (kD * kMhsaS));
    const int S = ls == 0 ? kMhsaS / 2 : kMhsaS, ph = ring_phase(n, ls == 0 ? Tr : T);
    f[kOffMhsa + e] = t < kMhsaS - S ? __float2half_rn(0.f)
                                     : rg[kRingConv + ((int64_t)ls * kMhsaS + (ph + t) % kMhsaS) * kD + c];
  }
}

hipError_t launch_ring_import(const __half* flat, int64_t fstride, __half* slab, int64_t sstride, const int* rows, __half* ring,
                              const int* ring_ids, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ring_import_kernel, dim3(n), dim3(256), 0, st, flat, fstride, slab, sstride, rows, ring, ring_ids);
  return hipGetLastError();
}

hipError_t launch_ring_export(const __half* slab, int64_t sstride, const int* rows, const __half* ring, const int* ring_ids,
                              __half* flat, int64_t fstride, int T, int Tr, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ring_export_kernel, dim3(n), dim3(256), 0, st, slab, sstride, rows, ring, ring_ids, flat, fstride, T, Tr);
  return hipGetLastError();
}

hipError_t launch_head(const void* x, const float* w, const float* b, float* logp, int32_t* frame_info, int rows, bool r16,
                       hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  if (rows <= 64) {
    if (r16) hipLaunchKernelGGL(head_rows_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
    else hipLaunchKernelGGL(head_rows_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
    return hipGetLastError();
  }
  if (knobs().head_mfma) {
    if (r16) hipLaunchKernelGGL(head_mfma_kernel<true>, dim3((rows + 31) / 32), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
    else hipLaunchKernelGGL(head_mfma_kernel<false>, dim3((rows + 31) / 32), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
    return hipGetLastError();
  }
  if (r16) hipLaunchKernelGGL(head_kernel<true>, dim3((rows + 63) / 64), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
  else hipLaunchKernelGGL(head_kernel<false>, dim3((rows + 63) / 64), dim3(256), 0, st, x, w, b, logp, frame_info, rows);
  return hipGetLastError();
}

}  // namespace tone
