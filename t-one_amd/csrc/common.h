// Shared device helpers for the T-one HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <utility>

namespace tone {

// f(std::integral_constant<int, I>) for I = 0 .. N-1, each call its own instantiation: loops whose index must be a
// compile-time constant but whose body is past the unroller's size limit
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- model constants (t-one_amd/config.py; tone/training/model_wrapper.py:27-115) -------------
constexpr int kChunk = 2400;                  // 300 ms (the defaults below; 400 ms: Geom)
constexpr int kPreState = 80;
constexpr int kWave = kChunk + kPreState;     // 2480 samples per mel pass
constexpr int kMelT = 30;                     // mel frames per chunk
constexpr int kWin = 160;
constexpr int kHop = 80;
constexpr int kBasisRows = 162;
constexpr int kBins = 81;
constexpr int kMels = 64;
constexpr int kD = 384;
constexpr int kHeads = 8;
constexpr int kDk = 48;
constexpr int kDff = 1536;
constexpr int kRope = 32;
constexpr int kConvK = 31;
constexpr int kConvS = 30;
constexpr int kMhsaS = 30;
constexpr int kT = 10;                        // acoustic frames per chunk
constexpr int kVocab = 35;
constexpr int kSub1C = 32, kSub1Kt = 11, kSub1Kf = 21, kSub1F = 44, kSub1S = 10;
constexpr int kSub2C = 64, kSub2Kt = 11, kSub2Kf = 11, kSub2F = 34, kSub2S = 8, kSub2Stride = 3;
constexpr int kSub2In = kSub2S + kMelT;       // 38 time rows into conv2
constexpr int kSubOut = kSub2C * kSub2F;      // 2176
constexpr int kConv2K = kSub2Kt * kSub2Kf * kSub1C;   // 3872 = 121 taps x 32 channels
constexpr int kConv2KPad = 3904;              // next multiple of 64 (bf16 K-step); pad tap has zero weights
constexpr int kMelPowCols = 128;              // 81 power bins padded to 4 x 32

// flat state offsets (elements, per stream)
// Chunk geometry.  The reference streams 300 ms (StreamingCTCModel.AUDIO_CHUNK_SAMPLES = 2400) and
// exports / serves a 400 ms variant (tone/scripts/export.py:139-157 chunk_duration_ms;
// triton/ensemble/config.pbtxt:12-18: 3200 samples).  The state layout is the same for both (its
// sizes are fixed by the model, conformer.py:235-290); what changes per chunk is:
//   wave   = chunk + 80 carried samples            2480 | 3280
//   melT   = (wave - 160) / 80 + 1                  30   | 40    (feats.py:95-102)
//   sub2In = 8 carried rows + melT                  38   | 48    (conformer_blocks.py:631-641)
//   T      = (sub2In - 11) / 3 + 1                  10   | 13    (conv2 stride 3; 400 ms leaves row 47 unread)
//   Tr     = (T + 1 - 3) / 2 + 1                    5    | 6     (CausalTemporalReduction, streaming branch)
// and the upsampling pads one frame back to T (conformer_blocks.py:978-981: live for T = 13).
struct Geom {
  int chunk, wave, melT, sub2In, T, Tr;
};
__host__ __device__ constexpr Geom make_geom(int chunk) {
  return Geom{chunk, chunk + 80, (chunk + 80 - 160) / 80 + 1, 8 + (chunk + 80 - 160) / 80 + 1,
              (8 + (chunk + 80 - 160) / 80 + 1 - 11) / 3 + 1, ((8 + (chunk + 80 - 160) / 80 + 1 - 11) / 3 + 1 + 1 - 3) / 2 + 1};
}
constexpr int kChunkMax = 3200, kWaveMax = 3280, kMelTMax = 40, kSub2InMax = 48, kTMax = 13, kTrMax = 6;
static_assert(make_geom(2400).T == 10 && make_geom(2400).Tr == 5 && make_geom(2400).melT == 30, "300 ms geometry");
static_assert(make_geom(3200).T == 13 && make_geom(3200).Tr == 6 && make_geom(3200).melT == 40, "400 ms geometry");

constexpr int64_t kOffPre = 0;
constexpr int64_t kOffMhsa = 80;
constexpr int64_t kOffConv = 23120;
constexpr int64_t kOffMhsaLen = 207440;
constexpr int64_t kOffSub1 = 207441;
constexpr int64_t kOffSub2 = 208081;
constexpr int64_t kOffRed = 219345;
constexpr int64_t kStateSize = 219729;

constexpr float kRmsEps = 1e-8f;
constexpr float kLnEps = 1e-5f;

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// Where stream b's state rows live: row b of state_in / state_out, or rows slots[b] of device-resident
// slabs; with slots_out, stream b reads row slots[b] and writes row slots_out[b] (ping-pong rows of one
// slab, so streams that sit out a step keep their state without a copy).
// Resident (ring) form, tone_session_run_ring: the conv-module caches and the layer 14 / 15 MHSA input caches of stream b
// live outside its row, in the ring ring + ring_ids[b] * kRingElems, time-major [16 conv layers + 2 MHSA layers][30
// frames][384 channels] fp16, updated in place: a step writes only its T new frames, over the T oldest (the flat form
// rewrites all 30 shifted by T).  Cache frame i of layer l sits at ring row (ph_l + i) mod 30, ph_l = (n T_l) mod 30,
// n = the stream's chunk counter mod 30, kept (as fp16) at the first element of the row's then unused conv section;
// T_l = the layer's frames per step (T, or Tr in layers 7-14).  The MHSA caches' frames older than the layer's S
// (layer 14: S = 15) are the flat form's zero padding: stale in the ring, zeros on export.
constexpr int64_t kRingConv = (int64_t)16 * 30 * 384;    // 184320 = the flat conv section's size
constexpr int64_t kRingMhsa = (int64_t)2 * 30 * 384;     // 23040 = the flat mhsa section's size
constexpr int64_t kRingElems = kRingConv + kRingMhsa;
__host__ __device__ __forceinline__ int ring_phase(int n, int T) { return (n * T) % 30; }

struct StateRef {
  const __half* in;
  __half* out;
  int64_t stride;          // elements between consecutive rows
  const int* slots;        // rows read (nullptr -> identity)
  const int* slots_out;    // rows written (nullptr -> the rows read)
  __half* ring = nullptr;  // resident form: the conv rings (nullptr: flat form, caches in the rows)
  const int* ring_ids = nullptr;   // ... and stream b's ring index
  __device__ __forceinline__ int64_t row_in(int b) const { return (int64_t)(slots ? slots[b] : b) * stride; }
  __device__ __forceinline__ int64_t row_out(int b) const {
    return slots_out ? (int64_t)slots_out[b] * stride : row_in(b);
  }
  __device__ __forceinline__ int chunk_counter(int b) const {   // resident form only
    return (int)__half2float(in[row_in(b) + kOffConv]);
  }
};

// MXFP8 (OCP MX, e4m3 values, one E8M0 scale per 32): the block exponent from the block's max |v|,
// E = floor(log2 amax) - 7 (biased by 127, clamped to 1 .. 254), and the inverse block scale 2^(127 - E).  Round 6: one
// binade of headroom below the OCP choice (- 8): the scaled values stay below 256 < 448, so no saturation can occur and
// gfx950's scaled conversion (v_cvt_scalef32_pk_fp8_f32: cvt(x / 2^(E - 127)), which does not saturate) encodes a block
// in one instruction per two values instead of a multiply, two clamps and a conversion; the lowest binade of e4m3
// (values below 2^-15 of the block max) is what the headroom costs.  Weights keep the OCP exponent (host, once).
__device__ __forceinline__ int mx_exp(float amax) {
  const int e = (int)((__float_as_uint(amax) >> 23) & 0xff);   // biased exponent of amax (0 for 0/subnormal)
  return max(1, min(254, e - 7));
}
// the block scale 2^(E - 127) as the float operand of the scaled conversion (E >= 1: a normal float)
__device__ __forceinline__ float mx_scale(int ebiased) { return __uint_as_float((uint32_t)ebiased << 23); }
typedef short mx_s16x2 __attribute__((ext_vector_type(2)));
// two floats -> two e4m3 bytes of x / 2^(E - 127) in the low (HI false) or high half of w; NaN stays NaN
template <bool HI>
__device__ __forceinline__ uint32_t mx_cvt2(float a, float b, float scale, uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(__builtin_bit_cast(mx_s16x2, w), a, b,
                                                                               scale, HI));
}
// clamp to e4m3's finite range (+-448) keeping a NaN a NaN: IEEE 754-2019 maximum / minimum (v_maximum3_f32 /
// v_minimum3_f32 on gfx950) propagate NaN, so two instructions do what fminf / fmaxf plus a NaN select did in four
// (identical bytes on every edge value, tools/cvt_probe.hip, profiles/r03_cvt_probe.jsonl)
__device__ __forceinline__ float sat_e4m3(float v) {
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, -448.f), 448.f);
}
__device__ __forceinline__ float exp2i(int ebiased) {
  return __uint_as_float((uint32_t)(254 - ebiased) << 23);
}

// fp8 mode: the folded-RMSNorm row factor of an MXFP8 GEMM operand comes from a sum-of-squares slab, kSsSlots floats
// per row, the sum of the row's squared bf16 values split over 32-column slots: a producer that sees the whole row
// (quant_mx, the fused rmsnorm) writes {ss, 0, ...}, a RESID GEMM epilogue the partial sum of each 32-column slot
// range its workgroup / wave covers (zeros in the slots it covers without a sum); the consumer adds the slots in a
// fixed order (three 4-slot groups) -- {ss, 0, ...} gives ss exactly
constexpr int kSsSlots = 12;   // 384 / 32
__device__ __forceinline__ float mx_row_inv(const float* __restrict__ ss_row) {
  const float4 a = reinterpret_cast<const float4*>(ss_row)[0];
  const float4 b = reinterpret_cast<const float4*>(ss_row)[1];
  const float4 c = reinterpret_cast<const float4*>(ss_row)[2];
  const float ss = (((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w))) + ((c.x + c.y) + (c.z + c.w));
  return 1.0f / (sqrtf(ss) * 0.05103103630798288f + kRmsEps);   // 384^-0.5
}
// 4 floats -> 4 e4m3 bytes (one dword) of the block with biased exponent e (mx_exp), NaN kept
__device__ __forceinline__ uint32_t quant4(float a, float b, float c, float d, int e) {
  const float sc = mx_scale(e);
  return mx_cvt2<true>(c, d, sc, mx_cvt2<false>(a, b, sc, 0u));
}

// One 1 KiB LDS-DMA piece (global_load_lds_dwordx4: lane l's 16 bytes at src land at lds_dst + 16 l) issued from
// inline asm.  After the builtin form the compiler's wait-count pass no longer counts LDS reads: every later
// ds_read wait became lgkmcnt(0), a full drain of the reads issued ahead (gemm_xw: 54 lgkmcnt(0) with the builtin,
// counted waits without the DMA).  The asm form is invisible to that pass; the kernels order their DMAs with explicit
// vmcnt waits and barriers, which is what makes this safe.  lds_dst must be wave-uniform (as for the builtin).
__device__ __forceinline__ void lds_dma16(const void* src, void* lds_dst) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
#else
  (void)src;
  (void)lds_dst;
#endif
}
// the 4-byte form (global_load_lds_dword: lane l's dword lands at lds_dst + 4 l)
__device__ __forceinline__ void lds_dma4(const void* src, void* lds_dst) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
#else
  (void)src;
  (void)lds_dst;
#endif
}

// s_waitcnt vmcnt(n) for a wave-uniform n known only at run time (a scalar branch to the immediate form)
__device__ __forceinline__ void vmcnt_dyn(int n) {
  switch (n) {
#define TONE_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    TONE_VMC(1) TONE_VMC(2) TONE_VMC(3) TONE_VMC(4) TONE_VMC(5) TONE_VMC(6) TONE_VMC(7) TONE_VMC(8) TONE_VMC(9)
    TONE_VMC(10) TONE_VMC(11) TONE_VMC(12) TONE_VMC(13) TONE_VMC(14) TONE_VMC(15) TONE_VMC(16) TONE_VMC(17)
    TONE_VMC(18) TONE_VMC(19) TONE_VMC(20) TONE_VMC(21) TONE_VMC(22) TONE_VMC(23) TONE_VMC(24) TONE_VMC(25)
    TONE_VMC(26) TONE_VMC(27) TONE_VMC(28) TONE_VMC(29) TONE_VMC(30) TONE_VMC(31) TONE_VMC(32)
#undef TONE_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Counted wait for an LDS-DMA ring of depth R over n tiles where tile t + R - 1's P pieces are issued at the START
// of iteration t (tiles 0 .. R - 2 before the loop) and iteration i >= 1 then issues S stores (the epilogue of tile
// i - 1): the number of this wave's vector-memory ops issued after tile j's DMA, i.e. the vmcnt that guarantees
// tile j landed.  (Ops the compiler adds only make the wait stricter.)
__device__ __forceinline__ int ring_younger(int j, int n, int R, int P, int S) {
  // closed form (checked against the iteration-by-iteration count for R 2-6, P 1-12, S 0-8, n 1-40, every j): the
  // loop form compiled to ~300 scalar instructions and branches per tile, enough to make the scalar unit a bottleneck
  // of the K = 384 kernels.  DMAs after tile j's: prologue tiles j+1 .. min(R-2, n-1) (only when j <= R-2) and the
  // in-loop DMAs of iterations a .. j-1 whose tile i+R-1 exists; stores: iterations max(1, a) .. j-1, plus the
  // iteration that issued tile j (j - R + 1) when it is >= 1
  const int pro = j <= R - 2 ? max(0, min(R - 2, n - 1) - j) : 0;
  const int a = max(0, j - R + 2);
  const int dm = max(0, min(j - 1, n - R) - a + 1);
  const int st = max(0, j - max(1, a)) + (j >= R ? 1 : 0);
  return (pro + dm) * P + st * S;
}

// The counted ring wait: the steady-state count (R - 2 later DMAs, R - 1 store groups) is one compile-time wait; the
// other counts (the first R and last R - 1 tiles of a run) go through vmcnt_dyn's switch, which compiles to a
// branch tree of ~60 scalar instructions -- too many to run on every tile.
template <int R, int P, int S>
__device__ __forceinline__ void ring_wait(int j, int n) {
  constexpr int kSteady = (R - 2) * P + (R - 1) * S;
  static_assert(kSteady <= 63, "vmcnt field");
  const int c = ring_younger(j, n, R, P, S);
  if (c >= kSteady) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kSteady) : "memory");
  else vmcnt_dyn(c);
}

// reductions over the four lanes l ^ {0, 16, 32, 48} (one value per 16-lane row): v_permlane16_swap then
// v_permlane32_swap, plain VALU (__shfl_xor's ds_bpermute goes through the LDS and its lgkmcnt(0) also waits for
// every fragment read in flight).  Same association as v + shfl_xor(v, 16), then + shfl_xor(., 32).
__device__ __forceinline__ float lg_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float lg_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// max |v| over 8 values and the lane group, as the bits of a non-negative float: the lane's own values by fmaxf, the
// lane swaps by integer max on the bits (finite and infinite magnitudes order like their bit patterns), which saves the
// canonicalizing v_max_f32 x, x, x fmaxf needs after every swap.  Identical to the all-fmaxf form unless a lane's own 8
// values are all NaN (fmaxf drops a NaN beside a number; that lane's NaN bits win the integer max); the NaN values stay
// NaN through quant4 either way
__device__ __forceinline__ uint32_t lg_max_abs_bits(const float (&v)[8]) {
  float f = 0.f;   // the lane's own 8 values: v_max3_f32 with |.| source modifiers
#pragma unroll
  for (int r = 0; r < 8; ++r) f = fmaxf(f, fabsf(v[r]));
  uint32_t m = __float_as_uint(f);
  const auto a = __builtin_amdgcn_permlane16_swap(m, m, false, false);
  m = max((uint32_t)a[0], (uint32_t)a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(m, m, false, false);
  return max((uint32_t)b[0], (uint32_t)b[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float round_h(float x) { return __half2float(__float2half_rn(x)); }

// Activation store: fp32, or bf16 bits when OBF (bf16 mode operands of the next GEMM).
template <bool OBF>
__device__ __forceinline__ void store_act(void* base, int64_t i, float v) {
  if constexpr (OBF) {
    __bf16 h = (__bf16)v;
    static_cast<uint16_t*>(base)[i] = __builtin_bit_cast(uint16_t, h);
  } else {
    static_cast<float*>(base)[i] = v;
  }
}
// activation loads matching store_act: element i of an fp32 or bf16 (OBF) array; four consecutive
// elements (16-byte / 8-byte aligned)
template <bool OBF>
__device__ __forceinline__ float load_act(const void* base, int64_t i) {
  if constexpr (OBF) {
    const uint32_t u = (uint32_t) static_cast<const uint16_t*>(base)[i] << 16;
    return __builtin_bit_cast(float, u);
  } else {
    return static_cast<const float*>(base)[i];
  }
}
template <bool OBF>
__device__ __forceinline__ float4 load_act4(const void* base, int64_t i) {
  if constexpr (OBF) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(base) + i);
    return make_float4(__builtin_bit_cast(float, u.x << 16), __builtin_bit_cast(float, u.x & 0xffff0000u),
                       __builtin_bit_cast(float, u.y << 16), __builtin_bit_cast(float, u.y & 0xffff0000u));
  } else {
    return *reinterpret_cast<const float4*>(static_cast<const float*>(base) + i);
  }
}
__device__ __forceinline__ void store_bf16(uint16_t* base, int64_t i, float v) {
  __bf16 h = (__bf16)v;
  base[i] = __builtin_bit_cast(uint16_t, h);
}
// Exact three-term bf16 split of an fp32 value: v = t0 + t1 + t2, t0 = bf16(v), t1 = bf16(v - t0),
// t2 = bf16(v - t0 - t1) (both residuals exact in fp32; |v - t0 - t1 - t2| <= 2^-27 |v|).
__device__ __forceinline__ void split3_f(float v, float& t0, float& t1, float& t2) {
  t0 = (float)(__bf16)v;
  const float r = v - t0;
  t1 = (float)(__bf16)r;
  t2 = (float)(__bf16)(r - t1);
}
// bf16 shadow of an fp32 activation for the next GEMM's A operand: one plane (bf16 mode), or with
// plane > 0 the exact split into planes s, s + plane, s + 2 plane (fp32 split mode, gemm_x3).
__device__ __forceinline__ void store_shadow(uint16_t* s, int64_t plane, int64_t i, float v) {
  if (!plane) {
    store_bf16(s, i, v);
    return;
  }
  float t0, t1, t2;
  split3_f(v, t0, t1, t2);
  store_bf16(s, i, t0);
  store_bf16(s, i + plane, t1);
  store_bf16(s, i + 2 * plane, t2);
}

// The bf16 FFN hidden h between the X-stationary up-projection (gemm_xw) and the row-panel down-projection (gemm_rp),
// "blocked": a [rows][ld] matrix (ld a multiple of 32, rows padded to a multiple of 32) as 32 x 32 tiles of 2 KiB, tile
// (row / 32, col / 32) at element ((row / 32) (ld / 32) + col / 32) 1024; inside a tile the 8-column chunk c (columns
// 8c .. 8c + 7) of row r at element (c >> 1) 512 + ((c & 1) 32 + r) 8.  That is the order in which the 32x32x16
// MFMA's accumulator registers leave gemm_xw (lane l = 32 h + r holds chunks h and 2 + h of token r): each of its
// store instructions writes 1 KiB contiguous (row-major h: 32-byte row segments 3 KiB apart), and gemm_rp's 1 KiB
// DMA pieces read four 256-byte runs (row-major: sixteen 64-byte row segments).  h never leaves that pair.
__host__ __device__ __forceinline__ int64_t hblk_off(int64_t row, int col, int64_t ld) {
  const int c = (col & 31) >> 3;
  return ((row >> 5) * (ld >> 5) + (col >> 5)) * 1024 + (c >> 1) * 512 + ((c & 1) * 32 + (row & 31)) * 8 + (col & 7);
}

// fp32 split mode: the operands of gemm_d3 (the N = 384 projections at small M) "fragment-packed", so that every one of
// its 16-byte-per-lane loads reads 1 KiB contiguous.  A [rows][K] fp32 activation (rows padded to a multiple of 32):
// per 32-row block and 32-column pair block 4 KiB, chunk 2 e + o (e = K-step of the pair, o = which half of the lane's
// 8 values) holding lane (h, r) = 32 h + r's four values row 32 rb + r, columns 32 p + 16 e + 8 h + 4 o .. + 3 -- the B
// operand of v_mfma_f32_32x32x16_bf16 for lane 32 h + r once split.  Written by the producers of those A operands
// (the fp32 SwiGLU epilogue, the attention kernels, the depthwise conv) when the consumer is routed to gemm_d3.
__host__ __device__ __forceinline__ int64_t xpk_off(int64_t row, int col, int K) {
  const int k = col & 31;
  return (((row >> 5) * (K >> 5) + (col >> 5)) * 4 + 2 * (k >> 4) + ((k >> 2) & 1)) * 256 +
         (((k >> 3) & 1) * 32 + (row & 31)) * 4 + (k & 3);
}
// The element offset of an fp32 activation stored row-major (ld K) or packed as above.
__host__ __device__ __forceinline__ int64_t act_off(int64_t row, int col, int K, bool packed) {
  return packed ? xpk_off(row, col, K) : row * K + col;
}
// W's three bf16 planes [3][N][K] for gemm_d3: per 32-row block and 32-column pair block 6 KiB, chunk 2 plane + e holding
// lane (h, r)'s 8 values row 32 nb + r, columns 32 p + 16 e + 8 h .. + 7 (the A operand of the same MFMA).
__host__ __device__ __forceinline__ int64_t wpk_off(int64_t n, int k, int plane, int K) {
  return ((((n >> 5) * (K >> 5) + (k >> 5)) * 3 + plane) * 2 + ((k >> 4) & 1)) * 512 + (((k >> 3) & 1) * 32 + (n & 31)) * 8 +
         (k & 7);
}

// The residual stream: fp32 in fp32 mode, fp16 in the bf16 / fp8 modes (as the reference's exported graph keeps it,
// tone/scripts/export.py:411).  Element i, and four consecutive elements (16 / 8-byte aligned),
// with the type fixed at compile time (R16) or chosen per launch (r16, the GEMM epilogues).
template <bool R16>
__device__ __forceinline__ float load_res(const void* base, int64_t i) {
  if constexpr (R16) return __half2float(static_cast<const __half*>(base)[i]);
  else return static_cast<const float*>(base)[i];
}
template <bool R16>
__device__ __forceinline__ void store_res(void* base, int64_t i, float v) {
  if constexpr (R16) static_cast<__half*>(base)[i] = __float2half_rn(v);
  else static_cast<float*>(base)[i] = v;
}
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4_t load_res4(const void* base, int64_t i, bool r16) {
  if (r16) {
    const f16x4_t h = *reinterpret_cast<const f16x4_t*>(static_cast<const __half*>(base) + i);
    return __builtin_convertvector(h, f32x4_t);
  }
  return *reinterpret_cast<const f32x4_t*>(static_cast<const float*>(base) + i);
}
__device__ __forceinline__ void store_res4(void* base, int64_t i, f32x4_t v, bool r16, bool nt = false) {
  if (r16) {
    const f16x4_t h = __builtin_convertvector(v, f16x4_t);   // round to nearest even, as __float2half_rn
    f16x4_t* d = reinterpret_cast<f16x4_t*>(static_cast<__half*>(base) + i);
    if (nt) __builtin_nontemporal_store(h, d);
    else *d = h;
    return;
  }
  f32x4_t* d = reinterpret_cast<f32x4_t*>(static_cast<float*>(base) + i);
  if (nt) __builtin_nontemporal_store(v, d);
  else *d = v;
}

}  // namespace tone
