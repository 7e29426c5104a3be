// Depthwise-conv (a9) microbenchmark: where the state stream's time goes.
//   v0  launch_dwconv (the library kernel)
//   v1  the same state traffic with no arithmetic (section window -> LDS -> other slab), no g / out
//   v2  the same number of bytes as v1, packed contiguously (float4 grid-stride copy)
//   ablate_D  the previous kernel (state write-back after the arithmetic) with parts compiled out (DBG bits below);
//       ablate_0 is checked bit for bit against v0
// (A persistent variant prefetching the next stream's state and frames into registers measured 86-117 us against
// 52-62 for the library kernel at B = 4096, and a lane-per-channel-pair v_pk_fma_f32 kernel 60-67 us; both removed.)
// Usage: dwconv_bench <B> <T> [obf=1] [reps=50]; one JSON line per variant.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../common.h"
#include "../kernels.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using namespace tone;

constexpr int kSecH = kD * kConvS;   // halves of one (stream, layer) conv-state section

template <int CPW>
__global__ void __launch_bounds__(CPW) state_copy_kernel(StateRef s, int layer) {
  constexpr int kSec = CPW * kConvS, kVec = kSec / 8 + 1;
  __shared__ uint4 lds[kVec];
  const int c = threadIdx.x, b = blockIdx.x, ch0 = blockIdx.y * CPW;
  const int64_t sec = kOffConv + (int64_t)layer * kSecH + ch0 * kConvS;
  const uintptr_t a = reinterpret_cast<uintptr_t>(s.in + s.row_in(b) + sec);
  const int nvec = ((int)((a & 15) >> 1) + kSec + 7) >> 3;
  const uint4* q = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
  for (int v = c; v < nvec; v += CPW) lds[v] = q[v];
  __syncthreads();
  uint4* d = reinterpret_cast<uint4*>(reinterpret_cast<uintptr_t>(s.out + s.row_out(b) + sec) & ~uintptr_t(15));
  for (int v = c; v < nvec; v += CPW) d[v] = lds[v];
}

__global__ void __launch_bounds__(256) dense_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

// ---- ablations of the library kernel (encoder.hip dwconv_kernel, 192 x 1 shape): DBG bits 1 no conv FMAs, 2 no SiLU,
// 4 no frame stores, 8 no frame loads, 16 no state reads from LDS, 32 no state write-back to HBM -------------------
template <int T, bool OBF, int DBG>
__global__ void __launch_bounds__(192) dw_ablate_kernel(const void* __restrict__ g, StateRef s, int layer,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        void* __restrict__ out, int B) {
  constexpr int CPW = 192, kSec = CPW * kConvS, kVec = kSec / 8 + 1;
  __shared__ uint4 lds[kVec];
  const int c = threadIdx.x, ch0 = blockIdx.y * CPW, ch = ch0 + c, b = blockIdx.x;
  const int64_t sec = kOffConv + (int64_t)layer * kSecH + ch0 * kConvS;
  const uintptr_t a = reinterpret_cast<uintptr_t>(s.in + s.row_in(b) + sec);
  const int shift = (int)((a & 15) >> 1), nvec = (shift + kSec + 7) >> 3;
  const uint4* q = reinterpret_cast<const uint4*>(a & ~uintptr_t(15));
  for (int v = c; v < nvec; v += CPW) lds[v] = q[v];
  float wr[kConvK];
#pragma unroll
  for (int k = 0; k < kConvK; ++k) wr[k] = w[k * kD + ch];
  const float bb = bias[ch];
  float gx[T];
#pragma unroll
  for (int t = 0; t < T; ++t) gx[t] = (DBG & 8) ? 0.f : load_act<OBF>(g, ((int64_t)b * T + t) * kD + ch);
  __syncthreads();
  __half* h = reinterpret_cast<__half*>(lds) + shift + c * kConvS;
  float x[kConvS + T];
#pragma unroll
  for (int t = 0; t < T; ++t) x[kConvS + t] = gx[t];
#pragma unroll
  for (int i = 0; i < kConvS; ++i) x[i] = (DBG & 16) ? (float)i : __half2float(h[i]);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    float acc = bb;
    if constexpr (DBG & 1) acc += x[t];
    else {
#pragma unroll
      for (int k = 0; k < kConvK; ++k) acc = fmaf(wr[k], x[t + k], acc);
    }
    const float y = (DBG & 2) ? acc : silu_f(acc);
    if constexpr (!(DBG & 4)) store_act<OBF>(out, ((int64_t)b * T + t) * kD + ch, y);
    else if (y == 1234.5f) store_act<OBF>(out, ch, y);
  }
#pragma unroll
  for (int i = 0; i < kConvS; ++i) h[i] = __float2half_rn(x[T + i]);
  __syncthreads();
  if constexpr (!(DBG & 32)) {
    uint4* d = reinterpret_cast<uint4*>(reinterpret_cast<uintptr_t>(s.out + s.row_out(b) + sec) & ~uintptr_t(15));
    for (int v = c; v < nvec; v += CPW) d[v] = lds[v];
  }
}

template <int T, bool OBF, int DBG>
static void launch_ablate(const void* g, StateRef s, int layer, const float* w, const float* b, void* out, int B,
                          hipStream_t st) {
  hipLaunchKernelGGL((dw_ablate_kernel<T, OBF, DBG>), dim3(B, 2), dim3(192), 0, st, g, s, layer, w, b, out, B);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096;
  const int T = argc > 2 ? atoi(argv[2]) : 10;
  const bool obf = argc > 3 ? atoi(argv[3]) != 0 : true;
  const int reps = argc > 4 ? atoi(argv[4]) : 50;
  const int layer = 5;
  const int64_t stride = kStateSize;
  const size_t sbytes = (size_t)B * stride * 2;
  const size_t act = (size_t)B * T * kD * (obf ? 2 : 4);
  __half *s_in, *s_out, *s_ref;
  void *g, *out, *out_ref;
  float *w, *bias;
  CK(hipMalloc(&s_in, sbytes));
  CK(hipMalloc(&s_out, sbytes));
  CK(hipMalloc(&s_ref, sbytes));
  CK(hipMalloc(&g, act));
  CK(hipMalloc(&out, act));
  CK(hipMalloc(&out_ref, act));
  CK(hipMalloc(&w, kConvK * kD * 4));
  CK(hipMalloc(&bias, kD * 4));
  {
    std::vector<uint16_t> hs((size_t)B * stride);
    uint32_t r = 12345;
    for (auto& v : hs) {
      r = r * 1664525u + 1013904223u;
      v = (uint16_t)(0x3000 + ((r >> 16) & 0x0fff));   // fp16 in [0.125, 1)
    }
    CK(hipMemcpy(s_in, hs.data(), sbytes, hipMemcpyHostToDevice));
    std::vector<uint16_t> hg(act / 2);
    for (auto& v : hg) {
      r = r * 1664525u + 1013904223u;
      v = (uint16_t)(0x3e00 + ((r >> 16) & 0x00ff));
    }
    CK(hipMemcpy(g, hg.data(), act, hipMemcpyHostToDevice));
    std::vector<float> hw(kConvK * kD), hb(kD);
    for (auto& v : hw) {
      r = r * 1664525u + 1013904223u;
      v = ((r >> 8) & 0xffff) / 65536.0f - 0.5f;
    }
    for (auto& v : hb) v = 0.01f;
    CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  }
  CK(hipMemset(s_out, 0, sbytes));
  CK(hipMemset(s_ref, 0, sbytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  StateRef sr{s_in, s_ref, stride, nullptr, nullptr};
  StateRef so{s_in, s_out, stride, nullptr, nullptr};
  const double state_bytes = 2.0 * B * kSecH * 2;
  const double io_bytes = 2.0 * act;

  auto timeit = [&](const char* name, double bytes, auto&& fn) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("{\"variant\": \"%s\", \"B\": %d, \"T\": %d, \"obf\": %d, \"us\": %.2f, \"GBps\": %.0f, \"bytes\": %.0f}\n", name,
           B, T, (int)obf, us, bytes / us * 1e-3, bytes);
    fflush(stdout);
  };
  auto run_ref = [&]() { CK(launch_dwconv(g, sr, layer, w, bias, out_ref, obf, T, B, st)); };
  timeit("library", state_bytes + io_bytes, run_ref);
  timeit("state_copy_192", state_bytes, [&]() {
    hipLaunchKernelGGL((state_copy_kernel<192>), dim3(B, 2), dim3(192), 0, st, so, layer);
  });
  {
    const int64_t n = (int64_t)B * kSecH * 2 / 16;
    uint4* a = reinterpret_cast<uint4*>(s_in);
    uint4* d = reinterpret_cast<uint4*>(s_out);
    timeit("dense_copy", state_bytes, [&]() {
      hipLaunchKernelGGL(dense_copy_kernel, dim3(2048), dim3(256), 0, st, a, d, n);
    });
  }
  CK(hipMemset(s_out, 0, sbytes));
  auto compare = [&](const char* name, const __half* sdst) {
    std::vector<uint16_t> o1(act / 2), o2(act / 2);
    CK(hipMemcpy(o1.data(), out_ref, act, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), out, act, hipMemcpyDeviceToHost));
    size_t bad = 0, bad1 = 0;   // differing 16-bit words; of which off by more than one bf16 ulp (obf)
    for (size_t k = 0; k < o1.size(); ++k) {
      if (o1[k] == o2[k]) continue;
      ++bad;
      if (!obf || (o1[k] > o2[k] ? o1[k] - o2[k] : o2[k] - o1[k]) > 1) ++bad1;
    }
    size_t bad_s = 0;
    std::vector<uint16_t> s1((size_t)kSecH), s2((size_t)kSecH);
    for (int b = 0; b < B; b += (B > 64 ? 7 : 1)) {
      const size_t off = (size_t)b * stride + kOffConv + (size_t)layer * kSecH;
      CK(hipMemcpy(s1.data(), s_ref + off, kSecH * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(s2.data(), sdst + off, kSecH * 2, hipMemcpyDeviceToHost));
      for (int k = 0; k < kSecH; ++k) bad_s += s1[k] != s2[k];
    }
    printf("{\"check\": \"%s\", \"out_words_differing\": %zu, \"out_beyond_1ulp\": %zu, \"state_mismatch\": %zu}\n", name,
           bad, bad1, bad_s);
    fflush(stdout);
  };
  CK(hipMemset(s_out, 0, sbytes));
#define ABL(d)                                                                                               \
  {                                                                                                          \
    char nm[32];                                                                                             \
    snprintf(nm, sizeof nm, "ablate_%d", d);                                                                 \
    timeit(nm, state_bytes + io_bytes, [&]() {                                                               \
      if (T == 10) { if (obf) launch_ablate<10, true, d>(g, so, layer, w, bias, out, B, st);                 \
                     else launch_ablate<10, false, d>(g, so, layer, w, bias, out, B, st); }                  \
      else { if (obf) launch_ablate<5, true, d>(g, so, layer, w, bias, out, B, st);                          \
             else launch_ablate<5, false, d>(g, so, layer, w, bias, out, B, st); }                           \
    });                                                                                                      \
  }
  ABL(0)
  CK(hipStreamSynchronize(st));
  compare("ablate_0_vs_library", s_out);   // the previous order (write-back last) against the library's
  ABL(1) ABL(2) ABL(3) ABL(4) ABL(8) ABL(12) ABL(16) ABL(32) ABL(7) ABL(15) ABL(31) ABL(63)
#undef ABL
  {
    // output rows aligned differently from the input rows (run_rows' ping-pong layout): the realignment path
    CK(hipMemset(s_out, 0, sbytes));
    StateRef so2{s_in, s_out + 1, stride, nullptr, nullptr};
    CK(launch_dwconv(g, so2, layer, w, bias, out, obf, T, B, st));
    CK(hipStreamSynchronize(st));
    compare("library_shifted_out", s_out + 1);
  }
  return 0;
}
