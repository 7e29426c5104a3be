// Sustained MFMA rate on the MI355X with no memory traffic: every wave runs NCH independent accumulator chains of
// one MFMA shape for ITERS iterations on register operands (8 waves per CU = 2 per SIMD, 256 workgroups), timed with
// HIP events.  The ceiling the K = 384 GEMMs are priced against: the dense peak at the clock
// the chip actually holds under a full MFMA load.
//   mfma_peak [iters]   -> one JSON line per shape
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// SHAPE 0: v_mfma_f32_32x32x16_bf16; 1: v_mfma_f32_16x16x32_bf16; 2: v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3);
// 3: v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3)
template <int SHAPE, int NCH>
__global__ void __launch_bounds__(512) mfma_kernel(float* out, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  bf16x8 a = bf16x8{} + (__bf16)(seed * lane), b = bf16x8{} + (__bf16)(seed + lane);
  i32x8 a8 = i32x8{} + (int)(lane * 0x01010101u), b8 = i32x8{} + (int)(lane * 0x02020202u);
  if constexpr (SHAPE == 0 || SHAPE == 3) {
    f32x16 acc[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[c] = f32x16{};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if constexpr (SHAPE == 0) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
        else acc[c] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[c], 0, 0, 0, 127, 0, 127);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += acc[c][0] + acc[c][15];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else {
    f32x4 acc[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) acc[c] = f32x4{};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if constexpr (SHAPE == 1) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
        else acc[c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[c], 0, 0, 0, 127, 0, 127);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += acc[c][0] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

template <int SHAPE, int NCH>
void run(const char* name, double flop_per_mfma, float* out, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((mfma_kernel<SHAPE, NCH>), dim3(256), dim3(512), 0, 0, out, iters, 0.001f);   // warm-up
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((mfma_kernel<SHAPE, NCH>), dim3(256), dim3(512), 0, 0, out, iters, 0.001f);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / 5;
  const double flop = flop_per_mfma * NCH * (double)iters * 256 * 8;
  printf("{\"shape\": \"%s\", \"chains\": %d, \"us\": %.1f, \"tflops\": %.1f}\n", name, NCH, us, flop / us * 1e-6);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  float* out;
  CK(hipMalloc(&out, 256 * 512 * 4));
  run<0, 4>("32x32x16_bf16", 2.0 * 32 * 32 * 16, out, iters);
  run<0, 2>("32x32x16_bf16", 2.0 * 32 * 32 * 16, out, iters);
  run<1, 8>("16x16x32_bf16", 2.0 * 16 * 16 * 32, out, iters);
  run<1, 4>("16x16x32_bf16", 2.0 * 16 * 16 * 32, out, iters);
  run<2, 8>("scale_16x16x128_f8", 2.0 * 16 * 16 * 128, out, iters);
  run<2, 4>("scale_16x16x128_f8", 2.0 * 16 * 16 * 128, out, iters);
  run<3, 4>("scale_32x32x64_f8", 2.0 * 32 * 32 * 64, out, iters);
  run<3, 2>("scale_32x32x64_f8", 2.0 * 32 * 32 * 64, out, iters);
  return 0;
}
