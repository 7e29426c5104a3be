// What v_cvt_pk_fp8_f32 does at the edges of e4m3 on the MI355X, and the gfx950 scaled conversion (scale 1), against the
// software saturation the MXFP8 kernels use (sat_e4m3 + the builtin): one line per input value.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ float sat_e4m3(float v) { return v != v ? v : fminf(fmaxf(v, -448.f), 448.f); }

__global__ void probe(const float* in, uint32_t* out, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  const float v = in[i];
  const uint32_t a = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);              // no clamp
  const uint32_t b = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(v), sat_e4m3(v), 0, false);   // software
  typedef short v2s __attribute__((ext_vector_type(2)));
  const v2s z = {0, 0};
  const v2s cs = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, v, v, 1.0f, false);             // gfx950 scaled convert
  const uint32_t c = (uint32_t)(uint16_t)cs[0];
  // NaN-propagating clamps: v_med3_f32, and IEEE-754-2019 maximum / minimum (llvm.maximum / llvm.minimum)
  const float m3 = __builtin_amdgcn_fmed3f(v, -448.f, 448.f);
  const float mm = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, -448.f), 448.f);
  const uint32_t d = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(m3, m3, 0, false);
  const uint32_t e = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(mm, mm, 0, false);
  out[3 * i] = a & 0xff;
  out[3 * i + 1] = b & 0xff;
  out[3 * i + 2] = c & 0xff;
  out[3 * n + 2 * i] = d & 0xff;
  out[3 * n + 2 * i + 1] = e & 0xff;
}

int main() {
  const float vals[] = {0.f, 1.f, -1.f, 0.3f, 240.f, 256.f, 416.f, 440.f, 448.f, 450.f, 463.f, 464.f, 470.f, 480.f, 500.f, 511.f,
                        1e6f, -450.f, -464.f, -500.f, -1e6f, INFINITY, -INFINITY, NAN, -NAN, 1e-9f, 0.0019f};
  const int n = sizeof(vals) / sizeof(vals[0]);
  float* din;
  uint32_t* dout;
  hipMalloc(&din, sizeof(vals));
  hipMalloc(&dout, 5 * n * 4);
  hipMemcpy(din, vals, sizeof(vals), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, din, dout, n);
  uint32_t h[5 * 64];
  hipMemcpy(h, dout, 5 * n * 4, hipMemcpyDeviceToHost);
  int diff = 0;
  for (int i = 0; i < n; ++i) {
    printf("{\"v\": \"%g\", \"noclamp\": \"0x%02x\", \"software\": \"0x%02x\", \"scalef32\": \"0x%02x\", \"med3\": \"0x%02x\", \"minmax2019\": \"0x%02x\"}\n",
           vals[i], h[3 * i], h[3 * i + 1], h[3 * i + 2], h[3 * n + 2 * i], h[3 * n + 2 * i + 1]);
    diff += (h[3 * i + 1] != h[3 * n + 2 * i]) + 100 * (h[3 * i + 1] != h[3 * n + 2 * i + 1]);
  }
  printf("{\"med3_differences_plus_100x_minmax_differences\": %d}\n", diff);
  return 0;
}
