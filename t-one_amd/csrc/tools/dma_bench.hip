// LDS-DMA fill-rate microbenchmark (MI355X): how many bytes per CU per second global_load_lds_dwordx4
// delivers into LDS as a function of waves per workgroup, pieces in flight per wave, the piece shape and
// where the source lines live (L2-resident buffer vs a buffer far larger than L2).
//
// One workgroup per CU; every wave streams ITER pieces (1 KiB each: 64 lanes x 16 B) into its own
// P-slot LDS ring, keeping P pieces in flight with a counted vmcnt (no barriers, no consumers).
// Piece shapes: 0 = one contiguous 1 KiB; 1 = 8 rows x 128 B (the GEMM staging shape, row pitch 1536 B).
// Usage: dma_bench <buffer MiB> <iters per wave>; prints one JSON line per (waves, pieces, shape).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int P>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P - 1) : "memory");
}

template <int W, int P, int SHAPE>
__global__ void __launch_bounds__(W * 64) dma_kernel(const uint8_t* __restrict__ src, int64_t nbytes, int iters,
                                                    unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[W * P * 1024];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* ring = lds + wid * P * 1024;
  // every wave starts at its own offset and wraps around the whole buffer
  const int64_t base = ((int64_t)blockIdx.x * W + wid) * 4096;
  int64_t off = 0;
  for (int i = 0; i < iters; ++i) {
    int64_t o;
    if constexpr (SHAPE == 0) o = off + lane * 16;
    else o = off + (lane >> 3) * 1536 + (lane & 7) * 16;
    const uint8_t* s = src + (((base + o) & (nbytes - 1)) & ~(int64_t)15);   // nbytes: a power of two
    if (i >= P) wait_vm<P>();
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds(s, ring + (i % P) * 1024, 16, 0, 0);
#else
    (void)s;
#endif
    off += SHAPE == 0 ? 1024 : 128;   // shape 1: walks along the rows (K-steps of 128 B)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[blockIdx.x & 1023];
}

// The GEMM pattern: per K-tile every wave issues IPW pieces, then waits until the K-tile issued R - 2
// iterations earlier has landed (counted vmcnt) and meets the other waves at an s_barrier.
template <int W, int IPW, int R>
__global__ void __launch_bounds__(W * 64) ring_kernel(const uint8_t* __restrict__ src, int64_t nbytes, int iters,
                                                     unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[R * W * IPW * 1024];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // disjoint regions per wave when the buffer is larger than all reads (streams from HBM / Infinity Cache),
  // overlapping 4 KiB-spaced starts otherwise (L2-resident)
  const int64_t total = (int64_t)gridDim.x * W * iters * IPW * 1024;
  const int64_t base = ((int64_t)blockIdx.x * W + wid) * (total <= nbytes ? (int64_t)iters * IPW * 1024 : 4096);
  int64_t off = 0;
  for (int t = 0; t < iters; ++t) {
    if (t >= R - 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 2) * IPW) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const uint8_t* s = src + (((base + off + lane * 16) & (nbytes - 1)) & ~(int64_t)15);
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_global_load_lds(s, lds + ((t % R) * W * IPW + wid * IPW + i) * 1024, 16, 0, 0);
#else
      (void)s;
#endif
      off += 1024;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[blockIdx.x & 1023];
}

template <int W, int IPW, int R>
void run_ring(const uint8_t* buf, int64_t nbytes, int iters, unsigned* sink, int ncu) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int kt = iters / IPW;
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL((ring_kernel<W, IPW, R>), dim3(ncu), dim3(W * 64), 0, 0, buf, nbytes, kt, sink);
  CK(hipEventRecord(e0, 0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((ring_kernel<W, IPW, R>), dim3(ncu), dim3(W * 64), 0, 0, buf, nbytes, kt, sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)ncu * W * kt * IPW * 1024.0;
  const double s = ms * 1e-3 / reps;
  printf("{\"buffer_mib\": %lld, \"ring\": 1, \"waves\": %d, \"pieces_per_ktile\": %d, \"slots\": %d, \"us\": %.2f, \"gbs_per_cu\": %.1f}\n",
         (long long)(nbytes >> 20), W, IPW, R, s * 1e6, bytes / s / ncu / 1e9);
  fflush(stdout);
}

template <int W, int P, int SHAPE>
void run(const uint8_t* buf, int64_t nbytes, int iters, unsigned* sink, int ncu) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL((dma_kernel<W, P, SHAPE>), dim3(ncu), dim3(W * 64), 0, 0, buf, nbytes, iters, sink);
  CK(hipEventRecord(e0, 0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((dma_kernel<W, P, SHAPE>), dim3(ncu), dim3(W * 64), 0, 0, buf, nbytes, iters, sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)ncu * W * iters * 1024.0;
  const double s = ms * 1e-3 / reps;
  printf("{\"buffer_mib\": %lld, \"waves\": %d, \"pieces_in_flight\": %d, \"shape\": %d, \"us\": %.2f, \"gbs_per_cu\": %.1f, \"tbs\": %.2f}\n",
         (long long)(nbytes >> 20), W, P, SHAPE, s * 1e6, bytes / s / ncu / 1e9, bytes / s / 1e12);
  fflush(stdout);
}

template <int SHAPE>
void sweep(const uint8_t* buf, int64_t nbytes, int iters, unsigned* sink, int ncu) {
  run<1, 8, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<2, 8, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<4, 2, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<4, 4, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<4, 8, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<4, 16, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<8, 2, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<8, 4, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<8, 8, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<8, 16, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<16, 4, SHAPE>(buf, nbytes, iters, sink, ncu);
  run<16, 8, SHAPE>(buf, nbytes, iters, sink, ncu);
}

int main(int argc, char** argv) {
  const int64_t mib = argc > 1 ? atoll(argv[1]) : 2;
  const int iters = argc > 2 ? atoi(argv[2]) : 2048;
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t nbytes = mib << 20;
  uint8_t* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, nbytes + (1 << 20)));
  CK(hipMemset(buf, 1, nbytes + (1 << 20)));
  CK(hipMalloc(&sink, 4096 * 4));
  if (argc > 3 && atoi(argv[3]) == 1) {   // the GEMM ring pattern
    run_ring<8, 6, 3>(buf, nbytes, iters, sink, ncu);
    run_ring<8, 4, 4>(buf, nbytes, iters, sink, ncu);
    run_ring<8, 2, 6>(buf, nbytes, iters, sink, ncu);
    run_ring<4, 4, 6>(buf, nbytes, iters, sink, ncu);
    run_ring<4, 8, 3>(buf, nbytes, iters, sink, ncu);
    run_ring<8, 1, 6>(buf, nbytes, iters, sink, ncu);
    return 0;
  }
  sweep<0>(buf, nbytes, iters, sink, ncu);
  sweep<1>(buf, nbytes, iters, sink, ncu);
  return 0;
}
