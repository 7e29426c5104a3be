// Microbenchmark + self-check of the bf16 GEMM tile/stage variants at the encoder's shapes.
//   gemm_bench M K N epi variants [nsplit] [iters]      (epi: 0 STORE 1 RESID 2 SWIGLU 3 GLU)
// Prints one JSON line per variant: average launch time, TFLOP/s and max |err| against a naive
// fp32-accumulate kernel on the same bf16 operands (FULLF32=1: full fp32 operands, fp64 reference;
// meaningful for the fp32 variants -2/-3, 30-33 and the split variants 50-55).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../kernels.h"

using namespace tone;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static uint16_t to_bf16(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

__device__ float bf(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// naive reference: out[m][o] for the epilogue (no rowscale)
__global__ void ref_kernel(const uint16_t* A, const uint16_t* W, const float* bias, const float* R, float* out, int M,
                           int N, int K, int epi, int rowscale) {
  const int m = blockIdx.y, o = blockIdx.x * blockDim.x + threadIdx.x;
  const int nout = (epi >= 2) ? N / 2 : N;
  if (o >= nout) return;
  float den = 1.f;
  if (rowscale) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += bf(A[(int64_t)m * K + k]) * bf(A[(int64_t)m * K + k]);
    den = sqrtf(s) / sqrtf((float)K) + 1e-8f;
  }
  auto dot = [&](int n) {
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc += bf(A[(int64_t)m * K + k]) * bf(W[(int64_t)n * K + k]);
    return acc / den + bias[n];
  };
  float v;
  if (epi <= 1) {
    v = dot(o);
    if (epi == 1) v = R[(int64_t)m * N + o] + v;
  } else {
    const int blk = o / 32, c = o % 32, n0 = blk * 64 + c;
    const float g = dot(n0), u = dot(n0 + 32);
    v = (epi == 2) ? g / (1.f + expf(-g)) * u : g / (1.f + expf(-u));
  }
  out[(int64_t)m * nout + o] = v;
}

// fp64 reference on fp32 operands (FULLF32=1: operands are full-precision fp32, not bf16 values)
__global__ void ref64_kernel(const float* A, const float* W, const float* bias, const float* R, float* out, int M,
                             int N, int K, int epi, int rowscale) {
  const int m = blockIdx.y, o = blockIdx.x * blockDim.x + threadIdx.x;
  const int nout = (epi >= 2) ? N / 2 : N;
  if (o >= nout) return;
  double den = 1.0;
  if (rowscale) {
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += (double)A[(int64_t)m * K + k] * A[(int64_t)m * K + k];
    den = sqrt(s) / sqrt((double)K) + 1e-8;
  }
  auto dot = [&](int n) {
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += (double)A[(int64_t)m * K + k] * W[(int64_t)n * K + k];
    return acc / den + bias[n];
  };
  double v;
  if (epi <= 1) {
    v = dot(o);
    if (epi == 1) v = R[(int64_t)m * N + o] + v;
  } else {
    const int blk = o / 32, c = o % 32, n0 = blk * 64 + c;
    const double g = dot(n0), u = dot(n0 + 32);
    v = (epi == 2) ? g / (1.0 + exp(-g)) * u : g / (1.0 + exp(-u));
  }
  out[(int64_t)m * nout + o] = (float)v;
}

__global__ void err_kernel(const void* C, int cbf, const float* ref, int64_t n, float* err) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float e = 0.f;
  for (; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float c = cbf == 2 ? __half2float(static_cast<const __half*>(C)[i])
                    : cbf ? bf(static_cast<const uint16_t*>(C)[i]) : static_cast<const float*>(C)[i];
    const float r = ref[i];
    e = fmaxf(e, fabsf(c - r) / (1.f + fabsf(r)));
  }
  atomicMax(reinterpret_cast<int*>(err), __float_as_int(e));
}

// MXFP8 helpers (variant 99): dequantize e4m3 + E8M0 to fp32, reference with a given row factor
__global__ void dequant_mx_kernel(const uint8_t* Q, const uint8_t* S, float* out, int64_t rows, int K) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * K) return;
  const int64_t r = i / K;
  const int k = (int)(i % K);
  const float sc = __uint_as_float((uint32_t)S[r * (K / 32) + k / 32] << 23);
  out[i] = __builtin_amdgcn_cvt_f32_fp8((int)Q[i], 0) * sc;
}
__global__ void ref_mx_kernel(const float* A, const float* W, const float* bias, const float* R, const float* inv,
                              float* out, int M, int N, int K, int epi) {
  const int m = blockIdx.y, o = blockIdx.x * blockDim.x + threadIdx.x;
  const int nout = (epi >= 2) ? N / 2 : N;
  if (o >= nout) return;
  const double f = inv ? inv[m] : 1.0;
  auto dot = [&](int n) {
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += (double)A[(int64_t)m * K + k] * W[(int64_t)n * K + k];
    return acc * f + bias[n];
  };
  double v;
  if (epi <= 1) {
    v = dot(o);
    if (epi == 1) v = R[(int64_t)m * N + o] + v;
  } else {
    const int blk = o / 32, c = o % 32, n0 = blk * 64 + c;
    const double g = dot(n0), u = dot(n0 + 32);
    v = g / (1.0 + exp(-g)) * u;
  }
  out[(int64_t)m * nout + o] = (float)v;
}

// the folded-RMSNorm row factor from the sum-of-squares slab (for the reference)
__global__ void ss_to_inv_kernel(const float* ss8, float* inv, int M) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) inv[m] = mx_row_inv(ss8 + (int64_t)m * kSsSlots);
}

// the fused block-final RMSNorm of a RESID row (NORMW=1): the residual sum rounded to fp16 as the stream stores it,
// then w * v / (||v|| / sqrt(N) + 1e-8) in fp64 -- one thread per row, in place over the un-normalized reference
__global__ void norm_ref_kernel(float* ref, const float* w, int M, int N) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float* r = ref + (int64_t)m * N;
  double ss = 0.0;
  for (int n = 0; n < N; ++n) {
    const double v = (double)__half2float(__float2half_rn(r[n]));
    ss += v * v;
  }
  const double den = sqrt(ss) / sqrt((double)N) + 1e-8;
  for (int n = 0; n < N; ++n) r[n] = (float)((double)w[n] * ((double)__half2float(__float2half_rn(r[n])) / den));
}

// Q8=1: the RESID epilogue's MXFP8 form of its bf16 shadow (e4m3 + E8M0) against quant_mx over the same shadow, byte
// for byte, and the row factor its sum-of-squares slab gives against quant_mx's (relative)
__global__ void q8_cmp_kernel(const uint8_t* q, const uint8_t* s, const float* ss, const uint8_t* q2, const uint8_t* s2,
                              const float* ss2, int M, int N, int* bad, float* inv_err) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  int nb = 0;
  for (int n = 0; n < N; ++n) nb += q[(int64_t)m * N + n] != q2[(int64_t)m * N + n];
  for (int n = 0; n < N / 32; ++n) nb += s[(int64_t)m * (N / 32) + n] != s2[(int64_t)m * (N / 32) + n];
  if (nb) atomicAdd(bad, nb);
  const float a = mx_row_inv(ss + (int64_t)m * kSsSlots), b = mx_row_inv(ss2 + (int64_t)m * kSsSlots);
  atomicMax(reinterpret_cast<int*>(inv_err), __float_as_int(fabsf(a - b) / fabsf(b)));
}

// the blocked FFN hidden (common.h hblk_off; HBLK=1): row-major -> blocked and back, bf16 [rows][ld]
// fragment-packed fp32 rows (common.h xpk_off, gemm_d3's A / the fp32 SwiGLU epilogue's c_packed) back to row-major
__global__ void xunpack_kernel(const float* src, float* dst, int64_t rows, int ld) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * ld) return;
  dst[i] = src[xpk_off(i / ld, (int)(i % ld), ld)];
}

__global__ void hblk_kernel(const uint16_t* src, uint16_t* dst, int64_t rows, int ld, int to_blocked) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * ld) return;
  const int64_t r = i / ld;
  const int c = (int)(i % ld);
  if (to_blocked) dst[hblk_off(r, c, ld)] = src[i];
  else dst[i] = src[hblk_off(r, c, ld)];
}

struct Q8Bufs {
  uint8_t *q = nullptr, *s = nullptr, *q2 = nullptr, *s2 = nullptr;
  float *ss = nullptr, *ss2 = nullptr, *inv_err = nullptr;
  int* bad = nullptr;
  void alloc(int M, int N) {
    CK(hipMalloc(&q, (size_t)M * N)); CK(hipMalloc(&s, (size_t)M * N / 32)); CK(hipMalloc(&ss, (size_t)M * kSsSlots * 4));
    CK(hipMalloc(&q2, (size_t)M * N)); CK(hipMalloc(&s2, (size_t)M * N / 32)); CK(hipMalloc(&ss2, (size_t)M * kSsSlots * 4));
    CK(hipMalloc(&bad, 4)); CK(hipMalloc(&inv_err, 4));
  }
  // mismatching bytes and the largest relative row-factor difference
  void check(const uint16_t* C2, int M, int N, int* hbad, float* herr) {
    CK(launch_quant_mx(C2, N, M, N, q2, s2, ss2, 0));
    CK(hipMemset(bad, 0, 4)); CK(hipMemset(inv_err, 0, 4));
    hipLaunchKernelGGL(q8_cmp_kernel, dim3((M + 255) / 256), dim3(256), 0, 0, q, s, ss, q2, s2, ss2, M, N, bad, inv_err);
    CK(hipMemcpy(hbad, bad, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(herr, inv_err, 4, hipMemcpyDeviceToHost));
  }
};

static void run_mx(const uint16_t* A, const uint16_t* W, const float* bias, const float* R, float* ref, float* err,
                   int M, int N, int K, int epi, int rowscale, int iters, int xs = 0, const __half* R16 = nullptr,
                   const float* normw = nullptr) {
  // xs: 98 = the X-stationary kernel (gemm_xs8, SWIGLU only; XSNC = W tiles per item, 0 auto)
  const int xsnc = getenv("XSNC") ? atoi(getenv("XSNC")) : 0;
  // RPMX=1 (RESID, with RES16): the row-panel kernel on MXFP8 operands (gemm_rp_mx) instead of gemm_mx
  const int rpmx = getenv("RPMX") ? atoi(getenv("RPMX")) : 0;
  auto mx = [&](const MxArgs& a) {
    return xs ? gemm_xs8(a, epi, xsnc, 0) : (rpmx && epi == 1) ? gemm_rp_mx(a, normw, 0) : gemm_mx(a, epi, 0);
  };
  // Q8=1 (gemm_rp_mx RESID): also the shadow's MXFP8 form + slab, checked against quant_mx of the shadow
  const bool q8 = rpmx && epi == 1 && getenv("Q8") && atoi(getenv("Q8"));
  const int nout = epi >= 2 ? N / 2 : N;
  uint8_t *A8, *As, *W8, *Ws, *C8, *C8s;
  float *inv, *ss8, *Af, *Wf, *C, *Cf;
  CK(hipMalloc(&ss8, (size_t)M * kSsSlots * 4));
  CK(hipMalloc(&A8, (size_t)M * K)); CK(hipMalloc(&As, (size_t)M * K / 32));
  CK(hipMalloc(&W8, (size_t)N * K)); CK(hipMalloc(&Ws, (size_t)N * K / 32));
  CK(hipMalloc(&inv, (size_t)M * 4)); CK(hipMalloc(&Af, (size_t)M * K * 4)); CK(hipMalloc(&Wf, (size_t)N * K * 4));
  CK(hipMalloc(&C, (size_t)M * nout * 4)); CK(hipMalloc(&Cf, (size_t)M * nout * 4));
  CK(hipMalloc(&C8, (size_t)M * nout)); CK(hipMalloc(&C8s, (size_t)M * nout / 32));
  CK(launch_quant_mx(A, K, M, K, A8, As, rowscale ? ss8 : nullptr, 0));
  if (rowscale) hipLaunchKernelGGL(ss_to_inv_kernel, dim3((M + 255) / 256), dim3(256), 0, 0, ss8, inv, M);
  CK(launch_quant_mx(W, K, N, K, W8, Ws, nullptr, 0));
  hipLaunchKernelGGL(dequant_mx_kernel, dim3((unsigned)(((int64_t)M * K + 255) / 256)), dim3(256), 0, 0, A8, As, Af, (int64_t)M, K);
  hipLaunchKernelGGL(dequant_mx_kernel, dim3((unsigned)(((int64_t)N * K + 255) / 256)), dim3(256), 0, 0, W8, Ws, Wf, (int64_t)N, K);
  // NOREF=1: no fp64 reference (timing / counter runs: under rocprofv3 --pmc the naive reference takes minutes)
  const bool noref = getenv("NOREF") && atoi(getenv("NOREF"));
  if (!noref) {
    hipLaunchKernelGGL(ref_mx_kernel, dim3((nout + 255) / 256, M), dim3(256), 0, 0, Af, Wf, bias, R, rowscale ? inv : nullptr,
                       ref, M, N, K, epi);
    if (normw && rpmx && epi == 1) hipLaunchKernelGGL(norm_ref_kernel, dim3((M + 255) / 256), dim3(256), 0, 0, ref, normw, M, N);
  }
  // LDAPAD: X rows at a pitch of K + LDAPAD bytes (L2 channel spread of the row-strided K-tile reads)
  const int pad = getenv("LDAPAD") ? atoi(getenv("LDAPAD")) : 0;
  uint8_t* A8p = A8;
  if (pad) {
    CK(hipMalloc(&A8p, (size_t)M * (K + pad)));
    CK(hipMemcpy2D(A8p, K + pad, A8, K, K, M, hipMemcpyDeviceToDevice));
  }
  MxArgs a{};
  a.A = A8p; a.lda = K + pad; a.As = As; a.ldas = K / 32; a.W = W8; a.Ws = Ws; a.rs_ss = rowscale ? ss8 : nullptr;
  a.bias = bias; a.C = C; a.ldc = nout; a.c_bf16 = 0; a.R = R16 ? reinterpret_cast<const float*>(R16) : R; a.ldr = N;
  a.alpha = 1.f;
  a.res16 = R16 != nullptr && epi == 1;
  a.C8 = C8; a.C8s = C8s; a.ldc8s = nout / 32; a.M = M; a.N = N; a.K = K;
  a.dbg = getenv("MXDBG") ? atoi(getenv("MXDBG")) : 0;   // gemm_mx.hip DBG bits (SWIGLU only)
  if (epi >= 2) a.ldc = nout;   // bytes of C8 rows
  Q8Bufs qb;
  uint16_t* C2q = nullptr;
  if (q8) {
    qb.alloc(M, N);
    CK(hipMalloc(&C2q, (size_t)M * N * 2));
    a.C2 = C2q; a.Q8 = qb.q; a.Q8s = qb.s; a.ss8 = qb.ss;
  }
  hipError_t rc = mx(a);
  if (rc != hipSuccess) { printf("{\"variant\": %d, \"error\": \"%s\"}\n", xs ? 98 : 99, hipGetErrorString(rc)); return; }
  CK(hipDeviceSynchronize());
  const float* chk = C;
  if (epi >= 2) {
    hipLaunchKernelGGL(dequant_mx_kernel, dim3((unsigned)(((int64_t)M * nout + 255) / 256)), dim3(256), 0, 0, C8, C8s, Cf, (int64_t)M, nout);
    chk = Cf;
  }
  CK(hipMemset(err, 0, 4));
  hipLaunchKernelGGL(err_kernel, dim3(1024), dim3(256), 0, 0, (const void*)chk, a.res16 ? 2 : 0, ref, (int64_t)M * nout, err);
  float herr, q8_inv_err = 0.f;
  int q8_bad = -1;
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  if (q8) qb.check(C2q, M, N, &q8_bad, &q8_inv_err);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(mx(a));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(mx(a));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch_quant_mx(A, K, M, K, A8, As, rowscale ? ss8 : nullptr, 0));   // the slab: M x kSsSlots
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float qms;
  CK(hipEventElapsedTime(&qms, e0, e1));
  printf("{\"M\": %d, \"K\": %d, \"N\": %d, \"epi\": %d, \"variant\": %d, \"us\": %.2f, \"tflops\": %.1f, \"max_rel_err\": %.3g, \"quant_us\": %.2f, \"norm\": %d, \"q8_bad\": %d, \"q8_inv_err\": %.3g}\n",
         M, K, N, epi, xs ? 98 : 99, us, 2.0 * M * N * (double)K / us * 1e-6, herr, qms * 1e3 / iters,
         normw && rpmx && epi == 1 ? 1 : 0, q8_bad, q8_inv_err);
  fflush(stdout);
}

static const int kRpRows[9] = {0, 16, 32, 48, 64, 80, 96, 128, 160};

int main(int argc, char** argv) {
  if (argc < 6) { fprintf(stderr, "usage: %s M K N epi v1,v2,.. [nsplit] [iters]\n", argv[0]); return 2; }
  const int M = atoi(argv[1]), K = atoi(argv[2]), N = atoi(argv[3]), epi = atoi(argv[4]);
  const int nsplit = argc > 6 ? atoi(argv[6]) : 1, iters = argc > 7 ? atoi(argv[7]) : 20;
  const int nout = epi >= 2 ? N / 2 : N;
  int cbf = epi >= 2 ? 1 : 0;   // as in the session: qkv/attn fp32, SWIGLU/GLU bf16
  if (getenv("CBF")) cbf = atoi(getenv("CBF"));   // STORE with a bf16 C (output-byte sensitivity of a shape)
  std::vector<uint16_t> hA((size_t)M * K), hW((size_t)N * K);
  std::vector<float> hb(N), hR((size_t)M * N);
  uint64_t x = 12345;
  auto rnd = [&]() { x = x * 6364136223846793005ull + 1442695040888963407ull; return (float)((x >> 40) & 0xffffff) / 16777216.f * 2.f - 1.f; };
  for (auto& v : hA) v = to_bf16(rnd());
  for (auto& v : hW) v = to_bf16(rnd() * 0.05f);
  for (auto& v : hb) v = rnd() * 0.1f;
  for (auto& v : hR) v = rnd();
  uint16_t *A, *W, *C2;
  float *bias, *R, *ref, *err, *ws;
  void* C;
  CK(hipMalloc(&A, hA.size() * 2)); CK(hipMalloc(&W, hW.size() * 2));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&R, hR.size() * 4));
  CK(hipMalloc(&C, ((size_t)M + 32) * nout * 4)); CK(hipMalloc(&C2, (size_t)M * nout * 2));
  CK(hipMalloc(&ref, (size_t)M * nout * 4)); CK(hipMalloc(&err, 4));
  const int64_t ws_cap = (int64_t)16 * M * N;
  CK(hipMalloc(&ws, ws_cap * 4));
  float* ws_ss;
  CK(hipMalloc(&ws_ss, (size_t)16 * M * 4));   // split-K row sums of squares (rowscale)
  // fp32 copies of the same (bf16-representable) operands for the fp32 path (variant -2)
  // FULLF32=1: full-precision fp32 operands and an fp64 reference (fp32 / x3 variants only)
  const int fullf32 = getenv("FULLF32") ? atoi(getenv("FULLF32")) : 0;
  float *Af, *Wf;
  uint16_t* W3;   // the three bf16 planes of Wf (gemm_x3)
  uint16_t* A3;   // the three bf16 planes of Af (gemm_x3 with a pre-split A, variants 60-65)
  uint16_t* W3P;  // W3 fragment-packed (gemm_d3)
  float* Afp;     // Af fragment-packed (gemm_d3 under PACKX=1)
  {
    std::vector<float> fa(hA.size()), fw(hW.size());
    for (size_t i = 0; i < hA.size(); ++i) { uint32_t u = (uint32_t)hA[i] << 16; memcpy(&fa[i], &u, 4); }
    for (size_t i = 0; i < hW.size(); ++i) { uint32_t u = (uint32_t)hW[i] << 16; memcpy(&fw[i], &u, 4); }
    if (fullf32) {
      for (auto& v : fa) v = rnd();
      for (auto& v : fw) v = rnd() * 0.05f;
    }
    std::vector<uint16_t> w3(3 * fw.size());
    auto bf2f = [](uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; };
    for (size_t i = 0; i < fw.size(); ++i) {
      const uint16_t h = to_bf16(fw[i]);
      const float r1 = fw[i] - bf2f(h);
      const uint16_t m = to_bf16(r1);
      w3[i] = h; w3[fw.size() + i] = m; w3[2 * fw.size() + i] = to_bf16(r1 - bf2f(m));
    }
    CK(hipMalloc(&Af, fa.size() * 4)); CK(hipMalloc(&Wf, fw.size() * 4)); CK(hipMalloc(&W3, w3.size() * 2));
    CK(hipMemcpy(Af, fa.data(), fa.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(Wf, fw.data(), fw.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W3, w3.data(), w3.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint16_t> a3(3 * fa.size());
    for (size_t i = 0; i < fa.size(); ++i) {
      const uint16_t h = to_bf16(fa[i]);
      const float r1 = fa[i] - bf2f(h);
      const uint16_t m = to_bf16(r1);
      a3[i] = h; a3[fa.size() + i] = m; a3[2 * fa.size() + i] = to_bf16(r1 - bf2f(m));
    }
    CK(hipMalloc(&A3, a3.size() * 2));
    // gemm_d3's fragment-packed operands: W's planes always, A's rows under PACKX=1 (padding rows NaN: they must
    // not reach any stored output)
    const size_t mp = (size_t)(M + 31) / 32 * 32;
    std::vector<uint16_t> w3p(w3.size());
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k)
        for (int pl = 0; pl < 3; ++pl) w3p[wpk_off(n, k, pl, K)] = w3[(size_t)pl * fw.size() + (size_t)n * K + k];
    CK(hipMalloc(&W3P, w3p.size() * 2));
    CK(hipMemcpy(W3P, w3p.data(), w3p.size() * 2, hipMemcpyHostToDevice));
    std::vector<float> afp(mp * K, std::nanf(""));
    for (int m = 0; m < M; ++m)
      for (int k = 0; k < K; ++k) afp[xpk_off(m, k, K)] = fa[(size_t)m * K + k];
    CK(hipMalloc(&Afp, afp.size() * 4));
    CK(hipMemcpy(Afp, afp.data(), afp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(A3, a3.data(), a3.size() * 2, hipMemcpyHostToDevice));
  }
  CK(hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(R, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
  const int rowscale = getenv("ROWSCALE") ? atoi(getenv("ROWSCALE")) : 0;
  if (fullf32) hipLaunchKernelGGL(ref64_kernel, dim3((nout + 255) / 256, M), dim3(256), 0, 0, Af, Wf, bias, R, ref, M, N, K, epi, rowscale);
  else hipLaunchKernelGGL(ref_kernel, dim3((nout + 255) / 256, M), dim3(256), 0, 0, A, W, bias, R, ref, M, N, K, epi, rowscale);
  CK(hipDeviceSynchronize());

  GemmArgs a{};
  a.A = A; a.lda = K; a.W = W; a.C = C; a.ldc = nout; a.bias = bias; a.R = R; a.ldr = N; a.alpha = 1.f;
  a.M = M; a.N = N; a.K = K; a.ws = ws; a.ws_ss = ws_ss; a.ws_cap = ws_cap; a.a_bf16 = 1; a.c_bf16 = cbf;
  a.C2 = (epi == 1 || (epi == 0 && !cbf)) ? C2 : nullptr;   // the session's shadowed outputs
  if (getenv("NOC2")) a.C2 = nullptr;                         // fp32 mode: no bf16 shadow
  // RES16=1: the bf16 / fp8 modes' fp16 residual stream (R and C fp16; the reference keeps its fp32 R)
  const bool res16 = getenv("RES16") && atoi(getenv("RES16"));
  __half* R16 = nullptr;
  if (res16) {
    std::vector<__half> h(hR.size());
    for (size_t i = 0; i < h.size(); ++i) h[i] = __float2half(hR[i]);
    CK(hipMalloc(&R16, h.size() * 2));
    CK(hipMemcpy(R16, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    a.R = reinterpret_cast<const float*>(R16);
    a.res16 = 1;
  }
  a.rowscale = rowscale;
  a.inv_sqrt_k = 1.0f / sqrtf((float)K);
  // NORMW=1: RESID with the fused row RMSNorm (gemm_rp / gemm_rp_mx only; gain = 1 + small noise), checked against the
  // reference row normalized the same way (norm_ref_kernel)
  float* normw = nullptr;
  if (getenv("NORMW") && atoi(getenv("NORMW"))) {
    std::vector<float> g(N);
    for (auto& v : g) v = 1.0f + 0.1f * rnd();
    CK(hipMalloc(&normw, N * 4));
    CK(hipMemcpy(normw, g.data(), N * 4, hipMemcpyHostToDevice));
  }
  float* refn = nullptr;
  if (normw) CK(hipMalloc(&refn, (size_t)M * nout * 4));
  uint16_t *Ablk = nullptr, *Cun = nullptr;
  float* Cunf = nullptr;
  Q8Bufs q8b;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double flop = 2.0 * M * N * (double)K;
  char* list = strdup(argv[5]);
  for (char* tok = strtok(list, ","); tok; tok = strtok(nullptr, ",")) {
    const int vv = atoi(tok);
    if (vv == 99 || vv == 98) {   // MXFP8 path: quant_mx + gemm_mx (99) / gemm_xs8 (98) vs an fp64 reference
      run_mx(A, W, bias, R, ref, err, M, N, K, epi, rowscale, iters, vv == 98, res16 ? R16 : nullptr, normw);
      continue;
    }
    // v % 100 = variant (20..23: gemm_t tiles); (v / 100) bits: 1 N-partitioned XCD order,
    // 2 non-temporal stores, 4.. debug (no epilogue / no K loop)
    const int v = vv < 0 ? vv : (vv % 100);   // -1 gemm() bf16, -2 gemm() fp32 (+W3), -3 gemm() fp32 (no W3)
    const int fl = vv < 0 ? 0 : vv / 100;
    a.order_n = fl & 1;
    a.nt_store = (fl >> 1) & 1;
    a.dbg = (fl >> 2) & 255;   // gemm_t: 1 no epilogue, 2 no MFMA, 4 no DMA; gemm_r3: see gemm_t.hip
    if (vv <= -300 && getenv("XSDBG")) a.dbg = atoi(getenv("XSDBG"));   // gemm_xw ablations
    // RESID writes C in place of R in the session; here R is separate so repeated launches are idempotent
    CK(hipMemset(C, 0, (size_t)M * nout * 4));
    const bool f32 = (vv == -2) || (vv == -3) || (vv == -4) || (vv <= -499) || (v >= 30 && v < 50) || (v >= 50 && v < 90);
    // -2: gemm() fp32 routing with W planes, -3: without, -4: with W and A planes
    a.W3 = (vv == -2 || vv == -4 || vv <= -499 || (v >= 50 && v < 90)) ? W3 : nullptr;
    a.a_plane = (vv == -4 || (v >= 60 && v < 70)) ? (int64_t)M * K : 0;
    a.A = a.a_plane ? (const void*)A3 : f32 ? (const void*)Af : (const void*)A;
    a.W3P = W3P;
    // PACKX=1: gemm_d3 reads A fragment-packed; CPACK=1: an fp32 SWIGLU variant writes C fragment-packed (unpacked
    // for the check)
    a.a_packed = vv <= -499 && getenv("PACKX") && atoi(getenv("PACKX"));   // -499: gemm()'s routing (gemm_d3 by shape)
    if (a.a_packed) a.A = Afp;
    a.c_packed = f32 && epi == 2 && (vv > -300 || vv == -499) && getenv("CPACK") && atoi(getenv("CPACK"));
    // CPOUT=1 (gemm_d3 STORE / RESID through gemm()): also the packed copy of C (GemmArgs::CP), checked unpacked
    const bool cpout = vv == -499 && (epi == 0 || epi == 1) && getenv("CPOUT") && atoi(getenv("CPOUT"));
    static float* CPbuf = nullptr;
    if (cpout && !CPbuf) CK(hipMalloc(&CPbuf, ((size_t)M + 32) * nout * 4));
    a.CP = cpout ? CPbuf : nullptr;
    a.W = f32 ? (const void*)Wf : (const void*)W;
    a.a_bf16 = !f32;
    a.c_bf16 = f32 ? 0 : cbf;
    a.res16 = res16 && !f32;
    // the residual buffer in the type the variant reads: an fp32 variant under RES16 must not be handed the fp16
    // buffer (half the bytes: it read past the end -- a GPU memory fault, round 6)
    a.R = a.res16 ? reinterpret_cast<const float*>(R16) : R;
    a.norm_w = (v >= 90 && v <= 98) ? normw : nullptr;
    // HBLK=1: gemm_xw SWIGLU writes / gemm_rp reads the blocked hidden (checked through a row-major copy / built from one)
    const bool hblk = getenv("HBLK") && atoi(getenv("HBLK")) && ((vv <= -300 && epi == 2) || (v >= 90 && v <= 98 && epi == 1));
    a.h_blocked = hblk;
    if (hblk && v >= 90) {
      if (!Ablk) {
        CK(hipMalloc(&Ablk, ((size_t)M + 32) * K * 2));
        hipLaunchKernelGGL(hblk_kernel, dim3((unsigned)(((int64_t)M * K + 255) / 256)), dim3(256), 0, 0, A, Ablk, (int64_t)M, K, 1);
      }
      a.A = Ablk;
    }
    const float* chk_ref = ref;
    if (a.norm_w && epi == 1) {   // the normalized reference (once per variant: cheap next to the fp32 reference)
      CK(hipMemcpy(refn, ref, (size_t)M * nout * 4, hipMemcpyDeviceToDevice));
      hipLaunchKernelGGL(norm_ref_kernel, dim3((M + 255) / 256), dim3(256), 0, 0, refn, normw, M, N);
      chk_ref = refn;
    }
    // Q8=1 (gemm_rp, RESID with the shadow): the shadow's MXFP8 form + slab, checked against quant_mx of the shadow
    const bool q8 = v >= 90 && v <= 98 && epi == 1 && a.C2 && getenv("Q8") && atoi(getenv("Q8"));
    if (q8) {
      if (!q8b.q) q8b.alloc(M, N);
      a.C8 = q8b.q; a.C8s = q8b.s; a.ss8 = q8b.ss;
    } else {
      a.C8 = nullptr; a.C8s = nullptr; a.ss8 = nullptr;
    }
    auto launch = [&]() {
      return vv <= -600 ? gemm_d3n(a, epi, -600 - vv, 0)   // -600 - c: gemm_d3n variant c
             : vv <= -500 ? gemm_d3(a, epi, -500 - vv, 0)   // -500 - c: gemm_d3 variant c
             : vv == -499 ? gemm(a, epi, false, 0)
             : vv <= -300 ? gemm_xw(a, epi, -300 - vv, 0)   // -300: gemm_xw auto run length, -300 - c: c W tiles per item
             : v < 0 ? gemm(a, epi, !f32, 0)
             : (v >= 90 && v <= 98) ? gemm_rp(a, 0, kRpRows[v - 90])   // 90: auto panel rows, 91-98: 16 .. 160
             : v >= 70 ? gemm_x3(a, epi, v - 70, 0)   // 70-89: fp32 A, any x3 tile variant
             : v >= 60 ? gemm_x3(a, epi, v - 60, 0)
             : (v >= 50 && nsplit > 1) ? gemm_x3_splitk(a, epi, v - 50, nsplit, 0)
             : v >= 50 ? gemm_x3(a, epi, v - 50, 0)
             : v >= 40 ? gemm_r3(a, epi, v - 40, 0)        // 40-49: fp32 W and X, K-tile ring
             : v >= 30 ? gemm_f32t(a, epi, v - 30, 0)
             : v >= 20 ? gemm_t(a, epi, v - 20, 0)
                       : gemm_bf16_variant(a, epi, v, nsplit, 0);
    };
    hipError_t rc = launch();
    if (rc != hipSuccess) { printf("{\"variant\": %d, \"error\": \"%s\"}\n", v, hipGetErrorString(rc)); continue; }
    CK(hipDeviceSynchronize());
    CK(hipMemset(err, 0, 4));
    const void* Cchk = C;
    if (a.c_packed) {
      if (!Cunf) CK(hipMalloc(&Cunf, (size_t)M * nout * 4));
      hipLaunchKernelGGL(xunpack_kernel, dim3((unsigned)(((int64_t)M * nout + 255) / 256)), dim3(256), 0, 0,
                         static_cast<const float*>(C), Cunf, (int64_t)M, nout);
      Cchk = Cunf;
    }
    if (hblk && vv <= -300) {   // the blocked output, back to row-major for the check
      if (!Cun) CK(hipMalloc(&Cun, (size_t)M * nout * 2));
      hipLaunchKernelGGL(hblk_kernel, dim3((unsigned)(((int64_t)M * nout + 255) / 256)), dim3(256), 0, 0,
                         static_cast<const uint16_t*>(C), Cun, (int64_t)M, nout, 0);
      Cchk = Cun;
    }
    float cp_err = -1.f;
    if (cpout) {   // the packed copy, unpacked, against the same reference
      if (!Cunf) CK(hipMalloc(&Cunf, (size_t)M * nout * 4));
      hipLaunchKernelGGL(xunpack_kernel, dim3((unsigned)(((int64_t)M * nout + 255) / 256)), dim3(256), 0, 0, CPbuf, Cunf,
                         (int64_t)M, nout);
      CK(hipMemset(err, 0, 4));
      hipLaunchKernelGGL(err_kernel, dim3(1024), dim3(256), 0, 0, (const void*)Cunf, 0, chk_ref, (int64_t)M * nout, err);
      CK(hipMemcpy(&cp_err, err, 4, hipMemcpyDeviceToHost));
      CK(hipMemset(err, 0, 4));
    }
    hipLaunchKernelGGL(err_kernel, dim3(1024), dim3(256), 0, 0, Cchk, a.res16 && epi <= 1 ? 2 : a.c_bf16, chk_ref, (int64_t)M * nout, err);
    float herr, herr2 = 0.f, q8_inv_err = 0.f;
    int q8_bad = -1;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    if (a.C2) {   // the bf16 shadow must hold the same values (bf16-rounded)
      CK(hipMemset(err, 0, 4));
      hipLaunchKernelGGL(err_kernel, dim3(1024), dim3(256), 0, 0, (const void*)a.C2, 1, chk_ref, (int64_t)M * nout, err);
      CK(hipMemcpy(&herr2, err, 4, hipMemcpyDeviceToHost));
    }
    if (q8) q8b.check(a.C2, M, N, &q8_bad, &q8_inv_err);
    for (int i = 0; i < 3; ++i) CK(launch());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) CK(launch());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("{\"M\": %d, \"K\": %d, \"N\": %d, \"epi\": %d, \"variant\": %d, \"nsplit\": %d, \"us\": %.2f, \"tflops\": %.1f, \"max_rel_err\": %.3g, \"shadow_err\": %.3g, \"norm\": %d, \"q8_bad\": %d, \"q8_inv_err\": %.3g, \"hblk\": %d, \"cp_err\": %.3g}\n",
           M, K, N, epi, vv, nsplit, us, flop / us * 1e-6, herr, herr2, a.norm_w && epi == 1 ? 1 : 0, q8_bad, q8_inv_err,
           (int)hblk, cp_err);
    fflush(stdout);
  }
  return 0;
}
