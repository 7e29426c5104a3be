// Element-wise check of the non-GEMM kernels of the streaming step at the bench's batches (tests/test_gpu_kernels.py).
//   kernel_check <check> <B> [T]
// Each check feeds ONE launch of a library kernel seeded synthetic inputs and a seeded state slab, runs it once, and
// compares every output element -- and every element of every state row the launch may touch -- with a naive GPU
// reference: one thread per output element, plain loops in the reference model's own order of operations
// (tone/nn/modules/conformer_blocks.py, submodules.py, conformer.py; the numpy oracle oracle/tone_oracle.py restates
// the same), fp64 accumulation unless stated.  The reference consumes the kernel's own operands (the bf16-rounded
// values where the kernel rounds), so a wrong tile, row, stream or a race shows as an O(1) error while the kernel's
// legitimate roundings stay at their own size.
//
// State handling: the slab holds 2B rows of 219729 fp16 (odd stride: the kernels see 2-byte-aligned rows); stream b
// reads row 2 p(b) and writes row 2 p(b) + 1 (p a permutation: the run_rows ping-pong form).  Read rows are filled with
// hashed values, written rows with a NaN sentinel.  After the launch every read row must be unchanged, every element
// of a written row outside the sections the kernel owns must still be the sentinel, and the owned sections must equal
// the reference (`state_ulp`: largest fp16 ulp distance, 0 for copies; `state_err`: largest |out - ref| / (1 + |ref|),
// the measure for recomputed values, whose ulp distance near zero says nothing).
//
// Prints one JSON line: {"check", "B", "T", outputs: {name: max |out - ref| / (1 + |ref|)}, "nan", "state_ulp",
// "state_err", "state_sentinel_bad", "state_in_changed", "us" (the launch's mean time over 20 warm repeats, measured
// after the checks)}.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <string>
#include <type_traits>
#include <vector>

#include "../kernels.h"

using namespace tone;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

// ---- seeded values -----------------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__host__ __device__ inline float urand(uint64_t seed, int64_t i) {   // uniform in [-1, 1)
  return (float)(mix64(seed * 0x100000001B3ull + (uint64_t)i) >> 40) / 16777216.f * 2.f - 1.f;
}
__device__ inline float bfr(float v) { return (float)(__bf16)v; }     // round to bf16 (RNE)
__device__ inline float h2f(__half h) { return __half2float(h); }

__global__ void fill_f32_kernel(float* p, int64_t n, uint64_t seed, float scale, float bias, int round_bf) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = bias + scale * urand(seed, i);
    p[i] = round_bf ? bfr(v) : v;
  }
}
__global__ void f32_to_bf16_kernel(const float* s, uint16_t* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    store_bf16(d, i, s[i]);
}
__global__ void f32_to_f16_kernel(const float* s, __half* d, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = __float2half_rn(s[i]);
}

static const dim3 kFillGrid(2048), kFillBlock(256);

struct Pool {   // every device allocation of a check, freed at exit
  std::vector<void*> ptrs;
  template <typename T>
  T* get(int64_t n) {
    void* p = nullptr;
    CK(hipMalloc(&p, (size_t)(n > 0 ? n : 1) * sizeof(T)));
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  ~Pool() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};
static Pool pool;

// fp32 array of seeded values (bf16-exact when round_bf)
static float* rand_f32(int64_t n, uint64_t seed, float scale, float bias = 0.f, bool round_bf = false) {
  float* p = pool.get<float>(n);
  hipLaunchKernelGGL(fill_f32_kernel, kFillGrid, kFillBlock, 0, 0, p, n, seed, scale, bias, (int)round_bf);
  return p;
}
static uint16_t* to_bf16(const float* s, int64_t n) {
  uint16_t* d = pool.get<uint16_t>(n);
  hipLaunchKernelGGL(f32_to_bf16_kernel, kFillGrid, kFillBlock, 0, 0, s, d, n);
  return d;
}
static __half* to_f16(const float* s, int64_t n) {
  __half* d = pool.get<__half>(n);
  hipLaunchKernelGGL(f32_to_f16_kernel, kFillGrid, kFillBlock, 0, 0, s, d, n);
  return d;
}
static std::vector<float> to_host(const float* d, int64_t n) {
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
  return h;
}

// ---- results -------------------------------------------------------------------------------------------------------
struct Res {
  float err;    // max |out - ref| / (1 + |ref|) per output
  int nan;      // non-finite outputs where the reference is finite
  int ulp;      // state: largest fp16 ulp distance in the owned sections
  int sent;     // state: written-row elements outside the owned sections that lost the sentinel
  int inchg;    // state: read-row elements that changed
  int pad;
};

__device__ inline float load_typed(const void* p, int ty, int64_t i) {
  if (ty == 1) return load_act<true>(p, i);
  if (ty == 2) return __half2float(static_cast<const __half*>(p)[i]);
  return static_cast<const float*>(p)[i];
}

// every element of a [rows][cols] output (row pitch ld) against the reference [rows][cols]
__global__ void cmp_kernel(const void* o, int ty, int64_t ld, const float* ref, int64_t rows, int cols, Res* r) {
  float e = 0.f;
  int nan = 0;
  const int64_t n = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / cols;
    const int c = (int)(i % cols);
    const float v = load_typed(o, ty, row * ld + c), f = ref[i];
    if (!isfinite(v) && isfinite(f)) {
      ++nan;
      continue;
    }
    e = fmaxf(e, fabsf(v - f) / (1.f + fabsf(f)));
  }
  atomicMax(reinterpret_cast<int*>(&r->err), __float_as_int(e));
  if (nan) atomicAdd(&r->nan, nan);
}

// ---- the state slab --------------------------------------------------------------------------------------------------
constexpr uint16_t kSentinel = 0x7E01;   // a NaN no kernel produces
constexpr uint64_t kStateSeed = 77;

__device__ inline float state_init_value(int64_t row, int64_t e) {
  if (e == kOffMhsaLen) return (float)(mix64(row * 131 + 7) % 31);   // mhsa_len: 0 .. 30
  return urand(kStateSeed, row * kStateSize + e);
}
__global__ void init_slab_kernel(__half* s, int64_t stride, int64_t rows) {
  const int64_t n = rows * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / stride, e = i % stride;
    if (row & 1) s[i] = __ushort_as_half(kSentinel);
    else s[i] = __float2half_rn(state_init_value(row, e));
  }
}

struct Sec {
  int64_t off, len;
};
struct Secs {
  Sec s[3];
  int n;
  int64_t total;
};

__device__ inline int f16_ord(uint16_t h) { return (h & 0x8000) ? -(int)(h & 0x7fff) : (int)h; }

// ex: the owned sections' expected fp16 values per stream, [B][secs.total] (sections concatenated in order)
__global__ void check_slab_kernel(const __half* s, int64_t stride, int B, const int* rows_in, const int* rows_out,
                                  Secs secs, const __half* ex, Res* r) {
  int ulp = 0, sent = 0, inchg = 0;
  float serr = 0.f;
  const int64_t n = (int64_t)B * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / stride);
    const int64_t e = i % stride;
    // the read row is unchanged
    const int64_t ri = rows_in[b];
    const uint16_t hin = __half_as_ushort(s[ri * stride + e]);
    if (hin != __half_as_ushort(__float2half_rn(state_init_value(ri, e)))) ++inchg;
    // the written row: owned sections against the reference, the rest still the sentinel
    const uint16_t hout = __half_as_ushort(s[(int64_t)rows_out[b] * stride + e]);
    int64_t base = 0, k = -1;
    for (int q = 0; q < secs.n; ++q) {
      if (e >= secs.s[q].off && e < secs.s[q].off + secs.s[q].len) k = base + (e - secs.s[q].off);
      base += secs.s[q].len;
    }
    if (k < 0) {
      if (hout != kSentinel) ++sent;
    } else {
      const uint16_t he = __half_as_ushort(ex[(int64_t)b * secs.total + k]);
      const int d = (hout == kSentinel) ? 1 << 20 : abs(f16_ord(hout) - f16_ord(he));
      ulp = max(ulp, d);
      const float fo = __half2float(__ushort_as_half(hout)), fe = __half2float(__ushort_as_half(he));
      serr = fmaxf(serr, hout == kSentinel ? 1e30f : fabsf(fo - fe) / (1.f + fabsf(fe)));
    }
  }
  if (ulp) atomicMax(&r->ulp, ulp);
  atomicMax(reinterpret_cast<int*>(&r->err), __float_as_int(serr));
  if (sent) atomicAdd(&r->sent, sent);
  if (inchg) atomicAdd(&r->inchg, inchg);
}

struct Slab {
  __half* p = nullptr;
  int64_t stride = kStateSize;
  int B = 0;
  int *rows_in = nullptr, *rows_out = nullptr;
  std::vector<int> hin, hout;
  void make(int b) {
    B = b;
    p = pool.get<__half>((int64_t)2 * B * stride);
    hipLaunchKernelGGL(init_slab_kernel, kFillGrid, kFillBlock, 0, 0, p, stride, (int64_t)2 * B);
    hin.resize(B);
    hout.resize(B);
    for (int i = 0; i < B; ++i) {   // p(b) = (7 b + 3) mod B: a permutation for B coprime with 7
      const int q = (int)(((int64_t)7 * i + 3) % B);
      hin[i] = 2 * q;
      hout[i] = 2 * q + 1;
    }
    rows_in = pool.get<int>(B);
    rows_out = pool.get<int>(B);
    CK(hipMemcpy(rows_in, hin.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(rows_out, hout.data(), B * 4, hipMemcpyHostToDevice));
  }
  StateRef ref() const { return StateRef{p, p, stride, rows_in, rows_out}; }
};

// ---- output bookkeeping ----------------------------------------------------------------------------------------------
struct Report {
  std::string check;
  int B, T;
  std::vector<std::pair<std::string, Res>> outs;
  Res st{};
  bool has_state = false;
  double us = 0;
  Res* dres = nullptr;
  Report() { CK(hipMalloc(&dres, sizeof(Res))); }
  void out(const char* name, const void* o, int ty, int64_t ld, const float* ref, int64_t rows, int cols) {
    CK(hipMemset(dres, 0, sizeof(Res)));
    hipLaunchKernelGGL(cmp_kernel, dim3(2048), dim3(256), 0, 0, o, ty, ld, ref, rows, cols, dres);
    Res h;
    CK(hipMemcpy(&h, dres, sizeof(Res), hipMemcpyDeviceToHost));
    outs.emplace_back(name, h);
  }
  void state(const Slab& sl, const Secs& secs, const __half* ex) {
    CK(hipMemset(dres, 0, sizeof(Res)));
    hipLaunchKernelGGL(check_slab_kernel, dim3(4096), dim3(256), 0, 0, sl.p, sl.stride, sl.B, sl.rows_in, sl.rows_out,
                       secs, ex, dres);
    CK(hipMemcpy(&st, dres, sizeof(Res), hipMemcpyDeviceToHost));
    has_state = true;
  }
  void print() const {
    printf("{\"check\": \"%s\", \"B\": %d, \"T\": %d, \"outputs\": {", check.c_str(), B, T);
    int nan = 0;
    for (size_t i = 0; i < outs.size(); ++i) {
      printf("%s\"%s\": %.4g", i ? ", " : "", outs[i].first.c_str(), outs[i].second.err);
      nan += outs[i].second.nan;
    }
    printf("}, \"nan\": %d", nan);
    if (has_state)
      printf(", \"state_ulp\": %d, \"state_err\": %.4g, \"state_sentinel_bad\": %d, \"state_in_changed\": %d", st.ulp,
             st.err, st.sent, st.inchg);
    printf(", \"us\": %.2f}\n", us);
    fflush(stdout);
  }
};

// the launch under test: run once here (the checks compare its outputs); Report::print times it afterwards (3 warm-up
// launches, then the mean of 20), when the results have been read -- later launches may change the state they read
static std::function<hipError_t()> g_launch;
template <typename F>
static double time_once(F&& f) {
  g_launch = f;
  CK(f());
  CK(hipDeviceSynchronize());
  return 0.0;
}
static double time_warm() {
  if (!g_launch) return 0.0;
  for (int i = 0; i < 3; ++i) CK(g_launch());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < 20; ++i) CK(g_launch());
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / 20;
}

static dim3 grid1(int64_t n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

// =====================================================================================================================
// a3: pre-encode (ConvSubsamplingPreEncode.forward, conformer_blocks.py:631-641)
// x1[b][r][m], r < 10 + MT: the carried sub1 rows, then RMSNorm_64(feats) (eps outside the sqrt, submodules.py:34-54)
__global__ void ref_x1_kernel(const float* feats, StateRef s, const float* pw, int MT, float* x1, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int R = kSub1S + MT;
  if (i >= (int64_t)B * R * kMels) return;
  const int m = (int)(i % kMels), r = (int)((i / kMels) % R), b = (int)(i / ((int64_t)kMels * R));
  if (r < kSub1S) {
    x1[i] = h2f(s.in[s.row_in(b) + kOffSub1 + r * kMels + m]);
    return;
  }
  const float* f = feats + ((int64_t)b * MT + (r - kSub1S)) * kMels;
  double ss = 0.0;
  for (int k = 0; k < kMels; ++k) ss += (double)f[k] * f[k];
  const double den = sqrt(ss) / 8.0 + 1e-8;
  x1[i] = (float)((double)pw[m] * ((double)f[m] / den));
}
// c1[b][t][f][c] = SiLU(scale (sum_{kt<11, kf<21} w1[c][kt][kf] x1[t + kt][f + kf]) + shift); bf: x1 rounded to bf16 as
// the bf16 kernels' operand
__global__ void ref_conv1_kernel(const float* x1, const float* w1, int bf, const float* sc, const float* sh, int MT,
                                 float* c1, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * MT * kSub1F * kSub1C) return;
  const int c = (int)(i % kSub1C), f = (int)((i / kSub1C) % kSub1F), t = (int)((i / (kSub1C * kSub1F)) % MT);
  const int b = (int)(i / ((int64_t)kSub1C * kSub1F * MT));
  const float* xb = x1 + (int64_t)b * (kSub1S + MT) * kMels;
  double acc = 0.0;
  for (int kt = 0; kt < kSub1Kt; ++kt)
    for (int kf = 0; kf < kSub1Kf; ++kf) {
      float xv = xb[(t + kt) * kMels + f + kf];
      if (bf) xv = bfr(xv);
      acc += (double)w1[(c * kSub1Kt + kt) * kSub1Kf + kf] * xv;
    }
  const double z = acc * sc[c] + sh[c];
  c1[i] = (float)(z / (1.0 + exp(-z)));
}
// the conv2 input [b][8 + MT][44][32] channels-last: the carried sub2 rows (state [c][8][44]), then c1; bf: as bf16
__global__ void ref_x2_kernel(StateRef s, const float* c1, int bf, int MT, float* x2, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int R = kSub2S + MT;
  if (i >= (int64_t)B * R * kSub1F * kSub1C) return;
  const int c = (int)(i % kSub1C), f = (int)((i / kSub1C) % kSub1F), r = (int)((i / (kSub1C * kSub1F)) % R);
  const int b = (int)(i / ((int64_t)kSub1C * kSub1F * R));
  float v;
  if (r < kSub2S) v = h2f(s.in[s.row_in(b) + kOffSub2 + (c * kSub2S + r) * kSub1F + f]);
  else v = c1[(((int64_t)b * MT + r - kSub2S) * kSub1F + f) * kSub1C + c];
  x2[i] = bf ? bfr(v) : v;
}
// expected next sub1 (the last 10 x1 rows) and sub2 (c1 rows MT - 8 .. MT - 1 as [c][8][44]), fp16, [B][640 + 11264]
__global__ void ref_sub_state_kernel(const float* x1, const float* c1, int MT, __half* ex, int B) {
  constexpr int n1 = kSub1S * kMels, n2 = kSub1C * kSub2S * kSub1F;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * (n1 + n2)) return;
  const int b = (int)(i / (n1 + n2)), e = (int)(i % (n1 + n2));
  float v;
  if (e < n1) {
    v = x1[((int64_t)b * (kSub1S + MT) + MT + e / kMels) * kMels + e % kMels];
  } else {
    const int q = e - n1, c = q / (kSub2S * kSub1F), r = (q / kSub1F) % kSub2S, f = q % kSub1F;
    v = c1[(((int64_t)b * MT + MT - kSub2S + r) * kSub1F + f) * kSub1C + c];
  }
  ex[i] = __float2half_rn(v);
}
// flat[b*T + t][f*64 + c] = SiLU(scale (sum_{kt, kf, ci} w2[c][(kt*11 + kf)*32 + ci] x2[3t + kt][f + kf][ci]) + shift)
// (w2 tap-major [64][kw]); F64: fp64 accumulation, else fp32 (the bf16 checks: 345 G MACs at B = 4096)
template <bool F64>
__global__ void ref_conv2_kernel(const float* x2, const float* w2, int kw, const float* sc, const float* sh, int IN, int T,
                                 float* flat, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * T * kSub2F * kSub2C) return;
  const int c = (int)(i % kSub2C), f = (int)((i / kSub2C) % kSub2F), t = (int)((i / (kSub2C * kSub2F)) % T);
  const int b = (int)(i / ((int64_t)kSub2C * kSub2F * T));
  const float* xb = x2 + (int64_t)b * IN * kSub1F * kSub1C;
  const float* wc = w2 + (int64_t)c * kw;
  typename std::conditional<F64, double, float>::type acc = 0;
  for (int kt = 0; kt < kSub2Kt; ++kt)
    for (int kf = 0; kf < kSub2Kf; ++kf) {
      const float* xr = xb + ((kSub2Stride * t + kt) * kSub1F + f + kf) * kSub1C;
      const float* wr = wc + (kt * kSub2Kf + kf) * kSub1C;
      for (int ci = 0; ci < kSub1C; ++ci) acc += (decltype(acc))wr[ci] * xr[ci];
    }
  const double z = (double)acc * sc[c] + sh[c];
  flat[i] = (float)(z / (1.0 + exp(-z)));
}

static Secs sub_secs() {
  Secs s{};
  s.s[0] = {kOffSub1, kSub1S * kMels};
  s.s[1] = {kOffSub2, kSub1C * kSub2S * kSub1F};
  s.n = 2;
  s.total = s.s[0].len + s.s[1].len;
  return s;
}

// host: bf16 bits of an fp32 value (RNE) and the exact 3-term split (session.hip upload_w)
static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// the pre-encode front: "sub_conv" (bf16, 300 ms: RMSNorm + conv1 + conv2 in one launch), "sub1" (fp32 / bf16 conv1
// alone, x2 written to HBM; 400 ms and the fp32 mode)
static void check_pre(const std::string& which, int B, int chunk, bool bf, Report& rep) {
  const Geom geo = make_geom(chunk);
  const int MT = geo.melT, IN = geo.sub2In, T = geo.T;
  Slab sl;
  sl.make(B);
  const float* feats = rand_f32((int64_t)B * MT * kMels, 11, 4.f, -2.f);
  const float* pw = rand_f32(kMels, 12, 0.1f, 1.f);
  // conv1 weights [32][11][21], bf16-exact values (one set for both modes); the bf16 kernels' [kt][c][32] copy
  std::vector<float> w1h(kSub1C * kSub1Kt * kSub1Kf);
  for (size_t i = 0; i < w1h.size(); ++i) w1h[i] = bf2f(f2bf(0.07f * urand(13, i)));
  std::vector<uint16_t> w1t((size_t)kSub1Kt * kSub1C * 32, 0);
  for (int c = 0; c < kSub1C; ++c)
    for (int kt = 0; kt < kSub1Kt; ++kt)
      for (int kf = 0; kf < kSub1Kf; ++kf) w1t[((size_t)kt * kSub1C + c) * 32 + kf] = f2bf(w1h[(c * kSub1Kt + kt) * kSub1Kf + kf]);
  float* w1 = pool.get<float>(w1h.size());
  uint16_t* w1td = pool.get<uint16_t>(w1t.size());
  CK(hipMemcpy(w1, w1h.data(), w1h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w1td, w1t.data(), w1t.size() * 2, hipMemcpyHostToDevice));
  const float* sc1 = rand_f32(kSub1C, 14, 0.2f, 1.f);
  const float* sh1 = rand_f32(kSub1C, 15, 0.3f);
  const float* sc2 = rand_f32(kSub2C, 16, 0.2f, 1.f);
  const float* sh2 = rand_f32(kSub2C, 17, 0.3f);
  // conv2 weights [64][3872] tap-major (bf16-exact) and the bf16 kernels' padded [64][3904]
  std::vector<float> w2h((size_t)kSub2C * kConv2K);
  for (size_t i = 0; i < w2h.size(); ++i) w2h[i] = bf2f(f2bf(0.03f * urand(18, i)));
  std::vector<uint16_t> w2c((size_t)kSub2C * kConv2KPad, 0);
  for (int c = 0; c < kSub2C; ++c)
    for (int k = 0; k < kConv2K; ++k) w2c[(size_t)c * kConv2KPad + k] = f2bf(w2h[(size_t)c * kConv2K + k]);
  float* w2 = pool.get<float>(w2h.size());
  uint16_t* w2cd = pool.get<uint16_t>(w2c.size());
  CK(hipMemcpy(w2, w2h.data(), w2h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w2cd, w2c.data(), w2c.size() * 2, hipMemcpyHostToDevice));

  // references
  float* x1 = pool.get<float>((int64_t)B * (kSub1S + MT) * kMels);
  float* c1 = pool.get<float>((int64_t)B * MT * kSub1F * kSub1C);
  float* x2r = pool.get<float>((int64_t)B * IN * kSub1F * kSub1C);
  const Secs secs = sub_secs();
  __half* exps = pool.get<__half>((int64_t)B * secs.total);
  hipLaunchKernelGGL(ref_x1_kernel, grid1((int64_t)B * (kSub1S + MT) * kMels), dim3(256), 0, 0, feats, sl.ref(), pw, MT, x1, B);
  hipLaunchKernelGGL(ref_conv1_kernel, grid1((int64_t)B * MT * kSub1F * kSub1C), dim3(256), 0, 0, x1, w1, (int)bf, sc1, sh1,
                     MT, c1, B);
  hipLaunchKernelGGL(ref_x2_kernel, grid1((int64_t)B * IN * kSub1F * kSub1C), dim3(256), 0, 0, sl.ref(), c1, (int)bf, MT, x2r, B);
  hipLaunchKernelGGL(ref_sub_state_kernel, grid1((int64_t)B * secs.total), dim3(256), 0, 0, x1, c1, MT, exps, B);
  CK(hipDeviceSynchronize());

  if (which == "sub_conv") {   // bf16, 300 ms: the flat conv2 output
    uint16_t* flat = pool.get<uint16_t>((int64_t)B * T * kSubOut);
    rep.us = time_once([=] {
      return launch_sub_conv_bf16(feats, sl.ref(), pw, w1td, sc1, sh1, w2cd, sc2, sh2, flat, B, 0);
    });
    float* fr = pool.get<float>((int64_t)B * T * kSubOut);
    hipLaunchKernelGGL(ref_conv2_kernel<false>, grid1((int64_t)B * T * kSubOut), dim3(256), 0, 0, x2r, w2, kConv2K, sc2, sh2,
                       IN, T, fr, B);
    rep.out("flat", flat, 1, kSubOut, fr, (int64_t)B * T, kSubOut);
  } else {                     // sub1: x2 (the conv2 input) in HBM
    void* x2 = bf ? (void*)pool.get<uint16_t>((int64_t)B * IN * kSub1F * kSub1C) : (void*)pool.get<float>((int64_t)B * IN * kSub1F * kSub1C);
    rep.us = time_once([=] { return launch_sub1(feats, sl.ref(), pw, w1, w1td, sc1, sh1, x2, bf, B, chunk, 0); });
    rep.out("x2", x2, bf ? 1 : 0, (int64_t)kSub1F * kSub1C, x2r, (int64_t)B * IN, kSub1F * kSub1C);
  }
  rep.state(sl, secs, exps);
}

// conv2 alone: fp32 split (conv2_p3, B > 8), exact fp32 (conv2_sm, B <= 8) or bf16 implicit GEMM (400 ms)
static void check_conv2(int B, int chunk, bool bf, Report& rep) {
  const Geom geo = make_geom(chunk);
  const int IN = geo.sub2In, T = geo.T;
  const int64_t nx = (int64_t)B * IN * kSub1F * kSub1C;
  float* x2f = rand_f32(nx, 21, 0.6f, 0.3f, bf);
  const float* sc = rand_f32(kSub2C, 22, 0.2f, 1.f);
  const float* sh = rand_f32(kSub2C, 23, 0.3f);
  std::vector<float> w2h((size_t)kSub2C * kConv2K);
  for (size_t i = 0; i < w2h.size(); ++i) {
    const float v = 0.03f * urand(24, i);
    w2h[i] = bf ? bf2f(f2bf(v)) : v;
  }
  float* w2 = pool.get<float>(w2h.size());
  CK(hipMemcpy(w2, w2h.data(), w2h.size() * 4, hipMemcpyHostToDevice));
  float* fr = pool.get<float>((int64_t)B * T * kSubOut);
  hipLaunchKernelGGL(ref_conv2_kernel<true>, grid1((int64_t)B * T * kSubOut), dim3(256), 0, 0, x2f, w2, kConv2K, sc, sh, IN,
                     T, fr, B);
  if (bf) {
    std::vector<uint16_t> w2c((size_t)kSub2C * kConv2KPad, 0);
    for (int c = 0; c < kSub2C; ++c)
      for (int k = 0; k < kConv2K; ++k) w2c[(size_t)c * kConv2KPad + k] = f2bf(w2h[(size_t)c * kConv2K + k]);
    uint16_t* w2cd = pool.get<uint16_t>(w2c.size());
    CK(hipMemcpy(w2cd, w2c.data(), w2c.size() * 2, hipMemcpyHostToDevice));
    uint16_t* x2 = to_bf16(x2f, nx);
    uint16_t* flat = pool.get<uint16_t>((int64_t)B * T * kSubOut);
    rep.us = time_once([=] { return conv2_gemm(x2, w2cd, sc, sh, flat, B, true, 0, chunk, nullptr); });
    rep.out("flat", flat, 1, kSubOut, fr, (int64_t)B * T, kSubOut);
    return;
  }
  // fp32 mode: the three bf16 planes packed for conv2_p3 (session.hip finalize_weights)
  const size_t n = w2h.size();
  std::vector<uint16_t> pl(3 * n), px(3 * n);
  for (size_t i = 0; i < n; ++i) {
    const uint16_t h = f2bf(w2h[i]);
    const float r1 = w2h[i] - bf2f(h);
    const uint16_t m = f2bf(r1);
    pl[i] = h;
    pl[n + i] = m;
    pl[2 * n + i] = f2bf(r1 - bf2f(m));
  }
  conv2_p3_pack(pl.data(), px.data());
  uint16_t* w2p = pool.get<uint16_t>(px.size());
  CK(hipMemcpy(w2p, px.data(), px.size() * 2, hipMemcpyHostToDevice));
  float* flat = pool.get<float>((int64_t)B * T * kSubOut);
  rep.us = time_once([=] { return conv2_gemm(x2f, w2, sc, sh, flat, B, false, 0, chunk, w2p); });
  rep.out("flat", flat, 0, kSubOut, fr, (int64_t)B * T, kSubOut);
}

// =====================================================================================================================
// a9: depthwise conv k31 with carried state + folded BatchNorm + SiLU (conformer_blocks.py:427-433, submodules.py:364-402)
// x = [state (30) ; g (T)] per channel; out[t] = SiLU(b + sum_k w[k] x[t + k]); next state = x[T:]
__global__ void ref_dwconv_kernel(const void* g, int gty, StateRef s, int layer, const float* w, const float* bias, int T,
                                  float* out, __half* ex, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * kD) return;
  const int b = (int)(i / kD), c = (int)(i % kD);
  const int64_t sec = s.row_in(b) + kOffConv + (int64_t)layer * kD * kConvS + c * kConvS;
  float x[kConvS + kTMax];
  for (int k = 0; k < kConvS; ++k) x[k] = h2f(s.in[sec + k]);
  for (int t = 0; t < T; ++t) x[kConvS + t] = load_typed(g, gty, ((int64_t)b * T + t) * kD + c);
  for (int t = 0; t < T; ++t) {
    double acc = bias[c];
    for (int k = 0; k < kConvK; ++k) acc += (double)w[k * kD + c] * x[t + k];
    out[((int64_t)b * T + t) * kD + c] = (float)(acc / (1.0 + exp(-acc)));
  }
  for (int k = 0; k < kConvS; ++k) ex[(int64_t)b * kD * kConvS + c * kConvS + k] = __float2half_rn(x[T + k]);
}

// "_pk" checks (fp32): the output written fragment-packed for gemm_d3 (common.h xpk_off), unpacked here for the compare
static bool g_pk = false;
__global__ void xunpack_kernel(const float* src, float* dst, int64_t rows, int ld) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * ld) return;
  dst[i] = src[xpk_off(i / ld, (int)(i % ld), ld)];
}
static const void* unpacked(const void* out, int64_t rows, int ld = kD, bool force = false) {
  if (!g_pk && !force) return out;
  float* u = pool.get<float>(rows * ld);
  hipLaunchKernelGGL(xunpack_kernel, grid1(rows * ld), dim3(256), 0, 0, static_cast<const float*>(out), u, rows, ld);
  CK(hipDeviceSynchronize());
  return u;
}

static void check_dwconv(int B, int T, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int layer = 5;
  const int64_t M = (int64_t)B * T;
  float* gf = rand_f32(M * kD, 31, 1.5f, 0.f, bf);
  const void* g = bf ? (const void*)to_bf16(gf, M * kD) : (const void*)gf;
  const float* w = rand_f32(kConvK * kD, 32, 0.2f);
  const float* bias = rand_f32(kD, 33, 0.2f);
  void* out = bf ? (void*)pool.get<uint16_t>(M * kD) : (void*)pool.get<float>((M + 32) * kD);
  float* ref = pool.get<float>(M * kD);
  Secs secs{};
  secs.s[0] = {kOffConv + (int64_t)layer * kD * kConvS, (int64_t)kD * kConvS};
  secs.n = 1;
  secs.total = secs.s[0].len;
  __half* exps = pool.get<__half>((int64_t)B * secs.total);
  hipLaunchKernelGGL(ref_dwconv_kernel, grid1((int64_t)B * kD), dim3(256), 0, 0, g, bf ? 1 : 0, sl.ref(), layer, w, bias, T,
                     ref, exps, B);
  CK(hipDeviceSynchronize());
  const bool pk = g_pk;
  rep.us = time_once([=] { return launch_dwconv(g, sl.ref(), layer, w, bias, out, bf, T, B, 0, pk); });
  rep.out("out", unpacked(out, M), bf ? 1 : 0, kD, ref, M, kD);
  rep.state(sl, secs, exps);
}

__global__ void cmp_bytes_kernel(const uint8_t* a, const uint8_t* b, int64_t n, int* bad);

// the resident form (common.h StateRef ring): stream b's counter n_b = (7 b + 3) mod 30 in its read row, its ring
// ring_ids[b] = a shuffle of B + 1 rings; the reference reads cache frame i at ring row (n_b T + i) mod 30 and writes the
// expected ring (the T new frames over rows (n_b T + j) mod 30, j < T) into a copy of the rings
__global__ void set_counter_kernel(StateRef s, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) const_cast<__half*>(s.in)[s.row_in(b) + kOffConv] = __float2half_rn((float)((7 * b + 3) % kConvS));
}
__global__ void ref_dwconv_ring_kernel(const void* g, int gty, StateRef s, const __half* ring0, int layer, const float* w,
                                       const float* bias, int T, float* out, __half* ring_exp, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * kD) return;
  const int b = (int)(i / kD), c = (int)(i % kD);
  const int n = (7 * b + 3) % kConvS, ph = (n * T) % kConvS;
  const int64_t base = (int64_t)s.ring_ids[b] * kRingElems + (int64_t)layer * kConvS * kD + c;
  float x[kConvS + kTMax];
  for (int k = 0; k < kConvS; ++k) x[k] = h2f(ring0[base + (int64_t)((ph + k) % kConvS) * kD]);
  for (int t = 0; t < T; ++t) x[kConvS + t] = load_typed(g, gty, ((int64_t)b * T + t) * kD + c);
  for (int t = 0; t < T; ++t) {
    double acc = bias[c];
    for (int k = 0; k < kConvK; ++k) acc += (double)w[k * kD + c] * x[t + k];
    out[((int64_t)b * T + t) * kD + c] = (float)(acc / (1.0 + exp(-acc)));
  }
  for (int j = 0; j < T; ++j) ring_exp[base + (int64_t)((ph + j) % kConvS) * kD] = __float2half_rn(x[kConvS + j]);
}

static void check_dwconv_ring(int B, int T, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int layer = 9, nr = B + 1;
  std::vector<int> ids(B);
  for (int b = 0; b < B; ++b) ids[b] = (int)(((int64_t)5 * b + 1) % nr);   // 5 coprime with B + 1 for the tested B
  int* dids = pool.get<int>(B);
  CK(hipMemcpy(dids, ids.data(), B * 4, hipMemcpyHostToDevice));
  StateRef sr = sl.ref();
  sr.ring = to_f16(rand_f32((int64_t)nr * kRingElems, 34, 1.f), (int64_t)nr * kRingElems);
  sr.ring_ids = dids;
  hipLaunchKernelGGL(set_counter_kernel, grid1(B), dim3(256), 0, 0, sr, B);
  __half* ring0 = pool.get<__half>((int64_t)nr * kRingElems);
  __half* ring_exp = pool.get<__half>((int64_t)nr * kRingElems);
  CK(hipMemcpy(ring0, sr.ring, (size_t)nr * kRingElems * 2, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(ring_exp, sr.ring, (size_t)nr * kRingElems * 2, hipMemcpyDeviceToDevice));
  const int64_t M = (int64_t)B * T;
  float* gf = rand_f32(M * kD, 31, 1.5f, 0.f, bf);
  const void* g = bf ? (const void*)to_bf16(gf, M * kD) : (const void*)gf;
  const float* w = rand_f32(kConvK * kD, 32, 0.2f);
  const float* bias = rand_f32(kD, 33, 0.2f);
  void* out = bf ? (void*)pool.get<uint16_t>(M * kD) : (void*)pool.get<float>((M + 32) * kD);
  float* ref = pool.get<float>(M * kD);
  hipLaunchKernelGGL(ref_dwconv_ring_kernel, grid1((int64_t)B * kD), dim3(256), 0, 0, g, bf ? 1 : 0, sr, ring0, layer, w, bias,
                     T, ref, ring_exp, B);
  CK(hipDeviceSynchronize());
  const bool pk = g_pk;
  rep.us = time_once([=] { return launch_dwconv(g, sr, layer, w, bias, out, bf, T, B, 0, pk); });
  rep.out("out", unpacked(out, M), bf ? 1 : 0, kD, ref, M, kD);
  // every ring element (all layers, the unused ring too) against the expected rings: bytes
  int* bad = pool.get<int>(1);
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(cmp_bytes_kernel, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const uint8_t*>(sr.ring),
                     reinterpret_cast<const uint8_t*>(ring_exp), (int64_t)nr * kRingElems * 2, bad);
  int hb = 0;
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  rep.outs.emplace_back("ring_bad_bytes", Res{(float)hb, 0, 0, 0, 0, 0});
}

// =====================================================================================================================
// a7 / a8: RoPE multi-head attention (conformer_blocks.py:688-726, submodules.py:204-271); recomputing layers:
// q, k -> LayerNorm(48) -> RoPE on dims [0, 32) (q at positions 0..T-1, k at -S..T-1) -> scores / sqrt(48) -> masked
// softmax (layers 14 / 15: offset 30 - mhsa_len, floor-divided by 2 in the reduced block; a pair is masked iff key j or
// query S + i lies before it: -10000 in, 0 out) -> P V.  One thread per (stream, head, query).
__device__ void ln_rope(const float* x, const float* lw, const float* lb, const float* cs, const float* sn, int pos, double* y) {
  double mu = 0.0;
  for (int d = 0; d < kDk; ++d) mu += x[d];
  mu /= kDk;
  double var = 0.0;
  for (int d = 0; d < kDk; ++d) var += (x[d] - mu) * (x[d] - mu);
  var /= kDk;
  const double rs = 1.0 / sqrt(var + 1e-5);
  double z[kDk];
  for (int d = 0; d < kDk; ++d) z[d] = (x[d] - mu) * rs * lw[d] + lb[d];
  for (int d = 0; d < kDk; ++d) y[d] = z[d];
  for (int d = 0; d < kRope / 2; ++d) {
    const double c = cs[(pos + kMhsaS) * (kRope / 2) + d], s = sn[(pos + kMhsaS) * (kRope / 2) + d];
    y[d] = z[d] * c - z[d + kRope / 2] * s;
    y[d + kRope / 2] = z[d + kRope / 2] * c + z[d] * s;
  }
}
__global__ void ref_attention_kernel(AttnArgs a, int ty, float* ctx, float* probs) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int T = a.T, S = a.S, TK = S + T;
  if (i0 >= (int64_t)a.B * kHeads * T) return;
  const int i = (int)(i0 % T), h = (int)((i0 / T) % kHeads), b = (int)(i0 / ((int64_t)T * kHeads));
  const int c0 = h * kDk;
  double p[30 + kTMax];
  if (a.recompute) {
    float xq[kDk];
    double q[kDk];
    for (int d = 0; d < kDk; ++d) xq[d] = load_typed(a.q, ty, ((int64_t)b * T + i) * a.ldq + c0 + d);
    ln_rope(xq, a.qln_w, a.qln_b, a.rope_cos, a.rope_sin, i, q);
    double off = -1e30;
    if (S > 0) {
      off = (double)kMhsaS - (double)h2f(a.s.in[a.s.row_in(b) + kOffMhsaLen]);
      if (a.reduced) off = floor(off / 2.0);
    }
    double mx = -1e300;
    for (int j = 0; j < TK; ++j) {
      float xk[kDk];
      double k[kDk];
      for (int d = 0; d < kDk; ++d) xk[d] = load_typed(a.k, ty, ((int64_t)b * TK + j) * a.ldk + c0 + d);
      ln_rope(xk, a.kln_w, a.kln_b, a.rope_cos, a.rope_sin, j - S, k);
      double sc = 0.0;
      for (int d = 0; d < kDk; ++d) sc += q[d] * k[d];
      sc /= sqrt((double)kDk);
      const bool masked = S > 0 && ((double)j < off || (double)(S + i) < off);
      p[j] = masked ? -10000.0 : sc;
      mx = fmax(mx, p[j]);
    }
    double sum = 0.0;
    for (int j = 0; j < TK; ++j) sum += (p[j] = exp(p[j] - mx));
    for (int j = 0; j < TK; ++j) {
      const bool masked = S > 0 && ((double)j < off || (double)(S + i) < off);
      p[j] = masked ? 0.0 : p[j] / sum;
      if (probs) probs[(((int64_t)b * kHeads + h) * T + i) * TK + j] = (float)p[j];
    }
  } else {
    for (int j = 0; j < TK; ++j) p[j] = a.probs[(((int64_t)b * kHeads + h) * T + i) * TK + j];
  }
  for (int d = 0; d < kDk; ++d) {
    double acc = 0.0;
    for (int j = 0; j < TK; ++j) acc += p[j] * load_typed(a.v, ty, ((int64_t)b * TK + j) * a.ldv + c0 + d);
    ctx[((int64_t)b * T + i) * kD + c0 + d] = (float)acc;
  }
}
// random softmax rows for the shared-probability layers: p[j] = e_j / sum e
__global__ void softmax_rows_kernel(float* p, int64_t rows, int n) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  double s = 0.0;
  for (int j = 0; j < n; ++j) s += (p[r * n + j] = expf(3.f * p[r * n + j]));
  for (int j = 0; j < n; ++j) p[r * n + j] = (float)(p[r * n + j] / s);
}

static void rope_tables(float** cs, float** sn) {   // session.hip make_rope: positions -30 .. 12, 16 frequencies
  std::vector<float> c((30 + kTMax) * 16), s(c.size());
  for (int j = 0; j < 16; ++j) {
    const float e = (float)(2 * j) / 32.0f;
    const float inv = 1.0f / powf(10000.0f, e);
    for (int p = -30; p < kTMax; ++p) {
      c[(p + 30) * 16 + j] = cosf((float)p * inv);
      s[(p + 30) * 16 + j] = sinf((float)p * inv);
    }
  }
  *cs = pool.get<float>(c.size());
  *sn = pool.get<float>(s.size());
  CK(hipMemcpy(*cs, c.data(), c.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(*sn, s.data(), s.size() * 4, hipMemcpyHostToDevice));
}

// recompute: (T, S) of an instantiated recomputing layer; else the shared-probability kernel at T
static void check_attention(int B, int T, int S, bool recompute, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int TK = S + T, ty = bf ? 1 : 0;
  AttnArgs a{};
  a.B = B;
  a.T = T;
  a.S = S;
  a.recompute = recompute;
  a.reduced = S == 15;   // layer 14 sits in the reduced block (conformer.py:221-225)
  a.ctx_bf16 = bf;
  a.s = sl.ref();
  float *cs, *sn;
  rope_tables(&cs, &sn);
  a.rope_cos = cs;
  a.rope_sin = sn;
  auto act = [&](int64_t n, uint64_t seed, float scale) -> const void* {
    float* f = rand_f32(n, seed, scale, 0.f, bf);
    return bf ? (const void*)to_bf16(f, n) : (const void*)f;
  };
  if (S == 0) {   // layers 0 / 7: q | k | v in one [M][1152] buffer (session.hip enqueue_step)
    const void* qkv = act((int64_t)B * T * 3 * kD, 41, 2.f);
    const int es = bf ? 2 : 4;
    a.q = qkv;
    a.k = static_cast<const char*>(qkv) + kD * es;
    a.v = static_cast<const char*>(qkv) + 2 * kD * es;
    a.ldq = a.ldk = a.ldv = 3 * kD;
  } else {        // layers 14 / 15: q [M][384], k | v [B(S+T)][768]
    a.q = act((int64_t)B * T * kD, 42, 2.f);
    const void* kv = act((int64_t)B * TK * 2 * kD, 43, 2.f);
    a.k = kv;
    a.v = static_cast<const char*>(kv) + kD * (bf ? 2 : 4);
    a.ldq = kD;
    a.ldk = a.ldv = 2 * kD;
  }
  a.qln_w = rand_f32(kDk, 44, 0.2f, 1.f);
  a.qln_b = rand_f32(kDk, 45, 0.1f);
  a.kln_w = rand_f32(kDk, 46, 0.2f, 1.f);
  a.kln_b = rand_f32(kDk, 47, 0.1f);
  const int64_t np = (int64_t)B * kHeads * T * TK;
  float* probs_ref = pool.get<float>(np);
  if (!recompute) {   // the shared layers read the last recomputing layer's probabilities
    float* pr = rand_f32(np, 48, 1.f);
    hipLaunchKernelGGL(softmax_rows_kernel, grid1((int64_t)B * kHeads * T), dim3(256), 0, 0, pr, (int64_t)B * kHeads * T, TK);
    a.probs = pr;
  } else {
    a.probs = S == 0 ? pool.get<float>(np) : nullptr;   // written by layers 0 / 7 only (session.hip)
  }
  void* ctx = bf ? (void*)pool.get<uint16_t>((int64_t)B * T * kD) : (void*)pool.get<float>(((int64_t)B * T + 32) * kD);
  a.ctx = ctx;
  a.ctx_packed = g_pk;
  float* ref = pool.get<float>((int64_t)B * T * kD);
  AttnArgs ar = a;
  hipLaunchKernelGGL(ref_attention_kernel, grid1((int64_t)B * kHeads * T, 64), dim3(64), 0, 0, ar, ty, ref,
                     recompute && a.probs ? probs_ref : nullptr);
  CK(hipDeviceSynchronize());
  rep.us = time_once([=] { return launch_attention(a, 0); });
  rep.out("ctx", unpacked(ctx, (int64_t)B * T), ty, kD, ref, (int64_t)B * T, kD);
  if (recompute && a.probs) rep.out("probs", a.probs, 0, TK, probs_ref, (int64_t)B * kHeads * T, TK);
  // the attention kernels read the state (mhsa_len) and write none of it
  Secs none{};
  rep.state(sl, none, nullptr);
}

// =====================================================================================================================
// a6: layers 14 / 15 MHSA input cache (conformer_blocks.py:147-163, submodules.py:295-302): xn = RMSNorm(r);
// kv = [cache rows 30-S..29 ; xn]; next cache = zeros(30 - S) ; [cache_S[T:] ; xn]
__global__ void ref_kv_kernel(const void* r, int rty, const float* nw, StateRef s, int slot, int T, int S, float* xn,
                              float* kv, __half* ex, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * kD) return;
  const int b = (int)(i / kD), c = (int)(i % kD);
  const int TK = S + T;
  const int64_t cache = s.row_in(b) + kOffMhsa + (int64_t)slot * kMhsaS * kD;
  float xr[kTMax];
  for (int t = 0; t < T; ++t) {
    double ss = 0.0;
    for (int k = 0; k < kD; ++k) {
      const double v = load_typed(r, rty, ((int64_t)b * T + t) * kD + k);
      ss += v * v;
    }
    const double den = sqrt(ss) / sqrt((double)kD) + 1e-8;
    xr[t] = (float)((double)nw[c] * ((double)load_typed(r, rty, ((int64_t)b * T + t) * kD + c) / den));
    xn[((int64_t)b * T + t) * kD + c] = xr[t];
    kv[((int64_t)b * TK + S + t) * kD + c] = xr[t];
  }
  for (int j = 0; j < S; ++j) kv[((int64_t)b * TK + j) * kD + c] = h2f(s.in[cache + (int64_t)(kMhsaS - S + j) * kD + c]);
  // next cache row rr: < 30 - S zero; then new[rr - (30 - S)] with new = [cache_S[T:] ; xn]
  for (int rr = 0; rr < kMhsaS; ++rr) {
    float v = 0.f;
    if (rr >= kMhsaS - S) {
      const int q = rr - (kMhsaS - S);
      v = q < S - T ? h2f(s.in[cache + (int64_t)(kMhsaS - S + T + q) * kD + c]) : xr[q - (S - T)];
    }
    ex[(int64_t)b * kMhsaS * kD + (int64_t)rr * kD + c] = __float2half_rn(v);
  }
}

// the resident form: cache frame j at ring row (n_b T + j) mod 30 of ring region 16 + slot; expected ring = the T new xn
// rows over rows (n_b T + i) mod 30 (counter n_b = (7 b + 3) mod 30 as set_counter_kernel writes it)
__global__ void ref_kv_ring_kernel(const void* r, int rty, const float* nw, StateRef s, const __half* ring0, int slot, int T,
                                   int S, float* xn, float* kv, __half* ring_exp, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * kD) return;
  const int b = (int)(i / kD), c = (int)(i % kD);
  const int TK = S + T, n = (7 * b + 3) % kMhsaS, ph = (n * T) % kMhsaS;
  const int64_t base = (int64_t)s.ring_ids[b] * kRingElems + kRingConv + (int64_t)slot * kMhsaS * kD + c;
  for (int t = 0; t < T; ++t) {
    double ss = 0.0;
    for (int k = 0; k < kD; ++k) {
      const double v = load_typed(r, rty, ((int64_t)b * T + t) * kD + k);
      ss += v * v;
    }
    const double den = sqrt(ss) / sqrt((double)kD) + 1e-8;
    const float y = (float)((double)nw[c] * ((double)load_typed(r, rty, ((int64_t)b * T + t) * kD + c) / den));
    xn[((int64_t)b * T + t) * kD + c] = y;
    kv[((int64_t)b * TK + S + t) * kD + c] = y;
    ring_exp[base + (int64_t)((ph + t) % kMhsaS) * kD] = __float2half_rn(y);
  }
  for (int j = 0; j < S; ++j)
    kv[((int64_t)b * TK + j) * kD + c] = h2f(ring0[base + (int64_t)((ph + kMhsaS - S + j) % kMhsaS) * kD]);
}

__global__ void set_counter_kernel(StateRef s, int B);
__global__ void cmp_bytes_kernel(const uint8_t* a, const uint8_t* b, int64_t n, int* bad);
// fp16 ulp distance of two fp16 buffers, max over elements (the recomputed xn rows of the ring)
__global__ void ulp_kernel(const __half* a, const __half* b, int64_t n, int* mx) {
  int d = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint16_t x = __half_as_ushort(a[i]), y = __half_as_ushort(b[i]);
    const int ox = (x & 0x8000) ? -(int)(x & 0x7fff) : (int)x, oy = (y & 0x8000) ? -(int)(y & 0x7fff) : (int)y;
    d = max(d, abs(ox - oy));
  }
  if (d) atomicMax(mx, d);
}

static void check_kv_ring(int B, int T, int S, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int slot = S == 15 ? 0 : 1, TK = S + T, nr = B + 1;
  std::vector<int> ids(B);
  for (int b = 0; b < B; ++b) ids[b] = (int)(((int64_t)5 * b + 1) % nr);
  int* dids = pool.get<int>(B);
  CK(hipMemcpy(dids, ids.data(), B * 4, hipMemcpyHostToDevice));
  StateRef sr = sl.ref();
  sr.ring = to_f16(rand_f32((int64_t)nr * kRingElems, 35, 2.f), (int64_t)nr * kRingElems);
  sr.ring_ids = dids;
  hipLaunchKernelGGL(set_counter_kernel, grid1(B), dim3(256), 0, 0, sr, B);
  __half* ring0 = pool.get<__half>((int64_t)nr * kRingElems);
  __half* ring_exp = pool.get<__half>((int64_t)nr * kRingElems);
  CK(hipMemcpy(ring0, sr.ring, (size_t)nr * kRingElems * 2, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(ring_exp, sr.ring, (size_t)nr * kRingElems * 2, hipMemcpyDeviceToDevice));
  const int64_t M = (int64_t)B * T;
  float* rf = rand_f32(M * kD, 51, 3.f);
  const void* r = bf ? (const void*)to_f16(rf, M * kD) : (const void*)rf;
  const float* nw = rand_f32(kD, 52, 0.2f, 1.f);
  void* xn = bf ? (void*)pool.get<uint16_t>(M * kD) : (void*)pool.get<float>(M * kD);
  void* kv = bf ? (void*)pool.get<uint16_t>((int64_t)B * TK * kD) : (void*)pool.get<float>((int64_t)B * TK * kD);
  float* xr = pool.get<float>(M * kD);
  float* kr = pool.get<float>((int64_t)B * TK * kD);
  hipLaunchKernelGGL(ref_kv_ring_kernel, grid1((int64_t)B * kD), dim3(256), 0, 0, r, bf ? 2 : 0, nw, sr, ring0, slot, T, S, xr,
                     kr, ring_exp, B);
  CK(hipDeviceSynchronize());
  rep.us = time_once([=] { return launch_kv_assemble(r, nw, sr, slot, T, S, xn, kv, bf, B, 0); });
  rep.out("xn", xn, bf ? 1 : 0, kD, xr, M, kD);
  rep.out("kv", kv, bf ? 1 : 0, kD, kr, (int64_t)B * TK, kD);
  // every ring element within one fp16 ulp of the expected rings (copies exact, the new xn rows one rounding of a
  // value computed in another order), the rest of every ring (conv layers, the other MHSA layer) byte-exact
  int* mx = pool.get<int>(1);
  CK(hipMemset(mx, 0, 4));
  hipLaunchKernelGGL(ulp_kernel, dim3(2048), dim3(256), 0, 0, sr.ring, ring_exp, (int64_t)nr * kRingElems, mx);
  int hm = 0;
  CK(hipMemcpy(&hm, mx, 4, hipMemcpyDeviceToHost));
  rep.outs.emplace_back("ring_max_ulp", Res{(float)hm, 0, 0, 0, 0, 0});
}

static void check_kv(int B, int T, int S, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int slot = S == 15 ? 0 : 1, TK = S + T;
  const int64_t M = (int64_t)B * T;
  float* rf = rand_f32(M * kD, 51, 3.f);
  const void* r = bf ? (const void*)to_f16(rf, M * kD) : (const void*)rf;   // the residual stream: fp16 in bf16 mode
  const float* nw = rand_f32(kD, 52, 0.2f, 1.f);
  void* xn = bf ? (void*)pool.get<uint16_t>(M * kD) : (void*)pool.get<float>(M * kD);
  void* kv = bf ? (void*)pool.get<uint16_t>((int64_t)B * TK * kD) : (void*)pool.get<float>((int64_t)B * TK * kD);
  float* xr = pool.get<float>(M * kD);
  float* kr = pool.get<float>((int64_t)B * TK * kD);
  Secs secs{};
  secs.s[0] = {kOffMhsa + (int64_t)slot * kMhsaS * kD, (int64_t)kMhsaS * kD};
  secs.n = 1;
  secs.total = secs.s[0].len;
  __half* exps = pool.get<__half>((int64_t)B * secs.total);
  hipLaunchKernelGGL(ref_kv_kernel, grid1((int64_t)B * kD), dim3(256), 0, 0, r, bf ? 2 : 0, nw, sl.ref(), slot, T, S, xr, kr,
                     exps, B);
  CK(hipDeviceSynchronize());
  rep.us = time_once([=] { return launch_kv_assemble(r, nw, sl.ref(), slot, T, S, xn, kv, bf, B, 0); });
  rep.out("xn", xn, bf ? 1 : 0, kD, xr, M, kD);
  rep.out("kv", kv, bf ? 1 : 0, kD, kr, (int64_t)B * TK, kD);
  rep.state(sl, secs, exps);
}

// =====================================================================================================================
// a11: CausalTemporalReduction streaming branch (conformer_blocks.py:888-907), grouped conv part:
// x = [state (1) ; frames (T)] per channel; y[o][t] = b[o] + sum_k w[o][k] x[o / 4][2 t + k]; next state = last frame
__global__ void ref_reduce_kernel(const void* x, int xty, StateRef s, const float* w, const float* bias, int T, float* y,
                                  __half* ex, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int TR = (T + 1 - 3) / 2 + 1;
  if (i >= (int64_t)B * 4 * kD) return;
  const int b = (int)(i / (4 * kD)), o = (int)(i % (4 * kD)), c = o / 4;
  float xc[kTMax + 1];
  xc[0] = h2f(s.in[s.row_in(b) + kOffRed + c]);
  for (int t = 0; t < T; ++t) xc[t + 1] = load_typed(x, xty, ((int64_t)b * T + t) * kD + c);
  for (int t = 0; t < TR; ++t) {
    double acc = bias[o];
    for (int k = 0; k < 3; ++k) acc += (double)w[o * 3 + k] * xc[2 * t + k];
    y[((int64_t)b * TR + t) * 4 * kD + o] = (float)acc;
  }
  if ((o & 3) == 0) ex[(int64_t)b * kD + c] = __float2half_rn(xc[T]);
}

static void check_reduce(int B, int T, bool bf, Report& rep) {
  Slab sl;
  sl.make(B);
  const int TR = (T + 1 - 3) / 2 + 1;
  const int64_t M = (int64_t)B * T;
  float* xf = rand_f32(M * kD, 61, 2.f);
  const void* x = bf ? (const void*)to_f16(xf, M * kD) : (const void*)xf;
  const float* w = rand_f32(4 * kD * 3, 62, 0.3f);
  const float* bias = rand_f32(4 * kD, 63, 0.2f);
  void* y = bf ? (void*)pool.get<uint16_t>((int64_t)B * TR * 4 * kD) : (void*)pool.get<float>(((int64_t)B * TR + 32) * 4 * kD);
  float* yr = pool.get<float>((int64_t)B * TR * 4 * kD);
  Secs secs{};
  secs.s[0] = {kOffRed, kD};
  secs.n = 1;
  secs.total = kD;
  __half* exps = pool.get<__half>((int64_t)B * kD);
  hipLaunchKernelGGL(ref_reduce_kernel, grid1((int64_t)B * 4 * kD), dim3(256), 0, 0, x, bf ? 2 : 0, sl.ref(), w, bias, T, yr,
                     exps, B);
  CK(hipDeviceSynchronize());
  const bool pk = g_pk;
  rep.us = time_once([=] { return launch_reduce_conv(x, sl.ref(), w, bias, y, bf, B, T, 0, pk); });
  rep.out("y", unpacked(y, (int64_t)B * TR, 4 * kD), bf ? 1 : 0, 4 * kD, yr, (int64_t)B * TR, 4 * kD);
  rep.state(sl, secs, exps);
}

// a12: TemporalUpsampling (conformer_blocks.py:955-988): x[t] += x5[t / 2] for t < 2 Tr (a later frame is the zero pad)
__global__ void ref_upsample_kernel(const float* x10, const float* x5, int T, float* out, int B) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int TR = (T + 1 - 3) / 2 + 1;
  if (i >= (int64_t)B * T * kD) return;
  const int c = (int)(i % kD), t = (int)((i / kD) % T), b = (int)(i / ((int64_t)kD * T));
  float v = x10[i];
  if (t < 2 * TR) v += x5[((int64_t)b * TR + t / 2) * kD + c];
  out[i] = v;
}
__global__ void round_f16_kernel(float* p, int64_t n) {   // the fp16 residual stream's values
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = __half2float(__float2half_rn(p[i]));
}

static void check_upsample(int B, int T, bool r16, Report& rep) {
  const int TR = (T + 1 - 3) / 2 + 1;
  const int64_t n10 = (int64_t)B * T * kD, n5 = (int64_t)B * TR * kD;
  float* a = rand_f32(n10, 71, 2.f);
  float* c = rand_f32(n5, 72, 2.f);
  if (r16) {
    hipLaunchKernelGGL(round_f16_kernel, kFillGrid, kFillBlock, 0, 0, a, n10);
    hipLaunchKernelGGL(round_f16_kernel, kFillGrid, kFillBlock, 0, 0, c, n5);
  }
  float* ref = pool.get<float>(n10);
  hipLaunchKernelGGL(ref_upsample_kernel, grid1(n10), dim3(256), 0, 0, a, c, T, ref, B);
  void* x10 = r16 ? (void*)to_f16(a, n10) : (void*)a;
  const void* x5 = r16 ? (const void*)to_f16(c, n5) : (const void*)c;
  uint16_t* shadow = pool.get<uint16_t>(n10);
  CK(hipDeviceSynchronize());
  float* xp = g_pk ? pool.get<float>(((int64_t)B * T + 32) * kD) : nullptr;
  rep.us = time_once([=] { return launch_upsample_add(x10, x5, B, T, shadow, 0, r16, 0, xp); });
  rep.out("x", x10, r16 ? 2 : 0, kD, ref, (int64_t)B * T, kD);
  rep.out("shadow", shadow, 1, kD, ref, (int64_t)B * T, kD);
  if (xp) rep.out("xp", unpacked(xp, (int64_t)B * T), 0, kD, ref, (int64_t)B * T, kD);
}

// =====================================================================================================================
// a14: ConvASRDecoder (conformer.py:338-354): logits = x W^T + b, log_softmax; frame_info = greedy token (first index on
// ties, decoder.py:57) | (exp(lp[33]) + exp(lp[34]) <= 0.9) << 8 (logprob_splitter.py:134).  The token and flag are
// compared where the reference's top-2 margin / distance to the threshold exceeds 1e-5 (a closer call may go either way
// in fp32).
__global__ void ref_head_kernel(const void* x, int xty, const float* w, const float* b, float* lp, int32_t* fi,
                                int32_t* fi_ok, int rows) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  double z[kVocab], m = -1e300;
  for (int v = 0; v < kVocab; ++v) {
    double acc = b[v];
    for (int k = 0; k < kD; ++k) acc += (double)w[v * kD + k] * load_typed(x, xty, (int64_t)r * kD + k);
    z[v] = acc;
    m = fmax(m, acc);
  }
  double se = 0.0;
  for (int v = 0; v < kVocab; ++v) se += exp(z[v] - m);
  const double lse = log(se);
  int tok = 0;
  double best = -1e300, second = -1e300;
  for (int v = 0; v < kVocab; ++v) {
    const double l = z[v] - m - lse;
    lp[(int64_t)r * kVocab + v] = (float)l;
    if (l > best) { second = best; best = l; tok = v; }
    else if (l > second) second = l;
  }
  const double sil = exp(z[kVocab - 2] - m - lse) + exp(z[kVocab - 1] - m - lse);
  fi[r] = tok | (sil <= 0.9 ? 256 : 0);
  fi_ok[r] = (best - second > 1e-5 ? 1 : 0) | (fabs(sil - 0.9) > 1e-5 ? 2 : 0);
}
__global__ void cmp_fi_kernel(const int32_t* fi, const int32_t* ref, const int32_t* ok, int rows, int* bad) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  int d = 0;
  if ((ok[r] & 1) && (fi[r] & 255) != (ref[r] & 255)) d = 1;
  if ((ok[r] & 2) && (fi[r] & 256) != (ref[r] & 256)) d = 1;
  if (d) atomicAdd(bad, 1);
}

static void check_head(int rows, bool r16, Report& rep) {
  float* xf = rand_f32((int64_t)rows * kD, 81, 2.f);
  if (r16) hipLaunchKernelGGL(round_f16_kernel, kFillGrid, kFillBlock, 0, 0, xf, (int64_t)rows * kD);
  const void* x = r16 ? (const void*)to_f16(xf, (int64_t)rows * kD) : (const void*)xf;
  const float* w = rand_f32(kVocab * kD, 82, 0.15f);
  const float* b = rand_f32(kVocab, 83, 1.f);
  float* lp = pool.get<float>((int64_t)rows * kVocab);
  float* lr = pool.get<float>((int64_t)rows * kVocab);
  int32_t* fi = pool.get<int32_t>(rows);
  int32_t* fr = pool.get<int32_t>(rows);
  int32_t* ok = pool.get<int32_t>(rows);
  hipLaunchKernelGGL(ref_head_kernel, grid1(rows), dim3(256), 0, 0, x, r16 ? 2 : 0, w, b, lr, fr, ok, rows);
  CK(hipDeviceSynchronize());
  rep.us = time_once([=] { return launch_head(x, w, b, lp, fi, rows, r16, 0); });
  rep.out("logprobs", lp, 0, kVocab, lr, rows, kVocab);
  int* bad = pool.get<int>(1);
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(cmp_fi_kernel, grid1(rows), dim3(256), 0, 0, fi, fr, ok, rows, bad);
  int hb = 0;
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  rep.outs.emplace_back("frame_info_bad", Res{(float)hb, 0, 0, 0, 0, 0});
}

// a4: RMSNorm (submodules.py:34-54) in place over the residual stream, with the bf16 shadow and (fp8 mode) the shadow's
// MXFP8 form + sum-of-squares slab, the latter compared byte for byte with quant_mx over the kernel's own shadow
__global__ void ref_rmsnorm_kernel(const float* x, const float* w, float* y, int rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * kD) return;
  const int64_t r = i / kD;
  double ss = 0.0;
  for (int k = 0; k < kD; ++k) ss += (double)x[r * kD + k] * x[r * kD + k];
  y[i] = (float)((double)w[i % kD] * ((double)x[i] / (sqrt(ss) / sqrt((double)kD) + 1e-8)));
}
__global__ void cmp_bytes_kernel(const uint8_t* a, const uint8_t* b, int64_t n, int* bad) {
  int d = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) d += a[i] != b[i];
  if (d) atomicAdd(bad, d);
}

__global__ void inv_cmp_kernel(const float* ss, const float* ss2, int rows, float* err) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float a = mx_row_inv(ss + (int64_t)r * kSsSlots), b = mx_row_inv(ss2 + (int64_t)r * kSsSlots);
  atomicMax(reinterpret_cast<int*>(err), __float_as_int(fabsf(a - b) / fabsf(b)));
}

static void check_rmsnorm(int rows, bool r16, bool q8, Report& rep) {
  const int64_t n = (int64_t)rows * kD;
  float* xf = rand_f32(n, 91, 3.f);
  if (r16) hipLaunchKernelGGL(round_f16_kernel, kFillGrid, kFillBlock, 0, 0, xf, n);
  const float* w = rand_f32(kD, 92, 0.2f, 1.f);
  float* ref = pool.get<float>(n);
  hipLaunchKernelGGL(ref_rmsnorm_kernel, grid1(n), dim3(256), 0, 0, xf, w, ref, rows);
  void* x = r16 ? (void*)to_f16(xf, n) : (void*)xf;
  uint16_t* shadow = pool.get<uint16_t>(n);
  uint8_t *q = nullptr, *s = nullptr;
  float* ss = nullptr;
  if (q8) {
    q = pool.get<uint8_t>(n);
    s = pool.get<uint8_t>(n / 32);
    ss = pool.get<float>((int64_t)rows * kSsSlots);
  }
  CK(hipDeviceSynchronize());
  float* xp = g_pk ? pool.get<float>(((int64_t)rows + 32) * kD) : nullptr;
  rep.us = time_once([=] { return launch_rmsnorm(x, w, rows, shadow, 0, r16, 0, q, s, ss, xp); });
  rep.out("x", x, r16 ? 2 : 0, kD, ref, rows, kD);
  if (xp) rep.out("xp", unpacked(xp, rows), 0, kD, ref, rows, kD);
  rep.out("shadow", shadow, 1, kD, ref, rows, kD);
  if (q8) {
    uint8_t* q2 = pool.get<uint8_t>(n);
    uint8_t* s2 = pool.get<uint8_t>(n / 32);
    float* ss2 = pool.get<float>((int64_t)rows * kSsSlots);
    CK(launch_quant_mx(shadow, kD, rows, kD, q2, s2, ss2, 0));
    int* bad = pool.get<int>(1);
    CK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(cmp_bytes_kernel, dim3(1024), dim3(256), 0, 0, q, q2, n, bad);
    hipLaunchKernelGGL(cmp_bytes_kernel, dim3(1024), dim3(256), 0, 0, s, s2, n / 32, bad);
    int hb = 0;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    rep.outs.emplace_back("q8_bad_bytes", Res{(float)hb, 0, 0, 0, 0, 0});
    // the slab: the same row factor (the two kernels add the squares in different orders)
    float* e = pool.get<float>(1);
    CK(hipMemset(e, 0, 4));
    hipLaunchKernelGGL(inv_cmp_kernel, grid1(rows), dim3(256), 0, 0, ss, ss2, rows, e);
    float he = 0.f;
    CK(hipMemcpy(&he, e, 4, hipMemcpyDeviceToHost));
    rep.outs.emplace_back("q8_row_factor", Res{he, 0, 0, 0, 0, 0});
  }
}

// =====================================================================================================================
int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr,
            "usage: %s <check> <B> [T]\n  checks: sub_conv sub1_f32 sub1_f32_400 sub1_bf16_400 conv2_f32 conv2_f32_400 "
            "conv2_bf16_400 dwconv[_bf16|_pk] dwconv_ring[_bf16|_pk] attn_rec[_bf16|_pk] (T S) attn_shared[_bf16|_pk] "
            "kv[_bf16] (T S) kv_ring[_bf16] (T S) reduce[_bf16|_pk] "
            "upsample[_r16|_pk] head[_r16] (rows) rmsnorm[_r16|_q8|_pk] (rows)\n",
            argv[0]);
    return 2;
  }
  const std::string ck = argv[1];
  const int B = atoi(argv[2]);
  const int T = argc > 3 ? atoi(argv[3]) : kT;
  const int S = argc > 4 ? atoi(argv[4]) : 0;
  Report rep;
  rep.check = ck;
  rep.B = B;
  rep.T = T;
  auto has = [&](const char* suf) { return ck.size() >= strlen(suf) && ck.compare(ck.size() - strlen(suf), strlen(suf), suf) == 0; };
  const bool bf = has("_bf16") || has("_bf16_400");
  g_pk = has("_pk");   // fp32 dwconv / attention: the packed output gemm_d3 reads
  if (g_pk && bf) {
    fprintf(stderr, "the packed layout is fp32 only\n");
    return 2;
  }
  if (ck == "sub_conv") check_pre("sub_conv", B, 2400, true, rep);
  else if (ck == "sub1_f32") check_pre("sub1", B, 2400, false, rep);
  else if (ck == "sub1_f32_400") check_pre("sub1", B, 3200, false, rep);
  else if (ck == "sub1_bf16_400") check_pre("sub1", B, 3200, true, rep);
  else if (ck == "conv2_f32") check_conv2(B, 2400, false, rep);
  else if (ck == "conv2_f32_400") check_conv2(B, 3200, false, rep);
  else if (ck == "conv2_bf16_400") check_conv2(B, 3200, true, rep);
  else if (ck.rfind("dwconv_ring", 0) == 0) check_dwconv_ring(B, T, bf, rep);
  else if (ck.rfind("dwconv", 0) == 0) check_dwconv(B, T, bf, rep);
  else if (ck.rfind("attn_rec", 0) == 0) check_attention(B, T, S, true, bf, rep);
  else if (ck.rfind("attn_shared", 0) == 0) check_attention(B, T, 0, false, bf, rep);
  else if (ck.rfind("kv_ring", 0) == 0) check_kv_ring(B, T, S, bf, rep);
  else if (ck.rfind("kv", 0) == 0) check_kv(B, T, S, bf, rep);
  else if (ck.rfind("reduce", 0) == 0) check_reduce(B, T, bf, rep);
  else if (ck.rfind("upsample", 0) == 0) check_upsample(B, T, has("_r16"), rep);
  else if (ck.rfind("head", 0) == 0) check_head(B, has("_r16"), rep);
  else if (ck.rfind("rmsnorm", 0) == 0) check_rmsnorm(B, has("_r16") || has("_q8"), has("_q8"), rep);
  else {
    fprintf(stderr, "unknown check %s\n", ck.c_str());
    return 2;
  }
  if (ck == "sub_conv" || ck.rfind("sub1", 0) == 0 || ck.rfind("conv2", 0) == 0) rep.T = ck.find("400") != std::string::npos ? 13 : kT;
  rep.us = time_warm();
  rep.print();
  return 0;
}
