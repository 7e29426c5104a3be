// libtonehip.so: C ABI (include/tonehip.h), weight folding/packing and the per-step launch
// sequence of the T-one streaming acoustic path.
//
// One step (Tone.forward_for_export, tone/nn/model.py:162-205) is a fixed sequence of ~200
// kernel launches over a batch of independent streams; the activations of every stream are laid
// out [stream * frames, 384] row-major so every pointwise projection is one GEMM with
// M = batch * frames.  The step can be captured once per (batch, I/O pointers) into a hipGraph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/tonehip.h"
#include "common.h"
#include "kernels.h"

using namespace tone;

namespace tone {

const Knobs& knobs() {
  static const Knobs k = [] {
    auto env = [](const char* n, int dflt) {
      const char* e = std::getenv(n);
      return e && *e ? std::atoi(e) : dflt;
    };
    Knobs r;
    r.fp8_normq = env("TONE_FP8_NORMQ", 1) != 0;
    r.rp_norm = env("TONE_RP_NORM", 1) != 0;
    r.h_blocked = env("TONE_H_BLOCKED", 1) != 0;
    r.d3 = env("TONE_D3", 1) != 0;
    r.d3x = env("TONE_D3X", 1) != 0;
    r.ring_nt = env("TONE_RING_NT", 1) != 0;
    r.x3_xcd = env("TONE_X3_XCD", 1) != 0;
    r.head_mfma = env("TONE_HEAD_MFMA", 1) != 0;
    return r;
  }();
  return k;
}

}  // namespace tone

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return fail(TONE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// MXFP8 weight (fp8 mode): e4m3 [N][K] + E8M0 scales [N][K/32]
struct MxW {
  uint8_t* q = nullptr;
  uint8_t* s = nullptr;
};

struct LayerW {
  MxW mx13[2], mx2[2], mxqkv, mxq, mxkv;   // fp8 mode: the q/k/v and FFN weights as MXFP8
  void* w13[2];       // [3072][384] SwiGLU-interleaved, norm folded
  float* b13[2];
  void* w2[2];        // [384][1536]
  float* b2[2];
  void* wqkv;         // recompute layers 0/7: [1152][384] folded; shared layers: [384][384] Wv folded
  float* bqkv;
  void* wq;           // layers 14/15: [384][384] unfolded
  float* bq;
  void* wkv;          // layers 14/15: [768][384] unfolded (k | v)
  float* bkv;
  float* norm_att;    // layers 14/15
  float *qln_w, *qln_b, *kln_w, *kln_b;
  void* wo;
  float* bo;
  void* wpw1;         // [768][384] GLU-interleaved, norm folded
  float* bpw1;
  float* wdw;         // [31][384] BN folded, tap-major
  float* bdw;
  void* wpw2;
  float* bpw2;
  float* norm_out;
};

}  // namespace

struct tone_session {
  int device = 0;
  int precision = TONE_PRECISION_FP32;
  Geom geo = make_geom(kChunk);   // chunk geometry (tone_session_set_chunk; 300 ms by default)
  int max_batch = 0;
  bool finalized = false;
  bool use_graph = false;
  int32_t* frame_info = nullptr;   // optional [batch*10] greedy token | speech flag << 8
  bool timing = false;
  int debug_stop = -1;
  std::map<std::string, std::vector<float>> host;
  std::vector<DevBuf> allocs;
  int64_t dev_bytes = 0;

  // weights
  float *basis_p, *fbank_p, *rope_cos, *rope_sin;
  float *pre_norm, *w1, *scale1, *shift1, *scale2, *shift2, *out_norm;
  void* w1t = nullptr;   // bf16 mode: conv1 weights [kt 11][c 32][kf 32] (kf >= 21 zero)
  void* w2c;
  uint16_t* w2p = nullptr;   // fp32 (split) mode: conv2 split planes packed for conv2_p3 (frontend.hip)
  void* wsub_out;
  float *wred, *bred, *bred_pw;
  void* wred_pw;
  float *whead, *bhead;
  LayerW L[16];
  std::map<const void*, const uint16_t*> w3;   // fp32 (split) mode: GEMM weight -> its bf16 planes
  std::map<const void*, const uint16_t*> w3p;  // fp32 mode, the gemm_d3-routed weights: planes fragment-packed

  // activations
  float *wave, *power, *feats, *rA, *rB, *qkv, *kvp, *g, *probs;
  void *x2, *flat, *h, *ctx, *d, *xn, *kv, *yred;   // bf16 in bf16 mode
  float *rAP = nullptr, *rBP = nullptr;   // fp32 mode: fragment-packed copies of rA / rB (gemm_d3n's A)
  uint16_t *xbA, *xbB;                              // bf16 shadows of rA / rB (bf16 mode)
  uint8_t *a8 = nullptr, *a8s = nullptr, *h8 = nullptr, *h8s = nullptr;   // fp8 mode: MXFP8 GEMM inputs
  float* ss8 = nullptr;                             // fp8 mode: sum-of-squares slab of a8's rows [rows][kSsSlots]
  float *ws, *ws_ss;
  int64_t ws_cap = 0;

  // graphs
  struct GraphKey {
    int batch;
    const void *a, *b, *c, *d, *e, *f, *g, *h, *i;
    int64_t stride;
    bool operator<(const GraphKey& o) const {
      return std::memcmp(this, &o, sizeof(GraphKey)) < 0;
    }
  };
  struct CachedGraph {
    hipGraphExec_t exec;
    uint64_t last_use;
  };
  static constexpr size_t kMaxGraphs = 16;
  std::map<GraphKey, CachedGraph> graphs;
  uint64_t graph_clock = 0;

  // timing
  struct Timed {
    std::string family;
    hipEvent_t a, b;
  };
  std::vector<Timed> timed;
  size_t timed_used = 0;
  std::map<std::string, std::pair<double, int64_t>> last_timing;
};

namespace {

template <typename T>
int dalloc(tone_session* s, T** out, size_t count) {
  void* p = nullptr;
  const size_t bytes = count * sizeof(T);
  HIP_TRY(hipMalloc(&p, bytes));
  HIP_TRY(hipMemset(p, 0, bytes));
  s->allocs.push_back({p, bytes});
  s->dev_bytes += (int64_t)bytes;
  *out = static_cast<T*>(p);
  return TONE_OK;
}

int upload(tone_session* s, float** out, const std::vector<float>& v) {
  int rc = dalloc(s, out, v.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpy(*out, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  return TONE_OK;
}

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// bf16 activations and GEMM operands: bf16 mode, and fp8 mode (bf16 everywhere except the MXFP8 GEMMs)
bool bfmode(const tone_session* s) {
  return s->precision == TONE_PRECISION_BF16 || s->precision == TONE_PRECISION_FP8;
}

// OCP e4m3fn, round to nearest even, saturating at 448 (0x7E; 0x7F is NaN)
uint8_t f32_to_e4m3(float x) {
  const uint8_t sg = std::signbit(x) ? 0x80 : 0;
  const float a = std::fabs(x);
  if (std::isnan(x)) return 0x7F;
  if (a >= 448.0f) return sg | 0x7E;
  if (a < 0.015625f) {                                   // below 2^-6: subnormal, step 2^-9
    const float m = std::nearbyint(a * 512.0f);          // default rounding mode: to nearest even
    return sg | (uint8_t)m;                              // m == 8 encodes 2^-6 (exp 1, mant 0)
  }
  int ex;
  const float f = std::frexp(a, &ex);                    // a = f 2^ex, f in [0.5, 1)
  int e = ex - 1;
  int m = (int)std::nearbyint((f * 2.0f - 1.0f) * 8.0f);
  if (m == 8) { m = 0; ++e; }
  if (e > 8 || (e == 8 && m == 7)) return sg | 0x7E;
  return sg | (uint8_t)(((e + 7) << 3) | m);
}

// MXFP8 upload (fp8 mode): per 32 consecutive values along K, E = floor(log2 max|w|) - 8 (E8M0, biased),
// values w / 2^(E - 127) in e4m3 -- the same rule as quant_mx_kernel (gemm_mx.hip)
int upload_mx(tone_session* s, MxW* out, const std::vector<float>& v, int N, int K) {
  std::vector<uint8_t> q((size_t)N * K), sc((size_t)N * K / 32);
  for (int n = 0; n < N; ++n)
    for (int b = 0; b < K / 32; ++b) {
      const float* w = v.data() + (size_t)n * K + 32 * b;
      float am = 0.f;
      for (int i = 0; i < 32; ++i) am = std::fmax(am, std::fabs(w[i]));
      uint32_t bits;
      std::memcpy(&bits, &am, 4);
      const int e = std::max(0, std::min(254, (int)((bits >> 23) & 0xff) - 8));
      sc[(size_t)n * (K / 32) + b] = (uint8_t)e;
      const float inv = std::ldexp(1.0f, 127 - e);
      for (int i = 0; i < 32; ++i) q[(size_t)n * K + 32 * b + i] = f32_to_e4m3(w[i] * inv);
    }
  int rc = dalloc(s, &out->q, q.size());
  if (!rc) rc = dalloc(s, &out->s, sc.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpy(out->q, q.data(), q.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(out->s, sc.data(), sc.size(), hipMemcpyHostToDevice));
  return TONE_OK;
}

// GEMM weight in the session's precision (fp32, or bf16 bits).  fp32 (split) mode also uploads the
// exact three-term bf16 split [3][N][K] (w = w0 + w1 + w2, each term the bf16 rounding of what the
// previous ones leave) that gemm_x3 reads.
// packK > 0 (fp32 mode, the N = 384 projections gemm_d3 can take): also the planes fragment-packed (common.h wpk_off)
int upload_w(tone_session* s, void** out, const std::vector<float>& v, int packK = 0) {
  if (!bfmode(s)) {
    float* p;
    int rc = upload(s, &p, v);
    *out = p;
    if (rc || s->precision != TONE_PRECISION_FP32) return rc;
    const size_t n = v.size();
    std::vector<uint16_t> pl(3 * n);
    for (size_t i = 0; i < n; ++i) {
      const uint16_t h = f2bf(v[i]);
      const float r1 = v[i] - bf2f(h);
      const uint16_t m = f2bf(r1);
      pl[i] = h;
      pl[n + i] = m;
      pl[2 * n + i] = f2bf(r1 - bf2f(m));
    }
    uint16_t* d;
    rc = dalloc(s, &d, pl.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(d, pl.data(), pl.size() * 2, hipMemcpyHostToDevice));
    s->w3[p] = d;
    if (packK > 0 && packK % 32 == 0 && n % ((size_t)32 * packK) == 0) {
      const int64_t N = (int64_t)(n / packK);
      std::vector<uint16_t> pk(pl.size());
      for (int64_t r = 0; r < N; ++r)
        for (int k = 0; k < packK; ++k)
          for (int q = 0; q < 3; ++q) pk[wpk_off(r, k, q, packK)] = pl[q * n + (size_t)r * packK + k];
      uint16_t* dp;
      rc = dalloc(s, &dp, pk.size());
      if (rc) return rc;
      HIP_TRY(hipMemcpy(dp, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
      s->w3p[p] = dp;
    }
    return TONE_OK;
  }
  std::vector<uint16_t> hb(v.size());
  for (size_t i = 0; i < v.size(); ++i) hb[i] = f2bf(v[i]);
  uint16_t* p;
  int rc = dalloc(s, &p, hb.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpy(p, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  *out = p;
  return TONE_OK;
}

const std::vector<float>* getw(tone_session* s, const std::string& name, size_t numel, std::string* missing) {
  auto it = s->host.find(name);
  if (it == s->host.end() || it->second.size() != numel) {
    if (missing->empty()) *missing = name;
    return nullptr;
  }
  return &it->second;
}

// ---- front-end constants ----------------------------------------------------------------------
// FilterbankFeatures._compute_forward_basis (feats.py:66-80): fft(eye(160)) rows 0..80 as
// [Re ; Im], times the float32 symmetric Hann window, pre-emphasis matrix folded in, as float32.
std::vector<float> make_basis() {
  const int n = kWin;
  std::vector<float> win(n);
  const float step = (float)(M_PI * 2.0 / (double)(n - 1));
  for (int k = 0; k < n; ++k) win[k] = 0.5f - 0.5f * std::cos((float)k * step);
  std::vector<double> fb((size_t)n * kBasisRows);  // [k][r]
  for (int k = 0; k < n; ++k)
    for (int r = 0; r < kBasisRows; ++r) {
      const int f = r < kBins ? r : r - kBins;
      const double ang = -2.0 * M_PI * (double)((k * f) % n) / (double)n;
      const double v = r < kBins ? std::cos(ang) : std::sin(ang);
      fb[(size_t)k * kBasisRows + r] = v * (double)win[k];
    }
  const double pe = 0.97;
  std::vector<float> basis((size_t)kBasisRows * n);
  for (int k = 0; k < n; ++k)
    for (int r = 0; r < kBasisRows; ++r) {
      double v = fb[(size_t)k * kBasisRows + r];
      if (k == 0) v = (1.0 - pe) * v;
      if (k + 1 < n) v -= pe * fb[(size_t)(k + 1) * kBasisRows + r];
      basis[(size_t)r * n + k] = (float)v;
    }
  return basis;
}

double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}

// torchaudio 2.7.1 functional.melscale_fbanks(81, 0, 4000, 64, 8000, norm="slaney",
// mel_scale="slaney") (called at feats.py:84-92), transposed to [64][81], float32 arithmetic.
std::vector<float> make_fbank() {
  const int nf = kBins, nm = kMels;
  std::vector<float> freqs(nf), mpts(nm + 2), fpts(nm + 2);
  for (int i = 0; i < nf; ++i) freqs[i] = (float)(4000.0 * i / (nf - 1));
  const double m0 = hz_to_mel(0.0), m1 = hz_to_mel(4000.0);
  const float f_sp = (float)(200.0 / 3), min_log_mel = (float)(1000.0 / (200.0 / 3));
  const float logstep = (float)(std::log(6.4) / 27.0);
  for (int i = 0; i < nm + 2; ++i) {
    mpts[i] = (float)(m0 + (m1 - m0) * i / (nm + 1));
    fpts[i] = mpts[i] >= min_log_mel ? 1000.0f * std::exp(logstep * (mpts[i] - min_log_mel)) : f_sp * mpts[i];
  }
  std::vector<float> fb((size_t)nm * nf);
  for (int m = 0; m < nm; ++m) {
    const float enorm = 2.0f / (fpts[m + 2] - fpts[m]);
    for (int f = 0; f < nf; ++f) {
      const float down = (-1.0f * (fpts[m] - freqs[f])) / (fpts[m + 1] - fpts[m]);
      const float up = (fpts[m + 2] - freqs[f]) / (fpts[m + 2] - fpts[m + 1]);
      fb[(size_t)m * nf + f] = std::fmax(0.0f, std::fmin(down, up)) * enorm;
    }
  }
  return fb;
}

// RotaryPositionalEmbeddings._build_state (submodules.py:120-140), positions -30..12 (cached keys of
// layer 15 through the last frame of a 400 ms chunk), 16 freqs.
void make_rope(std::vector<float>& cs, std::vector<float>& sn) {
  cs.resize((30 + kTMax) * 16);
  sn.resize((30 + kTMax) * 16);
  for (int j = 0; j < 16; ++j) {
    const float e = (float)(2 * j) / 32.0f;
    const float inv = 1.0f / std::pow(10000.0f, e);
    for (int p = -30; p < kTMax; ++p) {
      const float ang = (float)p * inv;
      cs[(p + 30) * 16 + j] = std::cos(ang);
      sn[(p + 30) * 16 + j] = std::sin(ang);
    }
  }
}

// ---- timing helpers ----------------------------------------------------------------------------
struct Scope {
  tone_session* s;
  hipStream_t st;
  size_t idx = (size_t)-1;
  Scope(tone_session* s_, hipStream_t st_, const char* fam) : s(s_), st(st_) {
    if (!s->timing) return;
    if (s->timed_used == s->timed.size()) {
      tone_session::Timed t;
      t.family = fam;
      (void)hipEventCreate(&t.a);
      (void)hipEventCreate(&t.b);
      s->timed.push_back(t);
    }
    idx = s->timed_used++;
    s->timed[idx].family = fam;
    (void)hipEventRecord(s->timed[idx].a, st);
  }
  ~Scope() {
    if (idx != (size_t)-1) (void)hipEventRecord(s->timed[idx].b, st);
  }
};

#define LAUNCH(fam, expr)                                                                      \
  do {                                                                                         \
    Scope _sc(s, st, fam);                                                                     \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return fail(TONE_E_HIP, std::string(fam) + ": " + hipGetErrorString(_e)); \
  } while (0)

int gemm_call(tone_session* s, hipStream_t st, const char* fam, const void* A, int64_t lda, const void* W, void* C,
              int64_t ldc, const float* bias, int M, int N, int K, int epi, int rowscale, const float* R = nullptr,
              float alpha = 1.0f, bool a_bf16 = false, bool c_bf16 = false, uint16_t* c2 = nullptr,
              bool mx_out = false, const DwFuse* dw = nullptr, const AttFuse* att = nullptr,
              const float* norm_w = nullptr, bool h_blocked = false, bool a_packed = false, bool c_packed = false,
              float* cp = nullptr) {
  GemmArgs a{};   // value-initialised: every field not set below is zero
  a.norm_w = norm_w;
  a.h_blocked = h_blocked;
  if (dw) a.dw = *dw;
  if (att) a.att = *att;
  a.A = A;
  a.lda = lda;
  a.W = W;
  a.C = C;
  a.ldc = ldc;
  a.bias = bias;
  a.R = R;
  a.ldr = ldc;
  a.alpha = alpha;
  a.M = M;
  a.N = N;
  a.K = K;
  a.rowscale = rowscale;
  a.inv_sqrt_k = (float)std::pow((double)K, -0.5);
  a.ws = s->ws;
  a.ws_ss = s->ws_ss;
  a.ws_cap = s->ws_cap;
  a.k_split = 0;
  const bool bf = bfmode(s);
  a.a_bf16 = bf && a_bf16;
  a.c_bf16 = bf && c_bf16;
  a.C2 = bf ? c2 : nullptr;
  // bf16 / fp8 modes: the residual stream rA / rB is fp16 (the RESID projections, and the STOREs that start it)
  a.res16 = bf && (epi == EPI_RESID || C == s->rA || C == s->rB);
  if (mx_out) {   // fp8 mode, RESID: also the MXFP8 form of the shadow and its sum-of-squares slab (the next MX GEMM's A)
    a.C8 = s->a8;
    a.C8s = s->a8s;
    a.ss8 = s->ss8;
  }
  if (s->precision == TONE_PRECISION_FP32) {
    auto it = s->w3.find(W);
    a.W3 = it == s->w3.end() ? nullptr : it->second;
    auto ip = s->w3p.find(W);
    a.W3P = ip == s->w3p.end() ? nullptr : ip->second;
  }
  a.a_packed = a_packed;
  a.c_packed = c_packed;
  a.CP = cp;
  LAUNCH(fam, gemm(a, epi, bf, st));
  return TONE_OK;
}

// fp8 mode: one MXFP8 GEMM (gemm_mx.hip); A8/As the e4m3 rows and their scales (K bytes / K/32 per row)
int mx_call(tone_session* s, hipStream_t st, const char* fam, const uint8_t* A8, const uint8_t* As, const MxW& w, void* C,
            int64_t ldc, const float* bias, int M, int N, int K, int epi, const float* rs_ss, const float* R = nullptr,
            float alpha = 1.0f, bool c_bf16 = false, uint16_t* C2 = nullptr, uint8_t* C8 = nullptr,
            uint8_t* C8s = nullptr, bool mx_out = false, const float* norm_w = nullptr) {
  MxArgs a{};
  a.A = A8;
  a.lda = K;
  a.As = As;
  a.ldas = K / 32;
  a.W = w.q;
  a.Ws = w.s;
  a.rs_ss = rs_ss;
  a.bias = bias;
  a.C = C;
  a.ldc = ldc;
  a.c_bf16 = c_bf16;
  a.R = R;
  a.ldr = ldc;
  a.alpha = alpha;
  a.C2 = C2;
  a.C8 = C8;
  a.C8s = C8s;
  a.ldc8s = N / 64;
  a.res16 = epi == EPI_RESID;   // fp8 mode: the residual stream is fp16
  if (mx_out) {   // RESID: also the MXFP8 form of the shadow and its sum-of-squares slab (the next MX GEMM's A)
    a.Q8 = s->a8;
    a.Q8s = s->a8s;
    a.ss8 = s->ss8;
  }
  a.M = M;
  a.N = N;
  a.K = K;
  // FFN up from 40 blocks of 256 rows: the X-stationary MXFP8 kernel (M = 40960: 110 vs 137 us, M = 10240: 34 vs
  // 39; profiles/r03_xs_route_sweep.jsonl)
  if (epi == EPI_SWIGLU && K == 384 && (M + 255) / 256 >= 40) {
    LAUNCH(fam, gemm_xs8(a, epi, 0, st));
    return TONE_OK;
  }
  // the residual-output projections at large M: whole rows per workgroup (gemm_rp.hip; optionally the fused norm)
  if (epi == EPI_RESID && N == kD && gemm_rp_routed(M, K)) {
    LAUNCH(fam, gemm_rp_mx(a, norm_w, st));
    return TONE_OK;
  }
  if (norm_w) return fail(TONE_E_HIP, std::string(fam) + ": a fused norm needs the row-panel route");
  LAUNCH(fam, gemm_mx(a, epi, st));
  return TONE_OK;
}

#define CALL(x)          \
  do {                   \
    int _rc = (x);       \
    if (_rc) return _rc; \
  } while (0)

// element `i` of an activation buffer held as fp32, or as bf16 bits in bf16 mode
const void* act_at(const float* base, int64_t i, bool bf) {
  return bf ? static_cast<const void*>(reinterpret_cast<const uint16_t*>(base) + i) : static_cast<const void*>(base + i);
}

// The whole streaming step (Tone.forward_for_export, model.py:162-205).
// bf16 mode: every GEMM operand is bf16 in memory -- the residual stream is kept in fp16 (as the reference's exported
// graph keeps it) plus a bf16 shadow written by each of its producers; the other operands are produced in bf16 directly.
// fp32 mode: the residual stream and every activation are fp32.
int enqueue_step(tone_session* s, const int32_t* signal, StateRef sr, float* logp, int B, hipStream_t st) {
  const int D = kD;
  const bool bf = bfmode(s), f8 = s->precision == TONE_PRECISION_FP8;
  uint16_t* shA = bf ? s->xbA : nullptr;
  uint16_t* shB = bf ? s->xbB : nullptr;
  const Geom& geo = s->geo;
  LAUNCH("mel_prep", launch_mel_prep(signal, sr, s->wave, B, geo.chunk, st));
  LAUNCH("mel", mel_gemms(s->wave, s->basis_p, s->fbank_p, s->power, s->feats, B, geo.chunk, st));
  if (s->debug_stop == 0) return TONE_OK;
  if (bf && geo.T == kT) {   // 300 ms bf16 / fp8: conv1 output straight into conv2's LDS slab
    LAUNCH("sub_conv", launch_sub_conv_bf16(s->feats, sr, s->pre_norm, s->w1t, s->scale1, s->shift1, s->w2c, s->scale2,
                                            s->shift2, s->flat, B, st));
  } else {
    LAUNCH("sub1", launch_sub1(s->feats, sr, s->pre_norm, s->w1, s->w1t, s->scale1, s->shift1, s->x2, bf, B,
                               geo.chunk, st));
    LAUNCH("conv2", conv2_gemm(s->x2, s->w2c, s->scale2, s->shift2, s->flat, B, bf, st, geo.chunk, s->w2p));
  }
  CALL(gemm_call(s, st, "gemm_sub_out", s->flat, kSubOut, s->wsub_out, s->rA, D, nullptr, B * geo.T, D, kSubOut,
                 EPI_STORE, 0, nullptr, 1.0f, /*a_bf16=*/true));
  // fp8 mode: the norms that feed a layer's FFN1 directly, FFN1's down-projection (before q|k|v) and pw2 (before FFN2)
  // also emit the next MX GEMM's MXFP8 operand and its sum-of-squares slab (no quant_mx launch)
  // (TONE_FP8_NORMQ=0 keeps the separate quant_mx launches; the operands are bit-identical either way,
  // tests/test_gpu_parity.py::test_fp8_norm_quant_fusion_matches_quant_mx; norms 0.6-1 % per step,
  // profiles/r02_fp8_normq_ab.txt)
  const bool f8n = f8 && knobs().fp8_normq;
  bool q8_fresh = f8n;
  LAUNCH("norm", launch_rmsnorm(s->rA, s->out_norm, B * geo.T, shA, 0, bf, st, f8n ? s->a8 : nullptr, s->a8s, s->ss8));
  if (s->debug_stop == 1) {
    // the fused-vs-separate check reads the first FFN1's MXFP8 operand here: make it the separate way too
    if (f8 && !f8n) LAUNCH("quant_mx", launch_quant_mx(shA, D, B * geo.T, D, s->a8, s->a8s, s->ss8, st));
    return TONE_OK;
  }
  float* x = s->rA;
  uint16_t* xs = shA;           // bf16 shadow of x (bf16 mode)
  int T = geo.T;
  for (int l = 0; l < 16; ++l) {
    const LayerW& w = s->L[l];
    const int M = B * T;
    const void* xa = bf ? static_cast<const void*>(xs) : x;   // A operand of the rowscale GEMMs
    // bf16 / fp8 modes: norm_out runs inside FFN2's down-projection when that launch is a row-panel one (whole rows);
    // in fp8 mode it then also emits the next layer's FFN1 operand
    const bool norm_fused = bf && knobs().rp_norm && gemm_rp_routed(M, kDff);
    // bf16 mode, FFN up on gemm_xw and FFN down on gemm_rp (M >= 16384, 64+ blocks of 256 rows): the hidden h in 32 x 32
    // tiles (common.h hblk_off), whole-KiB stores out of gemm_xw instead of 32-byte row segments
    const bool h_blocked = bf && !f8 && knobs().h_blocked && gemm_rp_routed(M, kDff) && (M + 255) / 256 >= 40;
    const bool q8_after_norm = f8n && l != 6 && l < 14;
    // fp32 mode, the N = 384 projections routed to gemm_d3 (M = B T in its range): their A operands (h, ctx, the
    // depthwise conv output) written fragment-packed by their producers (common.h xpk_off)
    const bool f32m = s->precision == TONE_PRECISION_FP32;
    const bool pk_h = f32m && gemm_d3_routed(M, kDff, D) && s->w3p.count(w.w2[0]) && s->w3p.count(w.w2[1]);
    const bool pk_d = f32m && gemm_d3_routed(M, D, D) && s->w3p.count(w.wo) && s->w3p.count(w.wpw2);
    // ... and pw1 (GLU, folded norm) on gemm_d3n over a packed copy of the residual rows that attn-out writes beside them
    // (GemmArgs::CP): 217 vs 267 us per fp32 B = 256 step.  FFN up and q|k|v on gemm_d3n measured no faster in the step
    // (1039 vs 1019, 163 vs 160 us: their 7 / 2.6 MB of packed W planes come cold from HBM each layer, where gemm_x3 keeps
    // its W tile in LDS across row blocks; profiles/r06_d3x_all_ab.jsonl, step_r06_d3x_all_fp32_b256.txt; pw1 alone:
    // r06_d3x_pw1_ab.jsonl) and the packed copies they need cost their writes, so they stay on gemm_x3
    const bool pk_pw1 = pk_d && knobs().d3x && s->w3p.count(w.wpw1);
    float* xp = pk_pw1 ? (x == s->rA ? s->rAP : s->rBP) : nullptr;
    // FFN1 (conformer_blocks.py:812-814); h in bf16 in bf16 mode
    // fp8 mode: the residual shadow quantized to MXFP8 (with its row factor), h produced as MXFP8 by the
    // up-projection's epilogue
    // fp8 mode: q8_fresh = a8 / a8s / ss8 already hold the MXFP8 form of the current shadow xs -- made by the norm
    // (norm_out / out_norm), or by the RESID GEMM that produced xs (FFN1 down before q|k|v, pw2 before FFN2), else
    // by a quant_mx launch here
    auto ffn = [&](int f) -> int {
      if (f8) {
        if (!q8_fresh) LAUNCH("quant_mx", launch_quant_mx(xs, D, M, D, s->a8, s->a8s, s->ss8, st));
        CALL(mx_call(s, st, "gemm_ffn_up", s->a8, s->a8s, w.mx13[f], nullptr, kDff, w.b13[f], M, 2 * kDff, D, EPI_SWIGLU,
                     s->ss8, nullptr, 1.0f, false, nullptr, s->h8, s->h8s));
        q8_fresh = f8n && f == 0 && l < 14;   // FFN1 down emits the MXFP8 operand of layers 0-13's q|k|v
        const bool fuse = f == 1 && norm_fused;   // FFN2 down + norm_out: the operand of the next layer's FFN1
        return mx_call(s, st, "gemm_ffn_down", s->h8, s->h8s, w.mx2[f], x, D, w.b2[f], M, D, kDff, EPI_RESID, nullptr, x,
                       0.5f, false, xs, nullptr, nullptr, fuse ? q8_after_norm : q8_fresh, fuse ? w.norm_out : nullptr);
      }
      CALL(gemm_call(s, st, "gemm_ffn_up", xa, D, w.w13[f], s->h, kDff, w.b13[f], M, 2 * kDff, D, EPI_SWIGLU, 1, nullptr,
                     1.0f, true, true, nullptr, false, nullptr, nullptr, nullptr, h_blocked, false, pk_h));
      // FFN2's down-projection on the row-panel kernel also applies the block-final RMSNorm (norm_out)
      return gemm_call(s, st, "gemm_ffn_down", s->h, kDff, w.w2[f], x, D, w.b2[f], M, D, kDff, EPI_RESID, 0, x, 0.5f, true,
                       false, xs, false, nullptr, nullptr, f == 1 && norm_fused ? w.norm_out : nullptr, h_blocked, pk_h);
    };
    CALL(ffn(0));
    // MHSA (conformer_blocks.py:816-825)
    AttnArgs aa{};
    aa.ctx = s->ctx;
    aa.ctx_bf16 = bf;
    aa.probs = s->probs;
    aa.qln_w = w.qln_w;
    aa.qln_b = w.qln_b;
    aa.kln_w = w.kln_w;
    aa.kln_b = w.kln_b;
    aa.rope_cos = s->rope_cos;
    aa.rope_sin = s->rope_sin;
    aa.s = sr;
    aa.T = T;
    aa.B = B;
    if (l < 14) {
      const bool rec = (l == 0 || l == 7);
      const int N = rec ? 3 * D : D;
      // q/k/v in bf16 in bf16 mode (half the attention kernel's input bytes)
      if (f8) {
        if (!q8_fresh) LAUNCH("quant_mx", launch_quant_mx(xs, D, M, D, s->a8, s->a8s, s->ss8, st));
        CALL(mx_call(s, st, "gemm_qkv", s->a8, s->a8s, w.mxqkv, s->qkv, N, w.bqkv, M, N, D, EPI_STORE, s->ss8, nullptr,
                     1.0f, true));
      } else {
        CALL(gemm_call(s, st, "gemm_qkv", xa, D, w.wqkv, s->qkv, N, w.bqkv, M, N, D, EPI_STORE, 1, nullptr, 1.0f, true,
                       bf));
      }
      aa.S = 0;
      aa.recompute = rec;
      aa.reduced = 0;
      if (rec) {
        aa.q = act_at(s->qkv, 0, bf); aa.ldq = N;
        aa.k = act_at(s->qkv, D, bf); aa.ldk = N;
        aa.v = act_at(s->qkv, 2 * D, bf); aa.ldv = N;
      } else {
        aa.v = s->qkv; aa.ldv = D;
      }
    } else {
      const int S = (l == 14) ? kMhsaS / 2 : kMhsaS;
      LAUNCH("kv_assemble", launch_kv_assemble(x, w.norm_att, sr, l - 14, T, S, s->xn, s->kv, bf, B, st));
      if (f8) {
        const int MK = B * (S + T);
        LAUNCH("quant_mx", launch_quant_mx(static_cast<const uint16_t*>(s->xn), D, M, D, s->a8, s->a8s, nullptr, st));
        CALL(mx_call(s, st, "gemm_qkv", s->a8, s->a8s, w.mxq, s->qkv, D, w.bq, M, D, D, EPI_STORE, nullptr, nullptr, 1.0f,
                     true));
        LAUNCH("quant_mx", launch_quant_mx(static_cast<const uint16_t*>(s->kv), D, MK, D, s->a8, s->a8s, nullptr, st));
        CALL(mx_call(s, st, "gemm_qkv", s->a8, s->a8s, w.mxkv, s->kvp, 2 * D, w.bkv, MK, 2 * D, D, EPI_STORE, nullptr,
                     nullptr, 1.0f, true));
      } else {
        CALL(gemm_call(s, st, "gemm_qkv", s->xn, D, w.wq, s->qkv, D, w.bq, M, D, D, EPI_STORE, 0, nullptr, 1.0f, true,
                       bf));
        CALL(gemm_call(s, st, "gemm_qkv", s->kv, D, w.wkv, s->kvp, 2 * D, w.bkv, B * (S + T), 2 * D, D, EPI_STORE, 0,
                       nullptr, 1.0f, true, bf));
      }
      aa.S = S;
      aa.recompute = 1;
      aa.reduced = (l == 14);
      aa.probs = nullptr;
      aa.q = s->qkv; aa.ldq = D;
      aa.k = act_at(s->kvp, 0, bf); aa.ldk = 2 * D;
      aa.v = act_at(s->kvp, D, bf); aa.ldv = 2 * D;
    }
    // fp32 mode at M <= 64, shared-probability layers: ctx = P V inside the attn-out projection (gemm_sm.hip)
    if (!aa.recompute && s->precision == TONE_PRECISION_FP32 && M <= 64 && s->w3.count(w.wo)) {
      const AttFuse af{aa.probs, static_cast<const float*>(aa.v), aa.ldv, T};
      CALL(gemm_call(s, st, "gemm_attn_out_ctx", s->ctx, D, w.wo, x, D, w.bo, M, D, D, EPI_RESID, 0, x, 1.0f, false,
                     false, nullptr, false, nullptr, &af));
    } else {
      aa.ctx_packed = pk_d;
      LAUNCH("attention", launch_attention(aa, st));
      CALL(gemm_call(s, st, "gemm_attn_out", s->ctx, D, w.wo, x, D, w.bo, M, D, D, EPI_RESID, 0, x, 1.0f, true, false,
                     xs, false, nullptr, nullptr, nullptr, false, pk_d, false, xp));
    }
    q8_fresh = false;
    // Convolution module (conformer_blocks.py:827-830)
    // fp32 mode at M <= 64 (the drop-in's per-call batch): the depthwise conv runs in pw1's epilogue (gemm_sm.hip)
    // (not with the resident state: the fused form reads the flat conv section)
    if (s->precision == TONE_PRECISION_FP32 && M <= 64 && s->w3.count(w.wpw1) && !sr.ring) {
      const DwFuse dw{w.wdw, w.bdw, sr, l, T, static_cast<float*>(s->d)};
      CALL(gemm_call(s, st, "gemm_pw1_dwconv", xa, D, w.wpw1, s->g, D, w.bpw1, M, 2 * D, D, EPI_GLU, 1, nullptr, 1.0f,
                     false, false, nullptr, false, &dw));
    } else {
      CALL(gemm_call(s, st, "gemm_pw1", pk_pw1 ? static_cast<const void*>(xp) : xa, D, w.wpw1, s->g, D, w.bpw1, M, 2 * D,
                     D, EPI_GLU, 1, nullptr, 1.0f, true, true, nullptr, false, nullptr, nullptr, nullptr, false, pk_pw1));
      // (g in bf16 in the bf16 / fp8 modes; fp32 in fp32 mode: gemm_call drops c_bf16 there)
      LAUNCH("dwconv", launch_dwconv(s->g, sr, l, w.wdw, w.bdw, s->d, bf, T, B, st, pk_d));
    }
    // fp8 mode: pw2 also emits FFN2's MXFP8 operand
    CALL(gemm_call(s, st, "gemm_pw2", s->d, D, w.wpw2, x, D, w.bpw2, M, D, D, EPI_RESID, 0, x, 1.0f, true, false, xs, f8n,
                   nullptr, nullptr, nullptr, false, pk_d));
    q8_fresh = f8n;
    if (s->debug_stop == 100 + l) {   // FFN2's MXFP8 operand: the pw2 epilogue's, or quant_mx's with the fusion off
      if (f8 && !f8n) LAUNCH("quant_mx", launch_quant_mx(xs, D, M, D, s->a8, s->a8s, s->ss8, st));
      return TONE_OK;
    }
    // FFN2 + norm_out (conformer_blocks.py:832-836)
    CALL(ffn(1));
    // the next layer's FFN1 reads this norm's output unless the reduction / upsampling comes in between
    q8_fresh = q8_after_norm;
    if (!norm_fused)
      LAUNCH("norm", launch_rmsnorm(x, w.norm_out, M, xs, 0, bf, st, q8_fresh ? s->a8 : nullptr, s->a8s, s->ss8));
    if (l == 6) {  // CausalTemporalReduction (conformer.py:221-222); rA keeps the residual
      // fp32 mode: the 1x1 (K = 1536, N = 384) on gemm_d3 over y written packed by reduce_conv
      const bool pk_y = s->precision == TONE_PRECISION_FP32 && gemm_d3_routed(B * geo.Tr, 4 * D, D) &&
                        s->w3p.count(s->wred_pw);
      LAUNCH("reduce_conv", launch_reduce_conv(s->rA, sr, s->wred, s->bred, s->yred, bf, B, geo.T, st, pk_y));
      CALL(gemm_call(s, st, "gemm_reduce", s->yred, 4 * D, s->wred_pw, s->rB, D, s->bred_pw, B * geo.Tr, D, 4 * D,
                     EPI_STORE, 0, nullptr, 1.0f, true, false, shB, false, nullptr, nullptr, nullptr, false, pk_y));
      x = s->rB;
      xs = shB;
      T = geo.Tr;
    }
    if (l == 14) {  // TemporalUpsampling (conformer.py:224-225)
      LAUNCH("upsample", launch_upsample_add(s->rA, s->rB, B, geo.T, shA, 0, bf, st));
      x = s->rA;
      xs = shA;
      T = geo.T;
    }
    if (s->debug_stop == 2 + l) return TONE_OK;
  }
  LAUNCH("head", launch_head(s->rA, s->whead, s->bhead, logp, s->frame_info, B * geo.T, bf, st));
  return TONE_OK;
}

int finalize_weights(tone_session* s) {
  std::string miss;
  const int D = kD;
  auto W = [&](const std::string& n, size_t numel) { return getw(s, n, numel, &miss); };
  const std::string pe = "encoder.pre_encode.";
  auto pre_norm = W(pe + "pre_norm.weight", 64);
  auto c1w = W(pe + "conv.0.0.weight", 32 * 231);
  auto c1b = W(pe + "conv.0.0.bias", 32);
  const std::vector<float>* bn1[4];
  const std::vector<float>* bn2[4];
  const char* bnn[4] = {"weight", "bias", "running_mean", "running_var"};
  for (int i = 0; i < 4; ++i) {
    bn1[i] = W(pe + "conv.0.1." + bnn[i], 32);
    bn2[i] = W(pe + "conv.1.1." + bnn[i], 64);
  }
  auto c2w = W(pe + "conv.1.0.weight", (size_t)64 * 32 * 121);
  auto c2b = W(pe + "conv.1.0.bias", 64);
  auto outw = W(pe + "out.weight", (size_t)D * kSubOut);
  auto outn = W(pe + "out_norm.weight", D);
  const std::string tr = "encoder.temportal_reduction.";
  auto rw = W(tr + "conv.weight", 4 * D * 3);
  auto rb = W(tr + "conv.bias", 4 * D);
  auto rpw = W(tr + "conv_pw.weight", (size_t)D * 4 * D);
  auto rpb = W(tr + "conv_pw.bias", D);
  auto hw = W("decoder.decoder_layers.0.weight", 35 * D);
  auto hb = W("decoder.decoder_layers.0.bias", 35);
  if (!miss.empty()) return fail(TONE_E_MISSING, "missing or mis-sized weight: " + miss);

  {  // spectrum GEMM weight [256][160]: 32-bin blocks of Re rows then Im rows (bins >= 81 zero)
    const std::vector<float> basis = make_basis();   // [162][160]: rows 0..80 Re, 81..161 Im
    std::vector<float> bp((size_t)2 * kMelPowCols * kWin, 0.f);
    for (int q = 0; q < kMelPowCols / 32; ++q)
      for (int r = 0; r < 32; ++r) {
        const int f = 32 * q + r;
        if (f >= kBins) continue;
        for (int k = 0; k < kWin; ++k) {
          bp[(size_t)(64 * q + r) * kWin + k] = basis[(size_t)f * kWin + k];
          bp[(size_t)(64 * q + 32 + r) * kWin + k] = basis[(size_t)(kBins + f) * kWin + k];
        }
      }
    CALL(upload(s, &s->basis_p, bp));
    const std::vector<float> fb = make_fbank();      // [64][81]
    std::vector<float> fp((size_t)128 * kMelPowCols, 0.f);
    for (int m = 0; m < kMels; ++m)
      for (int f = 0; f < kBins; ++f) fp[(size_t)m * kMelPowCols + f] = fb[(size_t)m * kBins + f];
    CALL(upload(s, &s->fbank_p, fp));
  }
  std::vector<float> cs, sn;
  make_rope(cs, sn);
  CALL(upload(s, &s->rope_cos, cs));
  CALL(upload(s, &s->rope_sin, sn));

  CALL(upload(s, &s->pre_norm, *pre_norm));
  {
    std::vector<float> sc(32), sh(32);
    for (int c = 0; c < 32; ++c) {
      const double scale = (double)(*bn1[0])[c] / std::sqrt((double)(*bn1[3])[c] + 1e-5);
      sc[c] = (float)scale;
      sh[c] = (float)(((double)(*c1b)[c] - (double)(*bn1[2])[c]) * scale + (double)(*bn1[1])[c]);
    }
    CALL(upload(s, &s->w1, *c1w));
    if (bfmode(s)) {
      std::vector<float> wt((size_t)kSub1Kt * kSub1C * 32, 0.f);
      for (int c = 0; c < kSub1C; ++c)
        for (int kt = 0; kt < kSub1Kt; ++kt)
          for (int kf = 0; kf < kSub1Kf; ++kf) wt[((size_t)kt * kSub1C + c) * 32 + kf] = (*c1w)[((size_t)c * kSub1Kt + kt) * kSub1Kf + kf];
      CALL(upload_w(s, &s->w1t, wt));
    }
    CALL(upload(s, &s->scale1, sc));
    CALL(upload(s, &s->shift1, sh));
  }
  {
    std::vector<float> sc(64), sh(64);
    for (int c = 0; c < 64; ++c) {
      const double scale = (double)(*bn2[0])[c] / std::sqrt((double)(*bn2[3])[c] + 1e-5);
      sc[c] = (float)scale;
      sh[c] = (float)(((double)(*c2b)[c] - (double)(*bn2[2])[c]) * scale + (double)(*bn2[1])[c]);
    }
    // conv2 weight tap-major [c2][kt][kf][ci] for the implicit GEMM over channels-last input
    const int kw = bfmode(s) ? kConv2KPad : kConv2K;   // bf16: zero pad tap
    std::vector<float> w2r((size_t)64 * kw, 0.f);
    for (int c2 = 0; c2 < 64; ++c2)
      for (int ci = 0; ci < 32; ++ci)
        for (int k = 0; k < 121; ++k) w2r[(size_t)c2 * kw + k * 32 + ci] = (*c2w)[((size_t)c2 * 32 + ci) * 121 + k];
    CALL(upload_w(s, &s->w2c, w2r));
    if (s->precision == TONE_PRECISION_FP32) {
      std::vector<uint16_t> pl((size_t)3 * w2r.size()), px(pl.size());
      const size_t n = w2r.size();
      for (size_t i = 0; i < n; ++i) {
        const uint16_t h = f2bf(w2r[i]);
        const float r1 = w2r[i] - bf2f(h);
        const uint16_t m = f2bf(r1);
        pl[i] = h;
        pl[n + i] = m;
        pl[2 * n + i] = f2bf(r1 - bf2f(m));
      }
      conv2_p3_pack(pl.data(), px.data());
      CALL(dalloc(s, &s->w2p, px.size()));
      HIP_TRY(hipMemcpy(s->w2p, px.data(), px.size() * 2, hipMemcpyHostToDevice));
    }
    CALL(upload(s, &s->scale2, sc));
    CALL(upload(s, &s->shift2, sh));
  }
  {  // out Linear columns permuted from c*34+f to f*64+c (the conv2 GEMM writes channel-minor rows)
    std::vector<float> wo((size_t)D * kSubOut);
    for (int n = 0; n < D; ++n)
      for (int c = 0; c < 64; ++c)
        for (int f = 0; f < 34; ++f) wo[(size_t)n * kSubOut + f * 64 + c] = (*outw)[(size_t)n * kSubOut + c * 34 + f];
    CALL(upload_w(s, &s->wsub_out, wo));
  }
  CALL(upload(s, &s->out_norm, *outn));
  CALL(upload(s, &s->wred, *rw));
  CALL(upload(s, &s->bred, *rb));
  CALL(upload_w(s, &s->wred_pw, *rpw, 4 * kD));
  CALL(upload(s, &s->bred_pw, *rpb));
  CALL(upload(s, &s->whead, *hw));
  CALL(upload(s, &s->bhead, *hb));

  for (int l = 0; l < 16; ++l) {
    const std::string p = "encoder.layers." + std::to_string(l) + ".";
    LayerW& lw = s->L[l];
    for (int f = 0; f < 2; ++f) {
      const std::string ff = f == 0 ? "feed_forward1" : "feed_forward2";
      auto nrm = W(p + "norm_" + ff + ".weight", D);
      auto w1 = W(p + ff + ".linear1.weight", (size_t)kDff * D);
      auto b1 = W(p + ff + ".linear1.bias", kDff);
      auto wv = W(p + ff + ".linearv.weight", (size_t)kDff * D);
      auto bv = W(p + ff + ".linearv.bias", kDff);
      auto w2 = W(p + ff + ".linear2.weight", (size_t)D * kDff);
      auto b2 = W(p + ff + ".linear2.bias", D);
      if (!miss.empty()) return fail(TONE_E_MISSING, "missing or mis-sized weight: " + miss);
      std::vector<float> w13((size_t)2 * kDff * D), b13(2 * kDff);
      for (int q = 0; q < kDff / 32; ++q)
        for (int r = 0; r < 32; ++r) {
          const int src = 32 * q + r;
          for (int k = 0; k < D; ++k) {
            w13[(size_t)(64 * q + r) * D + k] = (*w1)[(size_t)src * D + k] * (*nrm)[k];
            w13[(size_t)(64 * q + 32 + r) * D + k] = (*wv)[(size_t)src * D + k] * (*nrm)[k];
          }
          b13[64 * q + r] = (*b1)[src];
          b13[64 * q + 32 + r] = (*bv)[src];
        }
      CALL(upload_w(s, &lw.w13[f], w13));
      CALL(upload(s, &lw.b13[f], b13));
      CALL(upload_w(s, &lw.w2[f], *w2, kDff));
      if (s->precision == TONE_PRECISION_FP8) {
        CALL(upload_mx(s, &lw.mx13[f], w13, 2 * kDff, D));
        CALL(upload_mx(s, &lw.mx2[f], *w2, D, kDff));
      }
      CALL(upload(s, &lw.b2[f], *b2));
    }
    const std::string a = p + "self_attn.";
    auto natt = W(p + "norm_self_att.weight", D);
    auto wv = W(a + "linear_v.weight", (size_t)D * D);
    auto bv = W(a + "linear_v.bias", D);
    auto wo = W(a + "linear_out.weight", (size_t)D * D);
    auto bo = W(a + "linear_out.bias", D);
    if (!miss.empty()) return fail(TONE_E_MISSING, "missing or mis-sized weight: " + miss);
    const bool rec = (l == 0 || l == 7 || l >= 14);
    const std::vector<float>*wq = nullptr, *bq = nullptr, *wk = nullptr, *bk = nullptr;
    if (rec) {
      wq = W(a + "linear_q.weight", (size_t)D * D);
      bq = W(a + "linear_q.bias", D);
      wk = W(a + "linear_k.weight", (size_t)D * D);
      bk = W(a + "linear_k.bias", D);
      auto qw = W(a + "q_ln.weight", kDk), qb = W(a + "q_ln.bias", kDk);
      auto kw = W(a + "k_ln.weight", kDk), kb = W(a + "k_ln.bias", kDk);
      if (!miss.empty()) return fail(TONE_E_MISSING, "missing or mis-sized weight: " + miss);
      CALL(upload(s, &lw.qln_w, *qw));
      CALL(upload(s, &lw.qln_b, *qb));
      CALL(upload(s, &lw.kln_w, *kw));
      CALL(upload(s, &lw.kln_b, *kb));
    }
    if (l < 14) {
      const int nb = rec ? 3 : 1;
      std::vector<float> wqkv((size_t)nb * D * D), bqkv(nb * D);
      const std::vector<float>* mats[3] = {wq, wk, wv};
      const std::vector<float>* bias[3] = {bq, bk, bv};
      for (int m = 0; m < nb; ++m) {
        const int src = rec ? m : 2;
        for (int n = 0; n < D; ++n) {
          for (int k = 0; k < D; ++k) wqkv[(size_t)(m * D + n) * D + k] = (*mats[src])[(size_t)n * D + k] * (*natt)[k];
          bqkv[m * D + n] = (*bias[src])[n];
        }
      }
      CALL(upload_w(s, &lw.wqkv, wqkv));
      if (s->precision == TONE_PRECISION_FP8) CALL(upload_mx(s, &lw.mxqkv, wqkv, nb * D, D));
      CALL(upload(s, &lw.bqkv, bqkv));
    } else {
      std::vector<float> wkv((size_t)2 * D * D), bkv(2 * D);
      std::memcpy(wkv.data(), wk->data(), (size_t)D * D * 4);
      std::memcpy(wkv.data() + (size_t)D * D, wv->data(), (size_t)D * D * 4);
      std::memcpy(bkv.data(), bk->data(), D * 4);
      std::memcpy(bkv.data() + D, bv->data(), D * 4);
      CALL(upload_w(s, &lw.wq, *wq));
      CALL(upload(s, &lw.bq, *bq));
      CALL(upload_w(s, &lw.wkv, wkv));
      if (s->precision == TONE_PRECISION_FP8) {
        CALL(upload_mx(s, &lw.mxq, *wq, D, D));
        CALL(upload_mx(s, &lw.mxkv, wkv, 2 * D, D));
      }
      CALL(upload(s, &lw.bkv, bkv));
      CALL(upload(s, &lw.norm_att, *natt));
    }
    CALL(upload_w(s, &lw.wo, *wo, kD));
    CALL(upload(s, &lw.bo, *bo));

    const std::string c = p + "conv.";
    auto ncv = W(p + "norm_conv.weight", D);
    auto pw1 = W(c + "pointwise_conv1.weight", (size_t)2 * D * D);
    auto pb1 = W(c + "pointwise_conv1.bias", 2 * D);
    auto dww = W(c + "depthwise_conv.conv.weight", (size_t)D * kConvK);
    auto dwb = W(c + "depthwise_conv.conv.bias", D);
    const std::vector<float>* bn[4];
    for (int i = 0; i < 4; ++i) bn[i] = W(c + "batch_norm." + bnn[i], D);
    auto pw2 = W(c + "pointwise_conv2.weight", (size_t)D * D);
    auto pb2 = W(c + "pointwise_conv2.bias", D);
    auto nout = W(p + "norm_out.weight", D);
    if (!miss.empty()) return fail(TONE_E_MISSING, "missing or mis-sized weight: " + miss);
    std::vector<float> wp((size_t)2 * D * D), bp(2 * D);
    for (int q = 0; q < D / 32; ++q)
      for (int r = 0; r < 32; ++r) {
        const int src = 32 * q + r;
        for (int k = 0; k < D; ++k) {
          wp[(size_t)(64 * q + r) * D + k] = (*pw1)[(size_t)src * D + k] * (*ncv)[k];
          wp[(size_t)(64 * q + 32 + r) * D + k] = (*pw1)[(size_t)(D + src) * D + k] * (*ncv)[k];
        }
        bp[64 * q + r] = (*pb1)[src];
        bp[64 * q + 32 + r] = (*pb1)[D + src];
      }
    CALL(upload_w(s, &lw.wpw1, wp, kD));
    CALL(upload(s, &lw.bpw1, bp));
    std::vector<float> wd((size_t)D * kConvK), bd(D);
    for (int ch = 0; ch < D; ++ch) {
      const double scale = (double)(*bn[0])[ch] / std::sqrt((double)(*bn[3])[ch] + 1e-5);
      for (int k = 0; k < kConvK; ++k) wd[(size_t)k * D + ch] = (float)((double)(*dww)[(size_t)ch * kConvK + k] * scale);
      bd[ch] = (float)(((double)(*dwb)[ch] - (double)(*bn[2])[ch]) * scale + (double)(*bn[1])[ch]);
    }
    CALL(upload(s, &lw.wdw, wd));
    CALL(upload(s, &lw.bdw, bd));
    CALL(upload_w(s, &lw.wpw2, *pw2, kD));
    CALL(upload(s, &lw.bpw2, *pb2));
    CALL(upload(s, &lw.norm_out, *nout));
  }

  // activations
  const size_t MB = (size_t)s->max_batch;
  CALL(dalloc(s, &s->wave, MB * kWaveMax));
  CALL(dalloc(s, &s->power, MB * kMelTMax * kMelPowCols));
  CALL(dalloc(s, &s->feats, MB * kMelTMax * kMels));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->x2), MB * kSub2InMax * kSub1F * kSub1C));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->flat), MB * kTMax * kSubOut));
  CALL(dalloc(s, &s->rA, MB * kTMax * D));
  CALL(dalloc(s, &s->rB, MB * kTrMax * D));
  // h: rows padded to a multiple of 32 for the blocked layout (common.h hblk_off); bf16 in the bf16 mode, so this
  // fp32-sized buffer holds it twice over
  CALL(dalloc(s, reinterpret_cast<float**>(&s->h), (MB * kTMax + 32) * kDff));
  CALL(dalloc(s, &s->qkv, MB * kTMax * 3 * D));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->xn), MB * kTMax * D));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->kv), MB * (30 + kTMax) * D));
  CALL(dalloc(s, &s->kvp, MB * (30 + kTMax) * 2 * D));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->ctx), (MB * kTMax + 32) * D));   // + 32 rows: the packed form's last block
  CALL(dalloc(s, &s->g, MB * kTMax * D));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->d), (MB * kTMax + 32) * D));
  CALL(dalloc(s, &s->probs, MB * kHeads * kTMax * (30 + kTMax)));
  CALL(dalloc(s, reinterpret_cast<float**>(&s->yred), (MB * kTrMax + 32) * 4 * D));   // + 32 rows: packed form
  if (s->precision == TONE_PRECISION_FP32) {
    CALL(dalloc(s, &s->rAP, (MB * kTMax + 32) * D));
    CALL(dalloc(s, &s->rBP, (MB * kTrMax + 32) * D));
  }
  CALL(dalloc(s, &s->xbA, MB * kTMax * D));
  CALL(dalloc(s, &s->xbB, MB * kTrMax * D));
  if (s->precision == TONE_PRECISION_FP8) {
    CALL(dalloc(s, &s->a8, MB * (30 + kTMax) * D));            // the largest quantized input: layer 15's k/v rows
    CALL(dalloc(s, &s->a8s, MB * (30 + kTMax) * (D / 32)));
    CALL(dalloc(s, &s->ss8, MB * (30 + kTMax) * kSsSlots));
    CALL(dalloc(s, &s->h8, MB * kTMax * kDff));
    CALL(dalloc(s, &s->h8s, MB * kTMax * (kDff / 32)));
  }
  // split-K workspace: only small batches split (large ones fill the chip with whole-K tiles)
  s->ws_cap = 16ll << 20;
  CALL(dalloc(s, &s->ws, (size_t)s->ws_cap));
  CALL(dalloc(s, &s->ws_ss, (size_t)16 * MB * 40));
  HIP_TRY(hipDeviceSynchronize());
  return TONE_OK;
}

int run_common(tone_session* s, const int32_t* signal, StateRef sr, float* logp, int batch, void* stream,
               const void* key_a, const void* key_b) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  if (!s->finalized) return fail(TONE_E_STATE, "tone_session_finalize has not been called");
  if (batch <= 0 || batch > s->max_batch)
    return fail(TONE_E_INVALID, "batch " + std::to_string(batch) + " outside 1.." + std::to_string(s->max_batch));
  if (!signal || !sr.in || !sr.out || !logp) return fail(TONE_E_INVALID, "null I/O pointer");
  if (sr.stride < kStateSize) return fail(TONE_E_INVALID, "state stride < 219729");
  if (sr.in == sr.out && !sr.slots_out) return fail(TONE_E_INVALID, "state_out must not alias state_in");
  if (sr.ring && !sr.ring_ids) return fail(TONE_E_INVALID, "null ring ids");
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  // graphs replay a captured step keyed by (batch, I/O pointers); debug stops and timing run eagerly
  if (s->use_graph && st != nullptr && !s->timing && s->debug_stop < 0) {
    tone_session::GraphKey k;
    std::memset(&k, 0, sizeof(k));
    k.batch = batch;
    k.a = signal;
    k.b = sr.in;
    k.c = sr.out;
    k.d = logp;
    k.e = sr.slots;
    k.f = s->frame_info;
    k.g = sr.slots_out;
    k.h = sr.ring;
    k.i = sr.ring_ids;
    k.stride = sr.stride;
    (void)key_a;
    (void)key_b;
    auto it = s->graphs.find(k);
    if (it == s->graphs.end()) {
      HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      int rc = enqueue_step(s, signal, sr, logp, batch, st);
      hipGraph_t graph = nullptr;
      hipError_t e = hipStreamEndCapture(st, &graph);
      if (rc || e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        if (rc) return rc;
        return fail(TONE_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
      }
      hipGraphExec_t exec = nullptr;
      e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (e != hipSuccess) return fail(TONE_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
      // bounded cache: a server that keeps changing pointers or batch sizes evicts the least recently
      // used executable graph instead of growing without limit
      if (s->graphs.size() >= tone_session::kMaxGraphs) {
        auto lru = s->graphs.begin();
        for (auto g = s->graphs.begin(); g != s->graphs.end(); ++g)
          if (g->second.last_use < lru->second.last_use) lru = g;
        // the evicted executable may still be in flight on any stream it was launched on (the key does not
        // include the stream): wait for the device, which only happens on an eviction
        HIP_TRY(hipDeviceSynchronize());
        (void)hipGraphExecDestroy(lru->second.exec);
        s->graphs.erase(lru);
      }
      it = s->graphs.emplace(k, tone_session::CachedGraph{exec, 0}).first;
    }
    it->second.last_use = ++s->graph_clock;
    HIP_TRY(hipGraphLaunch(it->second.exec, st));
    return TONE_OK;
  }
  return enqueue_step(s, signal, sr, logp, batch, st);
}

}  // namespace

// =============================================================================================
extern "C" {

int tone_abi_version(void) { return TONE_ABI_VERSION; }

const char* tone_last_error(void) { return g_err.c_str(); }

int tone_session_create(tone_session** out, int device, int precision, int max_batch) {
  if (!out) return fail(TONE_E_INVALID, "null out pointer");
  if (precision != TONE_PRECISION_FP32 && precision != TONE_PRECISION_BF16 && precision != TONE_PRECISION_FP32_MFMA &&
      precision != TONE_PRECISION_FP8)
    return fail(TONE_E_INVALID, "unknown precision " + std::to_string(precision));
  if (max_batch <= 0) return fail(TONE_E_INVALID, "max_batch must be positive");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(TONE_E_INVALID, "device " + std::to_string(device) + " not present");
  HIP_TRY(hipSetDevice(device));
  auto* s = new tone_session();
  s->device = device;
  s->precision = precision;
  s->max_batch = max_batch;
  *out = s;
  return TONE_OK;
}

int tone_session_destroy(tone_session* s) {
  if (!s) return TONE_OK;
  (void)hipSetDevice(s->device);
  for (auto& kv : s->graphs) (void)hipGraphExecDestroy(kv.second.exec);
  for (auto& t : s->timed) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (auto& a : s->allocs) (void)hipFree(a.p);
  delete s;
  return TONE_OK;
}

int tone_session_set_weight(tone_session* s, const char* name, const float* host_data, int64_t numel) {
  if (!s || !name || !host_data || numel <= 0) return fail(TONE_E_INVALID, "bad set_weight arguments");
  if (s->finalized) return fail(TONE_E_STATE, "session already finalized");
  std::string n(name);
  if (n.rfind("tone.", 0) == 0) n = n.substr(5);
  s->host[n].assign(host_data, host_data + numel);
  return TONE_OK;
}

int tone_session_finalize(tone_session* s) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  if (s->finalized) return TONE_OK;
  HIP_TRY(hipSetDevice(s->device));
  int rc = finalize_weights(s);
  if (rc) return rc;
  s->host.clear();
  s->finalized = true;
  return TONE_OK;
}

int tone_session_set_chunk(tone_session* s, int chunk_samples) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  if (s->finalized) return fail(TONE_E_STATE, "tone_session_set_chunk must precede tone_session_finalize");
  if (chunk_samples != 2400 && chunk_samples != 3200)
    return fail(TONE_E_INVALID, "chunk_samples must be 2400 (300 ms) or 3200 (400 ms), got " + std::to_string(chunk_samples));
  s->geo = make_geom(chunk_samples);
  return TONE_OK;
}

int tone_session_frames_per_chunk(const tone_session* s) { return s ? s->geo.T : 0; }

int tone_session_set_graph(tone_session* s, int enable) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  s->use_graph = enable != 0;
  return TONE_OK;
}

int tone_session_set_frame_info(tone_session* s, int32_t* frame_info) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  s->frame_info = frame_info;
  return TONE_OK;
}

int tone_session_run(tone_session* s, const int32_t* signal, const uint16_t* state_in, float* logprobs,
                     uint16_t* state_out, int batch, int64_t state_stride, void* stream) {
  StateRef sr{reinterpret_cast<const __half*>(state_in), reinterpret_cast<__half*>(state_out), state_stride, nullptr,
              nullptr};
  return run_common(s, signal, sr, logprobs, batch, stream, nullptr, nullptr);
}

int tone_session_run_slots(tone_session* s, const int32_t* signal, const int32_t* slots, const uint16_t* slab_in,
                           uint16_t* slab_out, int64_t slab_stride, float* logprobs, int batch, void* stream) {
  if (!slots) return fail(TONE_E_INVALID, "null slots");
  StateRef sr{reinterpret_cast<const __half*>(slab_in), reinterpret_cast<__half*>(slab_out), slab_stride, slots,
              nullptr};
  return run_common(s, signal, sr, logprobs, batch, stream, nullptr, nullptr);
}

int tone_session_run_rows(tone_session* s, const int32_t* signal, const int32_t* rows_in, const int32_t* rows_out,
                          uint16_t* slab, int64_t slab_stride, float* logprobs, int batch, void* stream) {
  if (!rows_in || !rows_out) return fail(TONE_E_INVALID, "null rows");
  if (rows_in == rows_out) return fail(TONE_E_INVALID, "rows_out must differ from rows_in");
  StateRef sr{reinterpret_cast<const __half*>(slab), reinterpret_cast<__half*>(slab), slab_stride, rows_in, rows_out};
  return run_common(s, signal, sr, logprobs, batch, stream, nullptr, nullptr);
}

int tone_session_run_ring(tone_session* s, const int32_t* signal, const int32_t* rows_in, const int32_t* rows_out,
                          uint16_t* slab, int64_t slab_stride, uint16_t* rings, const int32_t* ring_ids, float* logprobs,
                          int batch, void* stream) {
  if (!rows_in || !rows_out || !rings || !ring_ids) return fail(TONE_E_INVALID, "null rows / rings / ring ids");
  if (rows_in == rows_out) return fail(TONE_E_INVALID, "rows_out must differ from rows_in");
  StateRef sr{reinterpret_cast<const __half*>(slab), reinterpret_cast<__half*>(slab), slab_stride, rows_in, rows_out,
              reinterpret_cast<__half*>(rings), ring_ids};
  return run_common(s, signal, sr, logprobs, batch, stream, nullptr, nullptr);
}

int tone_session_ring_import(tone_session* s, const uint16_t* flat, int64_t flat_stride, uint16_t* slab, int64_t slab_stride,
                             const int32_t* rows, uint16_t* rings, const int32_t* ring_ids, int n, void* stream) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  if (!flat || !slab || !rows || !rings || !ring_ids || n < 0) return fail(TONE_E_INVALID, "bad ring_import arguments");
  if (flat_stride < kStateSize || slab_stride < kStateSize) return fail(TONE_E_INVALID, "state stride < 219729");
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(launch_ring_import(reinterpret_cast<const __half*>(flat), flat_stride, reinterpret_cast<__half*>(slab), slab_stride,
                             rows, reinterpret_cast<__half*>(rings), ring_ids, n, static_cast<hipStream_t>(stream)));
  return TONE_OK;
}

int tone_session_ring_export(tone_session* s, const uint16_t* slab, int64_t slab_stride, const int32_t* rows,
                             const uint16_t* rings, const int32_t* ring_ids, uint16_t* flat, int64_t flat_stride, int n,
                             void* stream) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  if (!flat || !slab || !rows || !rings || !ring_ids || n < 0) return fail(TONE_E_INVALID, "bad ring_export arguments");
  if (flat_stride < kStateSize || slab_stride < kStateSize) return fail(TONE_E_INVALID, "state stride < 219729");
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(launch_ring_export(reinterpret_cast<const __half*>(slab), slab_stride, rows, reinterpret_cast<const __half*>(rings),
                             ring_ids, reinterpret_cast<__half*>(flat), flat_stride, s->geo.T, s->geo.Tr, n,
                             static_cast<hipStream_t>(stream)));
  return TONE_OK;
}

int64_t tone_session_ring_elems(void) { return kRingElems; }

int64_t tone_session_device_bytes(const tone_session* s) { return s ? s->dev_bytes : 0; }

int tone_session_debug_stop(tone_session* s, int stage) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  s->debug_stop = stage;
  return TONE_OK;
}

int tone_session_debug_read(tone_session* s, const char* buffer, void* host_dst, int64_t bytes) {
  if (!s || !buffer || !host_dst || bytes < 0) return fail(TONE_E_INVALID, "bad debug_read arguments");
  if (!s->finalized) return fail(TONE_E_STATE, "session not finalized");
  const size_t MB = (size_t)s->max_batch;
  const std::string n(buffer);
  const void* p = nullptr;
  size_t cap = 0;   // bytes
  if (n == "feats") { p = s->feats; cap = MB * kMelTMax * kMels * 4; }
  else if (n == "x2") { p = s->x2; cap = MB * kSub2InMax * kSub1F * kSub1C * 4; }
  else if (n == "flat") { p = s->flat; cap = MB * kTMax * kSubOut * 4; }
  else if (n == "rA" || n == "rB") {
    // the residual stream: fp16 in the bf16 / fp8 modes, returned as fp32 like the fp32 mode's
    const size_t cap_el = MB * (n == "rA" ? kTMax : kTrMax) * kD;
    if (bytes % 4 || (size_t)bytes / 4 > cap_el) return fail(TONE_E_INVALID, "debug_read larger than the buffer");
    const float* src = n == "rA" ? s->rA : s->rB;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    if (!bfmode(s)) {
      HIP_TRY(hipMemcpy(host_dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
      return TONE_OK;
    }
    std::vector<__half> h((size_t)bytes / 4);
    HIP_TRY(hipMemcpy(h.data(), src, h.size() * 2, hipMemcpyDeviceToHost));
    float* d = static_cast<float*>(host_dst);
    for (size_t i = 0; i < h.size(); ++i) d[i] = __half2float(h[i]);
    return TONE_OK;
  }
  // bf16 / fp8 modes: the bf16 shadow of the residual stream rA (the bits, [M][384])
  else if (n == "xbA" && s->xbA) { p = s->xbA; cap = MB * kTMax * kD * 2; }
  // fp8 mode: the MXFP8 operand of the next MX GEMM (e4m3 [M][384], E8M0 [M][12], fp32 row factors [M])
  else if (n == "a8" && s->a8) { p = s->a8; cap = MB * kTMax * kD; }
  else if (n == "a8s" && s->a8s) { p = s->a8s; cap = MB * kTMax * (kD / 32); }
  else if (n == "ss8" && s->ss8) { p = s->ss8; cap = MB * kTMax * kSsSlots * 4; }
  else return fail(TONE_E_INVALID, "unknown debug buffer " + n);
  if ((size_t)bytes > cap) return fail(TONE_E_INVALID, "debug_read larger than the buffer");
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(host_dst, p, (size_t)bytes, hipMemcpyDeviceToHost));
  return TONE_OK;
}

int tone_session_set_timing(tone_session* s, int enable) {
  if (!s) return fail(TONE_E_INVALID, "null session");
  s->timing = enable != 0;
  s->timed_used = 0;
  return TONE_OK;
}

double tone_session_kernel_us(const tone_session* cs, const char* family, int64_t* launches) {
  auto* s = const_cast<tone_session*>(cs);
  if (!s || !family) return -1.0;
  double tot = 0.0;
  int64_t n = 0;
  for (size_t i = 0; i < s->timed_used; ++i) {
    if (s->timed[i].family != family) continue;
    if (hipEventSynchronize(s->timed[i].b) != hipSuccess) return -1.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s->timed[i].a, s->timed[i].b) != hipSuccess) return -1.0;
    tot += ms * 1000.0;
    ++n;
  }
  if (launches) *launches = n;
  return n ? tot / n : 0.0;
}

}  // extern "C"
