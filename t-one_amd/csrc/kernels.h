// Host-side launchers of the T-one HIP kernels (one streaming step = a fixed sequence of these).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "common.h"

namespace tone {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GLU = 3, EPI_CONV2 = 4 };

struct GemmArgs {
  const float* A;
  int64_t lda;
  const void* W;      // [N][K], fp32 or bf16 (raw bits)
  float* C;
  int64_t ldc;
  const float* bias;  // packed like W's rows, or nullptr
  const float* R;     // residual (EPI_RESID); may alias C
  int64_t ldr;
  float alpha;
  int M, N, K;
  int rowscale;       // 1: divide each row by ||a_row||/sqrt(K) + 1e-8 (folded RMSNorm)
  float inv_sqrt_k;
  // split-K workspace (nullptr disables split-K)
  float* ws;          // [nsplit][M][N] fp32 partials
  float* ws_ss;       // [nsplit][M] partial row sums of squares (rowscale)
  int64_t ws_cap;     // floats available in ws
  int k_split;        // set by the launcher
  const float* scale; // EPI_CONV2: folded BatchNorm scale per output channel (bias = shift)
};

hipError_t gemm(const GemmArgs& a, int epi, bool bf16, hipStream_t st);

// a3 conv2 as an implicit GEMM over all streams: A rows gathered from the channels-last
// [B][38][44][32] input (one 32-deep K-step = one (kt,kf) tap), W [64][121*32] tap-major,
// epilogue SiLU(acc*scale + shift) -> flat [B*10][34*64] (f-major, channel-minor).
hipError_t conv2_gemm(const float* x2, const void* w, const float* scale, const float* shift, float* flat, int B,
                      bool bf16, hipStream_t st);

// a1/a2: PCM -> fp16 -> log-mel fp16 features [B][30][64] (stored as fp32 values); preproc state
// and mhsa_len of the next state.
hipError_t launch_mel(const int32_t* pcm, StateRef s, const float* basis, const float* fbank, float* feats, int B,
                      hipStream_t st);

// a3 part 1: pre-norm RMSNorm(64) + sub1 state + Conv2d(1->32,k11x21) + BN + SiLU, written with the
// carried sub2 rows as the channels-last conv2 input x2 [B][38][44][32]; next sub1/sub2 states.
hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const float* scale1,
                       const float* shift1, float* x2, int B, hipStream_t st);

// In-place RMSNorm over rows of 384 (norm_out, out_norm).
hipError_t launch_rmsnorm(float* x, const float* w, int rows, hipStream_t st);

// Layers 14/15: xn = RMSNorm(r); kv = [cache(S rows) ; xn]; next cache (left-padded to 30) -> state.
hipError_t launch_kv_assemble(const float* r, const float* norm_w, StateRef s, int layer_slot, int T, int S,
                              float* xn, float* kv, int B, hipStream_t st);

struct AttnArgs {
  const float* q; int64_t ldq;      // rows b*T+i
  const float* k; int64_t ldk;      // rows b*(S+T)+j
  const float* v; int64_t ldv;      // rows b*(S+T)+j
  float* ctx;                       // [B*T][384]
  float* probs;                     // [B][8][T][S+T]: written when scores are computed, read when shared
  const float* qln_w; const float* qln_b; const float* kln_w; const float* kln_b;
  const float* rope_cos;            // [40][16] positions -30..9 (row = pos + 30)
  const float* rope_sin;
  StateRef s;                       // for mhsa_len (masks)
  int T, S;
  int recompute;                    // 1: q,k -> LN -> RoPE -> scores; 0: reuse probs
  int reduced;                      // mask offset floor-divided by 2 (layer 14)
  int B;
};
hipError_t launch_attention(const AttnArgs& a, hipStream_t st);

// a9: depthwise causal conv k31 with carried state + folded BatchNorm + SiLU.
hipError_t launch_dwconv(const float* g, StateRef s, int layer, const float* w, const float* b, float* out, int T,
                         int B, hipStream_t st);

// a11: reduction state + grouped conv (384->1536, k3, s2) -> y [B*5][1536]
hipError_t launch_reduce_conv(const float* x, StateRef s, const float* w, const float* b, float* y, int B,
                              hipStream_t st);

// a12: x10[b*10+t] += x5[b*5+t/2]
hipError_t launch_upsample_add(float* x10, const float* x5, int B, hipStream_t st);

// a14: logits = x . Wd^T + bd, log_softmax over 35 classes -> logprobs [B*10][35]
hipError_t launch_head(const float* x, const float* w, const float* b, float* logp, int rows, hipStream_t st);

}  // namespace tone
