// Host-side launchers of the T-one HIP kernels (one streaming step = a fixed sequence of these).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "common.h"

namespace tone {

// Experiment switches, read from the environment ONCE per process (the first call; A/B runs compare separate
// processes).  Defaults are the measured best; none of them changes the formulas or the rounding points (rp_norm
// changes the last bit, see there).
struct Knobs {
  int fp8_normq;       // TONE_FP8_NORMQ=0: separate quant_mx launches instead of the norm-fused MXFP8 operand (bit-identical)
  int rp_norm;         // TONE_RP_NORM=0: norm_out as its own launch instead of inside FFN2 down (gemm_rp).  NOT
                       // bit-identical: the fused form adds the row's squares in another order and multiplies by one
                       // reciprocal per row instead of dividing each element (last-bit differences of the residual)
  int h_blocked;       // TONE_H_BLOCKED=0: the bf16 FFN hidden row-major instead of in 32 x 32 tiles (bit-identical)
  int ring_nt;         // TONE_RING_NT=0: dwconv_ring reads / writes the ring rows through the caches (bit-identical)
  int d3x;             // TONE_D3X=0: fp32 pw1 on gemm_x3 instead of gemm_d3n over the packed copy of the residual rows that
                       // attn-out writes (last-bit changes: the row factor's squares added in another order)
  int x3_xcd;          // TONE_X3_XCD=0: gemm_x3 tiles dealt to XCDs by N only (each L2 fills all of X) instead of 2 M halves
                       // x 4 N quarters (bit-identical)
  int head_mfma;       // TONE_HEAD_MFMA=0: the CTC head (rows > 64) on LDS-fed FMAs instead of the exact-fp32 MFMA (last-bit
                       // changes: the logits' K quarters added in another order)
  int d3;              // TONE_D3=0: fp32 N = 384 projections at small M on gemm_x3 instead of gemm_d3 (last-bit changes:
                       // the K-split partials are added in another order)
};
const Knobs& knobs();

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GLU = 3, EPI_CONV2 = 4, EPI_POWER = 5, EPI_LOGMEL = 6 };

// fp32 mode, M <= 64 (gemm_sm): the depthwise conv module part (dwconv_kernel's arithmetic, bit for bit) run in the
// GLU projection's epilogue, so the pointwise-1 output never leaves the workgroup; w == nullptr: off
struct DwFuse {
  const float* w;     // [31][384] folded taps
  const float* b;     // [384] folded bias
  StateRef s;         // conv state section of layer `layer`
  int layer;
  int T;              // frames per stream (M = streams x T)
  float* out;         // [M][384] SiLU output (pw2's A)
};
// fp32 mode, M <= 64 (gemm_sm): a shared-probability attention layer's context (ctx = P V, attention_kernel's fma
// order) computed in the attn-out projection's operand loads, so ctx never exists; probs == nullptr: off
struct AttFuse {
  const float* probs; // [B][8][T][T], the last recomputing layer's probabilities
  const float* v;     // V rows b*T + j, ldv apart
  int64_t ldv;
  int T;
};
struct GemmArgs {
  const void* A;      // [M][K] fp32, or bf16 bits when a_bf16
  int64_t lda;
  const void* W;      // [N][K], fp32 or bf16 (raw bits)
  void* C;            // fp32, or bf16 bits when c_bf16
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
  int a_bf16, c_bf16; // bf16 mode only: A stored bf16 / C stored bf16
  int rpg;            // A row grouping: row r at (r / rpg) * gstride + (r % rpg) * lda (0 = off)
  int64_t gstride;
  int n_out;          // EPI_LOGMEL: columns written
  uint16_t* C2;       // STORE/RESID: optional bf16 shadow of C (same ldc), feeds bf16 GEMMs
  uint8_t* C8;        // fp8 mode, RESID with C2: also the MXFP8 form of the shadow, e4m3 [M][ldc] ...
  uint8_t* C8s;       // ... E8M0 [M][ldc / 32] ...
  float* ss8;         // ... and the rows' sum-of-squares slab [M][kSsSlots] (common.h)
  int order_n;        // bf16 LDS-DMA kernel: XCD x owns N-tiles [x*ntn/8, (x+1)*ntn/8) (large W)
  int xcd_mn;         // gemm_x3: XCDs as 2 M halves x 4 N quarters of the tile grid (set by the launcher)
  int nt_store;       // non-temporal epilogue stores
  int dbg;            // microbenchmark only: 1 = no epilogue, 4 = no K loop
  const uint16_t* W3; // fp32 mode: W split into three bf16 planes [3][N][K] (gemm_x3), or nullptr
  // fp32 split mode (gemm_x3): an operand held as its exact 3-term bf16 split, planes `*_plane`
  // elements apart (0 = not split)
  int64_t a_plane;    // A given as 3 bf16 planes (lda in elements) instead of fp32
  int64_t c_plane;    // STORE / SWIGLU / GLU: C written as 3 bf16 planes instead of fp32
  int64_t c2_plane;   // C2 shadow written as 3 bf16 planes
  int conv_t, conv_in; // EPI_CONV2: frames per chunk and conv2 input rows per stream (chunk geometry, common.h Geom)
  int res16;          // bf16 / fp8 modes: the residual stream is fp16 -- RESID reads R and writes C as fp16, STORE
                      // writes C as fp16 (the shadow C2 stays bf16)
  DwFuse dw;          // EPI_GLU on gemm_sm only: the depthwise conv in the epilogue (C is not written)
  AttFuse att;        // EPI_RESID, K = 384 on gemm_sm only: A = ctx computed from P and V (A is not read)
  const float* norm_w; // EPI_RESID on the row-panel kernel only (gemm_rp): RMSNorm (gain norm_w) of each whole output
                       // row after the residual add; C and its shadows hold the normalized row
  int h_blocked;       // bf16 FFN hidden h in 32 x 32 tiles (common.h hblk_off): the SWIGLU output C of gemm_xw, the
                       // RESID input A of gemm_rp (the only two kernels that take it; gemm() routes it there or refuses)
  // fp32 split mode, gemm_d3 (common.h xpk_off / wpk_off): W's planes fragment-packed, A fragment-packed (the consumer),
  // C written fragment-packed (the fp32 SWIGLU epilogue of gemm_x3, producing FFN down's A)
  const uint16_t* W3P;
  int a_packed, c_packed;
  float* CP;           // fp32 STORE / RESID on gemm_d3: also C fragment-packed -- the next rowscale projection's A (gemm_d3n)
};

hipError_t gemm(const GemmArgs& a, int epi, bool bf16, hipStream_t st);
// fp32 split mode, STORE / RESID with N = 384 (gemm_d3.hip): fragment-packed operands loaded straight into registers, no
// LDS staging; variant = wave arrangement / K split / prefetch depth (-1: by shape; hipErrorInvalidValue when the shape
// does not fit it).  gemm_d3_routed: whether gemm() sends an fp32 projection of this shape there -- the session then has
// its A written packed by the producer (a_packed) and W packed at load (W3P).
hipError_t gemm_d3(const GemmArgs& a, int epi, int variant, hipStream_t st);
bool gemm_d3_routed(int M, int K, int N);
// the wide form (NT W tiles per wave, optional row factor; A packed or, SWIGLU only, row-major): experiments (variant)
hipError_t gemm_d3n(const GemmArgs& a, int epi, int variant, hipStream_t st);
// Row-panel residual GEMM (gemm_rp.hip): bf16 A / W, N = 384, the fp16 residual stream updated in place with the whole
// output row per workgroup (optional fused RMSNorm, norm_w); bm = panel rows (0: about one panel per CU)
hipError_t gemm_rp(const GemmArgs& a, hipStream_t st, int bm = 0);
// whether gemm() routes a bf16-mode RESID projection of M rows and depth K to gemm_rp (so a norm can be fused)
bool gemm_rp_routed(int M, int K);
// whether gemm_rp implements this argument set (it refuses row factors, grouped rows, split planes, a K split ...)
bool gemm_rp_accepts(const GemmArgs& a);

// W tiles per work item of the X-stationary MXFP8 kernel (gemm_xs8: one 256-row X block, one workgroup per
// CU): the run length minimising rounds x (run + 3), 3 tiles being the per-item cost of loading the X fragments and
// draining the last tile's epilogue; ties go to the longer run (profiles/r03_xs_route_sweep.jsonl)
inline int xs_run_length(int x_blocks, int w_tiles, int cus = 256) {
  int best = w_tiles;
  int64_t best_cost = INT64_MAX;
  for (int c = w_tiles; c >= 1; --c) {
    const int64_t items = (int64_t)x_blocks * ((w_tiles + c - 1) / c);
    const int64_t cost = (items + cus - 1) / cus * (c + 3);
    if (cost < best_cost) { best_cost = cost; best = c; }
  }
  return best;
}

// ---- MXFP8 (TONE_PRECISION_FP8; gemm_mx.hip) --------------------------------------------------------
// e4m3 values with one E8M0 scale per 32 consecutive values along K (OCP MX)
struct MxArgs {
  const uint8_t* A;       // e4m3 [M][K] (lda bytes)
  int64_t lda;
  const uint8_t* As;      // E8M0 [M][K/32] (ldas bytes)
  int64_t ldas;
  const uint8_t* W;       // e4m3 [N][K]
  const uint8_t* Ws;      // E8M0 [N][K/32]
  const float* rs_ss;     // folded RMSNorm: the rows' sum-of-squares slab [M][kSsSlots] (common.h), or nullptr
  const float* bias;      // [N] or nullptr
  void* C;                // STORE: fp32, or bf16 when c_bf16; RESID: fp32 (may alias R)
  int64_t ldc;            // elements (C, C2) / bytes (C8)
  int c_bf16;
  const float* R;         // RESID: C = R + alpha * (.)
  int64_t ldr;
  float alpha;
  uint16_t* C2;           // optional bf16 shadow of an fp32 C
  uint8_t* C8;            // SWIGLU: output as e4m3 [M][N/2] ...
  uint8_t* C8s;           // ... with E8M0 scales [M][N/64]
  int64_t ldc8s;
  uint8_t* Q8;            // RESID with C2: also the MXFP8 form of the bf16 shadow, e4m3 [M][ldc] ...
  uint8_t* Q8s;           // ... E8M0 [M][ldc / 32] ...
  float* ss8;             // ... and the rows' sum-of-squares slab [M][kSsSlots]
  int res16;              // RESID: R and C fp16 (the bf16 / fp8 modes' residual stream)
  int M, N, K;
  int dbg;                // microbenchmarks only (gemm_mx.hip DBG bits); 0 in the session
};
hipError_t gemm_mx(const MxArgs& a, int epi, hipStream_t st);
// the row-panel residual GEMM (gemm_rp.hip) on MXFP8 operands: RESID, N = 384, fp16 residual, optional fused RMSNorm
// (norm_w) and MXFP8 form of the shadow (a.Q8); bm = panel rows (0: about one panel per CU)
hipError_t gemm_rp_mx(const MxArgs& a, const float* norm_w, hipStream_t st, int bm = 0);
// X-stationary MXFP8 GEMM for K = 384 (gemm_mx.hip gemm_xs8_kernel): SWIGLU (-> MXFP8 h) / STORE (bf16 out)
hipError_t gemm_xs8(const MxArgs& a, int epi, int nc, hipStream_t st);
// bf16 [M][K] (ldx elements) -> e4m3 [M][K] + E8M0 [M][K/32]; ss8 (optional): the rows' sum-of-squares slab
// [M][kSsSlots] as {ss, 0, ...} (the folded-RMSNorm row factor's input, common.h mx_row_inv)
hipError_t launch_quant_mx(const uint16_t* X, int64_t ldx, int M, int K, uint8_t* Q, uint8_t* S, float* ss8,
                           hipStream_t st);
// bf16 operands, fixed tile/stage variant (microbenchmarks)
hipError_t gemm_bf16_variant(const GemmArgs& a, int epi, int variant, int nsplit, hipStream_t st);
// persistent transposed-orientation bf16 GEMM (gemm_t.hip); variant = tile shape, see there
hipError_t gemm_t(const GemmArgs& a, int epi, int variant, hipStream_t st);
// X-stationary bf16 GEMM for K = 384 (gemm_xw.hip): each wave's 32 X rows in registers, W tiles streamed through an
// LDS ring, v_mfma_f32_32x32x16_bf16, the ring and the epilogue pipeline running across work items; SWIGLU / GLU,
// bf16 out; nc = W tiles per work item (0: auto)
hipError_t gemm_xw(const GemmArgs& a, int epi, int nc, hipStream_t st);
// exact-fp32 MFMA projections with an in-workgroup K split (gemm_t.hip); variant = tile shape
hipError_t gemm_f32t(const GemmArgs& a, int epi, int variant, hipStream_t st);
// fp32 operands on the bf16 MFMA by exact 3-way bf16 splitting (6 products; gemm_t.hip); needs a.W3
hipError_t gemm_x3(const GemmArgs& a, int epi, int variant, hipStream_t st);
// exact-fp32 projections for M <= 64 (gemm_sm.hip): fp32 W streamed into registers, v_mfma_f32_16x16x4_f32, K split
// over the waves of a 16-column workgroup; STORE / RESID / SWIGLU / GLU, fp32 in and out
hipError_t gemm_sm(const GemmArgs& a, int epi, hipStream_t st);
// the same with the K range split over nsplit workgroups (partials in a.ws, fixed-order combine; gemm.hip)
hipError_t gemm_x3_splitk(const GemmArgs& a, int epi, int variant, int nsplit, hipStream_t st);
// the same arithmetic with fp32 W and X streamed through a K-tile ring (gemm_t.hip gemm_r3_kernel); needs a.W fp32
hipError_t gemm_r3(const GemmArgs& a, int epi, int variant, hipStream_t st);

// a3 conv2 as an implicit GEMM over all streams: A rows gathered from the channels-last
// [B][38][44][32] input (one 32-deep K-step = one (kt,kf) tap), W [64][121*32] tap-major,
// epilogue SiLU(acc*scale + shift) -> flat [B*10][34*64] (f-major, channel-minor).
hipError_t conv2_gemm(const void* x2, const void* w, const float* scale, const float* shift, void* flat, int B,
                      bool bf16, hipStream_t st, int chunk = kChunk, const void* w2p = nullptr);

// a3 conv2 in bf16 mode, one workgroup per stream over an LDS-resident input slab (frontend.hip);
// x2 bf16 [B][38][44][32], w2c bf16 [64][3904] tap-major, flat bf16 [B*10][34*64]
// a3 in bf16 mode at 300 ms: pre-encode RMSNorm + conv1 + conv2 in one launch (the conv2 input stays in LDS)
hipError_t launch_sub_conv_bf16(const float* feats, StateRef s, const float* pre_norm_w, const void* w1t,
                                const float* scale1, const float* shift1, const void* w2c, const float* scale2,
                                const float* shift2, void* flat, int B, hipStream_t st);
hipError_t launch_conv2_bf16(const void* x2, const void* w2c, const float* scale, const float* shift, void* flat, int B,
                             hipStream_t st);
// a3 conv2 in fp32 (split) mode, input rows split once per kernel row (frontend.hip conv2_p3_kernel);
// w2p from conv2_p3_pack
hipError_t launch_conv2_p3(const void* x2, const void* w2p, const float* scale, const float* shift, void* flat, int B,
                           int T, hipStream_t st);
void conv2_p3_pack(const uint16_t* planes, uint16_t* w2p);
// a3 conv2 in fp32 mode for a few streams: exact fp32 MFMA, one workgroup per (row, 16 channels, 16 positions),
// kernel rows over its 11 waves (frontend.hip); w2 fp32 [64][3872] tap-major
hipError_t launch_conv2_sm(const void* x2, const void* w2, const float* scale, const float* shift, void* flat, int B,
                           int T, hipStream_t st);

// a2 log-mel on the fp32 MFMA: power spectrum GEMM over overlapping windows, then filterbank GEMM
// with the log / fp16 epilogue.  wave [B][2480] fp32 (from launch_mel_prep).
hipError_t mel_gemms(const float* wave, const float* basis_p, const float* fbank_p, float* power, float* feats, int B,
                     int chunk, hipStream_t st);

// a1: PCM -> fp16 wave [B][2480] (fp32 storage) with the 80 carried samples; next preproc state
// and mhsa_len of the next state.
hipError_t launch_mel_prep(const int32_t* pcm, StateRef s, float* wave, int B, int chunk, hipStream_t st);

// a3 part 1: pre-norm RMSNorm(64) + sub1 state + Conv2d(1->32,k11x21) + BN + SiLU, written with the
// carried sub2 rows as the channels-last conv2 input x2 [B][38][44][32]; next sub1/sub2 states.
// w1: fp32 [32][11][21] (fp32 mode); w1t: bf16 [11][32][32] kf-padded (bf16 mode)
hipError_t launch_sub1(const float* feats, StateRef s, const float* pre_norm_w, const float* w1, const void* w1t,
                       const float* scale1, const float* shift1, void* x2, bool x2_bf16, int B, int chunk,
                       hipStream_t st);

// In-place RMSNorm over rows of 384 (norm_out, out_norm); optional bf16 shadow of the result
// (3 split planes `plane` elements apart when plane > 0).
// q8 / s8 / ss8 (fp8 mode, optional): also the MXFP8 form of the bf16 shadow row and its sum-of-squares slab,
// exactly what launch_quant_mx would make from the shadow
// r16: x is the bf16 / fp8 modes' fp16 residual stream (read and written as fp16)
// xp (fp32 only): also the normalized rows fragment-packed (common.h xpk_off), the next FFN up's A on gemm_d3n
hipError_t launch_rmsnorm(void* x, const float* w, int rows, uint16_t* shadow, int64_t plane, bool r16, hipStream_t st,
                          uint8_t* q8 = nullptr, uint8_t* s8 = nullptr, float* ss8 = nullptr, float* xp = nullptr);

// Layers 14/15: xn = RMSNorm(r); kv = [cache(S rows) ; xn]; next cache (left-padded to 30) -> state.
// r is the residual stream: fp16 in the bf16 / fp8 modes (obf), fp32 in fp32 mode
hipError_t launch_kv_assemble(const void* r, const float* norm_w, StateRef s, int layer_slot, int T, int S,
                              void* xn, void* kv, bool obf, int B, hipStream_t st);

struct AttnArgs {
  const void* q; int64_t ldq;       // rows b*T+i; fp32, or bf16 bits when ctx_bf16 (bf16 mode)
  const void* k; int64_t ldk;       // rows b*(S+T)+j, same type
  const void* v; int64_t ldv;       // rows b*(S+T)+j, same type
  void* ctx;                        // [B*T][384], fp32 or bf16 (ctx_bf16)
  float* probs;                     // [B][8][T][S+T]: written when scores are computed, read when shared
  const float* qln_w; const float* qln_b; const float* kln_w; const float* kln_b;
  const float* rope_cos;            // [40][16] positions -30..9 (row = pos + 30)
  const float* rope_sin;
  StateRef s;                       // for mhsa_len (masks)
  int T, S;
  int recompute;                    // 1: q,k -> LN -> RoPE -> scores; 0: reuse probs
  int reduced;                      // mask offset floor-divided by 2 (layer 14)
  int B;
  int ctx_bf16;
  int ctx_packed;                   // fp32 only: ctx fragment-packed (common.h xpk_off) for gemm_d3
};
hipError_t launch_attention(const AttnArgs& a, hipStream_t st);

// a9: depthwise causal conv k31 with carried state + folded BatchNorm + SiLU; g and out bf16 when obf, else fp32.
// With s.ring (the resident form) the caches are read from / the new frames written to the stream's ring.
// out_packed (fp32 only): out fragment-packed (common.h xpk_off) for gemm_d3.
hipError_t launch_dwconv(const void* g, StateRef s, int layer, const float* w, const float* b, void* out, bool obf,
                         int T, int B, hipStream_t st, bool out_packed = false);

// flat state <-> resident form (common.h StateRef, tone_session_ring_import / _export): stream i's flat row i <-> slab
// row rows[i] + ring ring_ids[i]; T / Tr = frames per step outside / inside the reduced block (the layers' phases)
hipError_t launch_ring_import(const __half* flat, int64_t fstride, __half* slab, int64_t sstride, const int* rows, __half* ring,
                              const int* ring_ids, int n, hipStream_t st);
hipError_t launch_ring_export(const __half* slab, int64_t sstride, const int* rows, const __half* ring, const int* ring_ids,
                              __half* flat, int64_t fstride, int T, int Tr, int n, hipStream_t st);

// a11: reduction state + grouped conv (384->1536, k3, s2) -> y [B*5][1536]; x fp16 (residual stream) when obf
// y_packed (fp32 only): y fragment-packed (common.h xpk_off, ld 1536) for the 1x1 projection on gemm_d3
hipError_t launch_reduce_conv(const void* x, StateRef s, const float* w, const float* b, void* y, bool obf, int B,
                              int T, hipStream_t st, bool y_packed = false);

// a12: x10[b*10+t] += x5[b*5+t/2]; both fp16 (residual stream) when r16
// xp (fp32 only): also the sum fragment-packed (common.h xpk_off), layer 15's FFN1 A on gemm_d3n
hipError_t launch_upsample_add(void* x10, const void* x5, int B, int T, uint16_t* shadow, int64_t plane, bool r16,
                               hipStream_t st, float* xp = nullptr);

// a14: logits = x . Wd^T + bd, log_softmax over 35 classes -> logprobs [B*10][35]
// a14 + decode flags: logprobs [rows][35]; optional frame_info[row] = greedy token | speech flag << 8
// x: the residual stream, fp16 when r16
hipError_t launch_head(const void* x, const float* w, const float* b, float* logp, int32_t* frame_info, int rows, bool r16,
                       hipStream_t st);

}  // namespace tone
