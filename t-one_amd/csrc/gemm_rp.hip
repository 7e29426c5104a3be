// Row-panel residual GEMM (bf16 / fp8 modes, round 5): the residual-output projections -- FFN down (K = 1536),
// attn-out and pw2 (K = 384), all N = 384 -- as
//
//   x[M][384] (fp16, in place) = x + alpha * (A[M][K] . W[384][K]^T + bias)      (conformer_blocks.py:814, 825, 830, 834)
//   optionally followed by the block-final RMSNorm of the whole row              (conformer_blocks.py:836, submodules.py:34-54)
//
// with one workgroup per row panel and the WHOLE output row in it:
//   * panel = BM rows x 384 columns, BM chosen so that the panels are about one per CU (M = 40960: 160 rows, 256
//     panels; M = 20480: 80 rows).  Each K-step moves BM + 384 rows of 64 bytes into LDS, so the operand fill per CU is
//     (BM + 384) K 2 bytes -- the 128 x 128 tiles of the LDS-DMA kernel moved 2.4x that for the same outputs, and that
//     fill, not the matrix pipe or HBM, bounded them;
//   * a 4-stage ring of 32-deep K-steps filled by global_load_lds_dwordx4, read one step ahead: while the MFMAs of step
//     kt run from registers, step kt + 1's fragments are read and steps kt + 2 .. kt + 4 are in flight (one barrier
//     per step, counted vmcnt); 8 waves as WM x WN, each wave FM x FN tiles of v_mfma_f32_16x16x32_bf16 (16-row granularity, so
//     BM = 160 / 80 split evenly); rows of 64 bytes with chunk c of row r at slot c ^ 3((r >> 3) & 1): every
//     ds_read_b128 16-lane group conflict-free, and the swizzle depends on the lane only (immediate-offset reads);
//   * epilogue in 16-row sweeps: a sweep's accumulators go to LDS as fp32 (pitch 392: conflict-free stores; two image
//     slots alternate), then 32 lanes per row read 16-byte vectors: residual (fp16, loaded during the last K-step) + alpha (acc + bias) -> fp16 residual,
//     its bf16 shadow (the next GEMM's A operand) and, in fp8 mode, its MXFP8 form + sum-of-squares slab; with a norm,
//     the row's RMSNorm first (the row's sum of squares closed over its 32 lanes), so the separate rmsnorm launch and
//     its HBM round trip of the residual are gone.
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

namespace tone {
namespace {

constexpr int kRpN = 384;        // whole output row
constexpr int kRpS = 4;          // ring stages (3 in flight)
constexpr int kRpRowB = 64;      // bytes per staged row: 32 bf16 = one 16x16x32 K-step
constexpr int kRpPitch = 392;    // fp32 pitch of the epilogue image (4 pitch = 32 mod 64 banks)
constexpr int kRpThreads = 512;
constexpr int kRpPre = 3;        // epilogue sweeps whose residual rows are in flight ahead

template <int WM_, int FM_>
struct RpCfg {
  static constexpr int WM = WM_, FM = FM_;
  static constexpr int WN = 8 / WM, FN = kRpN / 16 / WN;   // FN x WN = 24 column tiles of 16
  static constexpr int BM = 16 * FM * WM;
  static constexpr int RP = 16 * FM;                       // rows per wave row = per epilogue pass
  static constexpr int NA = BM / 16;                       // A DMA pieces (1 KiB = 16 rows x 64 B) per stage
  static constexpr int NI = NA + kRpN / 16;                // all pieces per stage
  static constexpr int PMAX = (NI + 7) / 8, PMIN = NI / 8, NHI = NI % 8;   // waves < NHI issue PMAX pieces
  static constexpr int kStage = (BM + kRpN) * kRpRowB;
  static constexpr int kImg = (2 * 16 * kRpPitch + 2 * kRpN) * 4;   // the epilogue's two 16-row image slots + bias / gain
  static constexpr int kLds = kRpS * kStage > kImg ? kRpS * kStage : kImg;
  // MXFP8 (fp8 mode): a stage is one 128-deep K-tile: A rows | W rows (128 B each) | the K-tile's 4 scale bytes per
  // A row (whole 256-byte DMA pieces) | per W row; two stages
  static constexpr int kMxScA = (BM + kRpN) * 128, kMxScW = kMxScA + (BM + 63) / 64 * 256;
  static constexpr int kMxStage = kMxScW + kRpN * 4;
  static constexpr int QA = BM / 8, QW = kRpN / 8, QAS = (BM + 63) / 64, QWS = kRpN / 64;   // DMA pieces per stage
  static constexpr int QN = QA + QW + QAS + QWS, QP = (QN + 7) / 8;
  static constexpr int kLdsMx = 2 * kMxStage > kImg ? 2 * kMxStage : kImg;
  static constexpr int NV = 3;                             // 16-byte vectors per lane per row (32 lanes x 3 x 4 = 384)
  static_assert(WM * WN == 8 && FN * WN == 24, "8 waves over the panel");
  static_assert(kLds <= 160 * 1024 && kLdsMx <= 160 * 1024, "LDS");
};

template <int N>
__device__ __forceinline__ void rp_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait for the stage `ahead` stages older than the youngest issued one (P pieces per stage for this wave)
template <int P>
__device__ __forceinline__ void rp_wait(int ahead) {
  if (ahead >= 3) rp_vmcnt<3 * P>();
  else if (ahead == 2) rp_vmcnt<2 * P>();
  else if (ahead == 1) rp_vmcnt<P>();
  else rp_vmcnt<0>();
}

// cross-lane steps of the epilogue on DPP (VALU) instead of ds_bpermute round trips: xor 1 / xor 2 inside a quad,
// mirror inside 8 / 16 lanes (the butterfly equivalents once the smaller groups are uniform), xor 16 by ds_swizzle
template <int CTRL>
__device__ __forceinline__ float rp_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float rp_sum32(float v) {   // over each 32-lane half
  v += rp_dpp<0xb1>(v);    // quad_perm [1,0,3,2]
  v += rp_dpp<0x4e>(v);    // quad_perm [2,3,0,1]
  v += rp_dpp<0x141>(v);   // row_half_mirror
  v += rp_dpp<0x140>(v);   // row_mirror
  return v + __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x401f));   // xor 16
}
__device__ __forceinline__ float rp_max8(float v) {    // over each 8-lane group
  v = fmaxf(v, rp_dpp<0xb1>(v));
  v = fmaxf(v, rp_dpp<0x4e>(v));
  return fmaxf(v, rp_dpp<0x141>(v));
}

typedef int rp_i32x8 __attribute__((ext_vector_type(8)));
typedef unsigned int rp_u32x4 __attribute__((ext_vector_type(4)));

// the kernel's arguments, from a GemmArgs (bf16 operands) or an MxArgs (MXFP8 operands)
struct RpArgs {
  const void* A;         // bf16 [M][K] (lda elements) or e4m3 [M][K] (lda bytes)
  int64_t lda;
  const uint8_t* As;     // MX: E8M0 [M][K/32] (ldas bytes)
  int64_t ldas;
  const void* W;         // bf16 or e4m3 [384][K]
  const uint8_t* Ws;     // MX: E8M0 [384][K/32]
  const float* bias;     // [384] or nullptr
  const void* R;         // fp16 residual (ldr elements); C may alias it
  int64_t ldr;
  void* C;               // fp16 [M][384] (ldc elements)
  int64_t ldc;
  uint16_t* C2;          // bf16 shadow or nullptr
  uint8_t* C8;           // Q8: the shadow's MXFP8 form [M][ldc], E8M0 [M][ldc / 32], sum-of-squares slab
  uint8_t* C8s;
  float* ss8;
  const float* norm_w;   // NORM: the row RMSNorm's gain
  float alpha;
  int M, K, dbg;
  int h_blocked;         // bf16: A in the blocked hidden layout (HB)
};

// NORM: RMSNorm the output row (gain p.norm_w); Q8: fp8 mode, also the MXFP8 form of the shadow + the slab;
// MX: MXFP8 operands (v_mfma_scale_f32_16x16x128_f8f6f4), else bf16 (v_mfma_f32_16x16x32_bf16);
// HB (bf16): A is the FFN hidden in gemm_xw's blocked tiles (common.h hblk_off), one 32 x 32 tile per K-step and row block
template <int WM, int FM, bool NORM, bool Q8, bool MX, bool HB = false>
__global__ void __launch_bounds__(kRpThreads, 1) gemm_rp_kernel(RpArgs p) {
  using Cfg = RpCfg<WM, FM>;
  constexpr int BM = Cfg::BM, RP = Cfg::RP, FN = Cfg::FN, NA = Cfg::NA, NV = Cfg::NV;
  constexpr int PMAX = Cfg::PMAX;
  __shared__ __attribute__((aligned(16))) uint8_t lds[MX ? Cfg::kLdsMx : Cfg::kLds];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / Cfg::WN, wn = wid % Cfg::WN;
  const int nk = p.K / (MX ? 128 : 32);
  const int npan = (p.M + BM - 1) / BM;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);
  [[maybe_unused]] const uint8_t* __restrict__ A8 = static_cast<const uint8_t*>(p.A);
  [[maybe_unused]] const uint8_t* __restrict__ W8 = static_cast<const uint8_t*>(p.W);
  const int np = wid < Cfg::NHI ? Cfg::PMAX : Cfg::PMIN;   // this wave's DMA pieces per stage (wave-uniform)
#ifdef RP_ABLATE
  // microbenchmark ablations (tools/gemm_bench, gemm_bench_ablate; timing only, results wrong): 1 no epilogue, 4 no K
  // loop, 8 no DMA, 16 no MFMA (a VALU use keeps the fragment reads), 32 no residual loads
  const int dbg = p.dbg;
#else
  constexpr int dbg = 0;
#endif

  // fragment read offset of this lane inside a 16-row block: row l & 15, chunk l >> 4 at its swizzled slot
  const int frag_off = (lane & 15) * kRpRowB + (((lane >> 4) ^ (((lane >> 3) & 1) * 3)) << 4);
  // epilogue lanes: row tid >> 5 of each 16-row sweep, columns 4 (q + 32 i)
  const int er = tid >> 5, eq = tid & 31;

  for (int pan = blockIdx.x; pan < npan; pan += gridDim.x) {
    const int m0 = pan * BM;
    // this wave's DMA sources: piece j = wave + 8 j of the stage's [A rows ; W rows] image, lane L -> image row
    // 16 q + L / 4, chunk slot L & 3 holding global chunk (L & 3) ^ 3((L >> 5) & 1)
    const uint16_t* src[PMAX];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
      const int q = wid + 8 * j;
      const int c = (lane & 3) ^ (((lane >> 5) & 1) * 3);
      const int r = 16 * q + (lane >> 2);
      if (q < NA) {
        const int m = min(m0 + r, p.M - 1);
        if constexpr (HB) src[j] = A + hblk_off(m, c * 8, p.lda);   // + 1024 per K-step (the next 32 columns' tile)
        else src[j] = A + (int64_t)m * p.lda + c * 8;
      } else {
        src[j] = W + (int64_t)(r - BM) * p.K + c * 8;
      }
    }
    auto stage = [&](int slot, int kt) {
      if (dbg & 8) return;
      uint8_t* base = lds + slot * Cfg::kStage;
#pragma unroll
      for (int j = 0; j < PMAX; ++j) {
        const int ks = (HB && wid + 8 * j < NA) ? 1024 : 32;   // A pieces of a blocked hidden step a whole tile
        if (j < np) lds_dma16(src[j] + kt * ks, base + (wid + 8 * j) * 1024);
      }
    };

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // the residual rows of the first kRpPre epilogue sweeps (this lane's vectors), requested under the last K-step; each
    // sweep then requests the one kRpPre ahead
    constexpr int NSW = WM * FM;                  // 16-row sweeps of the panel
    // sweeps whose residual is requested inside the last K-step (WM = 2 holds twice the accumulators: one)
    constexpr int kPreLoop = (WM == 2 ? 1 : kRpPre) < NSW ? (WM == 2 ? 1 : kRpPre) : NSW;
    f16x4_t rin[NSW][NV];
    auto load_res = [&](int s) {
      if (dbg & 32) {
#pragma unroll
        for (int i = 0; i < NV; ++i) rin[s][i] = f16x4_t{0, 0, 0, 0};
        return;
      }
      const int row = min(m0 + 16 * s + er, p.M - 1);
#pragma unroll
      for (int i = 0; i < NV; ++i)
        rin[s][i] = *reinterpret_cast<const f16x4_t*>(reinterpret_cast<const __half*>(p.R) + (int64_t)row * p.ldr +
                                                      4 * (eq + 32 * i));
    };

    if constexpr (MX) {
      // MXFP8: two stages of one 128-deep K-tile; stage kt + 1 is DMA'd while stage kt's MFMAs run.  The pieces of a
      // stage (8 rows x 128 B for A / W, 64 rows x 4 scale bytes for As / Ws) are dealt over the waves, piece q to wave
      // q % 8; a 128-byte row's chunk c sits at slot c ^ ((r >> 1) & 7) (gemm_mx.hip's swizzle: both fragment reads
      // conflict-free)
      constexpr int QA = Cfg::QA, QW = Cfg::QW, QAS = Cfg::QAS, QP = Cfg::QP;
      const int nq = (Cfg::QN - wid + 7) / 8;   // this wave's pieces (wave-uniform)
      // addresses are recomputed where they are used from an opaque copy of the lane id: hoisted out of the loop they
      // were ~30 loop-invariant VGPRs (and spills)
      auto stage_mx = [&](int slot, int kt) {
        if (dbg & 8) return;
        uint8_t* base = lds + slot * Cfg::kMxStage;
        (void)base;
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int j = 0; j < QP; ++j) {
          if (j >= nq) break;
          [[maybe_unused]] const int q = wid + 8 * j;
          if (q < QA + QW) {
            const int r = 8 * (q < QA ? q : q - QA) + (ln >> 3), c = (ln & 7) ^ ((r >> 1) & 7);
            if (q < QA)
              lds_dma16(A8 + (uint32_t)(min(m0 + r, p.M - 1) * p.lda + 128 * kt + 16 * c), base + q * 1024);
            else
              lds_dma16(W8 + (uint32_t)(r * p.K + 128 * kt + 16 * c), base + BM * 128 + (q - QA) * 1024);
          } else {
            const int r = 64 * (q < QA + QW + QAS ? q - QA - QW : q - QA - QW - QAS) + ln;
            if (q < QA + QW + QAS)
              lds_dma4(p.As + (uint32_t)(min(m0 + r, p.M - 1) * p.ldas + 4 * kt), base + Cfg::kMxScA + (q - QA - QW) * 256);
            else
              lds_dma4(p.Ws + (uint32_t)(r * (p.K / 32) + 4 * kt), base + Cfg::kMxScW + (q - QA - QW - QAS) * 256);
          }
        }
      };
      const int nkl = (dbg & 4) ? 0 : nk;
      if (nkl > 0) stage_mx(0, 0);
      for (int kt = 0; kt < nkl; ++kt) {
        rp_vmcnt<0>();   // stage kt landed (the only one in flight)
        barrier_lds();   // ... for every wave; every wave's reads of stage kt - 1 are done, its slot is free
        if (kt + 1 < nkl) stage_mx((kt + 1) & 1, kt + 1);
        if (kt == nkl - 1) {
#pragma unroll
          for (int s = 0; s < kPreLoop; ++s) load_res(s);
        }
        // fragment bases: the lane's row l & 15 of the wave's first 16-row block, chunks (l >> 4) and 4 + (l >> 4) at
        // their swizzled slots, scale byte (l >> 4) of the row; the other blocks are immediate offsets (2 KiB / 64 B)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int l15 = ln & 15, lg = ln >> 4, g = (l15 >> 1) & 7;
        const uint8_t* st = lds + (kt & 1) * Cfg::kMxStage;
        const uint8_t* pa = st + (wm * RP + l15) * 128;
        const uint8_t* pw = st + (BM + wn * FN * 16 + l15) * 128;
        const uint8_t* psa = st + Cfg::kMxScA + 4 * (wm * RP + l15) + lg;
        const uint8_t* psw = st + Cfg::kMxScW + 4 * (wn * FN * 16 + l15) + lg;
        const int c0 = 16 * (lg ^ g), c1 = 16 * ((4 + lg) ^ g);
        auto frag = [&](const uint8_t* row) {
          const rp_u32x4 a = *reinterpret_cast<const rp_u32x4*>(row + c0);
          const rp_u32x4 b = *reinterpret_cast<const rp_u32x4*>(row + c1);
          return rp_i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
        };
        rp_i32x8 af[FM];
        int as[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          af[i] = frag(pa + 2048 * i);
          as[i] = psa[64 * i];
        }
        // W fragments one column tile ahead of its MFMAs (two register sets: all six at once spilled)
        rp_i32x8 wf[2];
        int ws[2];
        auto rdw = [&](int j, int b) {
          wf[b] = frag(pw + 2048 * j);
          ws[b] = psw[64 * j];
        };
        rdw(0, 0);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if (j + 1 < FN) rdw(j + 1, (j + 1) & 1);
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], wf[j & 1], acc[i][j], 0, 0, 0, as[i], 0,
                                                                         ws[j & 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      // fragments of a stage (the lane's swizzled 16-byte chunk of each 16-row block)
      auto read_frags = [&](int slot, bf16x8(&fa)[FM], bf16x8(&fb)[FN]) {
        const uint8_t* st = lds + slot * Cfg::kStage;
  #pragma unroll
        for (int i = 0; i < FM; ++i)
          fa[i] = *reinterpret_cast<const bf16x8*>(st + (wm * RP + 16 * i) * kRpRowB + frag_off);
  #pragma unroll
        for (int j = 0; j < FN; ++j)
          fb[j] = *reinterpret_cast<const bf16x8*>(st + (BM + (wn * FN + j) * 16) * kRpRowB + frag_off);
      };
      auto wait_stage = [&](int younger) {   // this wave's DMAs of a stage landed, `younger` later stages may fly
        if (np == Cfg::PMAX) rp_wait<Cfg::PMAX>(younger);
        else rp_wait<Cfg::PMIN>(younger);
      };
      // read-ahead ring: stage kt + 1's fragments are read while stage kt's MFMAs run (from registers), so no MFMA
      // waits on LDS; stage kt's slot is refilled with stage kt + S right after the barrier that follows its reads
      const int nkl = (dbg & 4) ? 0 : nk;
  #pragma unroll
      for (int s0 = 0; s0 < kRpS; ++s0)
        if (s0 < nkl) stage(s0, s0);
      // two fragment sets, alternating (the loop is unrolled by two so no set is copied)
      bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
      wait_stage(max(0, min(kRpS - 1, nkl - 1)));
      barrier_lds();
      read_frags(0, a0, b0);   // unconditional, as in the loop
      auto step = [&](int kt, bf16x8(&a)[FM], bf16x8(&b)[FN], bf16x8(&na)[FM], bf16x8(&nb)[FN]) {
        if (kt + 1 < nkl) wait_stage(min(kRpS - 2, nkl - 2 - kt));
        barrier_lds();   // stage kt + 1 published; every wave's reads of stage kt are done, its slot is free
        if (kt + kRpS < nkl) stage(kt % kRpS, kt + kRpS);
        if (kt == nkl - 1) {
  #pragma unroll
          for (int s = 0; s < kPreLoop; ++s) load_res(s);
        }
        read_frags((kt + 1) % kRpS, na, nb);   // unconditional (the last step reads a spent slot): a conditional read
                                               // made the compiler merge and split the fragment vectors per element
  #ifdef RP_ABLATE
        if (dbg & 16) {   // (element reads of the fragments in any build split them into 16-bit halves: ablation only)
  #pragma unroll
          for (int i = 0; i < FM; ++i)
  #pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j][0] += (float)a[i][0] * (float)b[j][0];
          return;
        }
  #endif
  #pragma unroll
        for (int i = 0; i < FM; ++i)
  #pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      };
      for (int kt = 0; kt < nkl; kt += 2) {
        step(kt, a0, b0, a1, b1);
        if (kt + 1 < nkl) step(kt + 1, a1, b1, a0, b0);
      }
    }
    if (dbg & 4) {
#pragma unroll
      for (int s = 0; s < kPreLoop; ++s) load_res(s);
    }
#pragma unroll
    for (int s = kPreLoop; s < kRpPre && s < NSW; ++s) load_res(s);
    if (dbg & 1) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (t == 1234.5f) static_cast<float*>(p.C)[tid] = t;
      continue;
    }

    // MX: the last K-tile's fragments are read from stage slot (nk - 1) & 1 during that step, and the image, bias and
    // gain below sit on slot 0: with an odd K-tile count (K = 384: 3) a wave that finished its MFMAs early overwrote
    // fragments another wave was still reading (gemm_bench RPMX at M = 20480, K = 384: max rel error 0.76).  The
    // bf16 ring's last step reads only a spent slot ahead, so it needs no barrier here.
    if constexpr (MX) barrier_lds();

    // epilogue, one 16-row sweep at a time (its accumulators die as it goes): the wave row that owns sweep s writes
    // tile row s % FM to an LDS image slot (two slots alternate, one barrier per sweep), then every lane takes 3
    // 16-byte vectors of one row
    float* img = reinterpret_cast<float*>(lds);
    // bias and gain of the lane's columns through LDS (beside the two image slots; published by the first sweep's
    // barrier): held in registers they cost 12-24 VGPRs, loaded from L2 per sweep their latency stalled every sweep
    float* sbias = img + 2 * 16 * kRpPitch;
    float* sgain = sbias + kRpN;
    if (tid < kRpN / 4) {
      const f32x4 bv = p.bias ? reinterpret_cast<const f32x4*>(p.bias)[tid] : f32x4{0.f, 0.f, 0.f, 0.f};
      reinterpret_cast<f32x4*>(sbias)[tid] = bv;
      if constexpr (NORM) reinterpret_cast<f32x4*>(sgain)[tid] = reinterpret_cast<const f32x4*>(p.norm_w)[tid];
    }
    static_for<NSW>([&](auto sc) {
      constexpr int s = decltype(sc)::value, ti = s % FM, owner = s / FM;
      float* slot = img + (s & 1) * 16 * kRpPitch;
      if (wm == owner) {
        // D of tile (ti, j): column 16 j + (lane & 15) of the wave's columns, rows 4 (lane >> 4) + r
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            slot[(4 * (lane >> 4) + r) * kRpPitch + (wn * FN + j) * 16 + (lane & 15)] = acc[ti][j][r];
      }
      barrier_lds();   // slot s & 1 written; every lane is past sweep s - 1, so the other slot is free
      if constexpr (s + kRpPre < NSW) load_res(s + kRpPre);
      const int row = m0 + 16 * s + er;
      f32x4 v[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(slot + er * kRpPitch + 4 * (eq + 32 * i));
        const f32x4 r = __builtin_convertvector(rin[s][i], f32x4);
        // the residual add rounds to the fp16 residual stream, as the stored stream holds it
        const f32x4 bb = *reinterpret_cast<const f32x4*>(sbias + 4 * (eq + 32 * i));
        v[i] = __builtin_convertvector(__builtin_convertvector(r + p.alpha * (t + bb), f16x4_t), f32x4);
      }
      if constexpr (NORM) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) ss += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        ss = rp_sum32(ss);
        // IEEE sqrt and one IEEE reciprocal of (rms + eps) per row, then a multiply per element: rmsnorm_kernel
        // (encoder.hip) divides each element and adds the squares in another order, so the two forms differ in the last
        // bit (a true division per element here cost 5-7 us per launch: 63.7 -> 70.8 us at M = 40960, K = 1536,
        // profiles/r06_kt1_rp_norm_cost.jsonl)
        const float inv = 1.0f / (sqrtf(ss) * 0.05103103630798288f + kRmsEps);   // 384^-0.5
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const f32x4*>(sgain + 4 * (eq + 32 * i)) * (v[i] * inv);
      }
      const bool ok = row < p.M;
      float ssq = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t o = (int64_t)row * p.ldc + 4 * (eq + 32 * i);
        if (ok) store_res4(p.C, o, v[i], true);
        const uint32_t h0 = pk2(v[i].x, v[i].y), h1 = pk2(v[i].z, v[i].w);
        if (ok && p.C2) {
          typedef unsigned int rp_u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<rp_u32x2*>(p.C2 + o) = rp_u32x2{h0, h1};
        }
        if constexpr (Q8) {
          // the shadow's MXFP8 form as quant_mx makes it (a 32-column block = 8 lanes)
          const float b0 = __uint_as_float(h0 << 16), b1 = __uint_as_float(h0 & 0xffff0000u);
          const float b2 = __uint_as_float(h1 << 16), b3 = __uint_as_float(h1 & 0xffff0000u);
          const float am = rp_max8(fmaxf(fmaxf(fabsf(b0), fabsf(b1)), fmaxf(fabsf(b2), fabsf(b3))));
          const int e = mx_exp(am);
          const uint32_t q4 = quant4(b0, b1, b2, b3, e);
          ssq = fmaf(b3, b3, fmaf(b2, b2, fmaf(b1, b1, fmaf(b0, b0, ssq))));
          if (ok) {
            *reinterpret_cast<uint32_t*>(p.C8 + o) = q4;
            if ((eq & 7) == 0) p.C8s[(int64_t)row * (p.ldc / 32) + (eq + 32 * i) / 8] = (uint8_t)e;
          }
        }
      }
      if constexpr (Q8) {   // the row's sum of squares as {ss, 0, ...} (a producer that sees the whole row)
        ssq = rp_sum32(ssq);
        if (ok && eq < kSsSlots) p.ss8[(int64_t)row * kSsSlots + eq] = eq == 0 ? ssq : 0.f;
      }
    });
    barrier_lds();   // the image is read before the next panel's DMA overwrites the ring
  }
}

template <int WM, int FM, bool MX>
hipError_t launch_rp(const RpArgs& a, hipStream_t st) {
  using Cfg = RpCfg<WM, FM>;
  const int npan = (a.M + Cfg::BM - 1) / Cfg::BM;
  const dim3 grid(npan < 256 ? npan : 256), block(kRpThreads);
  const bool q8 = a.C8 != nullptr;
  if constexpr (!MX) {
    if (a.h_blocked) {   // bf16 FFN down from gemm_xw's blocked hidden (no MXFP8 output in the bf16 mode)
      if (q8) return hipErrorInvalidValue;
      if (a.norm_w) hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, true, false, false, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, false, false, false, true>), grid, block, 0, st, a);
      return hipGetLastError();
    }
  }
  if (a.norm_w) {
    if (q8) hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, true, true, MX>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, true, false, MX>), grid, block, 0, st, a);
  } else {
    if (q8) hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, false, true, MX>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, false, false, MX>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

int gemm_rp_panel_rows(int M) {
  // the smallest panel that keeps the panels within one per CU (256), from the instantiated heights
  const int need = (M + 255) / 256;
  const int rows[] = {16, 32, 48, 64, 80, 96, 128, 160};
  for (int r : rows)
    if (r >= need) return r;
  return 160;
}

template <bool MX>
hipError_t launch_rp_bm(const RpArgs& a, int bm, hipStream_t st) {
  switch (bm > 0 ? bm : gemm_rp_panel_rows(a.M)) {
    case 16: return launch_rp<1, 1, MX>(a, st);
    case 32: return launch_rp<1, 2, MX>(a, st);
    case 48: return launch_rp<1, 3, MX>(a, st);
    case 64: return launch_rp<1, 4, MX>(a, st);
    case 80: return launch_rp<1, 5, MX>(a, st);
    case 96: return launch_rp<2, 3, MX>(a, st);
    case 128: return launch_rp<2, 4, MX>(a, st);
    case 160: return launch_rp<2, 5, MX>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool gemm_rp_routed(int M, int K) {
  // from 64-row panels (M >= 16384): at M = 20480 (80-row panels) 40 vs 45 us (K = 1536) and 18 vs 21 (K = 384) for
  // the LDS-DMA 128 x 128 tiles, at M = 10240 (48 rows) 31 vs 24 and 13.5 vs 11.2 (tools/gemm_bench variants 14 / 90,
  // profiles/r05_rp_sweep_readahead.jsonl): the W fill per CU no longer shrinks with the panel
  return K % 32 == 0 && M >= 16384;
}

bool gemm_rp_accepts(const GemmArgs& a) {
  // what the kernel implements: RESID on bf16 A / W, N = 384, the fp16 residual, no row factor, no grouped A rows, no
  // split planes and no K split (those fields are not read by it, so an argument set using them is refused)
  if (a.N != kRpN || a.K % 32 || a.K < 32 || a.M <= 0 || !a.a_bf16 || !a.res16 || a.c_bf16 || a.lda % 8 ||
      a.ldc % 8 || a.ldr % 4 || !a.R || !a.W)
    return false;
  if (a.rowscale || a.rpg || a.a_plane || a.c_plane || a.c2_plane || a.k_split || a.W3 || a.dw.w || a.att.probs)
    return false;
  if (a.h_blocked && (a.lda % 32 || a.K > a.lda || a.C8)) return false;   // whole tiles; no MXFP8 output
  return !a.C8 || (a.C2 && a.C8s && a.ss8 && a.ldc == a.N);
}

hipError_t gemm_rp(const GemmArgs& a, hipStream_t st, int bm) {
  if (!gemm_rp_accepts(a)) return hipErrorInvalidValue;
  RpArgs r{};
  r.A = a.A; r.lda = a.lda; r.W = a.W; r.bias = a.bias; r.R = a.R; r.ldr = a.ldr; r.C = a.C; r.ldc = a.ldc;
  r.C2 = a.C2; r.C8 = a.C8; r.C8s = a.C8s; r.ss8 = a.ss8; r.norm_w = a.norm_w; r.alpha = a.alpha;
  r.M = a.M; r.K = a.K; r.dbg = a.dbg; r.h_blocked = a.h_blocked;
  return launch_rp_bm<false>(r, bm, st);
}

hipError_t gemm_rp_mx(const MxArgs& a, const float* norm_w, hipStream_t st, int bm) {
  // RESID with the fp16 residual stream; the optional MXFP8 operand (Q8) needs the shadow and whole rows
  if (a.N != kRpN || a.K % 128 || a.K < 128 || a.M <= 0 || !a.res16 || !a.R || a.c_bf16 || a.lda % 16 ||
      a.ldas != a.K / 32 || a.ldc % 8 || a.ldr % 4 || (int64_t)a.M * a.lda >= (1ll << 32))
    return hipErrorInvalidValue;
  if (a.Q8 && (!a.C2 || !a.Q8s || !a.ss8 || a.ldc != a.N)) return hipErrorInvalidValue;
  RpArgs r{};
  r.A = a.A; r.lda = a.lda; r.As = a.As; r.ldas = a.ldas; r.W = a.W; r.Ws = a.Ws; r.bias = a.bias; r.R = a.R;
  r.ldr = a.ldr; r.C = a.C; r.ldc = a.ldc; r.C2 = a.C2; r.C8 = a.Q8; r.C8s = a.Q8s; r.ss8 = a.ss8; r.norm_w = norm_w;
  r.alpha = a.alpha; r.M = a.M; r.K = a.K; r.dbg = a.dbg;
  return launch_rp_bm<true>(r, bm, st);
}

}  // namespace tone
