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
  static constexpr int NV = 3;                             // 16-byte vectors per lane per row (32 lanes x 3 x 4 = 384)
  static_assert(WM * WN == 8 && FN * WN == 24, "8 waves over the panel");
  static_assert(kLds <= 160 * 1024, "LDS");
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

// NORM: RMSNorm the output row (gain p.norm_w); Q8: fp8 mode, also the MXFP8 form of the shadow + the slab
template <int WM, int FM, bool NORM, bool Q8>
__global__ void __launch_bounds__(kRpThreads, 1) gemm_rp_kernel(GemmArgs p) {
  using Cfg = RpCfg<WM, FM>;
  constexpr int BM = Cfg::BM, RP = Cfg::RP, FN = Cfg::FN, NA = Cfg::NA, NV = Cfg::NV;
  constexpr int PMAX = Cfg::PMAX;
  __shared__ __attribute__((aligned(16))) uint8_t lds[Cfg::kLds];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / Cfg::WN, wn = wid % Cfg::WN;
  const int nk = p.K / 32;
  const int npan = (p.M + BM - 1) / BM;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ W = static_cast<const uint16_t*>(p.W);
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
        src[j] = A + (int64_t)m * p.lda + c * 8;
      } else {
        src[j] = W + (int64_t)(r - BM) * p.K + c * 8;
      }
    }
    auto stage = [&](int slot, int kt) {
      if (dbg & 8) return;
      uint8_t* base = lds + slot * Cfg::kStage;
#pragma unroll
      for (int j = 0; j < PMAX; ++j) {
        if (j < np) {
#if defined(__HIP_DEVICE_COMPILE__)
          __builtin_amdgcn_global_load_lds(src[j] + kt * 32, base + (wid + 8 * j) * 1024, 16, 0, 0);
#else
          (void)base;
#endif
        }
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
        const float inv = __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(ss) * 0.05103103630798288f + kRmsEps);   // 384^-0.5
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
          const uint32_t q4 = quant4(b0, b1, b2, b3, exp2i(e));
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

template <int WM, int FM>
hipError_t launch_rp(const GemmArgs& a, hipStream_t st) {
  using Cfg = RpCfg<WM, FM>;
  const int npan = (a.M + Cfg::BM - 1) / Cfg::BM;
  const dim3 grid(npan < 256 ? npan : 256), block(kRpThreads);
  const bool q8 = a.C8 != nullptr;
  if (a.norm_w) {
    if (q8) hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, true, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, true, false>), grid, block, 0, st, a);
  } else {
    if (q8) hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, false, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_rp_kernel<WM, FM, false, false>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace

static int gemm_rp_panel_rows(int M) {
  // the smallest panel that keeps the panels within one per CU (256), from the instantiated heights
  const int need = (M + 255) / 256;
  const int rows[] = {16, 32, 48, 64, 80, 96, 128, 160};
  for (int r : rows)
    if (r >= need) return r;
  return 160;
}

bool gemm_rp_routed(int M, int K) {
  // from 64-row panels (M >= 16384): at M = 20480 (80-row panels) 40 vs 45 us (K = 1536) and 18 vs 21 (K = 384) for
  // the LDS-DMA 128 x 128 tiles, at M = 10240 (48 rows) 31 vs 24 and 13.5 vs 11.2 (tools/gemm_bench variants 14 / 90,
  // profiles/r05_rp_sweep_readahead.jsonl): the W fill per CU no longer shrinks with the panel
  return K % 32 == 0 && M >= 16384;
}

hipError_t gemm_rp(const GemmArgs& a, hipStream_t st, int bm) {
  if (a.N != kRpN || a.K % 32 || a.K < 32 || a.M <= 0 || !a.a_bf16 || !a.res16 || a.c_bf16 || a.lda % 8 ||
      a.ldc % 8 || a.ldr % 4 || !a.R)
    return hipErrorInvalidValue;
  if (a.C8 && (!a.C2 || !a.C8s || !a.ss8 || a.ldc != a.N)) return hipErrorInvalidValue;
  switch (bm > 0 ? bm : gemm_rp_panel_rows(a.M)) {
    case 16: return launch_rp<1, 1>(a, st);
    case 32: return launch_rp<1, 2>(a, st);
    case 48: return launch_rp<1, 3>(a, st);
    case 64: return launch_rp<1, 4>(a, st);
    case 80: return launch_rp<1, 5>(a, st);
    case 96: return launch_rp<2, 3>(a, st);
    case 128: return launch_rp<2, 4>(a, st);
    case 160: return launch_rp<2, 5>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
