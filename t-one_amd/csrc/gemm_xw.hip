// X-stationary bf16 GEMM for K = 384 on the 32x32x16 MFMA, with the W ring and the epilogue pipeline running
// across work items (round 4; replaces round 3's gemm_xs): FFN up (SwiGLU) and pw1 (GLU) at large batch, bf16 h out.
//
//   * each of the 8 waves (two per SIMD) keeps its 32 X rows x 384 K in registers as the B operand of
//     v_mfma_f32_32x32x16_bf16 (24 K-steps x 8 bf16 = 96 VGPRs); W tiles of 64 rows x 384 (48 KiB) stream through a
//     3-deep LDS ring by global_load_lds_dwordx4 and are read as the 32-row A operand.  One 64-row W tile = the g | u
//     32-row block pair of 32 hidden columns (the session's 32-row SwiGLU / GLU interleave): acc_g, acc_u (16
//     registers each) hold g and u of the same (unit, row);
//   * the A operand's lane l reads W row c(l & 31) of the block, c = swap of bits 2 and 3: D row p of the 32x32
//     result (p = (r & 3) + 8 (r >> 2) + 4 h for register r, lane half h) then holds unit c(p) = 16 (r >> 3) + 8 h +
//     (r & 7), so each lane owns 8 consecutive hidden columns in registers 0-7 and 8 more in 8-15: two 16-byte stores
//     per lane and tile, no lane swaps.  c keeps every ds_read_b128 16-lane group on 16 distinct rows mod 16, so with
//     chunk c' of row r at slot c' ^ (r & 15) the reads stay conflict-free;
//   * one flat step sequence per workgroup over all its (item, W tile) pairs: tile s + 2 is DMA'd into ring slot
//     (s + 2) % 3 during step s (one piece every four K-steps) across item boundaries, the epilogue of step s - 1
//     (bias, SwiGLU, bf16, stores) runs between step s's MFMAs whatever item it belongs to, and the next item's X
//     fragments are loaded at the end of an item's last step (peeled, so the compiler waits for them only there).
// Measured (profiles/r04_xw_*): 116-125 us at M = 40960 in the microbenchmark (gemm_xs 116-129), 1.8 % (FFN up) and
// 3 % (pw1) below gemm_xs inside the bf16 B = 4096 step.  Ablations: without MFMAs 74-80 us, without MFMAs and
// epilogue 50-52, DMA / X loads / barriers alone 33-37; a ping-pong schedule (one wave's whole epilogue under its
// partner's MFMAs) 7-8 % slower; SQ counters: the matrix pipe busy 38 % of the launch at 1.96 GHz (gemm_xs 32 %).
// Work item = (256 X rows, a run of nc W tiles), dealt XCD-contiguously.
#include "common.h"
#include "kernels.h"

#include "gemm_common.h"

#include <type_traits>

namespace tone {
namespace {

constexpr int kXwK = 384;                    // K (d_model)
constexpr int kXwKS = kXwK / 16;             // 32x32x16 K-steps (24)
constexpr int kXwWaves = 8;                  // two per SIMD
constexpr int kXwBM = kXwWaves * 32;         // X rows per work item
constexpr int kXwBN = 64;                    // W rows per tile (g block | u block)
constexpr int kXwRowB = kXwK * 2;            // bytes per W row
constexpr int kXwTile = kXwBN * kXwRowB;     // 48 KiB
constexpr int kXwR = 3;                      // ring depth
constexpr int kXwP = kXwTile / 1024 / kXwWaves;   // 1 KiB DMA pieces per wave per tile (6)
// stores per lane per step (the previous step's epilogue): SwiGLU / GLU 2 (16 hidden columns), STORE 4 (the g and u
// halves of the tile are both outputs)
template <int EPI>
constexpr int xw_stores() { return EPI == EPI_STORE ? 4 : 2; }

typedef __bf16 xw_bf16x8 __attribute__((ext_vector_type(8)));
typedef float xw_f32x16 __attribute__((ext_vector_type(16)));
typedef float xw_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 xw_bf16x2 __attribute__((ext_vector_type(2)));
typedef float xw_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int xw_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xw_perm(int r) {   // swap bits 2 and 3 (an involution on 0..31)
  return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1);
}

// position of a step in the workgroup's sequence: item, tile j of the item's run, run length n, first W tile t0
struct XwPos {
  int item, j, n, t0, mt;
};

// DBG (XW_ABLATE microbenchmark builds only; 1-16 and 256 are timing only, the results are wrong): 256 no output stores,
// 1 no epilogue (the MFMAs
// and fragment reads are then dead code too), 2 no MFMA, 4 no W DMA after the prologue, 16 no W fragment reads, 64 a
// ping-pong schedule instead of the interleaved one (waves 0-3: half the K-steps, the whole VALU phase, the other
// half; waves 4-7: VALU phase first), 128 (with 64) the waves 0-3 order for all waves.  Measured at M = 40960
// (profiles/r04_xw_ablate.jsonl): the ping-pong is 7-8 % slower than the interleaved schedule.
// HB: SWIGLU / GLU output in the blocked tile layout (common.h hblk_off): each 16-byte-per-lane store instruction
// writes 1 KiB contiguous (lane l's chunk at 16 l of the tile half) instead of 32-byte segments of 32 rows
template <int EPI, bool RS, int DBG = 0, bool HB = false>
__global__ void __launch_bounds__(kXwWaves * 64, 1) gemm_xw_kernel(GemmArgs p, int nc) {
  static_assert(EPI == EPI_SWIGLU || EPI == EPI_GLU || EPI == EPI_STORE, "SWIGLU / GLU / STORE");
  constexpr int kXwS = xw_stores<EPI>();
  __shared__ __attribute__((aligned(16))) uint8_t lds[kXwR * kXwTile + 4 * kBiasMax];
  float* sbias = reinterpret_cast<float*>(lds + kXwR * kXwTile);

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int nwt = p.N / kXwBN, ntm = (p.M + kXwBM - 1) / kXwBM, nch = (nwt + nc - 1) / nc;
  const int items = ntm * nch;
  const int nxb = gridDim.x >> 3, xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = (items + 7) >> 3, ibeg = xcd * q, iend = min(items, ibeg + q);
  if (ibeg + jb >= iend) return;                                  // workgroup-uniform

  for (int i = tid; i < p.N; i += kXwWaves * 64) sbias[i] = p.bias ? p.bias[i] : 0.f;
  __syncthreads();                                                // no DMA in flight yet

  const uint16_t* __restrict__ X = static_cast<const uint16_t*>(p.A);
  const uint8_t* __restrict__ Wb = static_cast<const uint8_t*>(p.W);
  uint16_t* __restrict__ Cout = static_cast<uint16_t*>(p.C);

  auto pos_of = [&](int item) {
    XwPos ps;
    ps.item = item;
    ps.j = 0;
    ps.mt = item / nch;
    const int ch = item - ps.mt * nch;
    ps.t0 = ch * nc;
    ps.n = min(nwt, ps.t0 + nc) - ps.t0;
    return ps;
  };
  auto advance = [&](XwPos& ps) {
    if (++ps.j == ps.n) ps = pos_of(ps.item + nxb);
  };
  int total = 0;
  for (int it = ibeg + jb; it < iend; it += nxb) total += pos_of(it).n;

  // DMA of W tile t into ring slot sl: wave w moves pieces 6 w .. 6 w + 5; lane i of piece pc lands at linear 16-byte
  // slot 64 pc + i of the tile = (row, slot) with 48 slots per row, fetching chunk slot ^ (row & 15) of that row
  uint32_t doff[kXwP];
#pragma unroll
  for (int i = 0; i < kXwP; ++i) {
    const int pc = wid * kXwP + i, lin = pc * 64 + lane, row = lin / 48, slot = lin % 48;
    doff[i] = (uint32_t)(row * kXwRowB + ((slot ^ (row & 15)) << 4));
  }
  auto dma_piece = [&](int t, int sl, int i) __attribute__((always_inline)) {
    const uint8_t* src = Wb + (int64_t)t * kXwTile;
    uint8_t* base = lds + sl * kXwTile + wid * kXwP * 1024;
    lds_dma16(src + doff[i], base + i * 1024);
  };
  auto dma = [&](int t, int sl) {
#pragma unroll
    for (int i = 0; i < kXwP; ++i) dma_piece(t, sl, i);
  };
  // A-operand reads: lane row c(lr) of the g block, the same of the u block 32 rows on; chunk 2 ks + lh
  const int ra = xw_perm(lr);
  const uint32_t roff = (uint32_t)(ra * kXwRowB), rsw = (uint32_t)(ra & 15);
  uint32_t soff[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) soff[k] = roff + ((((uint32_t)(2 * k + lh)) ^ rsw) << 4);

  xw_bf16x8 xf[kXwKS];
  auto xload = [&](const XwPos& ps) {
    const int64_t row = min(ps.mt * kXwBM + wid * 32 + lr, p.M - 1);
    const uint16_t* xr = X + row * p.lda + 8 * lh;
#pragma unroll
    for (int ks = 0; ks < kXwKS; ++ks) xf[ks] = *reinterpret_cast<const xw_bf16x8*>(xr + 16 * ks);
  };
  // the row's RMS (sqrt(mean x^2) + eps, the row factor's reciprocal)
  auto row_rms = [&]() {
    if constexpr (RS) {
      float ss = 0.f;
#pragma unroll
      for (int ks = 0; ks < kXwKS; ++ks) ss = sumsq8(xf[ks], ss);
      ss += __shfl_xor(ss, 32, 64);
      return sqrtf(ss) * p.inv_sqrt_k + kRmsEps;
    } else {
      return 1.0f;
    }
  };

  xw_f32x16 acc[2][2];       // [buffer][g, u]
  uint32_t po[8], pu[8];     // packed bf16 pairs of the epilogue in flight (pu: STORE's second half)
  // epilogue part k (registers 2k, 2k + 1) of the step held in buffer b: W tile t, output row mrow, row factor inv.
  // The accumulators start from bias x RMS (RS) or the bias, so acc x inv = A.W^T x inv + bias and the part reads
  // no LDS: a bias read here was the youngest LDS op at its use, i.e. an lgkmcnt(0) that also drained the W
  // fragment reads in flight
  auto epi_part = [&](int b, int t, int64_t mrow, int blk, float inv, float cz, float inv2, int k) __attribute__((always_inline)) {
    if constexpr (EPI == EPI_STORE) {
      // output columns 64 t + u, + 1 (rows 0-31 of the tile) and 64 t + 32 + u, + 1 (rows 32-63)
      float y[2], z[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        y[e] = RS ? acc[b][0][2 * k + e] * inv : acc[b][0][2 * k + e];
        z[e] = RS ? acc[b][1][2 * k + e] * inv : acc[b][1][2 * k + e];
      }
      po[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(xw_f32x2{y[0], y[1]}, xw_bf16x2));
      pu[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(xw_f32x2{z[0], z[1]}, xw_bf16x2));
      if ((k & 3) == 3) {   // 8 consecutive columns of each half: two 16-byte stores
        uint16_t* dst = Cout + mrow * p.ldc + kXwBN * t + 16 * (k >> 2) + 8 * lh;
        *reinterpret_cast<xw_u32x4*>(dst) = xw_u32x4{po[k - 3], po[k - 2], po[k - 1], po[k]};
        *reinterpret_cast<xw_u32x4*>(dst + 32) = xw_u32x4{pu[k - 3], pu[k - 2], pu[k - 1], pu[k]};
      }
    } else {
      float y[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {   // scalar fp32 (packed f32 VALU beside MFMAs costs more than two plain ops)
        // the row factor rides on the sigmoid's exp2 scale (cz = inv * -log2 e) and, for SwiGLU, on the product once
        // (inv2 = inv^2): g * sigmoid(g) * v = (acc_g acc_u inv^2) / (1 + exp2(acc_g cz)), one multiply per output
        // fewer than scaling g and v first
        const float ag = acc[b][0][2 * k + e], au = acc[b][1][2 * k + e];
        const float za = (EPI == EPI_SWIGLU ? ag : au) * (RS ? cz : -1.4426950408889634f);
        const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(za));
        y[e] = (EPI == EPI_SWIGLU) ? (RS ? (ag * au) * inv2 : ag * au) * sg : (RS ? ag * inv : ag) * sg;
      }
      po[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(xw_f32x2{y[0], y[1]}, xw_bf16x2));
      if ((k & 3) == 3) {   // registers 0-7 / 8-15 done: 8 consecutive hidden columns, one 16-byte store
        const xw_u32x4 w = {po[k - 3], po[k - 2], po[k - 1], po[k]};
        if constexpr ((DBG & 256) != 0) asm volatile("" ::"v"(w));   // no stores (timing only)
        else if constexpr (HB)   // tile (blk, t) of the 32-row block / 32 hidden columns, half k >> 2, lane-contiguous
          *reinterpret_cast<xw_u32x4*>(Cout + ((int64_t)blk * (p.ldc >> 5) + t) * 1024 + 512 * (k >> 2) + 8 * lane) = w;
        else *reinterpret_cast<xw_u32x4*>(Cout + mrow * p.ldc + 32 * t + 16 * (k >> 2) + 8 * lh) = w;
      }
    }
  };

  // ---- prologue: first item's X, ring steps 0 and 1 ------------------------------------------------------------
  // Every run has an even length (gemm_xw picks nc among the even divisors of N / 64), so a run's steps use the
  // accumulator buffers 0, 1, ..., 1: the run's first step (X wait, row factors) and last step (next X load) are
  // peeled, and the compiler sees the X loads pending only on the path into a first step -- one explicit wait
  // there, no wait on X anywhere else.
  XwPos cur = pos_of(ibeg + jb);
  XwPos ahead = cur;
  xload(cur);
  dma(cur.t0 + cur.j, 0);
  advance(ahead);
  if (total > 1) dma(ahead.t0 + ahead.j, 1);
  advance(ahead);                                                 // ahead = step 2
  int s = 0;
  float inv = 1.f, rms = 1.f;
  int64_t mrow = 0;
  int mblk = 0;                                                   // the wave's 32-row block (HB tile row)
  int pt = 0;                                                     // previous step's W tile, row, row factor
  int64_t prow = 0;
  int pblk = 0;
  float pinv = 1.f, pcz = -1.4426950408889634f, pinv2 = 1.f;   // previous step's row factor, inv * -log2 e, inv^2

  auto step = [&](auto Bc, auto Fc, auto Lc) __attribute__((always_inline)) {
    constexpr int b = decltype(Bc)::value;
    constexpr bool first = decltype(Fc)::value, last = decltype(Lc)::value;
    const int t = cur.t0 + cur.j;
    if constexpr (first) {
      // the run's X loads (issued last in the previous step, or in the prologue) are the youngest ops: vmcnt(0),
      // as a builtin so the compiler's own wait counters see it
      __builtin_amdgcn_s_waitcnt(0x0F70);                         // vmcnt(0) expcnt(7) lgkmcnt(15)
    } else {
      // ring slot s landed: step s's DMA went out one piece at a time during step s - 2 (every four K-steps, or
      // between the epilogue parts of the ping-pong's VALU phase), its last piece before that step's last epilogue
      // part; younger ops: that part's stores, step s - 1's pieces (tile s + 1) and its stores
      constexpr int kLate = kXwS / 2;
      const int younger = kLate * (s >= 3) + kXwP + kXwS * (s >= 2);
      if (younger == kLate + kXwP + kXwS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLate + kXwP + kXwS) : "memory");
      else vmcnt_dyn(younger);
    }
    barrier_lds();                                                // ... for every wave; slot (s + 2) % 3 free
    if constexpr (first) {
      rms = row_rms();
      inv = 1.0f / rms;
      mrow = min(cur.mt * kXwBM + wid * 32 + lr, p.M - 1);
      mblk = cur.mt * (kXwBM / 32) + wid;
    }
    // every step DMAs a tile (the last two of the workgroup re-fetch their own into the free slot): a conditional DMA
    // or epilogue part is a branch around an LDS op, and at each such join the compiler's wait counter fell back to
    // lgkmcnt(0) -- a full drain of the fragment reads -- before the next MFMA
    constexpr bool dma_next = !(DBG & 4);
    const int t2 = s + 2 < total ? ahead.t0 + ahead.j : t, sl2 = (s + 2) % kXwR;
    const uint8_t* base = lds + (s % kXwR) * kXwTile;
    {   // accumulators from the bias: register r of lane half h is hidden unit 16 (r >> 3) + 8 h + (r & 7)
      const float* bt = sbias + kXwBN * t + 8 * lh;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const xw_f32x4 b0 = *reinterpret_cast<const xw_f32x4*>(bt + 32 * i), b1 = *reinterpret_cast<const xw_f32x4*>(bt + 32 * i + 4);
        const xw_f32x4 b2 = *reinterpret_cast<const xw_f32x4*>(bt + 32 * i + 16), b3 = *reinterpret_cast<const xw_f32x4*>(bt + 32 * i + 20);
        acc[b][i] = xw_f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                              b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
        if constexpr (RS) acc[b][i] *= rms;
      }
    }
    // W fragments two K-steps ahead of the MFMAs that use them (three register sets)
    xw_bf16x8 wf[3][2];
    auto rdw = [&](int ks, xw_bf16x8(&w)[2]) __attribute__((always_inline)) {
      if constexpr ((DBG & 16) != 0) {
        w[0] = xf[ks];
        w[1] = xf[(ks + 1) % kXwKS];
      } else {
        // chunk 2 ks + lh at slot (2 ks + lh) ^ rsw: the XOR touches bits 0-3 only, so the slot is 16 (ks >> 3) plus
        // one of eight per-lane offsets -- eight address registers, the rest immediate offsets
        const uint8_t* a = base + soff[ks & 7] + 256 * (ks >> 3);
        w[0] = *reinterpret_cast<const xw_bf16x8*>(a);
        w[1] = *reinterpret_cast<const xw_bf16x8*>(a + 32 * kXwRowB);
      }
    };
    const bool epi = (!first || s > 0) && !(DBG & 1);   // compile-time true past a run's first step
    // K-steps k0 .. k1 - 1, fragments read two steps ahead within the range (none live across a VALU phase)
    auto mfmas = [&](int k0, int k1) __attribute__((always_inline)) {
      rdw(k0, wf[k0 % 3]);
      rdw(k0 + 1, wf[(k0 + 1) % 3]);
#pragma unroll
      for (int ks = k0; ks < k1; ++ks) {
        xw_bf16x8(&cw)[2] = wf[ks % 3];
        if (ks + 2 < k1) rdw(ks + 2, wf[(ks + 2) % 3]);
        if constexpr ((DBG & 2) != 0) {
          asm volatile("" ::"v"(cw[0]), "v"(cw[1]), "v"(xf[ks]));
        } else {
          acc[b][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cw[0], xf[ks], acc[b][0], 0, 0, 0);
          acc[b][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cw[1], xf[ks], acc[b][1], 0, 0, 0);
        }
        if constexpr ((DBG & 64) == 0) {   // interleaved schedule: DMA piece / epilogue part between the MFMAs
          if (dma_next && ks % 4 == 2) dma_piece(t2, sl2, ks / 4);
          if (epi && ks % 3 == 1) epi_part(b ^ 1, pt, prow, pblk, pinv, pcz, pinv2, ks / 3);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // the VALU phase: the previous step's epilogue (8 parts) with this step's 6 DMA pieces (tile s + 2) between them
    auto valu_phase = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (epi) epi_part(b ^ 1, pt, prow, pblk, pinv, pcz, pinv2, k);
        if (k < kXwP && dma_next) dma_piece(t2, sl2, k);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if constexpr ((DBG & 64) == 0) {
      mfmas(0, kXwKS);
    } else {
      // ping-pong between the two waves of a SIMD (waves w and w + 4): waves 0-3 run half the K-steps, then their VALU
      // phase, then the other half; waves 4-7 their VALU phase first -- so one wave's epilogue issues while its
      // partner's MFMAs hold the matrix pipe, instead of both waves interleaving VALU and MFMA at K-step grain
      if (wid < 4 || (DBG & 128)) {
        mfmas(0, kXwKS / 2);
        valu_phase();
        mfmas(kXwKS / 2, kXwKS);
      } else {
        valu_phase();
        mfmas(0, kXwKS);
      }
    }
    pt = t;
    prow = mrow;
    pblk = mblk;
    pinv = inv;
    pcz = inv * -1.4426950408889634f;
    pinv2 = inv * inv;
    advance(cur);
    advance(ahead);
    ++s;
    if constexpr (last) {
      if (s < total) xload(cur);                                  // next run's X into the registers just freed
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T = std::true_type;
  using F = std::false_type;
  for (int it = ibeg + jb; it < iend; it += nxb) {                // cur is at (it, 0)
    const int n = cur.n;
    step(I0{}, T{}, F{});
    for (int j = 1; j < n - 1; j += 2) {
      step(I1{}, F{}, F{});
      step(I0{}, F{}, F{});
    }
    step(I1{}, F{}, T{});
  }
  // the last step's epilogue (buffer 1: runs have even lengths)
#pragma unroll
  for (int k = 0; k < 8; ++k) epi_part(1, pt, prow, pblk, pinv, pcz, pinv2, k);
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the re-fetch DMAs landed before the workgroup's LDS is released
}

// W tiles per work item: among the even divisors of the W tile count (runs of even length), the one minimising
// rounds x (run + 1.5), 1.5 tiles being the per-item X load and ring refill that the pipeline does not hide
inline int xw_run_length(int x_blocks, int w_tiles, int cus = 256) {
  int best = 0;
  double best_cost = 1e30;
  for (int c = 2; c <= w_tiles; c += 2) {
    if (w_tiles % c) continue;
    const int64_t items = (int64_t)x_blocks * (w_tiles / c);
    const double cost = (double)((items + cus - 1) / cus) * (c + 1.5);
    if (cost < best_cost) { best_cost = cost; best = c; }
  }
  return best;
}

template <int EPI>
hipError_t launch_xw(const GemmArgs& a, int nc, hipStream_t st) {
  const int items = ((a.M + kXwBM - 1) / kXwBM) * ((a.N / kXwBN + nc - 1) / nc);
  int grid = 256;
  const int need = (items + 7) / 8 * 8;
  if (grid > need) grid = need;
#ifdef XW_ABLATE
  if constexpr (EPI == EPI_SWIGLU) {
    switch (a.rowscale ? a.dbg : 0) {
#define XW_D(d) case d: hipLaunchKernelGGL((gemm_xw_kernel<EPI, true, d>), dim3(grid), dim3(kXwWaves * 64), 0, st, a, nc); return hipGetLastError();
      XW_D(1) XW_D(2) XW_D(3) XW_D(4) XW_D(16) XW_D(19) XW_D(64) XW_D(192) XW_D(256) XW_D(258)
#undef XW_D
      default: break;
    }
  }
#endif
  if constexpr (EPI == EPI_SWIGLU) {
    if (a.h_blocked) {
      if (a.rowscale) hipLaunchKernelGGL((gemm_xw_kernel<EPI, true, 0, true>), dim3(grid), dim3(kXwWaves * 64), 0, st, a, nc);
      else hipLaunchKernelGGL((gemm_xw_kernel<EPI, false, 0, true>), dim3(grid), dim3(kXwWaves * 64), 0, st, a, nc);
      return hipGetLastError();
    }
  }
  if (a.rowscale) hipLaunchKernelGGL((gemm_xw_kernel<EPI, true>), dim3(grid), dim3(kXwWaves * 64), 0, st, a, nc);
  else hipLaunchKernelGGL((gemm_xw_kernel<EPI, false>), dim3(grid), dim3(kXwWaves * 64), 0, st, a, nc);
  return hipGetLastError();
}

}  // namespace

// nc = W tiles per work item, an even divisor of N / 64 (0: xw_run_length); SWIGLU / GLU / STORE with bf16 output only
hipError_t gemm_xw(const GemmArgs& a, int epi, int nc, hipStream_t st) {
  if (!a.a_bf16 || !a.c_bf16 || a.K != kXwK || a.N % kXwBN || a.N > kBiasMax || a.M <= 0 || a.rpg || a.lda % 8 ||
      a.ldc % 8 || a.k_split || a.C2)
    return hipErrorInvalidValue;
  // the blocked hidden: SwiGLU only, whole 32-column tiles per row block (the caller pads the rows to 32)
  if (a.h_blocked && (epi != EPI_SWIGLU || a.ldc % 32 || a.ldc < a.N / 2)) return hipErrorInvalidValue;
  const int nwt = a.N / kXwBN, ntm = (a.M + kXwBM - 1) / kXwBM;
  if (nc <= 0) nc = xw_run_length(ntm, nwt);
  if (nc < 2 || nc % 2 || nwt % nc) return hipErrorInvalidValue;   // runs of even length (see the kernel)
  switch (epi) {
    case EPI_SWIGLU: return launch_xw<EPI_SWIGLU>(a, nc, st);
    case EPI_GLU: return launch_xw<EPI_GLU>(a, nc, st);
    case EPI_STORE: return launch_xw<EPI_STORE>(a, nc, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tone
