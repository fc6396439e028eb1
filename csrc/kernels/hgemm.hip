// Persistent dense bf16 GEMM for gfx950 (the transformer Linear path: GPT-2
// projections / MLP / LM head, fwd "NT", dgrad "NN", wgrad "TN").
//
// Replaces ATen addmm/mm (hipBLASLt) behind the reference's nn.Linear
// (/root/reference/train.py:39,42,45).  Design, MI355X-first:
//
//  * one workgroup per CU (two for the 128x128 tile) walks a list of work
//    units (output tile x K-split); tile order is XCD-aware (consecutive
//    logical units run on one XCD and share A rows / B columns in its L2);
//  * main loop = LDS-DMA (global_load_lds_dwordx4) into "half images" with a
//    4-phase-per-K-tile schedule: each phase ds_reads one accumulator
//    quadrant's fragments, restages one half image two phases after its last
//    read, and runs that quadrant's MFMA cluster (16x16x32 bf16) between raw
//    s_barriers under s_setprio(1); one counted vmcnt per K-tile keeps the two
//    newest half-images in flight across the barrier; the second half of the
//    waves runs one barrier behind (ping-pong: one wave per SIMD in MFMA while
//    its partner issues reads/DMA) -- cdna_hip_programming.md §5 T1-T5;
//  * epilogue straight from the accumulators (no LDS): its math runs first,
//    then the NEXT unit's prologue DMA is issued, then the stores -- the store
//    drain overlaps the next tile's first loads instead of serialising;
//  * fused epilogues: bias, GELU with the pre-activation kept (aux_out),
//    GELU-backward multiply (aux_in), fp32 residual add, fp32 accumulate into
//    gradient buckets, fp32 K-split partial slabs (+ hgemm_finalize).
//
// Layout conventions (D^T issue: every lane holds 4 consecutive output columns):
//   A: K-contiguous A[m][k] or M-contiguous A[k][m];  B: K-contiguous B[n][k] or N-contiguous B[k][n]
//   fwd   y = x w^T   : A K, B K      dgrad dx = dy w : A K, B N      wgrad dw = dy^T x : A M, B N
//
// Half images: the wave grid is WR x WC; wave (wr, wc) owns tile rows
// wr*(BM/WR) + [0, BM/WR) and columns wc*(BN/WC) + [0, BN/WC), each split in
// two halves (RH rows / CH columns).  A half image h holds rows
// {wr*(BM/WR) + h*RH + [0,RH)} of every wr, B half h columns {wc*(BN/WC) +
// h*CH + [0,CH)} of every wc, so one phase-quadrant of every wave reads exactly
// one A half and one B half.  K images are [rows][64 k] (128-B rows, chunk ^=
// (row>>1)&7); M/N-contiguous images are [64 k][128] (256-B rows, read with
// ds_read_b64_tr_b16).  LDS-DMA writes lane-linearly, so the swizzle is applied
// to the per-lane SOURCE address and undone on the read.
#include "common.h"
#include "igemm.h"
#include "hgemm.h"

namespace dpe {
namespace hg {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int TK = 64;

// Main-loop schedule: 1 (default) = reads retired before each phase's first barrier, restage one
// phase after the last read, three half images in flight across the per-K-tile wait;
// 0 = round-1 gemm256 schedule (restage two phases after, two half images in flight).
#ifndef HG_SCHED
#define HG_SCHED 1
#endif
#define HG_SCHED_LINE 256  // words between two dynamic-schedule counters (hgemm.h HGEMM_SCHED_BYTES)

template <int BM, int BN, int WR, int WC>
struct Geo {
  static constexpr int NW = WR * WC, NT = NW * 64;
  static constexpr int RH = BM / WR / 2, CH = BN / WC / 2;  // rows / columns per wave per half
  static constexpr int FMH = RH / 16, FNH = CH / 16;        // 16x16 fragments per wave per half
  static constexpr int AHB = BM * 64, BHB = BN * 64;        // bytes per half image (dim/2 x 64 k x 2 B)
  static constexpr int GA = AHB / 1024 / NW, GB = BHB / 1024 / NW;  // 1-KiB DMA pieces per wave per half
  static constexpr int B_REGION = 4 * AHB;
  static constexpr int LDS = 4 * (AHB + BHB);
  static constexpr int NKEEP = GA + GB;  // DMA instructions left in flight by the per-K-tile wait
  static_assert(GA >= 1 && GB >= 1 && GA * NW * 1024 == AHB && GB * NW * 1024 == BHB, "piece split");
  static_assert(FMH >= 1 && FNH >= 1, "fragments");
};

DPE_DEVICE int kswz(int row) { return (row >> 1) & 7; }
DPE_DEVICE int mnswz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// half-image index -> tile row / column
template <int D, int W, int HH>
DPE_DEVICE int hmap(int h, int r) { return (r / HH) * (D / W) + h * HH + (r % HH); }

template <int N>
DPE_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
  asm volatile("" ::: "memory");
}

// LDS-DMA of one 16-B chunk per lane to dst + 16 * lane (dst wave-uniform).  Issued through inline
// asm on purpose: after a compiler-visible LDS-DMA, hipcc (ROCm 7.2) puts s_waitcnt vmcnt(0) in
// front of every ds_read_b64_tr_b16 (not of ds_read_b128) -- in the M- / N-contiguous layouts that
// drained the whole prefetch pipeline four times per K-tile (TN ran at 885 TF vs NT 1334,
// scripts/gpu_pmc_hgemm.sh: equal LDS-array cycles, 2.3x the LDS-wait).  The kernel's own counted
// wait_vm<N> calls are what order the DMA against the LDS reads; a VMEM op the compiler does not
// see can only make its own vmcnt waits stricter, never wrong.  No other code in these kernels
// uses M0.
DPE_DEVICE void glds(const char* src, char* dst) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}

// LDS-DMA of one 16-B chunk per lane through a buffer resource (voffset past num_records -> zeros: the
// implicit-im2col padding), same inline-asm reasoning as glds
DPE_DEVICE void bdma16(__amdgpu_buffer_rsrc_t r, char* dst, uint32_t voff, uint32_t soff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(m0), "v"(voff), "s"(r), "s"(soff) : "memory");
}

// K-image fragment read, rows r0 + [0,16), k-step s
DPE_DEVICE int kread_off(int r0, int s) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15), ch = s * 4 + (lane >> 4);
  return row * 128 + ((ch ^ kswz(row)) << 4);
}
// MN-image fragment read, columns c0 + [0,16), k-step 0 (k-step 1 = +8192)
DPE_DEVICE int mnread_off(int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k1 = 8 * g + q;
  const int mc = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 8;
  return k1 * 256 + ((mc ^ mnswz(k1)) << 4) + sub;
}
DPE_DEVICE bf16x8 lds_b128(const char* a) { return __builtin_bit_cast(bf16x8, *(const u32x4*)a); }
DPE_DEVICE bf16x8 lds_tr(const char* a) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 1024));  // rows k1 + 4
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

// per-lane LDS-DMA source offsets (bytes, 32-bit) of one operand's two half images
template <int D, int W, int HH, int NG, bool KC>
DPE_DEVICE void stage_setup(int64_t ld, int dim, int d0, int kb, uint32_t (&g)[2][NG]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int pc = wid * NG + i;  // this lane's 1-KiB piece of the half image
      if constexpr (KC) {
        const int r = 8 * pc + (lane >> 3);
        const int gr = min(d0 + hmap<D, W, HH>(h, r), dim - 1);
        const int ch = (lane & 7) ^ kswz(r);
        g[h][i] = (uint32_t)(((int64_t)gr * ld + kb + ch * 8) * 2);
      } else {
        const int k = 4 * pc + (lane >> 4);
        const int c = (lane & 15) ^ mnswz(k);
        const int gc = min(d0 + hmap<D, W, HH>(h, c * 8), dim - 8);
        g[h][i] = (uint32_t)(((int64_t)(kb + k) * ld + gc) * 2);
      }
    }
}

#define HG_BARRIER()                   \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_s_barrier();      \
    asm volatile("" ::: "memory");     \
  } while (0)

DPE_DEVICE float gelu_fwd(float x) {
  // 0.5 x (1 + tanh(u)) == x / (1 + exp(-2u)),  u = sqrt(2/pi) (x + 0.044715 x^3)
  const float u2 = -1.5957691216057308f * (x + 0.044715f * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(u2));
}
DPE_DEVICE float gelu_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // tanh(u) = 1 - 2 / (1 + exp(2u)) (exp overflow -> t = 1, underflow -> t = -1)
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * k0 * (x + k1 * x * x * x)));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
}

// BG (TN weight grads, A = dy^T M-contiguous): the same launch also produces the bias gradient
// db[m] += alpha * sum_k A[k][m] -- the units of the first tile column sum the A fragments they
// already hold in registers (wave wc takes fragment row-block wc, v_dot2 with ones: 8 VALU per half
// image per K-tile), so dy is not streamed a second time by a column-sum kernel.
// AC: A is the implicit im2col of an NHWC conv input (HgemmArgs::conv; K-contiguous A): the A half images
// are staged by buffer_load ... lds with per-row tap-validity masks (padding reads as zeros) and the
// K-tile's filter-tap offset in soffset -- the forward-form 3x3 convolutions on this kernel's schedule.
// CV = 2 (BC): B is the implicit im2col of an NHWC conv input in the TN weight-grad layout (B[k][n], k = output
// pixel, n = (r, s, ci); N-contiguous): every lane's 16-B chunk is one (tap, 8 channels) column for the whole
// unit, and its pixel row is decomposed per K-tile (padding and the pixel tail read as zeros).
template <int BM, int BN, int WR, int WC, bool AK, bool BK, int EPI, int ACT, bool BG = false, int CV = 0,
          bool SKM = false>
// (4-wave tiles run 2 blocks per CU: 2 waves per SIMD, so at most 256 VGPRs + AGPRs per wave)
__global__ __launch_bounds__(WR * WC * 64, WR * WC == 4 ? 2 : 1) void hgemm_kernel(HgemmArgs p) {
  constexpr bool AC = CV == 1, BC = CV == 2, ACAT = CV == 3;
  using G = Geo<BM, BN, WR, WC>;
  constexpr int NW = G::NW, RH = G::RH, CH = G::CH, FMH = G::FMH, FNH = G::FNH, GA = G::GA, GB = G::GB;
  constexpr int AHB = G::AHB, BHB = G::BHB;
  static_assert(AK || BM == 256, "M-contiguous A needs 128-column half images (BM = 256)");
  static_assert(BK || BN == 256, "N-contiguous B needs 128-column half images (BN = 256)");
  // + 16 B: the next-unit slot of the dynamic schedule (in the one LDS array: a second __shared__
  // object can make the compiler drain vmcnt before the main loop's ds_reads)
  __shared__ __attribute__((aligned(16))) char smem[G::LDS + 16];

  // Grouped launch (HE_GROUP): several TN weight-grad problems share one persistent grid; decode()
  // switches these per unit.  Otherwise they are the launch's single problem.
  constexpr bool GRP = EPI == HE_GROUP;
  const void* qA = p.A;
  const void* qB = p.B;
  void* qC = p.C;
  float* qdbias = p.dbias;
  int qM = p.M, qN = p.N, qadim = p.a_dim, qover = 0;
  int64_t qlda = p.lda, qldb = p.ldb, qldc = p.ldc;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WC, wc = wid % WC;
  const bool late = NW == 8 && wid >= 4;  // second-dispatched half runs one barrier behind
  int tilesM = (qM + BM - 1) / BM, tilesN = (qN + BN - 1) / BN;
  int ntile = tilesM * tilesN;
  const int nunits = GRP ? p.grp[p.ngroup - 1].tile_end : ntile * p.splits;
  static_assert(!SKM || (NW == 8 && !GRP && !BG && EPI == HE_BF16), "stream-K: 1-block-per-CU tiles, bf16 epilogues");
  const float alpha = p.alpha * (p.alpha_ptr ? *p.alpha_ptr : 1.f);

  // Schedule.  Without p.sched (or with one round of units) block b computes units
  // xcd_remap(b), +grid, +2 grid, ...  With p.sched and more units than blocks, the leading 7/8 of
  // the grid start on static units (no claim latency at launch) and every other unit is claimed at
  // run time from 8 per-XCD queues (umap below), stealing from the other queues when its own is
  // empty.  So a block whose CU is shared with foreign work (RCCL channel blocks, another
  // stream's kernel) computes fewer units, and the grid's tail -- the blocks the dispatcher cannot
  // place while foreign workgroups hold slots -- holds no unit hostage: by the time it is placed the
  // queues are usually drained and it exits at once.  The claim for a block's next unit is issued
  // during the current unit's third-to-last K-tile and consumed after its main loop, so its latency
  // overlaps MFMA work.  No unit depends on which block computes it (no cross-unit reduction): outputs are
  // bitwise independent of the schedule.
  const int G0 = gridDim.x;
#if HG_SCHED == 1
  const bool dsched = !SKM && p.sched != nullptr && nunits > G0;
#else
  // only the HG_SCHED == 1 main loop issues the next-unit claim: any other build runs the static
  // schedule (a dynamic one would re-resolve the same unit forever)
  const bool dsched = false;
#endif
  const int S = dsched ? (G0 - G0 / 8) & ~7 : G0;  // blocks [0, S) start on a static unit
  const int dyn = dsched ? nunits - S : 0;         // units [S, nunits) are claimed
  const int xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;  // hwreg(HW_REG_XCC_ID, 0, 4)
  // counters, each on a 1 KB line of its own (HG_SCHED_LINE words apart): [0, 8) claim queues,
  // [8, 16) exit counts per block group b % 8, 16 the groups done.  (Packed in one cache line, all
  // claims of the chip serialise on one memory-side atomic unit.)
  auto ctr = [&](int k) { return p.sched + k * HG_SCHED_LINE; };
  // queue q's j-th ticket: chunk (j / CK) * 8 + q of CK = grid/8 consecutive claimed units -- XCD q
  // takes the q-th eighth of every grid-sized stretch of the grouped unit order, as under the static
  // round-robin (its blocks in flight share A rows / B columns in its L2)
  const unsigned CK = (unsigned)max(1, G0 >> 3);
  auto umap = [&](int q, unsigned j) -> int64_t { return S + ((int64_t)(j / CK) * 8 + q) * CK + (j % CK); };
  int claim_v = 0;  // wave 0 lane 0: the in-flight fetch_add of its own queue
  const int claimer = dyn > 0 && wid == 0 && lane == 0;
  int* const slot = (int*)(smem + G::LDS);
  // wave 0: the unit for own-queue ticket c0, else one stolen from another queue, else -1
  auto resolve = [&](int c0) -> int {
    if (umap(xcc, (unsigned)c0) < nunits) return (int)umap(xcc, (unsigned)c0);
    // (the opaque copy keeps the lane-dependent values below from being hoisted out of the unit
    // loop, where they would stay live -- and spill -- across every unit's main loop)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    while (true) {  // each pass either claims or sees every queue drained
      const int q = (xcc + ln) & 7;
      unsigned c = 0xffffffffu;
      if (ln < 8) c = __hip_atomic_load(ctr(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t has = __ballot(ln < 8 && umap(q, c) < nunits);
      if (!has) return -1;
      const int pick = (xcc + (int)__builtin_ctzll(has)) & 7;
      int w = 0;
      if (ln == 0) w = (int)__hip_atomic_fetch_add(ctr(pick), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w = __builtin_amdgcn_readfirstlane(w);
      if (umap(pick, (unsigned)w) < nunits) return (int)umap(pick, (unsigned)w);
    }
  };
  // the last block out resets every counter for the next launch on this stream (every block's final,
  // failed claim precedes its exit count, so no claim can follow the reset).  Exits are counted per
  // block group b % 8 (sizes known exactly, whatever the placement), then per group.
  auto sched_exit = [&]() {
    if (dyn > 0 && wid == 0 && lane == 0) {
      const int g = blockIdx.x & 7;
      const unsigned in_g = (unsigned)(G0 - g + 7) / 8u;
      if (__hip_atomic_fetch_add(ctr(8 + g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_g - 1u &&
          __hip_atomic_fetch_add(ctr(16), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)min(G0, 8) - 1u)
        for (int k = 0; k <= 16; ++k) __hip_atomic_store(ctr(k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  // Stream-K (SKM, hgemm.h): block lb (XCD-remapped) owns K-steps [lo(lb), lo(lb + 1)) of the tiles'
  // concatenated K-step sequence (ntk steps per tile, tile order = unit order): the first r blocks q + 1
  // steps, the rest q (32-bit: tiles x ntk < 2^31).  A segment is a block's part of one tile: unit u = its
  // tile, kb its first K.  A range that ends inside a tile it did not start in runs that last segment
  // FIRST (its partial is handed off early, while the other blocks still compute), then the rest in
  // order.  Nothing of this is kept live across the main loop (the epilogue recomputes it from u, kb and
  // the grid): the 256x256 tile has no SGPRs or VGPRs to spare.
  const int ntk = p.K / TK;
  int sk_kb0 = 0, sk_nt0 = 0;
  struct SkGrid {
    unsigned q, r, lb, nk;
    DPE_DEVICE unsigned lo(unsigned b) const { return b * q + min(b, r); }
    DPE_DEVICE unsigned blk(unsigned st) const {  // the block whose range holds K-step st
      const unsigned big = r * (q + 1u);
      return __builtin_amdgcn_readfirstlane(st < big ? st / (q + 1u) : r + (st - big) / q);
    }
    // first step of the tile holding block b's last step, if b runs that tile's segment first; else ~0u
    DPE_DEVICE unsigned lead(unsigned b) const {
      const unsigned l = lo(b), h = lo(b + 1u);
      const unsigned tb = __builtin_amdgcn_readfirstlane((h - 1u) / nk) * nk;
      return (tb > l && h != tb + nk) ? tb : ~0u;
    }
    // block b's segment of the tile starting at step t0: steps from b's start until it is done
    DPE_DEVICE unsigned done_at(unsigned b, unsigned t0) const {
      const unsigned l = lo(b), h = lo(b + 1u), tb = lead(b);
      const unsigned e = min(h, t0 + nk);
      return tb == ~0u ? e - l : (t0 == tb ? h - tb : (h - tb) + (e - l));
    }
  };
  auto sk_grid = [&]() -> SkGrid {
    unsigned g = (unsigned)G0;
    asm volatile("" : "+s"(g));  // recomputed where used, not hoisted out of the unit loop
    const unsigned total = (unsigned)ntile * (unsigned)ntk;
    const unsigned q = __builtin_amdgcn_readfirstlane(total / g);
    return SkGrid{q, total - q * g, (unsigned)xcd_remap(blockIdx.x, (int)g), (unsigned)ntk};
  };
  // the segment of K-steps [cur, bound): its tile (returned) and kb / nt
  auto sk_seg = [&](unsigned cur, unsigned bound) -> int {
    const int t = __builtin_amdgcn_readfirstlane((int)(cur / (unsigned)ntk));
    const unsigned t0 = (unsigned)t * (unsigned)ntk;
    sk_kb0 = (int)(cur - t0) * TK;
    sk_nt0 = (int)(min(t0 + (unsigned)ntk, bound) - cur);
    return t;
  };

  int u;
  if constexpr (SKM) {
    const SkGrid sg = sk_grid();
    const unsigned lo = sg.lo(sg.lb), hi = sg.lo(sg.lb + 1u), tb = sg.lead(sg.lb);
    if (lo >= hi) return;
    u = tb != ~0u ? sk_seg(tb, hi) : sk_seg(lo, hi);
  } else if ((int)blockIdx.x < S) {
    u = xcd_remap(blockIdx.x, S);
    if (u >= nunits) return;  // (the planner's grid never exceeds the unit count)
  } else {
    if (wid == 0) {
      int c0 = 0;
      if (lane == 0) c0 = (int)__hip_atomic_fetch_add(ctr(xcc), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int nx = resolve(__builtin_amdgcn_readfirstlane(c0));
      if (lane == 0) *slot = nx;
    }
    __syncthreads();
    u = __builtin_amdgcn_readfirstlane(*slot);
    __syncthreads();  // the slot is rewritten before this unit's epilogue
    if (u < 0) {
      sched_exit();
      return;
    }
  }

  const char* Ab = (const char*)qA;
  const char* Bb = (const char*)qB;
  int64_t astep = AK ? (int64_t)TK * 2 : (int64_t)TK * qlda * 2;
  int64_t bstep = BK ? (int64_t)TK * 2 : (int64_t)TK * qldb * 2;
  char* const wdA = smem + wid * GA * 1024;             // this wave's pieces in every A half image
  char* const wdB = smem + G::B_REGION + wid * GB * 1024;

  // fragment-read lane offsets
  int ra[FMH][2], rb[FNH][2];
#pragma unroll
  for (int i = 0; i < FMH; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) ra[i][s] = AK ? kread_off(wr * RH + i * 16, s) : mnread_off(wr * RH + i * 16) + s * 8192;
#pragma unroll
  for (int j = 0; j < FNH; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      rb[j][s] = G::B_REGION + (BK ? kread_off(wc * CH + j * 16, s) : mnread_off(wc * CH + j * 16) + s * 8192);

  uint32_t ga[2][GA], gb[2][GB];
  uint32_t gam[2][AC ? GA : 1];  // AC: per-row tap-validity masks of the A pieces
  uint32_t ga2[2][ACAT ? GA : 1];  // ACAT: the A pieces' offsets in the second segment (lda2)
  uint32_t gbt[2][BC ? GB : 1];  // BC: per-column tap displacement (r dh - ph, s dw - pw) as two int16
  static_assert(!AC || AK, "implicit-im2col A is K-contiguous");
  static_assert(!BC || (!AK && !BK && !GRP), "implicit-im2col B: the TN weight-grad layout");
  const ConvGeom& cg = p.conv_g;
  // (the conv resource is built for every instantiation -- unused without CV -- as it has no null value)
  const int64_t apre = CV ? ((int64_t)cg.ph * cg.W + cg.pw) * cg.C : 0;  // every in-range tap offset >= 0
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>((const void*)((const uint16_t*)(BC ? p.B : p.A) - apre)), (short)0,
      CV ? (int)((((int64_t)cg.N * cg.H * cg.W * cg.C) + apre) * 2) : 0, 0x00020000);
  const int cshift = CV ? 31 - __builtin_clz(cg.C) : 0;
  const float inv_ow = BC ? 1.f / (float)cg.OW : 0.f, inv_hw = BC ? 1.f / (float)(cg.OH * cg.OW) : 0.f;
  // BC: each B half stages the unit's K-tiles in order (half 0: 0, 1, 2, ..; half 1: 0, 1, 2, ..), so the
  // output pixel of a lane's piece is a cursor advanced by TK pixels per staging instead of decoded from
  // scratch (two float-reciprocal divisions with corrections): bq = the pixel's input offset
  // (img H + oh sh) W + ow sw, bohw = oh << 16 | ow.  Per-TK-step increments (wave-uniform):
  const int bc_dow = BC ? TK % cg.OW : 0, bc_doh = BC ? (TK / cg.OW) % cg.OH : 0,
            bc_dimg = BC ? (TK / cg.OW) / cg.OH : 0;
  const int bc_dq = BC ? bc_dow * cg.sw + bc_doh * cg.sh * cg.W + bc_dimg * cg.H * cg.W : 0;
  const int bc_cw = BC ? cg.sh * cg.W - cg.OW * cg.sw : 0;        // ow wrapped: oh + 1
  const int bc_ch = BC ? cg.H * cg.W - cg.OH * cg.sh * cg.W : 0;  // oh wrapped: img + 1
  uint32_t bq[2][BC ? GB : 1], bohw[2][BC ? GB : 1];
  int m0, n0, kb, nt, split;
  // Grouped tile order: consecutive unit ids (which run together on one XCD -- xcd_remap) walk
  // GROUP_M tile rows before moving one tile column, so an XCD's concurrent tiles form a
  // GROUP_M x (chunk / GROUP_M) block sharing A rows AND B columns in its L2 (row-major order
  // shares only A: L2 hit rate 50 % on 8192^3, measured -- profiles/hgemm_pmc_r2.txt in git history).
  const int gm_rows = p.group_m > 0 ? p.group_m : 1;
  auto decode = [&](int uu) {
    int tile;
    if constexpr (GRP) {
      int g = 0;  // (wave-uniform: a few scalar compares)
      while (g + 1 < p.ngroup && uu >= p.grp[g].tile_end) ++g;
      const HgemmProblem& q = p.grp[g];
      qA = q.A; qB = q.B; qC = q.C; qdbias = q.dbias;
      qM = q.M; qN = q.N; qadim = q.a_dim; qover = q.overwrite;
      qlda = q.lda; qldb = q.ldb; qldc = q.ldc;
      Ab = (const char*)qA;
      Bb = (const char*)qB;
      tilesM = (qM + BM - 1) / BM;
      tilesN = (qN + BN - 1) / BN;
      ntile = tilesM * tilesN;
      tile = uu - (g > 0 ? p.grp[g - 1].tile_end : 0);
      split = 0;
    } else if constexpr (SKM) {
      tile = uu;
      split = 0;
    } else {
      tile = uu % ntile;
      split = uu / ntile;
    }
    const int gsz = gm_rows * tilesN;
    const int g0 = (tile / gsz) * gm_rows;
    const int grows = min(tilesM - g0, gm_rows);
    const int in = tile % gsz;
    m0 = (g0 + in % grows) * BM;
    n0 = (in / grows) * BN;
    kb = SKM ? sk_kb0 : split * p.kps;
    nt = SKM ? sk_nt0 : (min(p.K, kb + p.kps) - kb) / TK;
    if constexpr (AC) {
      // per A piece row: the input pixel of output row m (byte offset from the resource base) and the
      // filter taps that stay inside the image
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          const int r = 8 * (wid * GA + i) + (lane >> 3);
          const int m = m0 + hmap<BM, WR, RH>(h, r);
          const int ch = (lane & 7) ^ kswz(r);
          uint32_t off = 0u, mask = 0u;
          if (m < qM) {
            const int ow = m % cg.OW, t = m / cg.OW, oh = t % cg.OH, n = t / cg.OH;
            const int ih0 = oh * cg.sh - cg.ph, iw0 = ow * cg.sw - cg.pw;
            off = (uint32_t)((((int64_t)n * cg.H + oh * cg.sh) * cg.W + ow * cg.sw) * cg.C * 2) + ch * 16u;
            for (int rr = 0; rr < cg.R; ++rr) {
              const bool vr = (unsigned)(ih0 + rr * cg.dh) < (unsigned)cg.H;
              for (int ss = 0; ss < cg.S; ++ss)
                if (vr && (unsigned)(iw0 + ss * cg.dw) < (unsigned)cg.W) mask |= 1u << (rr * cg.S + ss);
            }
          }
          ga[h][i] = off;
          gam[h][i] = mask;
        }
    } else {
      stage_setup<BM, WR, RH, GA, AK>(qlda, qadim > 0 ? qadim : qM, m0, AK ? kb : 0, ga);
      if constexpr (ACAT) stage_setup<BM, WR, RH, GA, true>(p.lda2, qM, m0, 0, ga2);
    }
    if constexpr (BC) {
      // per B piece column chunk: its filter tap's byte offset + channel, and the tap's displacement
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const int k = 4 * (wid * GB + i) + (lane >> 4);
          const int c = (lane & 15) ^ mnswz(k);
          const int gc = n0 + hmap<BN, WC, CH>(h, c * 8);
          uint32_t off = 0u, disp = 0x80008000u;  // invalid column: displacement never in range
          if (gc < qN) {
            const int tap = gc >> cshift, ci = gc & (cg.C - 1);
            const int r = (tap * p.conv_smagic) >> 16, s = tap - r * cg.S;
            off = (uint32_t)(((r * cg.dh * cg.W + s * cg.dw) << cshift) + ci) * 2u;
            disp = ((uint32_t)(r * cg.dh - cg.ph) << 16) | ((uint32_t)(s * cg.dw - cg.pw) & 0xffffu);
          }
          gb[h][i] = off;
          gbt[h][i] = disp;
        }
      // the pixel cursors at K-tile 0 of this unit (same for both halves: the pixel depends on the lane's
      // row of the piece, not on the column half)
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int px = kb + 4 * (wid * GB + i) + (lane >> 4);
        int img = (int)((float)px * inv_hw);
        img -= img * cg.OH * cg.OW > px;
        img += (img + 1) * cg.OH * cg.OW <= px;
        const int rem = px - img * cg.OH * cg.OW;
        int oh = (int)((float)rem * inv_ow);
        oh -= oh * cg.OW > rem;
        oh += (oh + 1) * cg.OW <= rem;
        const int ow = rem - oh * cg.OW;
        const uint32_t q = (uint32_t)((img * cg.H + oh * cg.sh) * cg.W + ow * cg.sw);
        bq[0][i] = bq[1][i] = q;
        bohw[0][i] = bohw[1][i] = ((uint32_t)oh << 16) | (uint32_t)ow;
      }
    } else {
      stage_setup<BN, WC, CH, GB, BK>(qldb, p.b_dim > 0 ? p.b_dim : qN, n0, BK ? kb : 0, gb);
    }
    if constexpr (GRP) {
      astep = AK ? (int64_t)TK * 2 : (int64_t)TK * qlda * 2;
      bstep = BK ? (int64_t)TK * 2 : (int64_t)TK * qldb * 2;
    }
    if constexpr (!AK) { for (int h = 0; h < 2; ++h) for (int i = 0; i < GA; ++i) ga[h][i] += (uint32_t)((int64_t)kb * qlda * 2); }
    if constexpr (!BK && !BC) { for (int h = 0; h < 2; ++h) for (int i = 0; i < GB; ++i) gb[h][i] += (uint32_t)((int64_t)kb * qldb * 2); }
  };

#define STAGE_A(h, buf, t)                                                                   \
  do {                                                                                       \
    if constexpr (AC) {                                                                      \
      const int k0_ = kb + (t) * TK, tap_ = k0_ >> cshift;                                   \
      const int r_ = (tap_ * p.conv_smagic) >> 16, s_ = tap_ - r_ * cg.S;                    \
      const uint32_t so_ = (uint32_t)(((r_ * cg.dh * cg.W + s_ * cg.dw) << cshift) + (k0_ & (cg.C - 1))) * 2u; \
      _Pragma("unroll") for (int i_ = 0; i_ < GA; ++i_)                                      \
        bdma16(arsrc, wdA + ((buf) * 2 + (h)) * AHB + i_ * 1024,                             \
               ((gam[h][i_] >> tap_) & 1u) ? ga[h][i_] : 0x80000000u, so_);                  \
    } else if constexpr (ACAT) {                                                             \
      const int k0_ = (t) * TK;                                                              \
      if (k0_ < p.k1) {                                                                      \
        const char* b_ = Ab + (int64_t)k0_ * 2;                                              \
        _Pragma("unroll") for (int i_ = 0; i_ < GA; ++i_)                                    \
          glds(b_ + ga[h][i_], wdA + ((buf) * 2 + (h)) * AHB + i_ * 1024);                   \
      } else {                                                                               \
        const char* b_ = (const char*)p.A2 + (int64_t)(k0_ - p.k1) * 2;                      \
        _Pragma("unroll") for (int i_ = 0; i_ < GA; ++i_)                                    \
          glds(b_ + ga2[h][i_], wdA + ((buf) * 2 + (h)) * AHB + i_ * 1024);                  \
      }                                                                                      \
    } else {                                                                                 \
      const char* b_ = Ab + (int64_t)(t) * astep;                                            \
      _Pragma("unroll") for (int i_ = 0; i_ < GA; ++i_)                                      \
        glds(b_ + ga[h][i_], wdA + ((buf) * 2 + (h)) * AHB + i_ * 1024);                     \
    }                                                                                        \
  } while (0)
#define STAGE_B(h, buf, t)                                                                   \
  do {                                                                                       \
    if constexpr (BC) {                                                                      \
      _Pragma("unroll") for (int i_ = 0; i_ < GB; ++i_) {                                    \
        /* this lane's pixel of K-tile t: half h's cursor (tile t exactly: stagings are in order) */ \
        const int ow_ = (int)(bohw[h][i_] & 0xffffu), oh_ = (int)(bohw[h][i_] >> 16);       \
        const int ih_ = oh_ * cg.sh + ((int)gbt[h][i_] >> 16);                               \
        const int iw_ = ow_ * cg.sw + (int)(int16_t)(gbt[h][i_] & 0xffffu);                  \
        const bool v_ = 4 * (wid * GB + i_) + (lane >> 4) < p.K - kb - (t) * TK &&           \
                        (unsigned)ih_ < (unsigned)cg.H && (unsigned)iw_ < (unsigned)cg.W;    \
        const uint32_t po_ = (bq[h][i_] << cshift) * 2u;                                     \
        bdma16(arsrc, wdB + ((buf) * 2 + (h)) * BHB + i_ * 1024, v_ ? po_ + gb[h][i_] : 0x80000000u, 0u); \
        /* advance the cursor one K-tile (TK pixels) */                                      \
        int ow2_ = ow_ + bc_dow, oh2_ = oh_ + bc_doh;                                        \
        uint32_t q2_ = bq[h][i_] + (uint32_t)bc_dq;                                          \
        if (ow2_ >= cg.OW) { ow2_ -= cg.OW; oh2_ += 1; q2_ += (uint32_t)bc_cw; }             \
        if (oh2_ >= cg.OH) { oh2_ -= cg.OH; q2_ += (uint32_t)bc_ch; }                         \
        bq[h][i_] = q2_;                                                                     \
        bohw[h][i_] = ((uint32_t)oh2_ << 16) | (uint32_t)ow2_;                               \
      }                                                                                      \
    } else {                                                                                 \
      const char* b_ = Bb + (int64_t)(t) * bstep;                                            \
      _Pragma("unroll") for (int i_ = 0; i_ < GB; ++i_)                                      \
        glds(b_ + gb[h][i_], wdB + ((buf) * 2 + (h)) * BHB + i_ * 1024);                     \
    }                                                                                        \
  } while (0)
#if HG_SCHED == 1
  // tile 0 -> buf 0 (all halves), tile 1 -> buf 1 (A0, B1, A1; B0(1) is staged in tile 0's phase 1)
#define PROLOGUE()                                                                           \
  do {                                                                                       \
    STAGE_A(0, 0, 0); STAGE_B(0, 0, 0); STAGE_B(1, 0, 0); STAGE_A(1, 0, 0);                  \
    if (nt > 1) { STAGE_A(0, 1, 1); STAGE_B(1, 1, 1); STAGE_A(1, 1, 1); }                    \
  } while (0)
#else
#define PROLOGUE()                                                                           \
  do {                                                                                       \
    STAGE_A(0, 0, 0); STAGE_B(1, 0, 0); STAGE_A(1, 0, 0); STAGE_B(0, 0, 0);                  \
    if (nt > 1) { STAGE_A(0, 1, 1); STAGE_B(1, 1, 1); }                                      \
  } while (0)
#endif

  f32x4 acc[2 * FMH][2 * FNH];
  bf16x8 af[FMH][2], bfr[FNH][2];
  static_assert(!BG || (!AK && FMH == WC), "bias-grad fusion: M-contiguous A, one fragment row-block per wave column");
  float rsum[2] = {0.f, 0.f};  // BG: this lane's partial row sums (rows of half images 0 / 1)
  bool bg_on = false;
  const bf16x2_t ones2 = {(__bf16)1.f, (__bf16)1.f};
#define BG_SUM(hh)                                                                           \
  do {                                                                                       \
    if (BG && bg_on) {                                                                       \
      _Pragma("unroll") for (int i_ = 0; i_ < FMH; ++i_)                                     \
        if (i_ == wc) {                                                                      \
          _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                 \
            const bf16x8 q_ = af[i_][s_];                                                    \
            rsum[hh] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(q_, q_, 0, 1), ones2, rsum[hh], false); \
            rsum[hh] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(q_, q_, 2, 3), ones2, rsum[hh], false); \
            rsum[hh] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(q_, q_, 4, 5), ones2, rsum[hh], false); \
            rsum[hh] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(q_, q_, 6, 7), ones2, rsum[hh], false); \
          }                                                                                  \
        }                                                                                    \
    }                                                                                        \
  } while (0)

#define LOAD_A(buf, h)                                                                       \
  do {                                                                                       \
    _Pragma("unroll") for (int i_ = 0; i_ < FMH; ++i_)                                       \
      _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                     \
        const char* a_ = smem + ((buf) * 2 + (h)) * AHB + ra[i_][s_];                        \
        af[i_][s_] = AK ? lds_b128(a_) : lds_tr(a_);                                         \
      }                                                                                      \
  } while (0)
#define LOAD_B(buf, h)                                                                       \
  do {                                                                                       \
    _Pragma("unroll") for (int j_ = 0; j_ < FNH; ++j_)                                       \
      _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                     \
        const char* a_ = smem + ((buf) * 2 + (h)) * BHB + rb[j_][s_];                        \
        bfr[j_][s_] = BK ? lds_b128(a_) : lds_tr(a_);                                        \
      }                                                                                      \
  } while (0)
#define QUAD(mh, nh)                                                                         \
  do {                                                                                       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                       \
    MFMAQ(mh, nh);                                                                           \
  } while (0)
#define MFMAQ(mh, nh)                                                                        \
  do {                                                                                       \
    __builtin_amdgcn_s_setprio(1);                                                           \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < FMH; ++i_)                                     \
        _Pragma("unroll") for (int j_ = 0; j_ < FNH; ++j_)                                   \
          acc[(mh) * FMH + i_][(nh) * FNH + j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(   \
              bfr[j_][s_], af[i_][s_], acc[(mh) * FMH + i_][(nh) * FNH + j_], 0, 0, 0);      \
    __builtin_amdgcn_s_setprio(0);                                                           \
  } while (0)

  decode(u);
  PROLOGUE();
  wait_vm<0>();
  HG_BARRIER();

  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  while (true) {
#pragma unroll
    for (int i = 0; i < 2 * FMH; ++i)
#pragma unroll
      for (int j = 0; j < 2 * FNH; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (BG) {
      bg_on = qdbias != nullptr && n0 == 0;  // one tile column carries the row sums
      rsum[0] = rsum[1] = 0.f;
    }
    if (late) HG_BARRIER();

#if HG_SCHED == 1
    // One K-tile per iteration, buffer b = t & 1.  Every phase retires its own
    // fragment reads (lgkmcnt(0)) BEFORE its first barrier, so a half image can
    // be restaged one phase after its last read: P1 B0(t+1)->b^1, P2 A0(t+2)->b,
    // P3 B1(t+2)->b, P4 A1(t+2)->b.  Phase 4's counted vmcnt retires B0(t+1)
    // and everything older and leaves three half images (A0/B1/A1 of t+2) in
    // flight across the barrier.
    for (int t = 0; t < nt; ++t) {
      const int b = t & 1;
      const bool h1 = t + 1 < nt, h2 = t + 2 < nt;

      LOAD_A(b, 0); LOAD_B(b, 0);
      if (h1) STAGE_B(0, b ^ 1, t + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      HG_BARRIER();
      MFMAQ(0, 0);
      HG_BARRIER();

      LOAD_B(b, 1);
      if (h2) STAGE_A(0, b, t + 2);
      {
        // the next unit's claim, consumed after the main loop: issued behind A0(t+2), fewer DMAs than
        // this tile's counted wait keeps in flight are younger than it, so it may stay in flight until
        // the drain (wait_vm<0>) of tile nt-2 -- about six phases (claimer goes through an empty asm
        // every iteration: the loop must not be unswitched on it, a second loop copy for wave 0
        // would double the hot loop's instruction footprint)
        int cl = claimer;
        asm volatile("" : "+v"(cl));
        if (t == (nt >= 3 ? nt - 3 : 0) && cl)
          claim_v = (int)__hip_atomic_fetch_add(ctr(xcc), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      HG_BARRIER();
      MFMAQ(0, 1);
      BG_SUM(0);  // A half 0 fragments: last used by this phase's MFMAs
      HG_BARRIER();

      LOAD_A(b, 1);
      if (h2) STAGE_B(1, b, t + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      HG_BARRIER();
      MFMAQ(1, 1);
      HG_BARRIER();

      LOAD_B(b, 0);
      if (h2) {
        STAGE_A(1, b, t + 2);
        wait_vm<2 * GA + GB>();
      } else {
        wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      HG_BARRIER();
      MFMAQ(1, 0);
      BG_SUM(1);  // A half 1 fragments
      HG_BARRIER();
    }
#else
    // One K-tile per iteration, buffer b = t & 1.  Phase p restages one half
    // image: A1(t+1)->b^1, B0(t+1)->b^1, A0(t+2)->b, B1(t+2)->b; each target was
    // last read two phases earlier, and phase 4's counted vmcnt retires tile t+1.
    for (int t = 0; t < nt; ++t) {
      const int b = t & 1;
      const bool h1 = t + 1 < nt, h2 = t + 2 < nt;

      LOAD_A(b, 0); LOAD_B(b, 0);
      if (h1) STAGE_A(1, b ^ 1, t + 1);
      HG_BARRIER();
      QUAD(0, 0);
      HG_BARRIER();

      LOAD_B(b, 1);
      if (h1) STAGE_B(0, b ^ 1, t + 1);
      HG_BARRIER();
      QUAD(0, 1);
      HG_BARRIER();

      LOAD_A(b, 1);
      if (h2) STAGE_A(0, b, t + 2);
      HG_BARRIER();
      QUAD(1, 1);
      HG_BARRIER();

      LOAD_B(b, 0);
      if (h2) {
        STAGE_B(1, b, t + 2);
        wait_vm<G::NKEEP>();
      } else {
        wait_vm<0>();
      }
      HG_BARRIER();
      QUAD(1, 0);
      HG_BARRIER();
    }
#endif
    // resolve the next unit (wave 0; its result reaches the other waves through the LDS slot and the
    // barrier below: the late waves' last loop barrier pairs with this rebalance barrier)
    if (dyn > 0 && wid == 0) {
      const int nx = resolve(__builtin_amdgcn_readfirstlane(claim_v));  // lane 0 (the wave is whole here)
      if (lane == 0) *slot = nx;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // s_barrier does not wait for the ds_write
    }
    if (!late) HG_BARRIER();  // rebalance the stagger: every wave is past its last LDS read

    // ------------------------------------------------------------ epilogue
    // acc[i][j][e]: row m0 + wr*(BM/WR) + (i/FMH)*RH + (i%FMH)*16 + lm,
    //               col n0 + wc*(BN/WC) + (j/FNH)*CH + (j%FNH)*16 + ln4 + e
    const int rbase = m0 + wr * (BM / WR) + lm, cbase = n0 + wc * (BN / WC) + ln4;
    // (readfirstlane: the value is uniform; keeping it scalar keeps the tile indexing in SGPRs)
    int next = dyn > 0 ? __builtin_amdgcn_readfirstlane(*slot)
                       : (u + (int)gridDim.x < nunits ? u + (int)gridDim.x : -1);
    const int cur_split = split;

    // Stream-K: a tile cut over P > 1 blocks.  Its owner is the segment that is done last (SkGrid::done_at;
    // ties: the lowest block); the others store their fp32 partials write-through (sc1, 16 B per lane per
    // fragment; two slabs per block: the segment starting the block's range, and the one it runs first),
    // issue their next segment's prologue, and after the loop-end drain (every wave's vmcnt(0), then the
    // barrier) one lane adds to the tile's counter.  The owner polls the counter (sc1, one lane) until the
    // P - 1 others have added, resets it, and after a barrier adds their slabs to its registers in block
    // order with sc1 loads (MI355X_MICROARCH.md, hand-off table row 1): run-to-run identical.  It only
    // waits on segments scheduled to be done before it, in blocks that are all resident (one block per CU,
    // grid <= free CUs); the poll is bounded and flags a timeout in sk_cnt[HGEMM_SK_MAX_TILES - 1]
    // instead of hanging.
    bool do_epi = true;
    int sk_sig = -1;  // tile whose counter this block adds to after the loop-end drain
    if constexpr (SKM) {
      constexpr int NF = 4 * FMH * FNH, SLAB = NF * G::NT * 16;  // fragments per lane, bytes per slab
      const SkGrid sg = sk_grid();
      const unsigned t0 = (unsigned)u * (unsigned)ntk, lo = sg.lo(sg.lb), hi = sg.lo(sg.lb + 1u), tb = sg.lead(sg.lb);
      const unsigned cs = t0 + (unsigned)(kb / TK), ce = cs + (unsigned)nt;  // this segment
      const int bf = (int)sg.blk(t0), P = (int)sg.blk(t0 + (unsigned)ntk - 1u) - bf + 1;
      if (P > 1) {
        int own = bf;
        unsigned best = 0u;
        for (int b = bf; b < bf + P; ++b) {
          const unsigned d = sg.done_at((unsigned)b, t0);
          if (d > best) {
            best = d;
            own = b;
          }
        }
        const __amdgpu_buffer_rsrc_t skr = __builtin_amdgcn_make_buffer_rsrc(p.sk_ws, (short)0, 2 * G0 * SLAB, 0x00020000);
        // block b's slab of this tile: slot 0 if its segment starts b's range, else 1; fragment f of thread x
        // at + (f * threads + x) * 16 (each store / load instruction moves 1 KB per wave; f in soffset)
        auto slab_of = [&](int b) -> uint32_t { return (uint32_t)(2 * b + (sg.lo((unsigned)b) >= t0 ? 0 : 1)) * (uint32_t)SLAB; };
        const uint32_t lofs = (uint32_t)tid * 16u;
        if ((int)sg.lb != own) {
          const uint32_t mine = slab_of((int)sg.lb) + lofs;
#pragma unroll
          for (int i = 0; i < 2 * FMH; ++i)
#pragma unroll
            for (int j = 0; j < 2 * FNH; ++j)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), skr, mine,
                                                     (i * 2 * FNH + j) * G::NT * 16, 16);
          sk_sig = u;
          do_epi = false;
        } else {
          if (tid == 0) {
            unsigned* const cnt = p.sk_cnt + u;
            for (unsigned n = 0; __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned)(P - 1); ++n) {
              if (n == (1u << 22)) {  // ~seconds: a block that never ran; give up rather than hang the GPU
                __hip_atomic_store(p.sk_cnt + (HGEMM_SK_MAX_TILES - 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
            }
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          __syncthreads();
          for (int b = bf; b < bf + P; ++b) {
            if (b == own) continue;
            const uint32_t base = slab_of(b) + lofs;
            constexpr int HI = FMH;  // fragment rows per batch of loads: half the tile
#pragma unroll
            for (int i0 = 0; i0 < 2 * FMH; i0 += HI) {
              u32x4 v[HI][2 * FNH];
#pragma unroll
              for (int i = 0; i < HI; ++i)
#pragma unroll
                for (int j = 0; j < 2 * FNH; ++j)
                  v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(skr, base, ((i0 + i) * 2 * FNH + j) * G::NT * 16, 16);
#pragma unroll
              for (int i = 0; i < HI; ++i)
#pragma unroll
                for (int j = 0; j < 2 * FNH; ++j) acc[i0 + i][j] += __builtin_bit_cast(f32x4, v[i][j]);
            }
          }
        }
      }
      // next: after the lead segment the range from its start (up to the lead tile), else onward
      const unsigned bound = tb != ~0u ? tb : hi;
      next = (tb != ~0u && ce == hi) ? sk_seg(lo, bound) : (ce < bound ? sk_seg(ce, bound) : -1);
    }

    // 0) bias gradient: the 4 lane groups hold k-slices of the same 16 rows
    if constexpr (BG) {
      if (bg_on) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v = rsum[hh];
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          const int row = m0 + wr * (BM / WR) + hh * RH + wc * 16 + lm;
          if (lane < 16 && row < qM) {
            if (p.splits > 1) p.ws_bias[(int64_t)cur_split * qM + row] = v;  // summed in split order by finalize
            else qdbias[row] += alpha * v;                                   // the row's only writer
          }
        }
      }
    }

    if constexpr (SKM) {
      if (!do_epi) {  // a partial for the tile's head: the next segment's prologue, then the drain and the add
        if (next >= 0) {
          u = next;
          decode(u);
          PROLOGUE();
        }
        wait_vm<0>();
        HG_BARRIER();
        if (tid == 0) __hip_atomic_fetch_add(p.sk_cnt + sk_sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (next < 0) break;
        continue;
      }
    }

    // 1) math (every global load of the epilogue happens here, before any DMA is in flight)
    u32x2 pk[2 * FMH][2 * FNH];
    u32x2 pv[(EPI == HE_BF16 && ACT == ACT_GELU) ? 2 * FMH : 1][(EPI == HE_BF16 && ACT == ACT_GELU) ? 2 * FNH : 1];
    if constexpr (EPI == HE_BF16) {
      f32x4 bias[2 * FNH];
#pragma unroll
      for (int j = 0; j < 2 * FNH; ++j) {
        const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
        bias[j] = (p.bias && c < qN) ? *(const f32x4*)(p.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 2 * FMH; ++i) {
        const int r = min(rbase + (i / FMH) * RH + (i % FMH) * 16, qM - 1);
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = alpha * acc[i][j][e] + bias[j][e];
          if constexpr (ACT == ACT_GELU) {
            pv[i][j][0] = pack_bf2(v[0], v[1]);
            pv[i][j][1] = pack_bf2(v[2], v[3]);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu_fwd(v[e]);
          } else if constexpr (ACT == HACT_GELU_BWD) {
            // unconditional load (clamped column): a load under the lane-divergent c < qN test got a full
            // vmcnt wait of its own; a column past N is never stored, so its value does not matter
            const u32x2 a = *(const u32x2*)(p.aux_in + (int64_t)r * qldc + (c < qN ? c : 0));
            v[0] *= gelu_grad(__uint_as_float(a[0] << 16));
            v[1] *= gelu_grad(__uint_as_float(a[0] & 0xffff0000u));
            v[2] *= gelu_grad(__uint_as_float(a[1] << 16));
            v[3] *= gelu_grad(__uint_as_float(a[1] & 0xffff0000u));
          } else if constexpr (ACT == ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          pk[i][j][0] = pack_bf2(v[0], v[1]);
          pk[i][j][1] = pack_bf2(v[2], v[3]);
        }
        if constexpr (ACT == HACT_GELU_BWD) __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (ACT == HACT_BNB || ACT == HACT_BNF) {
        // BN-backward partials of the stored (rounded) values over this wave's rows of the tile: per
        // column j-fragment, sum over the row fragments in registers, then over the 16 lanes (lm) that
        // hold the same 4 columns; lane lm == 0 writes the wave row's partial column
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
          const bool cv = c < qN;
          const int cc = cv ? c : 0;
          f32x4 sc{}, sh{}, mu{};
          if constexpr (ACT == HACT_BNB) {
            sc = *(const f32x4*)(p.st_coef + cc);
            sh = *(const f32x4*)(p.st_coef + qN + cc);
            mu = *(const f32x4*)(p.st_coef + 2 * qN + cc);
          }
          f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = f32x4{0.f, 0.f, 0.f, 0.f};
          // the pre-BN inputs of this column fragment's rows, all loads issued before the first use and
          // unconditionally (clamped row / column; invalid rows masked below): under the lane-divergent
          // row test each load was followed by its own full vmcnt wait -- 2*FMH round trips per fragment
          u32x2 xr[ACT == HACT_BNB ? 2 * FMH : 1];
          if constexpr (ACT == HACT_BNB) {
#pragma unroll
            for (int i = 0; i < 2 * FMH; ++i) {
              const int r = min(rbase + (i / FMH) * RH + (i % FMH) * 16, qM - 1);
              xr[i] = *(const u32x2*)(p.st_x + (int64_t)r * qldc + cc);
            }
          }
#pragma unroll
          for (int i = 0; i < 2 * FMH; ++i) {
            const int r = rbase + (i / FMH) * RH + (i % FMH) * 16;
            const bool rv = r < qM && cv;
            const float v4[4] = {__uint_as_float(pk[i][j][0] << 16), __uint_as_float(pk[i][j][0] & 0xffff0000u),
                                 __uint_as_float(pk[i][j][1] << 16), __uint_as_float(pk[i][j][1] & 0xffff0000u)};
            {
              if constexpr (ACT == HACT_BNB) {
                const float x4[4] = {__uint_as_float(xr[i][0] << 16), __uint_as_float(xr[i][0] & 0xffff0000u),
                                     __uint_as_float(xr[i][1] << 16), __uint_as_float(xr[i][1] & 0xffff0000u)};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float dz = (rv && fmaf(x4[e], sc[e], sh[e]) > 0.f) ? v4[e] : 0.f;
                  s1[e] += dz;
                  s2[e] = fmaf(dz, x4[e] - mu[e], s2[e]);
                }
              } else if (rv) {  // forward statistics of the stored values
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  s1[e] += v4[e];
                  s2[e] = fmaf(v4[e], v4[e], s2[e]);
                }
              }
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
              s1[e] += __shfl_xor(s1[e], o, 64);
              s2[e] += __shfl_xor(s2[e], o, 64);
            }
          }
          if (lm == 0 && cv) {
            const int col = (m0 / BM) * WR + wr;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              p.col_stats[(int64_t)(c + e) * p.stats_ld + col] = s1[e];
              p.col_stats[(int64_t)(qN + c + e) * p.stats_ld + col] = s2[e];
            }
          }
        }
      }
    } else if constexpr (EPI == HE_F32) {
      f32x4 bias[2 * FNH];
#pragma unroll
      for (int j = 0; j < 2 * FNH; ++j) {
        const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
        bias[j] = (p.bias && c < qN) ? *(const f32x4*)(p.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 2 * FMH; ++i) {
        const int r = min(rbase + (i / FMH) * RH + (i % FMH) * 16, qM - 1);
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
          f32x4 res = f32x4{0.f, 0.f, 0.f, 0.f};
          if (p.residual_f32 && c < qN) res = *(const f32x4*)(p.residual_f32 + (int64_t)r * qldc + c);
          // stored right away (holding 128 fp32 results across the next prologue spills)
          if (c < qN && rbase + (i / FMH) * RH + (i % FMH) * 16 < qM)
            *(f32x4*)((float*)qC + (int64_t)r * qldc + c) = acc[i][j] * alpha + bias[j] + res;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (EPI == HE_ACC_F32 || EPI == HE_GROUP) {
#pragma unroll
      for (int i = 0; i < 2 * FMH; ++i) {
        const int r = min(rbase + (i / FMH) * RH + (i % FMH) * 16, qM - 1);
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
          f32x4 old = f32x4{0.f, 0.f, 0.f, 0.f};
          if (c < qN && !(GRP && qover)) old = *(const f32x4*)((const float*)qC + (int64_t)r * qldc + c);
          if (c < qN && rbase + (i / FMH) * RH + (i % FMH) * 16 < qM)
            *(f32x4*)((float*)qC + (int64_t)r * qldc + c) = acc[i][j] * alpha + old;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // 2) the next unit's prologue DMA (LDS is free: every wave passed the rebalance barrier)
    if (next >= 0) {
      u = next;
      decode(u);
      PROLOGUE();
    }

    // 3) stores (drain while the prologue loads are in flight)
    if constexpr (EPI == HE_BF16) {
      // Widened to 16 B per lane (T21 with a 16-lane exchange): fragments i, i+1 (rows r, r+16) hold
      // columns 4g..4g+3 in lane group g; v_permlane16_swap gives even groups row r's columns
      // 8(g/2)..+7 and odd groups row r+16's, so every lane stores 8 consecutive bf16 -- half the
      // store instructions of the 8-B form (the epilogue tail is store-issue-bound).
      const int g = lane >> 4;
      const int c_off = (g >> 1) * 8 - ln4;  // this lane's 8-column chunk relative to cbase
#pragma unroll
      for (int i = 0; i < 2 * FMH; i += 2) {
        const int r = rbase + (i / FMH) * RH + (i % FMH) * 16 + (g & 1) * 16;
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16 + c_off;
          u32x2 a = pk[i][j], b = pk[i + 1][j];
          auto x = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
          auto y = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
          if (r < qM && c < qN) *(u32x4*)((uint16_t*)qC + (int64_t)r * qldc + c) = u32x4{x[0], y[0], x[1], y[1]};
          if constexpr (ACT == ACT_GELU) {
            u32x2 va = pv[i][j], vb = pv[i + 1][j];
            auto vx = __builtin_amdgcn_permlane16_swap(va[0], vb[0], false, false);
            auto vy = __builtin_amdgcn_permlane16_swap(va[1], vb[1], false, false);
            if (p.aux_out && r < qM && c < qN)
              *(u32x4*)(p.aux_out + (int64_t)r * qldc + c) = u32x4{vx[0], vy[0], vx[1], vy[1]};
          }
        }
      }
    } else if constexpr (EPI == HE_SLAB) {
#pragma unroll
      for (int i = 0; i < 2 * FMH; ++i) {
        const int r = rbase + (i / FMH) * RH + (i % FMH) * 16;
        if (r >= qM) continue;
#pragma unroll
        for (int j = 0; j < 2 * FNH; ++j) {
          const int c = cbase + (j / FNH) * CH + (j % FNH) * 16;
          if (c < qN) *(f32x4*)(p.ws + ((int64_t)cur_split * qM + r) * qN + c) = acc[i][j];
        }
      }
    }
    if (next < 0) break;
    wait_vm<0>();
    HG_BARRIER();
  }
  sched_exit();
#undef STAGE_A
#undef STAGE_B
#undef PROLOGUE
#undef LOAD_A
#undef LOAD_B
#undef QUAD
#undef MFMAQ
#undef BG_SUM
}

// sum of K-split partial slabs -> the real epilogue.  A block is FQ = 256 / FG output quads (4 columns
// each) x FG split groups (FG = 8 from 32 splits on): thread (quad, group g) sums slabs g, g + 8, g + 16, ... (loads issued 4 at a time),
// the 8 group sums are added in group order in LDS (fixed: run-to-run identical), and the group-0 threads
// run the epilogue.  (One thread per quad over every split left the many-split weight grads -- 100-200
// slabs of a 512 x 128 output in 64 blocks -- latency-bound at ~17 us.)
// FG = 1 (few splits: the per-thread loop is short, and the quads of 256 threads keep the grid small) is the
// plain per-quad sum.
template <int EPI, int ACT, int FG>
__global__ __launch_bounds__(256) void hgemm_finalize_kernel(HgemmArgs p) {
  constexpr int FQ = 256 / FG;
  __shared__ f32x4 part[FG][FQ];
  __shared__ float bpart[FG][FQ];
  const int qi = threadIdx.x % FQ, grp = threadIdx.x / FQ;
  const int64_t q = (int64_t)blockIdx.x * FQ + qi;
  const int nq = p.N >> 2;
  const bool ok = q < (int64_t)p.M * nq;
  const int r = ok ? (int)(q / nq) : 0, c = ok ? (int)(q % nq) * 4 : 0;
  const float alpha = p.alpha * (p.alpha_ptr ? *p.alpha_ptr : 1.f);
  const int64_t plane = (int64_t)p.M * p.N;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  float bs = 0.f;
  if (ok) {
    const float* src = p.ws + (int64_t)r * p.N + c;
    int k = grp;
    for (; k + 3 * FG < p.splits; k += 4 * FG) {
      const f32x4 a0 = *(const f32x4*)(src + k * plane), a1 = *(const f32x4*)(src + (k + FG) * plane);
      const f32x4 a2 = *(const f32x4*)(src + (k + 2 * FG) * plane), a3 = *(const f32x4*)(src + (k + 3 * FG) * plane);
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; k < p.splits; k += FG) s += *(const f32x4*)(src + k * plane);
    if (p.dbias && c == 0)  // fused bias gradient: the units' partial row sums, same grouping
      for (int kk = grp; kk < p.splits; kk += FG) bs += p.ws_bias[(int64_t)kk * p.M + r];
  }
  part[grp][qi] = s;
  bpart[grp][qi] = bs;
  __syncthreads();
  if (grp != 0 || !ok) return;
#pragma unroll
  for (int g = 1; g < FG; ++g) s += part[g][qi];
  s *= alpha;
  if (p.bias) s += *(const f32x4*)(p.bias + c);
  if (p.dbias && c == 0) {
#pragma unroll
    for (int g = 1; g < FG; ++g) bs += bpart[g][qi];
    p.dbias[r] += alpha * bs;
  }
  const int64_t o = (int64_t)r * p.ldc + c;
  if constexpr (EPI == HE_BF16) {
    float v[4] = {s[0], s[1], s[2], s[3]};
    if constexpr (ACT == ACT_GELU) {
      if (p.aux_out) *(u32x2*)(p.aux_out + o) = u32x2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_fwd(v[e]);
    } else if constexpr (ACT == HACT_GELU_BWD) {
      const u32x2 a = *(const u32x2*)(p.aux_in + o);
      v[0] *= gelu_grad(__uint_as_float(a[0] << 16));
      v[1] *= gelu_grad(__uint_as_float(a[0] & 0xffff0000u));
      v[2] *= gelu_grad(__uint_as_float(a[1] << 16));
      v[3] *= gelu_grad(__uint_as_float(a[1] & 0xffff0000u));
    } else if constexpr (ACT == ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    *(u32x2*)((uint16_t*)p.C + o) = u32x2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
  } else if constexpr (EPI == HE_F32) {
    if (p.residual_f32) s += *(const f32x4*)(p.residual_f32 + o);
    *(f32x4*)((float*)p.C + o) = s;
  } else {  // HE_ACC_F32
    *(f32x4*)((float*)p.C + o) = s + *(const f32x4*)((const float*)p.C + o);
  }
}

}  // namespace hg
}  // namespace dpe

using namespace dpe;

namespace {

template <int BM, int BN, int WR, int WC, bool AK, bool BK>
int launch_epi(const HgemmArgs& p, int epi, int grid, hipStream_t st) {
  const dim3 g((unsigned)grid), b(WR * WC * 64);
  if (p.dbias) {  // fused bias gradient: TN weight grads (raw slabs, fp32 accumulate or overwrite) only
    if constexpr (!AK && !BK && BM == 256 && BN == 256) {
      if (p.act != ACT_NONE || (p.splits > 1 && !p.ws_bias)) return -3;
      if (epi == HE_SLAB) hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, AK, BK, HE_SLAB, ACT_NONE, true>), g, b, 0, st, p);
      else if (epi == HE_ACC_F32) hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, AK, BK, HE_ACC_F32, ACT_NONE, true>), g, b, 0, st, p);
      else if (epi == HE_F32 && !p.bias && !p.residual_f32)  // overwrite (the gradient's first writer of the step)
        hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, AK, BK, HE_F32, ACT_NONE, true>), g, b, 0, st, p);
      else return -3;
      return 0;
    } else {
      return -5;
    }
  }
#define HL(E, A) hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, AK, BK, E, A>), g, b, 0, st, p)
  if (epi == HE_SLAB) {  // raw partials: the activation belongs to hgemm_finalize
    HL(HE_SLAB, ACT_NONE);
  } else if (epi == HE_BF16) {
    if (p.act == ACT_NONE) HL(HE_BF16, ACT_NONE);
    else if (p.act == ACT_GELU) HL(HE_BF16, ACT_GELU);
    else if (p.act == HACT_GELU_BWD) HL(HE_BF16, HACT_GELU_BWD);
    else if (p.act == ACT_RELU) HL(HE_BF16, ACT_RELU);
    else if (p.act == HACT_BNB && AK && !BK && p.splits == 1 && p.col_stats && p.st_x && p.st_coef) HL(HE_BF16, HACT_BNB);
    else if (p.act == HACT_BNF && AK && BK && p.splits == 1 && p.col_stats && !p.bias) HL(HE_BF16, HACT_BNF);
    else return -3;
  } else if (p.act != ACT_NONE) {
    return -3;
  } else if (epi == HE_F32) {
    HL(HE_F32, ACT_NONE);
  } else if (epi == HE_ACC_F32) {
    HL(HE_ACC_F32, ACT_NONE);
  } else {
    return -2;
  }
#undef HL
  return 0;
}

// implicit-im2col A (NT layout, bf16 out, no K split): plain, BN-forward or BN-backward partials epilogue
template <int BM, int BN, int WR, int WC>
int launch_conv(const HgemmArgs& p, int epi, int grid, hipStream_t st) {
  if (epi != HE_BF16 || p.splits != 1 || p.dbias || p.bias) return -3;
  const dim3 g((unsigned)grid), b(WR * WC * 64);
#define HC(A)                                                                                                     \
  do {                                                                                                            \
    if constexpr (WR * WC == 8) {                                                                                 \
      if (p.sk) {                                                                                                 \
        hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, true, true, HE_BF16, A, false, 1, true>), g, b, 0, st, p); \
        break;                                                                                                    \
      }                                                                                                           \
    }                                                                                                             \
    hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, true, true, HE_BF16, A, false, 1>), g, b, 0, st, p);      \
  } while (0)
  if (p.act == ACT_NONE) HC(ACT_NONE);
  else if (p.act == HACT_BNF && p.col_stats) HC(HACT_BNF);
  else if (p.act == HACT_BNB && p.col_stats && p.st_x && p.st_coef) HC(HACT_BNB);
  else return -3;
#undef HC
  return 0;
}

// implicit-im2col B (TN weight grads, 256x256 only): K-split slabs or fp32 accumulate
int launch_conv_wgrad(const HgemmArgs& p, int epi, int grid, hipStream_t st) {
  if (p.act != ACT_NONE || p.dbias || p.bias) return -3;
  const dim3 g((unsigned)grid), b(512);
  if (epi == HE_SLAB) hipLaunchKernelGGL((hg::hgemm_kernel<256, 256, 2, 4, false, false, HE_SLAB, ACT_NONE, false, 2>), g, b, 0, st, p);
  else if (epi == HE_ACC_F32 && p.splits == 1)
    hipLaunchKernelGGL((hg::hgemm_kernel<256, 256, 2, 4, false, false, HE_ACC_F32, ACT_NONE, false, 2>), g, b, 0, st, p);
  else return -3;
  return 0;
}

// concatenated-K A (NN layout, bf16 out with bias, BN-backward partials or none; no K split)
template <int BM, int BN, int WR, int WC>
int launch_cat(const HgemmArgs& p, int epi, int grid, hipStream_t st) {
  if (epi != HE_BF16 || p.splits != 1 || p.dbias) return -3;
  const dim3 g((unsigned)grid), b(WR * WC * 64);
  if (p.act == HACT_BNB && p.col_stats && p.st_x && p.st_coef)
    hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, true, false, HE_BF16, HACT_BNB, false, 3>), g, b, 0, st, p);
  else if (p.act == ACT_NONE)
    hipLaunchKernelGGL((hg::hgemm_kernel<BM, BN, WR, WC, true, false, HE_BF16, ACT_NONE, false, 3>), g, b, 0, st, p);
  else return -3;
  return 0;
}

template <int BM, int BN, int WR, int WC>
int launch_layout(const HgemmArgs& p, int a_k, int b_k, int epi, int grid, hipStream_t st) {
  if (p.conv == 3) {
    if constexpr (BN == 256) return (a_k && !b_k) ? launch_cat<BM, BN, WR, WC>(p, epi, grid, st) : -2;
    return -2;
  }
  if (p.conv == 2) {
    if constexpr (BM == 256 && BN == 256) return (!a_k && !b_k) ? launch_conv_wgrad(p, epi, grid, st) : -2;
    return -2;
  }
  if (p.conv) return (a_k && b_k) ? launch_conv<BM, BN, WR, WC>(p, epi, grid, st) : -2;
  if (a_k && b_k) return launch_epi<BM, BN, WR, WC, true, true>(p, epi, grid, st);
  if constexpr (BN == 256) {
    if (a_k && !b_k) return launch_epi<BM, BN, WR, WC, true, false>(p, epi, grid, st);
    if constexpr (BM == 256) {
      if (!a_k && !b_k) return launch_epi<BM, BN, WR, WC, false, false>(p, epi, grid, st);
    }
  }
  return -2;
}

}  // namespace

extern "C" int dpe_hgemm_launch(const HgemmArgs* a, int cfg, int a_k, int b_k, int epi, int grid, hipStream_t st) {
  const HgemmArgs& p = *a;
  if (p.K % 64 || p.kps % 64 || p.kps <= 0 || p.N % 4 || grid <= 0) return -1;
  if (epi == HE_BF16 && (p.N % 8 || p.ldc % 8)) return -1;  // 16-B output chunks
  if (p.splits < 1 || (p.splits > 1 && epi != HE_SLAB)) return -1;
  const int adim = p.a_dim > 0 ? p.a_dim : p.M, bdim = p.b_dim > 0 ? p.b_dim : p.N;
  if (adim < p.M || bdim < p.N) return -1;
  if (!a_k && (adim % 8 || p.lda < adim)) return -1;  // M-contiguous A: 16-B chunks of 8 rows
  if (!b_k && (bdim % 8 || p.ldb < bdim)) return -1;
  if (p.lda % 8 || p.ldb % 8) return -1;
  // per-lane LDS-DMA source offsets are 32-bit
  if (p.conv == 1) {
    const ConvGeom& g = p.conv_g;
    if (!a_k || g.C < 64 || (g.C & (g.C - 1)) || g.R * g.S > 32 || g.R * g.S * g.C != p.K || p.kps != p.K ||
        (int64_t)g.N * g.OH * g.OW != p.M || p.conv_smagic != (65536 + g.S - 1) / g.S)
      return -1;
    if ((((int64_t)g.N * g.H * g.W * g.C) + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2 >= (1ll << 31) - 4096) return -4;
  } else if (p.conv == 3) {
    if (!a_k || !p.A2 || p.k1 <= 0 || p.k1 % 64 || p.k1 >= p.K || p.kps != p.K || p.lda < p.k1 ||
        p.lda2 < p.K - p.k1 || p.lda2 % 8)
      return -1;
    if ((int64_t)p.M * p.lda * 2 >= (1ll << 32) || (int64_t)p.M * p.lda2 * 2 >= (1ll << 32)) return -4;
  } else if (p.conv == 2) {
    // pixel decomposition by float reciprocals: exact for pixel indices < 2^24 with the +-1 correction
    const ConvGeom& g = p.conv_g;
    if (a_k || b_k || g.C < 8 || (g.C & (g.C - 1)) || g.R * g.S > 32 || g.R * g.S * g.C != p.N ||
        (int64_t)g.N * g.OH * g.OW != p.K || p.K >= (1 << 24) || p.conv_smagic != (65536 + g.S - 1) / g.S ||
        g.ph > 32767 || g.pw > 32767)
      return -1;
    if ((((int64_t)g.N * g.H * g.W * g.C) + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2 >= (1ll << 31) - 4096) return -4;
    if ((int64_t)p.K * p.lda * 2 >= (1ll << 32)) return -4;
  } else if ((a_k ? (int64_t)adim * p.lda : (int64_t)p.K * p.lda) * 2 >= (1ll << 32)) {
    return -4;
  }
  if ((b_k ? (int64_t)bdim * p.ldb : (int64_t)p.K * p.ldb) * 2 >= (1ll << 32)) return -4;
  if (p.sk) {
    // stream-K: one block per CU, whole-K units, static grid; two slabs per block, one counter per tile
    const int bm = cfg == HC_128x256 ? 128 : 256, bn = cfg == HC_256x128 ? 128 : 256;
    const int64_t tiles = (int64_t)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn);
    if (cfg == HC_128x128 || p.conv != 1 || epi != HE_BF16 || p.splits != 1 || p.kps != p.K || !p.sk_ws || !p.sk_cnt ||
        tiles >= HGEMM_SK_MAX_TILES || (int64_t)grid * 2 * (bm * bn * 4) >= (1ll << 31))
      return -1;
  }
  switch (cfg) {
    case HC_256x256: return launch_layout<256, 256, 2, 4>(p, a_k, b_k, epi, grid, st);
    case HC_128x256: return launch_layout<128, 256, 2, 4>(p, a_k, b_k, epi, grid, st);
    case HC_256x128: return launch_layout<256, 128, 4, 2>(p, a_k, b_k, epi, grid, st);
    case HC_128x128: return launch_layout<128, 128, 2, 2>(p, a_k, b_k, epi, grid, st);
    default: return -1;
  }
}

extern "C" int dpe_hgemm_group_launch(const HgemmArgs* a, int grid, hipStream_t st) {
  const HgemmArgs& p = *a;
  if (p.ngroup < 1 || p.ngroup > HGEMM_MAX_GROUP || p.K % 64 || p.K <= 0 || grid <= 0) return -1;
  if (p.splits != 1 || p.kps != p.K || p.act != ACT_NONE) return -1;
  int prev = 0;
  for (int g = 0; g < p.ngroup; ++g) {
    const HgemmProblem& q = p.grp[g];
    const int adim = q.a_dim > 0 ? q.a_dim : q.M;
    if (!q.A || !q.B || !q.C || q.M <= 0 || q.N <= 0 || q.N % 8 || adim < q.M || adim % 8) return -1;
    if (q.lda < adim || q.ldb < q.N || q.lda % 8 || q.ldb % 8 || q.ldc < q.N) return -1;
    if ((int64_t)p.K * q.lda * 2 >= (1ll << 32) || (int64_t)p.K * q.ldb * 2 >= (1ll << 32)) return -4;
    const int tiles = ((q.M + 255) / 256) * ((q.N + 255) / 256);
    if (q.tile_end != prev + tiles) return -1;  // host and kernel agree on the unit -> problem map
    prev = q.tile_end;
  }
  hipLaunchKernelGGL((hg::hgemm_kernel<256, 256, 2, 4, false, false, HE_GROUP, ACT_NONE, true>), dim3((unsigned)grid),
                     dim3(512), 0, st, p);
  return 0;
}

extern "C" int dpe_hgemm_finalize(const HgemmArgs* a, int epi, hipStream_t st) {
  const HgemmArgs& p = *a;
  if (p.N % 4) return -1;
  const int64_t n = (int64_t)p.M * (p.N / 4);
  const bool grouped = p.splits >= 32;
  const dim3 g((unsigned)(grouped ? (n + 31) / 32 : (n + 255) / 256)), b(256);
#define FL(E, A)                                                                   \
  do {                                                                             \
    if (grouped) hipLaunchKernelGGL((hg::hgemm_finalize_kernel<E, A, 8>), g, b, 0, st, p); \
    else hipLaunchKernelGGL((hg::hgemm_finalize_kernel<E, A, 1>), g, b, 0, st, p);        \
  } while (0)
  if (epi == HE_BF16) {
    if (p.act == ACT_NONE) FL(HE_BF16, ACT_NONE);
    else if (p.act == ACT_GELU) FL(HE_BF16, ACT_GELU);
    else if (p.act == HACT_GELU_BWD) FL(HE_BF16, HACT_GELU_BWD);
    else if (p.act == ACT_RELU) FL(HE_BF16, ACT_RELU);
    else return -3;
  } else if (p.act != ACT_NONE) {
    return -3;
  } else if (epi == HE_F32) {
    FL(HE_F32, ACT_NONE);
  } else if (epi == HE_ACC_F32) {
    FL(HE_ACC_F32, ACT_NONE);
  } else {
    return -2;
  }
#undef FL
  return 0;
}
