// Streaming pointwise (1x1, stride 1) convolution GEMMs for the write-heavy ResNet shapes
// (K in {64, 128, 256}, N >= 2K: every bottleneck's conv3 forward and conv1 data grad):
//   PW_FWD:   y[M][N] = x[M][K] . W[N][K]^T, with the BatchNorm-forward sums of the stored y;
//   PW_DGRAD: y[M][N] = dy[M][K] . W[K][N] (+ residual, optionally ReLU-masked by its producer's
//             bits), with the BatchNorm-backward partials (sum dz, sum dz*(x - mean)) of the BN
//             whose output this y is the gradient of (ReLU from its coefficients, or from the
//             saved output's mask bits -- then the stored y is the masked dz itself).
//
// Why a separate kernel: at K <= 256 the implicit-GEMM tile does 2-8 K-steps and then spends
// most of its life in the prologue DMA wait and the LDS-staged epilogue; one tile per block at
// 4 blocks per CU streamed the bottleneck conv3 shapes (64->256 @ 56^2 ... 256->1024 @ 14^2)
// at only 2.1-3.6 TB/s.  Here
//   * every block is persistent over a fixed column slice: its weights (WN columns x K per wave)
//     sit in VGPRs for the whole launch as MFMA A operands (no B traffic per tile);
//   * the x row tiles (64 rows x K) stream through an NS-deep LDS ring by buffer_load ... lds
//     (NS-1 tiles in flight while one is consumed), so the HBM latency overlaps the MFMAs and
//     the stores of earlier tiles; every wave reads the same tile (A = x fragments via the
//     swizzled K-image, as igemm);
//   * the output is staged per wave, half a tile at a time, through the wave's own LDS region
//     and stored as whole 16-B row chunks (one store instruction = 8 full 128-B row segments;
//     stores straight from the accumulator layout -- 16 rows x 32 B per instruction -- ran at
//     ~4 TB/s and were the limiter); the epilogue operands (residual, pre-BN input, mask bits)
//     are loaded in the same row-chunk layout before the staging writes;
//   * BatchNorm sums accumulate in registers over all of the block's rows and are reduced once
//     at the end: one partial column per row group ([2][N][row groups]) instead of one per
//     128-row tile, and no per-tile LDS reduction or barrier.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "igemm.h"
#include "pwconv.h"

namespace dpe {
namespace pw {

constexpr int BM = 64;  // rows per tile
typedef __attribute__((address_space(3))) void lds_void_t;

DPE_DEVICE int kimg_off(int row, int chunk) {
  const int g = (0x78 >> (((row >> 2) & 3) << 1)) & 3;
  return row * 64 + ((chunk ^ g) << 4);
}
DPE_DEVICE bf16x8 kfrag(const char* img, int r0) {
  const int lane = threadIdx.x & 63;
  return __builtin_bit_cast(bf16x8, *(const u32x4*)(img + kimg_off(r0 + (lane & 15), lane >> 4)));
}
DPE_DEVICE __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <int N>
DPE_DEVICE void wait_vm() {  // s_waitcnt vmcnt(N): loads, LDS-DMA and stores count together, in order
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
  asm volatile("" ::: "memory");
}

// K: reduction depth; WN: output columns per wave (4 waves -> 4*WN per block); NS: ring depth
// DYN: the dynamic row-group schedule (a compile-time variant: the static kernels keep their registers)
template <int K, int WN, int NS, int EPI, bool DYN = false>
__global__ __launch_bounds__(256, (K == 64 && EPI == PW_FWD) ? 3 : 2) void pw_stream_kernel(PwArgs a) {
  constexpr int KC = K / 32;                  // 32-deep K chunks
  constexpr int TILE = BM * K * 2;            // bytes of one x tile in LDS ([KC][64 rows][64 B])
  constexpr int P = TILE / 1024 / 4;          // 1-KiB DMA pieces per wave per tile
  constexpr int NI = WN / 16, MI = BM / 16;
  static_assert(P >= 1 && P * 4096 == TILE, "pieces");
  // output staging: each wave stages half a tile (32 rows x WN channels, padded rows) in its own
  // LDS region and stores whole 16-B row chunks: one store instruction = RPP full row segments
  constexpr int ROWB = WN * 2 + 16, CPRW = WN / 8, RPP = 64 / CPRW, NPS = 32 / RPP;
  constexpr int STG = 32 * ROWB;
  // stores outstanding per wave per tile, for the counted vmcnt below (the epilogue's operand
  // loads are consumed -- waited for -- inside the tile, so they are not outstanding here)
  constexpr int S = (EPI == PW_APPLY ? 4 : 2) * NPS;  // (PW_APPLY: the y chunk and its ReLU-mask byte)
  constexpr int VM = (NS - 1) * S + (NS - 2) * P;
  static_assert(VM < 64, "vmcnt range");
  // ONE LDS object: ring, staging, in_coef's [scale | shift] of the K input channels, the claim slot.  (With a
  // second __shared__ object the compiler cannot tell the ring DMA's LDS writes from the other accesses and
  // drains vmcnt(0) -- the next tile's DMA -- before each tile's fragment reads.)
  __shared__ __attribute__((aligned(16))) char smem[NS * TILE + 4 * STG + 2 * K * 4 + 16];
  float* const bnin = (float*)(smem + NS * TILE + 4 * STG);
  int* const claim_slot = (int*)(smem + NS * TILE + 4 * STG + 2 * K * 4);

  // PW_DSUM: the data grad's BN-backward partials are the sums of dz only (no pre-BN input)
  constexpr bool DG = EPI == PW_DGRAD || EPI == PW_DSUM;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = (int)a.M, N = (int)a.N, RG = a.rg;
  const int nbN = N / (4 * WN);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the nbN column slices of a row group share an XCD
  const int nb = bid % nbN;
  int rg = bid / nbN;
  // Dynamic schedule (a.sched, RG > resident row groups SRG): row groups [0, SRG) start statically, the
  // rest are claimed per column slice from counter nb, so a block whose CU is shared with foreign work
  // (RCCL channel blocks) takes fewer of them.  A row group's tiles, their summation order and its
  // partial column do not depend on which block runs it: results are schedule-independent, bitwise.
  const int SRG = (int)gridDim.x / nbN;  // row groups started statically (DYN: the rest are claimed)
  const int n0w = nb * 4 * WN + wid * WN;  // the wave's first output channel
  const int tiles = (M + BM - 1) / BM;
  const int ch = lane % CPRW;              // the lane's 16-B chunk of each staged row
  const int nch = n0w + ch * 8;            // its first channel

  // weights as MFMA A operands: wf[ni][kc] = W^T[n0w + 16 ni + li][32 kc + 8 g .. +7]
  bf16x8 wf[NI][KC];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int n = n0w + 16 * ni + li, k0 = 32 * kc + 8 * g;
      if constexpr (!DG) {
        wf[ni][kc] = __builtin_bit_cast(bf16x8, *(const u32x4*)(a.w + (int64_t)n * K + k0));
      } else {  // W stored [K][N]: gather the column (once per block)
        s16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (short)a.w[(int64_t)(k0 + e) * N + n];
        wf[ni][kc] = __builtin_bit_cast(bf16x8, v);
      }
    }
  // BatchNorm-backward coefficients of the lane's 8 channels
  float bsc[8], bsh[8], bmu[8];
  const bool bnb = EPI == PW_DSUM || (EPI == PW_DGRAD && a.st_x != nullptr);
  const bool bnx = EPI == PW_DGRAD && a.st_x != nullptr;
  if (bnx) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = a.st_coef[nch + e];
      bsh[e] = a.st_coef[N + nch + e];
      bmu[e] = a.st_coef[2 * N + nch + e];
    }
  }

  // DMA pieces: piece q (of 4P per tile) = K chunk q / 4, rows 16 (q % 4) .. +15; lane -> (row, 16-B chunk)
  const __amdgpu_buffer_rsrc_t xr = rsrc(a.x, (uint32_t)((int64_t)M * K * 2));
  uint32_t voff[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int q = wid * P + i, kc = q >> 2, row = (q & 3) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
    voff[i] = (uint32_t)(row * K * 2 + kc * 64 + lc * 16);
  }
  auto issue = [&](int t, int slot) {
    char* dst = smem + slot * TILE;
    const int64_t base = t >= 0 ? (int64_t)t * BM * K * 2 : 0;
    const int valid_rows = t >= 0 ? M - t * BM : 0;  // rows past M (or t < 0: no tile) read as zeros
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int q = wid * P + i, row = (q & 3) * 16 + (lane >> 2);
      const uint32_t v = row < valid_rows ? voff[i] + (uint32_t)base : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(dst + q * 1024), 16, v, 0, 0, 0);
    }
  };

  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
  // PW_APPLY: the BN applied to this lane's 8 output channels (+ the residual's own BN)
  float osc[8], osh[8], rsc[8], rsh[8];
  if constexpr (EPI == PW_APPLY) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      osc[e] = a.out_coef[nch + e];
      osh[e] = a.out_coef[N + nch + e];
      rsc[e] = a.res_coef ? a.res_coef[nch + e] : 1.f;
      rsh[e] = a.res_coef ? a.res_coef[N + nch + e] : 0.f;
    }
  }
  // residual element offset of output row m (chunk nch); -1: no residual term at this row (the odd
  // positions of a stride-2 downsample branch's compact data grad)
  const int rh = a.res_h, rw = a.res_w;
  auto res_off = [&](int m) -> int64_t {
    if (rh <= 0) return (int64_t)m * N + nch;
    const int hw = rh * rw, n = m / hw, r = m - n * hw, h = r / rw, w = r - h * rw;
    if ((h | w) & 1) return -1;
    return ((int64_t)(n * (rh >> 1) + (h >> 1)) * (rw >> 1) + (w >> 1)) * N + nch;
  };

  // Epilogue operands and outputs through buffer resources (a null operand: a 0-byte resource): every
  // load and store of a tile is issued unconditionally -- out-of-range offsets read 0 / drop the store --
  // so the number of memory ops between a hoisted load and its use is the same on every path and the
  // compiler's wait for it is a counted vmcnt.  (A load or store under a branch, or the DMA issue skipped
  // for the last tiles, made those waits vmcnt(0): each tile's epilogue then also waited for the NEXT
  // tile's ring DMA -- the layer-2/3 data grads and applies ran at 55-77 % of their HBM roofline.)
  constexpr uint32_t OOB = 0xfffffff0u;  // past every resource here (M N < 2^31 - 256: pw_plan)
  const uint32_t ybytes = (uint32_t)((int64_t)M * N * 2), mbytes = (uint32_t)((int64_t)M * N / 8);
  const uint32_t rbytes = rh > 0 ? (uint32_t)((int64_t)(M / (rh * rw)) * (rh >> 1) * (rw >> 1) * N * 2) : ybytes;
  const __amdgpu_buffer_rsrc_t yrs = rsrc(a.y, ybytes);
  const __amdgpu_buffer_rsrc_t rrs = rsrc(a.residual, a.residual ? rbytes : 0u);
  const __amdgpu_buffer_rsrc_t rmrs = rsrc(a.res_mask, a.res_mask ? mbytes : 0u);
  const __amdgpu_buffer_rsrc_t xsrs = rsrc(a.st_x, bnx ? ybytes : 0u);
  const __amdgpu_buffer_rsrc_t smrs = rsrc(a.st_mask, (bnb && a.st_mask) ? mbytes : 0u);
  const __amdgpu_buffer_rsrc_t obrs = rsrc(a.out_bits, (EPI == PW_APPLY && a.out_bits) ? mbytes : 0u);

  if (!DG && a.in_coef) {  // before the ring's first DMA (its counted waits start after this)
    for (int i = tid; i < 2 * K; i += 256) bnin[i] = a.in_coef[i];
    __syncthreads();
  }

  // one tile: its epilogue operands, the DMA of the ring stage NS-1 ahead (nxt_tile < 0: none), the MFMAs
  // over the landed tile in ring slot cur_slot, the staged stores and the statistics
  auto tile_body = [&](const int m0, const int cur_slot, const int nxt_tile, const int nxt_slot) {
    // K = 256 data grads: this tile's epilogue operands (residual, pre-BN input, masks) are issued
    // before the next ring stage's DMAs and the MFMAs, so their latency overlaps the K loop (issued
    // in the epilogue they stalled each half for a full HBM round trip).  They are older than the
    // stage's DMAs, so the compiler's wait for them leaves the ring's counted vmcnt intact.  The
    // wider-WN tiles have no registers for it (they would spill).
    constexpr bool HOIST = (EPI != PW_FWD) && (WN == 32);
    constexpr int HN = HOIST ? NPS : 1;
    u32x4 hrv[2][HN], hxv[2][HN];
    uint32_t hrmb[2][HN], hsmb[2][HN];
    if constexpr (HOIST) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int ps = 0; ps < HN; ++ps) {
          const int m = min(m0 + 32 * hf + ps * RPP + lane / CPRW, M - 1);
          const int64_t off = (int64_t)m * N + nch;
          const int64_t ro = EPI == PW_APPLY ? off : res_off(m);
          // (absent operands skipped -- uniform branches; the explicit wait before the epilogue covers every
          // path.  A null mask's 0xff is selected at the use.)
          if (a.residual) hrv[hf][ps] = __builtin_amdgcn_raw_buffer_load_b128(rrs, ro >= 0 ? (uint32_t)(ro * 2) : OOB, 0, 0);
          if constexpr (DG) {
            if (a.res_mask) hrmb[hf][ps] = __builtin_amdgcn_raw_buffer_load_b8(rmrs, (uint32_t)(off >> 3), 0, 0);
            if (bnx) hxv[hf][ps] = __builtin_amdgcn_raw_buffer_load_b128(xsrs, (uint32_t)(off * 2), 0, 0);
            if (bnb && a.st_mask) hsmb[hf][ps] = __builtin_amdgcn_raw_buffer_load_b8(smrs, (uint32_t)(off >> 3), 0, 0);
          }
        }
    }
    if (!DG && a.in_coef) {
      // BN + ReLU of the producer applied to the landed tile ONCE, cooperatively in LDS (every wave reads
      // the whole tile as its MFMA operand: transformed in each wave's registers it was done four times
      // -- the layer-1/2 kernels were VALU-bound).  Chunk c: K slab c / 256, row (c % 256) / 4, physical
      // 16-B chunk c % 4 = logical chunk ^ swizzle(row) (an involution).  Rows past M: relu(shift)
      // values that are never stored and kept out of the statistics.
      char* timg = smem + cur_slot * TILE;
#pragma unroll
      for (int q = 0; q < TILE / 16 / 256; ++q) {
        const int c = q * 256 + tid, kc = c / (BM * 4), rem = c % (BM * 4), row = rem >> 2, pc = rem & 3;
        const int lc = pc ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
        u32x4* pch = (u32x4*)(timg + kc * (BM * 64) + row * 64 + pc * 16);
        const f32x4* cs = (const f32x4*)(bnin + 32 * kc + 8 * lc);
        const f32x4* chh = (const f32x4*)(bnin + K + 32 * kc + 8 * lc);
        const f32x4 s0 = cs[0], s1 = cs[1], h0 = chh[0], h1 = chh[1];
        const float sc8[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        const float sh8[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        float f[8];
        unpack8(*pch, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc8[e], sh8[e]), 0.f);
        *pch = pack8(f);
      }
      lds_barrier();
    }
    // (unconditional: past the stream's end a zero-filled DMA into the free slot -- see the resources above)
    issue(nxt_tile, nxt_slot);
    const char* img = smem + cur_slot * TILE;
    f32x4 acc[MI][NI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      bf16x8 xf[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) xf[mi] = kfrag(img + kc * (BM * 64), 16 * mi);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ni][kc], xf[mi], acc[mi][ni], 0, 0, 0);
    }
    // y rows: lane holds channels n0w + 16 ni + 4 g + e of pixel m0 + 16 mi + li; staged per
    // 32-row half through the wave's LDS region (LDS ops of one wave complete in order, so the
    // next half's writes never overtake this half's reads), then finished per 16-B row chunk
    char* stg = smem + NS * TILE + wid * STG;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // the half's epilogue operands first: their latency overlaps the staging below
      u32x4 rv[NPS], xv[NPS];
      uint32_t rmb[NPS], smb[NPS];
      if constexpr (HOIST) {
#pragma unroll
        for (int ps = 0; ps < HN; ++ps) {
          rv[ps] = hrv[hf][ps];
          xv[ps] = hxv[hf][ps];
          rmb[ps] = a.res_mask ? hrmb[hf][ps] : 0xffu;
          smb[ps] = (bnb && a.st_mask) ? hsmb[hf][ps] : 0xffu;
        }
      } else if constexpr (DG) {
#pragma unroll
        for (int ps = 0; ps < NPS; ++ps) {
          const int m = min(m0 + 32 * hf + ps * RPP + lane / CPRW, M - 1);
          const int64_t off = (int64_t)m * N + nch;
          if (a.residual) {
            const int64_t ro = res_off(m);
            rv[ps] = ro >= 0 ? *(const u32x4*)(a.residual + ro) : u32x4{0u, 0u, 0u, 0u};
          }
          rmb[ps] = a.res_mask ? (uint32_t)a.res_mask[off >> 3] : 0xffu;
          if (bnx) xv[ps] = *(const u32x4*)(a.st_x + off);
          smb[ps] = (bnb && a.st_mask) ? (uint32_t)a.st_mask[off >> 3] : 0xffu;
        }
      }
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        const int mi = 2 * hf + mh;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          u32x2 pk;
          pk[0] = pack_bf2(acc[mi][ni][0], acc[mi][ni][1]);
          pk[1] = pack_bf2(acc[mi][ni][2], acc[mi][ni][3]);
          *(u32x2*)(stg + (16 * mh + li) * ROWB + (16 * ni + 4 * g) * 2) = pk;
        }
      }
      // the hoisted epilogue operands (both halves): everything but the P ring DMAs issued after them has
      // landed.  (The DMA issue is unconditional, so P younger ops exist on every path; with this counted
      // wait the compiler needs no wait of its own for the conditionally loaded operands.)
      if (HOIST && hf == 0) wait_vm<P>();
#pragma unroll
      for (int ps = 0; ps < NPS; ++ps) {
        const int row = ps * RPP + lane / CPRW;
        u32x4 v = *(const u32x4*)(stg + row * ROWB + ch * 16);
        const int m = m0 + 32 * hf + row;
        const bool valid = m < M;
        float f[8];
        unpack8(v, f);
        if constexpr (EPI == PW_APPLY) {
          // y = relu(v * scale + shift + residual) from the rounded conv output v, as bn_apply /
          // bn_apply2 compute it from the stored pre-BN tensor (a BN'd residual rounded to bf16 first)
          float r[8];
          if (a.residual) unpack8(rv[ps], r);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float t = fmaf(f[e], osc[e], osh[e]);
            if (a.residual) t += a.res_coef ? bf2f(f2bf(fmaf(r[e], rsc[e], rsh[e]))) : r[e];
            f[e] = fmaxf(t, 0.f);
          }
          v = pack8(f);
          if constexpr (HOIST)
            __builtin_amdgcn_raw_buffer_store_b8(relu_mask_byte(v), obrs, valid ? (uint32_t)(((int64_t)m * N + nch) >> 3) : OOB, 0, 0);
          else if (valid && a.out_bits)
            a.out_bits[((int64_t)m * N + nch) >> 3] = relu_mask_byte(v);
        } else if constexpr (EPI == PW_FWD) {
          // statistics of the stored (rounded) values (rows past M: zeros, or relu(shift) terms
          // with in_coef -- masked)
          const float vm = valid ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float fv = f[e] * vm;
            s[e] += fv;
            ss[e] = fmaf(fv, fv, ss[e]);
          }
        } else {
          if (a.residual) {  // + residual (dz of a BN + residual + ReLU output: masked by its bits)
            float r[8];
            unpack8(rv[ps], r);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += ((rmb[ps] >> e) & 1u) ? r[e] : 0.f;
            v = pack8(f);
            unpack8(v, f);
          }
          if (bnb && valid) {  // (sum dz, sum dz*(x - mean)), dz = v * relu'(BN output)
            float x8[8];
            if (bnx) unpack8(xv[ps], x8);
            if (a.st_mask) {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                f[e] = ((smb[ps] >> e) & 1u) ? f[e] : 0.f;
                s[e] += f[e];
                if (bnx) ss[e] = fmaf(f[e], x8[e] - bmu[e], ss[e]);
              }
              v = pack8(f);  // the stored gradient is dz itself
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float dz = fmaf(x8[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
                s[e] += dz;
                ss[e] = fmaf(dz, x8[e] - bmu[e], ss[e]);
              }
            }
          }
        }
        if constexpr (HOIST) __builtin_amdgcn_raw_buffer_store_b128(v, yrs, valid ? (uint32_t)(((int64_t)m * N + nch) * 2) : OOB, 0, 0);
        else if (valid) *(u32x4*)(a.y + (int64_t)m * N + nch) = v;
      }
    }
  };
  // statistics: reduce over the lanes holding the same channel chunk (lane = row * CPRW + ch),
  // one partial column per row group
  auto flush_stats = [&](int col) {
    if (EPI != PW_APPLY && a.stats) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = CPRW; o < 64; o <<= 1) {
          s[e] += __shfl_xor(s[e], o, 64);
          ss[e] += __shfl_xor(ss[e], o, 64);
        }
      }
      if (lane < CPRW) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a.stats[(int64_t)(nch + e) * RG + col] = s[e];
          if (EPI != PW_DSUM) a.stats[(int64_t)(N + nch + e) * RG + col] = ss[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
    }
  };
  // Tile p of the block's stream landed.  In steady state NS-2 later tiles' DMAs and NS-1 tiles' stores
  // were issued after it (VM); a prologue tile p < NS-1 has only the NS-2 prologue DMAs and p tiles'
  // stores behind it, so it waits for fewer (a larger count would let the wave read a tile still in
  // flight); near the end fewer DMAs follow -> vmcnt(0).  (Any extra younger memory op -- a claim, a
  // statistics store -- only makes a count stricter.)
  auto ring_wait = [&](int p, bool ending) {
    if (ending) wait_vm<0>();
    else if (p == 0) wait_vm<(NS - 2) * P>();
    else if (NS >= 3 && p == 1) wait_vm<S + (NS - 2) * P>();
    else if (NS >= 4 && p == 2) wait_vm<2 * S + (NS - 2) * P>();
    else wait_vm<VM>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile p are in; slot (p-1)%NS is free
    asm volatile("" ::: "memory");
  };

  // the preamble's loads (weights, coefficients -- some under uniform branches) retired here, before the
  // ring starts: left pending, the compiler's first-use waits for them sat inside the tile loop as vmcnt(0),
  // which also waits for the ring's in-flight DMAs every tile
  wait_vm<0>();
  if constexpr (!DYN) {
    // static: this row group's tiles rg, rg + RG, ...
    const int nt = rg < tiles ? (tiles - 1 - rg) / RG + 1 : 0;
#pragma unroll
    for (int j = 0; j < NS - 1; ++j)
      if (j < nt) issue(rg + j * RG, j);
    for (int j = 0; j < nt; ++j) {
      ring_wait(j, j + NS - 2 >= nt);
      tile_body((rg + j * RG) * BM, j % NS, j + NS - 1 < nt ? rg + (j + NS - 1) * RG : -1, (j + NS - 1) % NS);
    }
    flush_stats(rg);
  } else {
    // Dynamic: one continuous tile stream over the row groups this block runs -- the static one, then
    // row groups claimed per column slice from counter nb, each claimed near the end of the previous one
    // but early enough that the ring never drains at a row-group boundary (every row group has >= NS + 3
    // tiles: pw_plan).  A row group's tiles, their summation order and its partial column do not depend
    // on which block runs it: results are schedule-independent, bitwise.
    auto ntiles = [&](int u) { return (tiles - 1 - u) / RG + 1; };
    int cu = rg, ntc = ntiles(cu), jc = 0;  // consumption: row group, its tile count, index
    int nu = -2;                            // the next row group (-2: not yet known, -1: none)
    int iu = cu, ij = 0;                    // issue cursor: row group, index
    int p = 0;                              // stream position being consumed
    int claimv = 0;                         // tid 0: the in-flight claim
    auto next_issue = [&]() -> int {        // tile at the issue cursor (advancing it), or -1
      if (iu < 0) return -1;
      if (ij == ntiles(iu)) {
        iu = iu == cu ? nu : -1;  // (the cursor never runs more than one row group ahead)
        ij = 0;
        if (iu < 0) return -1;
      }
      return iu + (ij++) * RG;
    };
    int issued = 0;
#pragma unroll
    for (int j = 0; j < NS - 1; ++j) {
      const int t = next_issue();
      if (t >= 0) { issue(t, j); ++issued; }
    }
    while (true) {
      ring_wait(p, issued < p + NS - 1);
      // the claim for the next row group is issued 8 + NS tiles before this one ends (late: a block that
      // claimed at the start of a row group would hold its next one while still slow; early enough that
      // the agent-scope atomic -- microseconds -- has returned when wave 0 publishes it), published
      // NS + 1 tiles before the end and read after the next barrier, one tile before the issue cursor
      // crosses over
      const int jpub = ntc - (NS + 1), jcl = max(0, jpub - 7);
      if (jc == jcl && tid == 0)
        claimv = SRG + (int)__hip_atomic_fetch_add(a.sched + nb * 256, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (jc == jpub && tid == 0) *claim_slot = claimv;  // published by the next barrier
      if (jc == jpub + 1) {
        const int c = __builtin_amdgcn_readfirstlane(*claim_slot);
        nu = c < RG ? c : -1;
      }
      const int t = next_issue();
      if (t >= 0) ++issued;
      tile_body((cu + jc * RG) * BM, p % NS, t, (p + NS - 1) % NS);
      ++p;
      if (++jc == ntc) {
        flush_stats(cu);
        if (nu < 0) break;
        cu = nu;
        ntc = ntiles(cu);
        jc = 0;
        nu = -2;
      }
    }
    if (tid == 0) {
      // the last block out re-zeroes the counters for the next launch on this stream (every block's final,
      // failed claim precedes its exit count, so no claim follows the reset)
      if (__hip_atomic_fetch_add(a.sched + 16 * 256, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
        for (int k = 0; k < nbN; ++k) __hip_atomic_store(a.sched + k * 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.sched + 16 * 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Concatenated-K data grad (PwCatArgs, pwconv.h): y = [dz | relu(BN2(h2))] . Bcat + e, + BN2-backward
// partials.  NW = K2 / 16 waves, wave w owning output channels 16 w .. +15 for the whole launch (their
// Bcat columns gathered once into VGPRs as MFMA A operands: KC = (K1 + K2) / 32 fragments).  Row tiles of
// CBM = 32 rows stream through an NS-deep LDS ring by LDS-DMA: K1 / 32 dz images then K2 / 32 raw h2
// images, each [32 rows][64 B] with the kimg swizzle.  Per tile the raw h2 images are transformed ONCE,
// cooperatively, into a separate a2 image (relu(h2 s + t), rounded to bf16 as every on-load BN here); the
// MFMAs read dz / a2 fragments; the epilogue adds e, rounds, and takes the BN2 mask and h2 - mean from the
// RAW h2 images still in the ring slot -- no second HBM read of h2.  One partial column per block.
constexpr int CBM = 32;
template <int K1, int K2, int NS>
__global__ __launch_bounds__(64 * (K2 / 16), K2 == 64 ? 2 : 1) void pw_cat_kernel(PwCatArgs a) {
  constexpr int NW = K2 / 16, NT = 64 * NW, N = K2;
  constexpr int KC1 = K1 / 32, KC2 = K2 / 32, KC = KC1 + KC2;
  constexpr int IMG = CBM * 64;               // one 32-K image of a tile
  constexpr int TILE = KC * IMG;
  constexpr int P = KC * 2 / NW;              // 1-KiB DMA pieces per wave per tile
  static_assert(P * NW == KC * 2, "piece split");
  constexpr int ROWB = 16 * 2 + 16;           // staged output row: 16 channels + pad
  constexpr int STG = CBM * ROWB;             // per wave
  constexpr int S = 1;                        // stores per lane per tile (32 rows x 2 chunks / 64 lanes)
  constexpr int VM = (NS - 1) * S + (NS - 2) * P;
  static_assert(VM < 64, "vmcnt range");
  // one LDS object (see pw_stream_kernel): ring, a2 image, staging, BN2's [scale | shift]
  __shared__ __attribute__((aligned(16))) char smem[NS * TILE + KC2 * IMG + NW * STG + 2 * K2 * 4];
  float* const bnin = (float*)(smem + NS * TILE + KC2 * IMG + NW * STG);
  char* const a2img = smem + NS * TILE;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = (int)a.M, RG = a.rg;
  const int tiles = (M + CBM - 1) / CBM;
  const int n0w = wid * 16;
  char* const stg = smem + NS * TILE + KC2 * IMG + wid * STG;
  auto swz = [](int row) { return (0x78 >> (((row >> 2) & 3) << 1)) & 3; };

  // Bcat columns of the wave's 16 channels: wf[kc] = A rows n0w + li, K = 32 kc + 8 g .. +7
  bf16x8 wf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    s16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)a.bcat[(int64_t)(32 * kc + 8 * g + e) * N + n0w + li];
    wf[kc] = __builtin_bit_cast(bf16x8, v);
  }
  // epilogue lane map: pixel row lane >> 1 of the 32, 8 channels nch = n0w + 8 (lane & 1)
  const int erow = lane >> 1, nch = n0w + 8 * (lane & 1);
  float eb[4], bsc[8], bsh[8], bmu[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) eb[e] = a.ebias[n0w + 4 * g + e];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bsc[e] = a.coef[nch + e];
    bsh[e] = a.coef[K2 + nch + e];
    bmu[e] = a.coef[2 * K2 + nch + e];
  }
  for (int i = tid; i < 2 * K2; i += NT) bnin[i] = a.coef[i];

  // DMA: piece q (of 2 KC per tile) = image q >> 1, rows 16 (q & 1) .. +15; lane -> (row, 16-B chunk)
  const __amdgpu_buffer_rsrc_t r1 = rsrc(a.dz, (uint32_t)((int64_t)M * K1 * 2));
  const __amdgpu_buffer_rsrc_t r2 = rsrc(a.h2, (uint32_t)((int64_t)M * K2 * 2));
  uint32_t voff[P];
  int prow[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int q = wid * P + i, kc = q >> 1, row = (q & 1) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ swz(row);
    prow[i] = row;
    voff[i] = kc < KC1 ? (uint32_t)(row * K1 * 2 + kc * 64 + lc * 16) : (uint32_t)(row * K2 * 2 + (kc - KC1) * 64 + lc * 16);
  }
  auto issue = [&](int t, int slot) {
    char* dst = smem + slot * TILE;
    const int valid_rows = M - t * CBM;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int q = wid * P + i, kc = q >> 1;
      if (kc < KC1) {
        const uint32_t v = prow[i] < valid_rows ? voff[i] + (uint32_t)t * (CBM * K1 * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_void_t*)(dst + q * 1024), 16, v, 0, 0, 0);
      } else {
        const uint32_t v = prow[i] < valid_rows ? voff[i] + (uint32_t)t * (CBM * K2 * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_void_t*)(dst + q * 1024), 16, v, 0, 0, 0);
      }
    }
  };
  auto ring_wait = [&](int p, bool ending) {  // as pw_stream_kernel's
    if (ending) wait_vm<0>();
    else if (p == 0) wait_vm<(NS - 2) * P>();
    else if (NS >= 3 && p == 1) wait_vm<S + (NS - 2) * P>();
    else wait_vm<VM>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
  const int rgb = blockIdx.x;
  const int nt = rgb < tiles ? (tiles - 1 - rgb) / RG + 1 : 0;
  wait_vm<0>();  // the preamble's loads retired before the ring starts (see pw_stream_kernel)
  __syncthreads();  // bnin
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nt) issue(rgb + j * RG, j);
  for (int j = 0; j < nt; ++j) {
    ring_wait(j, j + NS - 2 >= nt);
    const int slot = j % NS, m0 = (rgb + j * RG) * CBM;
    if (j + NS - 1 < nt) issue(rgb + (j + NS - 1) * RG, (j + NS - 1) % NS);
    const char* img = smem + slot * TILE;
    // raw h2 images -> a2 image (same physical positions), once per tile
#pragma unroll
    for (int c = tid; c < KC2 * CBM * 4; c += NT) {
      const int kc2 = c / (CBM * 4), rem = c % (CBM * 4), row = rem >> 2, pc = rem & 3;
      const int lc = pc ^ swz(row);
      const int off = kc2 * IMG + row * 64 + pc * 16;
      const f32x4* cs = (const f32x4*)(bnin + 32 * kc2 + 8 * lc);
      const f32x4* ch = (const f32x4*)(bnin + K2 + 32 * kc2 + 8 * lc);
      const f32x4 s0 = cs[0], s1 = cs[1], h0 = ch[0], h1 = ch[1];
      const float sc8[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float sh8[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      float f[8];
      unpack8(*(const u32x4*)(img + KC1 * IMG + off), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc8[e], sh8[e]), 0.f);
      *(u32x4*)(a2img + off) = pack8(f);
    }
    lds_barrier();
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const char* im = kc < KC1 ? img + kc * IMG : a2img + (kc - KC1) * IMG;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) acc[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kc], kfrag(im, 16 * mi), acc[mi], 0, 0, 0);
    }
    // stage (lane: channels n0w + 4 g + e of pixel row 16 mi + li), + e, rounded
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      u32x2 pk;
      pk[0] = pack_bf2(acc[mi][0] + eb[0], acc[mi][1] + eb[1]);
      pk[1] = pack_bf2(acc[mi][2] + eb[2], acc[mi][3] + eb[3]);
      *(u32x2*)(stg + (16 * mi + li) * ROWB + (4 * g) * 2) = pk;
    }
    const u32x4 v = *(const u32x4*)(stg + erow * ROWB + (lane & 1) * 16);
    const int m = m0 + erow;
    if (m < M) {
      float f[8], x8[8];
      unpack8(v, f);
      const int kc2 = nch >> 5, lc = (nch & 31) >> 3;
      unpack8(*(const u32x4*)(img + (KC1 + kc2) * IMG + erow * 64 + ((lc ^ swz(erow)) << 4)), x8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = fmaf(x8[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
        s[e] += dz;
        ss[e] = fmaf(dz, x8[e] - bmu[e], ss[e]);
      }
      *(u32x4*)(a.y + (int64_t)m * N + nch) = v;
    }
  }
  // one partial column per block: reduce over the lanes holding the same chunk (lane & 1)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {
      s[e] += __shfl_xor(s[e], o, 64);
      ss[e] += __shfl_xor(ss[e], o, 64);
    }
  }
  if (lane < 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a.stats[(int64_t)(nch + e) * RG + rgb] = s[e];
      a.stats[(int64_t)(N + nch + e) * RG + rgb] = ss[e];
    }
  }
}

}  // namespace pw
}  // namespace dpe

using namespace dpe;

extern "C" int dpe_cu_reserve();  // comm.cpp

// blocks of the concatenated-K data grad: the resident capacity (2 x 4-wave blocks per CU at K2 = 64,
// 1 x 8-wave at 128), twice that while a CU budget is in force (two dispatch rounds: the CUs that share
// with RCCL's blocks get fewer); 0 outside (K1, K2) in {(256, 64), (512, 128)} or a row count whose
// 32-bit byte offsets would overflow.
extern "C" int dpe_pw_cat_blocks(int64_t M, int64_t K1, int64_t K2) {
  static const bool on = [] { const char* e = getenv("DPE_PW_CAT"); return !(e && e[0] == '0'); }();
  if (!on || !((K1 == 256 && K2 == 64) || (K1 == 512 && K2 == 128))) return 0;
  if (M <= 0 || M * K1 * 2 >= (1ll << 31) - 4096) return 0;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int per = K2 == 64 ? 2 : 1;
  const int64_t tiles = (M + pw::CBM - 1) / pw::CBM;
  const int64_t nb = (int64_t)std::max(1, cus) * per * (dpe_cu_reserve() > 0 ? 2 : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>(nb, tiles));
}

extern "C" int dpe_pw_cat_launch(const PwCatArgs* args, int64_t K1, int64_t K2, hipStream_t st) {
  const PwCatArgs& a = *args;
  if (a.rg <= 0 || a.rg != dpe_pw_cat_blocks(a.M, K1, K2)) return -1;
  if (K1 == 256 && K2 == 64) hipLaunchKernelGGL((pw::pw_cat_kernel<256, 64, 3>), dim3(a.rg), dim3(256), 0, st, a);
  else if (K1 == 512 && K2 == 128) hipLaunchKernelGGL((pw::pw_cat_kernel<512, 128, 3>), dim3(a.rg), dim3(512), 0, st, a);
  else return -1;
  return 0;
}

extern "C" int dpe_cu_reserve();  // comm.cpp

// columns per wave.  The data grads at K = 64 / 128 use 32 (like K = 256) so that the epilogue operands
// (residual, pre-BN input, masks) can be hoisted ahead of the tile's MFMAs: with 64 columns per wave
// they were loaded in the epilogue and each half-tile stalled a full HBM round trip (layer-2 conv1
// data grads ran at ~61 % of their HBM roofline).
#ifndef DPE_PW64_DGRAD_WN
#define DPE_PW64_DGRAD_WN 32  // (64: the previous layout, for A/B)
#endif
// The forward (stats-only epilogue, no operand loads) keeps 64 columns per wave: 32 measured slower
// at K = 64 and 128 (ResNet-50 +0.1-0.2 ms/step: each row tile's DMA and BN-on-load transform then
// run in twice as many blocks); the defines are the compile-time A/B arms.
#ifndef DPE_PW64_FWD_WN
#define DPE_PW64_FWD_WN 64
#endif
#ifndef DPE_PW128_FWD_WN
#define DPE_PW128_FWD_WN 64
#endif
static int pw_wn(int K, int epi) {
  if (epi == PW_APPLY) return 32;  // epilogue operand (the residual) hoisted ahead of the MFMAs, as the data grads
  if (epi == PW_DSUM) epi = PW_DGRAD;
  if (K == 64) return epi == PW_DGRAD ? DPE_PW64_DGRAD_WN : DPE_PW64_FWD_WN;
  if (K == 128) return epi == PW_FWD ? DPE_PW128_FWD_WN : 32;
  return 32;
}

// Every block carries the same number of tiles, so the grid must be exactly the resident
// capacity (blocks per CU from the occupancy API x CUs): a grid that lets the dispatcher put
// 3 blocks on some CUs and 1 on others finishes at the pace of the fullest CU.
template <int K, int WN, int NS, int EPI, bool DYN>
static int pw_slots() {
  static int slots = [] {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pw::pw_stream_kernel<K, WN, NS, EPI, DYN>, 256, 0);
    return std::max(1, per) * std::max(1, cus);
  }();
  return slots;
}
// resident blocks of the static (DYN = false) or the dynamic-schedule variant
template <int EPI, bool DYN = false>
static int pw_capacity(int K) {
  if constexpr (EPI == PW_APPLY || EPI == PW_DSUM) {
    if (K == 64) return pw_slots<64, 32, 4, EPI, DYN>();
    if (K == 128) return pw_slots<128, 32, 3, EPI, DYN>();
    return pw_slots<256, 32, 2, EPI, DYN>();
  } else {
    if (K == 64) return EPI == PW_FWD ? pw_slots<64, DPE_PW64_FWD_WN, 4, EPI, DYN>() : pw_slots<64, DPE_PW64_DGRAD_WN, 4, EPI, DYN>();
    if (K == 128) return EPI == PW_FWD ? pw_slots<128, DPE_PW128_FWD_WN, 3, EPI, DYN>() : pw_slots<128, 32, 3, EPI, DYN>();
    return pw_slots<256, 32, 2, EPI, DYN>();
  }
}

// DPE_PW_DYNAMIC=0: the static schedule under a CU budget too (A/B)
static bool pw_dynamic() {
  static const bool on = [] { const char* e = getenv("DPE_PW_DYNAMIC"); return !(e && e[0] == '0'); }();
  return on;
}

template <bool DYN>
static int pw_cap(int64_t K, int epi) {
  return epi == PW_FWD ? pw_capacity<PW_FWD, DYN>((int)K)
                       : epi == PW_APPLY ? pw_capacity<PW_APPLY, DYN>((int)K)
                       : epi == PW_DSUM  ? pw_capacity<PW_DSUM, DYN>((int)K) : pw_capacity<PW_DGRAD, DYN>((int)K);
}

// Row groups of a launch: rg (= partial columns) and srg, the row groups started statically (the grid is
// srg x nbN blocks).  srg == rg: static schedule, one resident wave of blocks over the whole launch,
// sized to the resident capacity minus the slots left to in-flight RCCL channel blocks (comm.cpp CU
// budget).  srg < rg (CU budget in force): the dynamic variant, rg = 8 srg row groups of >= 7 tiles each
// (>= NS + 3: the stream claims the next row group NS + 2 tiles before the current one ends).
struct PwPlan { int rg, srg; };
static PwPlan pw_plan(int64_t M, int64_t N, int64_t K, int epi) {
  if (K != 64 && K != 128 && K != 256) return {0, 0};
  if (epi != PW_FWD && epi != PW_DGRAD && epi != PW_APPLY && epi != PW_DSUM) return {0, 0};
  const int bnb = 4 * pw_wn((int)K, epi);
  if (N % bnb || N < 2 * K) return {0, 0};  // write-heavy shapes only (N >= 2K)
  if (M * K * 2 >= (1ll << 31) - 4096 || M * N >= (1ll << 31) - 256) return {0, 0};
  const int64_t tiles = (M + pw::BM - 1) / pw::BM;
  const int64_t nbN = N / bnb;
  const int reserve = dpe_cu_reserve();
  if (reserve > 0 && pw_dynamic()) {
    const int64_t srg = std::max<int64_t>(1, (pw_cap<true>(K, epi) - reserve) / nbN);
    // (an eighth static, the rest claimed: a block two or three times slower than its peers -- a
    // VALU-bound foreign wave on its SIMD -- ends its static row group well before the launch's end, and
    // the launch's tail is one short row group at its speed.  Worst-case hog probe, same box: 8 vs 3 row
    // groups per resident block 36.41 / 36.56 vs 36.92 / 37.10 ms/step, 16 twice 36.49 / 36.92 -- the
    // >= 7-tile floor binds at layers 3-4; DPE_PW_DYN_FACTOR: A/B)
    static const int64_t fac = [] { const char* e = getenv("DPE_PW_DYN_FACTOR"); return (int64_t)(e ? std::max(2, atoi(e)) : 8); }();
    const int64_t rg = std::min<int64_t>(fac * srg, tiles / 7);
    if (rg > srg) return {(int)rg, (int)srg};
  }
  int64_t rg = (pw_cap<false>(K, epi) - reserve) / nbN;
  rg = std::max<int64_t>(1, std::min<int64_t>(rg, tiles));
  return {(int)rg, (int)rg};
}

extern "C" int dpe_pw_rowgroups(int64_t M, int64_t N, int64_t K, int epi) { return pw_plan(M, N, K, epi).rg; }

extern "C" int dpe_pw_launch(const PwArgs* args, int epi, hipStream_t st) {
  const PwArgs& a = *args;
  if (a.rg <= 0 || a.rg != dpe_pw_rowgroups(a.M, a.N, a.K, epi)) return -1;
  if (epi == PW_FWD && (a.residual || a.st_x)) return -1;
  if (a.st_x && !a.st_coef) return -1;
  if (epi == PW_DSUM && (a.st_x || !a.st_mask || !a.stats)) return -1;
  if (epi == PW_APPLY && (!a.out_coef || a.st_x || a.stats || a.res_h > 0 || (a.res_coef && !a.residual))) return -1;
  if (a.res_h > 0 && ((epi != PW_DGRAD && epi != PW_DSUM) || a.res_mask || a.res_h % 2 || a.res_w % 2 || a.M % ((int64_t)a.res_h * a.res_w)))
    return -1;
  // resident row groups: all of them, or (CU budget in force) the first half, the rest claimed
  // (no claim counters -- a stream being captured: the static variant over all rg row groups)
  const int srg = a.sched ? pw_plan(a.M, a.N, a.K, epi).srg : a.rg;
  const bool dyn = srg < a.rg;
  const int wn = pw_wn((int)a.K, epi);
  const dim3 grid((unsigned)(srg * (a.N / (4 * wn)))), block(256);
#define PW_GO(K_, WN_, NS_, E_)                                                                            \
  if (a.K == K_ && wn == WN_ && epi == E_) {                                                             \
    if (dyn) hipLaunchKernelGGL((pw::pw_stream_kernel<K_, WN_, NS_, E_, true>), grid, block, 0, st, a);    \
    else hipLaunchKernelGGL((pw::pw_stream_kernel<K_, WN_, NS_, E_, false>), grid, block, 0, st, a);       \
    return 0;                                                                                            \
  }
  PW_GO(64, 32, 4, PW_APPLY) PW_GO(128, 32, 3, PW_APPLY) PW_GO(256, 32, 2, PW_APPLY)
  PW_GO(64, 32, 4, PW_DSUM) PW_GO(128, 32, 3, PW_DSUM) PW_GO(256, 32, 2, PW_DSUM)
  PW_GO(64, DPE_PW64_DGRAD_WN, 4, PW_DGRAD) PW_GO(64, DPE_PW64_FWD_WN, 4, PW_FWD)
  PW_GO(128, 32, 3, PW_DGRAD) PW_GO(128, DPE_PW128_FWD_WN, 3, PW_FWD)
  PW_GO(256, 32, 2, PW_DGRAD) PW_GO(256, 32, 2, PW_FWD)
#undef PW_GO
  return -1;
}
