// Causal flash attention for GPT-2 (head dim 64) on gfx950 bf16 MFMA
// (v_mfma_f32_16x16x32_bf16).  qkv is the QKV projection output [B, T, 3, H, 64]
// (no split/transpose copies); out is [B, T, H, 64] (feeds the out-projection).
//
// Every wave owns 32 rows (two 16-row MFMA blocks) of the dimension it keeps on the
// lane, so each K/V (or Q/dO) fragment read from LDS feeds two MFMAs: with 16 rows per
// wave the 1 KiB-per-MFMA operand stream alone saturated the 256 B/clk LDS array.
//
// Forward (one workgroup = 128 queries of one (b, h), 4 waves x 32 queries, 64-key tiles):
//   S^T = K . Q^T with K as the A operand, so each lane holds ONE query (lane&15) of each
//   16-query block and 16 keys in registers: the online-softmax max/sum are lane-local
//   plus two permlane swaps (cdna_hip_programming.md App. B, "swapped QK^T").
//   P is converted to bf16 in registers and used directly as the B operand of
//   O^T += V^T . P; the key order inside each 32-key MFMA step is permuted
//   ({4g..4g+3} u {16+4g..}) and the V operand is read with transposing
//   ds_read_b64_tr_b16 from exactly those rows (§3 "accumulator tile as the
//   next MFMA's operand").  K/V tiles are register-prefetched one tile ahead
//   into double-buffered, XOR-swizzled LDS.  The running max is only moved when a
//   row's new maximum exceeds it by more than 2^8 (T13 "defer-max": P <= 256, exact
//   after the final 1/l), so the O rescale is skipped wave-uniformly on most tiles.
//   Waves skip key tiles that lie entirely above their causal diagonal.  Heaviest
//   (latest) query tiles are scheduled first.  Saves lse2 = m + log2(l) (log2 units,
//   scale folded).
// Backward = two kernels:
//   dK/dV (one workgroup = 128 keys, 4 waves x 32 keys; loops over 64-query tiles):
//   key-on-the-lane: S = Q.K^T and dP = dO.V^T have the key on the lane, so
//   their accumulators ARE the B operands of dV^T += dO^T.P and
//   dK^T += Q^T.dS (permuted-k trick again, Q/dO read transposed from LDS,
//   double-buffered, one barrier per tile).
//   dQ (one workgroup = 128 queries; loops over key tiles; runs first and also writes
//   delta = rowsum(dO*O) for the dK/dV kernel): the forward's query-on-lane structure
//   recomputing S and dP; dQ^T += K^T.dS^T.  Both kernels start the dP accumulation
//   from -delta, so dS = P*(dP - delta) is one multiply.  Two
//   extra MFMA passes replace fp32 dQ atomics across key tiles (the chip's
//   ~1.3 TB/s atomic rate: ~210 MB per layer).
#include <type_traits>

#include "common.h"

namespace dpe {

constexpr int AD = 64;      // head dim
constexpr int AQ = 64;      // queries per dK/dV loop tile
constexpr int AKV = 64;     // keys per forward / dQ loop tile
constexpr int FQ = 128;     // queries per forward / dQ workgroup (4 waves x 32)
constexpr int BKW = 128;    // keys per dK/dV workgroup (4 waves x 32)
constexpr float RESCALE_TH = 8.f;  // log2 units: defer the running-max update below 2^8

typedef __attribute__((address_space(3))) s16x4 lds4;

// [64 rows][32 bf16] K-contiguous image (64-B rows), swizzled for ds_read_b128 (as igemm)
DPE_DEVICE int kimg(int row, int chunk) {
  const int g = (0x78 >> (((row >> 2) & 3) << 1)) & 3;
  return row * 64 + ((chunk ^ g) << 4);
}
// [rows][64 bf16] image (128-B rows) read transposed, permuted-key rows {4g+q, 16+4g+q}:
// conflict-free with h = 2*((k>>1)&3)
DPE_DEVICE int pimg(int k, int chunk) {
  const int h = ((k >> 1) & 3) << 1;
  return k * 128 + ((chunk ^ h) << 4);
}

DPE_DEVICE bf16x8 kfrag64(const char* img, int r0) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15);
  return __builtin_bit_cast(bf16x8, *(const u32x4*)(img + kimg(row, lane >> 4)));
}

// A/B operand with k = rows k0 + {4g+q, 16+4g+q} (permuted), cols c0..c0+15 = lane&15
DPE_DEVICE bf16x8 trfrag(const char* img, int k0, int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r1 = k0 + 4 * g + q, r2 = r1 + 16;
  const int ch = (c0 >> 3) + (p >> 1), sub = (p & 1) * 8;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + pimg(r1, ch) + sub));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(img + pimg(r2, ch) + sub));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

DPE_DEVICE bf16x8 pack_frag(const f32x4& a, const f32x4& b) {
  u32x4 u;
  u[0] = pack_bf2(a[0], a[1]); u[1] = pack_bf2(a[2], a[3]);
  u[2] = pack_bf2(b[0], b[1]); u[3] = pack_bf2(b[2], b[3]);
  return __builtin_bit_cast(bf16x8, u);
}

// No inline asm here: an asm consumer of a v_exp_f32 / MFMA result gets none of the wait states
// the compiler inserts for its own instructions (gfx950 transcendental-use and MFMA-read hazards).
// Single-issue max / add / mul come from this file's build flags instead (_build.py FILE_FLAGS:
// no NaN-quieting canonicalisation before v_max, no SLP packing into v_pk_*_f32).
DPE_DEVICE float rowmax4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
DPE_DEVICE float rowsum4(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// K (two d-halves, K-contiguous) and V (permuted-row image) of one 64-key tile:
// global -> registers (one tile ahead) -> LDS.  Chunk c in [0,512): key = c>>3, dchunk = c&7.
// The per-thread row pointers are formed once; a tile step adds a wave-uniform offset.
struct KVStage {
  u32x4 rk[2], rv[2];
  const uint16_t* pk[2];
  int64_t vdelta, tstep;  // V - K distance, one tile's row advance (elements)
  DPE_DEVICE void init(const uint16_t* kb, const uint16_t* vb, int64_t RS) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + 256 * i, key = c >> 3, dc = c & 7;
      pk[i] = kb + (int64_t)key * RS + dc * 8;
    }
    vdelta = vb - kb;
    tstep = (int64_t)AKV * RS;
  }
  DPE_DEVICE void load(int kt) {
    const int64_t off = kt * tstep;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      rk[i] = *(const u32x4*)(pk[i] + off);
      rv[i] = *(const u32x4*)(pk[i] + off + vdelta);
    }
  }
};

// ======================================================================= fwd
// 3 waves per SIMD (<= 168 VGPRs): all 768 workgroups of the GPT-2 shape resident at once
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_fwd_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                                       float* __restrict__ lse2, int B, int T, int H, float sl2) {
  constexpr int KB = 2 * AKV * 64, STG = KB + AKV * 128;  // K halves 8K + V 8K per buffer
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nq = (T + FQ - 1) / FQ, BH = B * H;
  const int qt = nq - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const uint16_t* vb = qb + 2 * H * AD;
  const int q0w = qt * FQ + 32 * w;               // the wave's first query
  const bool live = q0w < T;                      // T % 64 == 0: a wave is all-valid or all-past-T
  const int ktw = live ? (q0w + 31) / AKV : -1;   // last key tile the wave needs
  const int nkt = min((qt * FQ + FQ - 1) / AKV, T / AKV - 1) + 1;

  bf16x8 qf[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      qf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(qb + (int64_t)(q0w + 16 * r + li) * RS + 32 * kk + 8 * g))
                       : bf16x8{};

  KVStage st;
  st.init(kb, vb, RS);
  auto lstore = [&](int buf) {
    char* s = smem + buf * STG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, key = c >> 3, dc = c & 7;
      *(u32x4*)(s + (dc >> 2) * (AKV * 64) + kimg(key, dc & 3)) = st.rk[i];
      *(u32x4*)(s + KB + pimg(key, dc)) = st.rv[i];
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[r][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};  // an inline-constant src2 for the first MFMA of each chain
  // key tiles below kd lie entirely at or below the wave's first query: no causal mask
  const int kd = (q0w + 1) / AKV;

  // one key tile: S^T, online softmax, O^T += V^T.P.  MASK (the diagonal tiles) is a separate
  // instantiation, so the common path is one basic block apart from the rare rescale branch.
  auto compute = [&](int kt, const char* s, auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;
    f32x4 sc[2][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16x8 k0 = kfrag64(s, 16 * nt), k1 = kfrag64(s + AKV * 64, 16 * nt);
#pragma unroll
      for (int r = 0; r < 2; ++r) sc[r][nt] = MFMA(k1, qf[r][1], MFMA(k0, qf[r][0], zero));
    }
    float mc[2];
    bool need[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if constexpr (MASK) {
        const int lim = q0w + 16 * r + li - kt * AKV - 4 * g;  // key offset e + 16nt allowed up to lim
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (16 * nt + e > lim) sc[r][nt][e] = -INFINITY;
      }
      float mx = sc[r][0][0];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = (nt == 0); e < 4; ++e) mx = fmaxf(mx, sc[r][nt][e]);
      mc[r] = rowmax4(mx) * sl2;
      need[r] = mc[r] > m[r] + RESCALE_TH;
    }
    if (__builtin_amdgcn_ballot_w64(need[0] || need[1])) {  // rare after the first tile
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float alpha = need[r] ? __builtin_amdgcn_exp2f(m[r] - mc[r]) : 1.f;
        m[r] = need[r] ? mc[r] : m[r];
        lsum[r] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] *= alpha;
      }
    }
    bf16x8 pk[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float nm = -m[r];
      float ps = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r][nt][e], sl2, nm));
          sc[r][nt][e] = pv;
          ps += pv;
        }
      lsum[r] += ps;
      pk[r][0] = pack_frag(sc[r][0], sc[r][1]);
      pk[r][1] = pack_frag(sc[r][2], sc[r][3]);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const bf16x8 v0 = trfrag(s + KB, 0, 16 * d), v1 = trfrag(s + KB, 32, 16 * d);
#pragma unroll
      for (int r = 0; r < 2; ++r) acc[r][d] = MFMA(v1, pk[r][1], MFMA(v0, pk[r][0], acc[r][d]));
    }
  };

  st.load(0);
  lstore(0);
  __syncthreads();
  // the tile loop unrolled by two: the LDS buffer of each step is a compile-time constant, so every
  // fragment address is a hoisted per-lane offset plus an immediate
  auto step = [&](int kt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = kt + 1 < nkt;
    if (more) st.load(kt + 1);
    if (kt < kd) compute(kt, smem + cur * STG, std::false_type{});
    else if (kt <= ktw) compute(kt, smem + cur * STG, std::true_type{});
    if (more) lstore(cur ^ 1);
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nkt) step(kt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int myq = q0w + 16 * r + li;
    const float l = rowsum4(lsum[r]);
    const float inv = 1.f / l;
    uint16_t* o = out + ((int64_t)(b * T + myq) * H + h) * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 pk2;
      pk2[0] = pack_bf2(acc[r][d][0] * inv, acc[r][d][1] * inv);
      pk2[1] = pack_bf2(acc[r][d][2] * inv, acc[r][d][3] * inv);
      *(u32x2*)(o + 16 * d + 4 * g) = pk2;
    }
    if (g == 0) lse2[(int64_t)bh * T + myq] = m[r] + __log2f(l);
  }
}

// Forward, VALU-lean form of attn_fwd_kernel.  The forward is VALU-throughput-bound per SIMD (three
// waves share one VALU; ~166 VALU vs 32 MFMA per 64-key tile and wave), so:
//  * the softmax row sum l comes from the MFMA unit: a constant all-ones A operand against the same
//    bf16 P fragments (4 extra MFMAs per tile) replaces 32 fp32 adds and the final cross-lane sum --
//    l is then the sum of exactly the rounded P that O accumulated;
//  * K/V go global -> LDS by LDS-DMA (no staging registers or ds_writes; the 8 accumulator registers
//    of l fit in 3 waves per SIMD).  Each lane fetches the chunk that the swizzled image places at its
//    slot (the XOR swizzles are involutions).
// (A software-pipelined variant -- next tile's S MFMAs issued under this tile's softmax, three LDS
// buffers -- measured 26.0 vs 26.2 us: the MFMA unit is not what the softmax waits on.)
typedef __attribute__((address_space(3))) void alds_void_t;
// LDS-DMA of one 16-B chunk per lane to wave_dst + 16 * lane, issued through inline asm so the
// compiler puts no vmcnt(0) drain in front of the LDS reads it cannot prove disjoint (as igemm.hip's
// dma16); the kernel orders it with its own vmcnt(0) before the step's barrier.  M0 is used by
// nothing else here.
DPE_DEVICE void attn_dma16(__amdgpu_buffer_rsrc_t r, char* wave_dst, uint32_t voff, uint32_t soff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(alds_void_t*)wave_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(m0), "v"(voff), "s"(r), "s"(soff) : "memory");
}
DPE_DEVICE void attn_vm_drain() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));  // vmcnt(0) only
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_fwd_dma_kernel(
    const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out, float* __restrict__ lse2, int B, int T, int H,
    float sl2) {
  constexpr int KB = 2 * AKV * 64, STG = KB + AKV * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nq = (T + FQ - 1) / FQ, BH = B * H;
  const int qt = nq - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const int q0w = qt * FQ + 32 * w;
  const bool live = q0w < T;
  const int ktw = live ? (q0w + 31) / AKV : -1;
  const int nkt = min((qt * FQ + FQ - 1) / AKV, T / AKV - 1) + 1;

  bf16x8 qf[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      qf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(qb + (int64_t)(q0w + 16 * r + li) * RS + 32 * kk + 8 * g))
                       : bf16x8{};

  // the sequence's qkv rows from K of head h on: one buffer resource, tile advance in soffset
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(kb), (short)0, (int)(T * RS * 2), 0x00020000);
  uint32_t voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = (w + 4 * i) * 1024 + lane * 16;  // this lane's byte slot in the 16 KiB tile image
    int key, dc, vo;
    if (i < 2) {  // K halves: kimg(key, c) = key * 64 + ((c ^ sw(key)) << 4), half dc >> 2
      const int dh = o >> 12, oo = o & 4095;
      key = oo >> 6;
      dc = 4 * dh + (((oo >> 4) & 3) ^ ((0x78 >> (((key >> 2) & 3) << 1)) & 3));
      vo = 0;
    } else {      // V: pimg(key, c) = key * 128 + ((c ^ h(key)) << 4)
      const int oo = o - KB;
      key = oo >> 7;
      dc = ((oo >> 4) & 7) ^ (((key >> 1) & 3) << 1);
      vo = H * AD;
    }
    voff[i] = (uint32_t)(((int64_t)key * RS + vo + dc * 8) * 2);
  }
  auto dma_tile = [&](int kt, char* s) {
    const uint32_t so = (uint32_t)((int64_t)kt * AKV * RS * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) attn_dma16(rs, s + (w + 4 * i) * 1024, voff[i], so);
  };

  f32x4 acc[2][4], accl[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    accl[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[r][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float m[2] = {-INFINITY, -INFINITY};
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  const int kd = (q0w + 1) / AKV;

  auto compute = [&](int kt, const char* s, auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;
    f32x4 sc[2][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16x8 k0 = kfrag64(s, 16 * nt), k1 = kfrag64(s + AKV * 64, 16 * nt);
#pragma unroll
      for (int r = 0; r < 2; ++r) sc[r][nt] = MFMA(k1, qf[r][1], MFMA(k0, qf[r][0], zero));
    }
    float mc[2];
    bool need[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if constexpr (MASK) {
        const int lim = q0w + 16 * r + li - kt * AKV - 4 * g;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (16 * nt + e > lim) sc[r][nt][e] = -INFINITY;
      }
      float mx = sc[r][0][0];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = (nt == 0); e < 4; ++e) mx = fmaxf(mx, sc[r][nt][e]);
      mc[r] = rowmax4(mx) * sl2;
      need[r] = mc[r] > m[r] + RESCALE_TH;
    }
    if (__builtin_amdgcn_ballot_w64(need[0] || need[1])) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float alpha = need[r] ? __builtin_amdgcn_exp2f(m[r] - mc[r]) : 1.f;
        m[r] = need[r] ? mc[r] : m[r];
        accl[r] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] *= alpha;
      }
    }
    bf16x8 pk[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float nm = -m[r];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) sc[r][nt][e] = __builtin_amdgcn_exp2f(fmaf(sc[r][nt][e], sl2, nm));
      pk[r][0] = pack_frag(sc[r][0], sc[r][1]);
      pk[r][1] = pack_frag(sc[r][2], sc[r][3]);
      accl[r] = MFMA(ones, pk[r][1], MFMA(ones, pk[r][0], accl[r]));
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const bf16x8 v0 = trfrag(s + KB, 0, 16 * d), v1 = trfrag(s + KB, 32, 16 * d);
#pragma unroll
      for (int r = 0; r < 2; ++r) acc[r][d] = MFMA(v1, pk[r][1], MFMA(v0, pk[r][0], acc[r][d]));
    }
  };

  dma_tile(0, smem);
  attn_vm_drain();
  __syncthreads();
  // the tile loop unrolled by two: each step's LDS buffer is a compile-time constant
  auto step = [&](int kt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = kt + 1 < nkt;
    if (more) dma_tile(kt + 1, smem + (cur ^ 1) * STG);  // read last in step kt - 1, before its barrier
    if (kt < kd) compute(kt, smem + cur * STG, std::false_type{});
    else if (kt <= ktw) compute(kt, smem + cur * STG, std::true_type{});
    if (more) attn_vm_drain();
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nkt) step(kt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int myq = q0w + 16 * r + li;
    const float l = accl[r][0];  // every row of the all-ones product is the sum over keys for query li
    const float inv = 1.f / l;
    uint16_t* o = out + ((int64_t)(b * T + myq) * H + h) * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 pk2;
      pk2[0] = pack_bf2(acc[r][d][0] * inv, acc[r][d][1] * inv);
      pk2[1] = pack_bf2(acc[r][d][2] * inv, acc[r][d][3] * inv);
      *(u32x2*)(o + 16 * d + 4 * g) = pk2;
    }
    if (g == 0) lse2[(int64_t)bh * T + myq] = m[r] + __log2f(l);
  }
}

// ======================================================================= bwd
// dK / dV: one workgroup = 128 keys of one (b, h), 4 waves x 32 keys, looping over the
// 64-query tiles at or after the key tile.  The query tile's Q / dO images are double-
// buffered in LDS (register-prefetched one tile ahead): one barrier per tile.
__global__ __launch_bounds__(256) void attn_bwd_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dout,
                                                       const float* __restrict__ lse2, const float* __restrict__ delta,
                                                       uint16_t* __restrict__ dqkv, int B, int T, int H, float sl2,
                                                       float scale) {
  // per buffer: Qk Qm dOk dOm (8 KB each) + lse, delta (512 B)
  constexpr int BUF = 4 * 8192 + 512;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nqt = T / AQ, BH = B * H;
  const int kt = (int)(blockIdx.x / BH);  // heaviest key tiles (most query tiles) first
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const uint16_t* vb = qb + 2 * H * AD;
  const int64_t ORS = (int64_t)H * AD;  // dO / O row stride
  const uint16_t* ob = dout + (int64_t)b * T * ORS + (int64_t)h * AD;
  const int k0w = kt * BKW + 32 * w;  // the wave's first key
  const bool live = k0w < T;
  const int qtw = k0w / AQ;           // first query tile that reaches the wave's keys

  // wave's own 32 keys as B operands (key on lane)
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int64_t off = (int64_t)(k0w + 16 * r + li) * RS + 32 * kk + 8 * g;
      kf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(kb + off)) : bf16x8{};
      vf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(vb + off)) : bf16x8{};
    }
  // Q / dO / lse / delta of a query tile: global -> registers (prefetched one tile ahead) -> LDS
  u32x4 qv[2], ov[2];
  float lv = 0.f;
  const uint16_t* pq[2];
  const uint16_t* po[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, q = c >> 3, dc = c & 7;
    pq[i] = qb + (int64_t)q * RS + dc * 8;
    po[i] = ob + (int64_t)q * ORS + dc * 8;
  }
  const float* pl = (tid < 64 ? lse2 + tid : delta + (tid - 64)) + (int64_t)bh * T;
  auto fetch = [&](int qt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      qv[i] = *(const u32x4*)(pq[i] + (int64_t)qt * AQ * RS);
      ov[i] = *(const u32x4*)(po[i] + (int64_t)qt * AQ * ORS);
    }
    if (tid < 128) lv = pl[qt * AQ];
  };
  auto stash = [&](int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, q = c >> 3, dc = c & 7;
      *(u32x4*)(base + (dc >> 2) * 4096 + kimg(q, dc & 3)) = qv[i];
      *(u32x4*)(base + 8192 + pimg(q, dc)) = qv[i];
      *(u32x4*)(base + 2 * 8192 + (dc >> 2) * 4096 + kimg(q, dc & 3)) = ov[i];
      *(u32x4*)(base + 3 * 8192 + pimg(q, dc)) = ov[i];
    }
    if (tid < 128) ((float*)(base + 4 * 8192))[tid] = tid < 64 ? lv : -lv;  // [0,64) lse, [64,128) -delta
  };
  const int qs = (kt * BKW) / AQ;
  fetch(qs);
  stash(0);
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) { dk[r][d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[r][d] = dk[r][d]; }
  __syncthreads();

  // the tile loop unrolled by two: the LDS buffer of each step is a compile-time constant, so every
  // fragment address is a hoisted per-lane offset plus an immediate
  auto step = [&](int qt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = qt + 1 < nqt;
    if (more) fetch(qt + 1);  // in flight during this tile's MFMAs
    auto compute = [&](const char* base, auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      const char* Qk = base;
      const char* Qm = base + 8192;
      const char* Ok = base + 2 * 8192;
      const char* Om = base + 3 * 8192;
      const float* sl = (const float*)(base + 4 * 8192);
      const float* snd = sl + 64;
      // S[q][key], dP[q][key] - delta[q]: lane = key, rows q = 16mt + 4g + e (the dP chain starts
      // from -delta, so dS = P * dP' needs no subtraction)
      f32x4 ps[2][4], dp[2][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 q0 = kfrag64(Qk, 16 * mt), q1 = kfrag64(Qk + 4096, 16 * mt);
        const bf16x8 o0 = kfrag64(Ok, 16 * mt), o1 = kfrag64(Ok + 4096, 16 * mt);
        const f32x4 nd4 = *(const f32x4*)(snd + 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          ps[r][mt] = MFMA(q1, kf[r][1], MFMA(q0, kf[r][0], (f32x4{0.f, 0.f, 0.f, 0.f})));
          dp[r][mt] = MFMA(o1, vf[r][1], MFMA(o0, vf[r][0], nd4));
        }
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 l4 = *(const f32x4*)(sl + 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float p = __builtin_amdgcn_exp2f(fmaf(ps[r][mt][e], sl2, -l4[e]));
            if constexpr (MASK)
              if (k0w + 16 * r + li > qt * AQ + 16 * mt + 4 * g + e) p = 0.f;
            ps[r][mt][e] = p;                        // P
            dp[r][mt][e] = p * dp[r][mt][e];  // dS (unscaled)
          }
      }
      // dV^T += dO^T . P ; dK^T += Q^T . dS   (k = q, permuted order matches the accumulators)
      bf16x8 pp[2][2], ss[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        pp[r][0] = pack_frag(ps[r][0], ps[r][1]); pp[r][1] = pack_frag(ps[r][2], ps[r][3]);
        ss[r][0] = pack_frag(dp[r][0], dp[r][1]); ss[r][1] = pack_frag(dp[r][2], dp[r][3]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 a0 = trfrag(Om, 0, 16 * d), a1 = trfrag(Om, 32, 16 * d);
        const bf16x8 c0 = trfrag(Qm, 0, 16 * d), c1 = trfrag(Qm, 32, 16 * d);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          dv[r][d] = MFMA(a1, pp[r][1], MFMA(a0, pp[r][0], dv[r][d]));
          dk[r][d] = MFMA(c1, ss[r][1], MFMA(c0, ss[r][0], dk[r][d]));
        }
      }
    };
    // query tiles whose first query is past the wave's last key need no causal mask
    if (live && qt >= qtw) {
      if (qt * AQ >= k0w + 31) compute(smem + cur * BUF, std::false_type{});
      else compute(smem + cur * BUF, std::true_type{});
    }
    if (more) stash(cur ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  };
  for (int qt = qs; qt < nqt; qt += 2) {
    step(qt, std::integral_constant<int, 0>{});
    if (qt + 1 < nqt) step(qt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
  // dK, dV (bf16) -> dqkv[b, key, 1|2, h, :]
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint16_t* dkb = dqkv + (int64_t)b * T * RS + (int64_t)(k0w + 16 * r + li) * RS + H * AD + (int64_t)h * AD;
    uint16_t* dvb = dkb + H * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 a, c;
      a[0] = pack_bf2(dk[r][d][0] * scale, dk[r][d][1] * scale);
      a[1] = pack_bf2(dk[r][d][2] * scale, dk[r][d][3] * scale);
      c[0] = pack_bf2(dv[r][d][0], dv[r][d][1]);
      c[1] = pack_bf2(dv[r][d][2], dv[r][d][3]);
      *(u32x2*)(dkb + 16 * d + 4 * g) = a;
      *(u32x2*)(dvb + 16 * d + 4 * g) = c;
    }
  }
}

// dK / dV with the query tile's four images (Q and dO, each K-contiguous and permuted-row) staged
// global -> LDS by LDS-DMA one tile ahead (no staging registers, no ds_write_b128 per image: 8 of
// them per thread and tile in attn_bwd_kernel); lse / -delta still go through registers (128 floats).
// Each lane fetches the chunk the swizzled image places at its slot (the swizzles are involutions).
__global__ __launch_bounds__(256) void attn_bwd_dma_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ dout,
                                                       const float* __restrict__ lse2, const float* __restrict__ delta,
                                                       uint16_t* __restrict__ dqkv, int B, int T, int H, float sl2,
                                                       float scale) {
  // per buffer: Qk Qm dOk dOm (8 KB each) + lse, delta (512 B)
  constexpr int BUF = 4 * 8192 + 512;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nqt = T / AQ, BH = B * H;
  const int kt = (int)(blockIdx.x / BH);  // heaviest key tiles (most query tiles) first
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const uint16_t* vb = qb + 2 * H * AD;
  const int64_t ORS = (int64_t)H * AD;  // dO / O row stride
  const uint16_t* ob = dout + (int64_t)b * T * ORS + (int64_t)h * AD;
  const int k0w = kt * BKW + 32 * w;  // the wave's first key
  const bool live = k0w < T;
  const int qtw = k0w / AQ;           // first query tile that reaches the wave's keys

  // wave's own 32 keys as B operands (key on lane)
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int64_t off = (int64_t)(k0w + 16 * r + li) * RS + 32 * kk + 8 * g;
      kf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(kb + off)) : bf16x8{};
      vf[r][kk] = live ? __builtin_bit_cast(bf16x8, *(const u32x4*)(vb + off)) : bf16x8{};
    }
  // Q / dO of a query tile: LDS-DMA into [Qk | Qm | Ok | Om] (8 KiB each); lse / -delta via registers
  float lv = 0.f;
  const float* pl = (tid < 64 ? lse2 + tid : delta + (tid - 64)) + (int64_t)bh * T;
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(qb), (short)0, (int)(T * RS * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rdo =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(ob), (short)0, (int)(T * ORS * 2), 0x00020000);
  uint32_t voff[8];  // piece w + 4 i of the 32 KiB image set: i < 4 Q, else dO; (i & 2) permuted-row image
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int oo = ((w + 4 * i) * 1024 + lane * 16) & 8191;  // byte slot inside its 8 KiB image
    int row, dc;
    if ((i & 2) == 0) {  // K-contiguous halves: (dc >> 2) * 4096 + kimg(row, dc & 3)
      const int o2 = oo & 4095;
      row = o2 >> 6;
      dc = 4 * (oo >> 12) + (((o2 >> 4) & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3));
    } else {             // permuted-row image: pimg(row, dc)
      row = oo >> 7;
      dc = ((oo >> 4) & 7) ^ (((row >> 1) & 3) << 1);
    }
    voff[i] = (uint32_t)(((int64_t)row * (i < 4 ? RS : ORS) + dc * 8) * 2);
  }
  auto dma_tile = [&](int qt, int buf) {
    char* base = smem + buf * BUF;
    const uint32_t sq = (uint32_t)((int64_t)qt * AQ * RS * 2), so = (uint32_t)((int64_t)qt * AQ * ORS * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) attn_dma16(i < 4 ? rq : rdo, base + (w + 4 * i) * 1024, voff[i], i < 4 ? sq : so);
    if (tid < 128) lv = pl[qt * AQ];
  };
  auto stash = [&](int buf) {  // after the tile's DMA has landed (attn_vm_drain)
    if (tid < 128) ((float*)(smem + buf * BUF + 4 * 8192))[tid] = tid < 64 ? lv : -lv;  // [0,64) lse, [64,128) -delta
  };
  const int qs = (kt * BKW) / AQ;
  dma_tile(qs, 0);
  attn_vm_drain();
  stash(0);
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) { dk[r][d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[r][d] = dk[r][d]; }
  __syncthreads();

  // the tile loop unrolled by two: the LDS buffer of each step is a compile-time constant, so every
  // fragment address is a hoisted per-lane offset plus an immediate
  auto step = [&](int qt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = qt + 1 < nqt;
    if (more) dma_tile(qt + 1, cur ^ 1);  // in flight during this tile's MFMAs (cur ^ 1 last read before the previous barrier)
    auto compute = [&](const char* base, auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      const char* Qk = base;
      const char* Qm = base + 8192;
      const char* Ok = base + 2 * 8192;
      const char* Om = base + 3 * 8192;
      const float* sl = (const float*)(base + 4 * 8192);
      const float* snd = sl + 64;
      // S[q][key], dP[q][key] - delta[q]: lane = key, rows q = 16mt + 4g + e (the dP chain starts
      // from -delta, so dS = P * dP' needs no subtraction)
      f32x4 ps[2][4], dp[2][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const bf16x8 q0 = kfrag64(Qk, 16 * mt), q1 = kfrag64(Qk + 4096, 16 * mt);
        const bf16x8 o0 = kfrag64(Ok, 16 * mt), o1 = kfrag64(Ok + 4096, 16 * mt);
        const f32x4 nd4 = *(const f32x4*)(snd + 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          ps[r][mt] = MFMA(q1, kf[r][1], MFMA(q0, kf[r][0], (f32x4{0.f, 0.f, 0.f, 0.f})));
          dp[r][mt] = MFMA(o1, vf[r][1], MFMA(o0, vf[r][0], nd4));
        }
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 l4 = *(const f32x4*)(sl + 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float p = __builtin_amdgcn_exp2f(fmaf(ps[r][mt][e], sl2, -l4[e]));
            if constexpr (MASK)
              if (k0w + 16 * r + li > qt * AQ + 16 * mt + 4 * g + e) p = 0.f;
            ps[r][mt][e] = p;                        // P
            dp[r][mt][e] = p * dp[r][mt][e];  // dS (unscaled)
          }
      }
      // dV^T += dO^T . P ; dK^T += Q^T . dS   (k = q, permuted order matches the accumulators)
      bf16x8 pp[2][2], ss[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        pp[r][0] = pack_frag(ps[r][0], ps[r][1]); pp[r][1] = pack_frag(ps[r][2], ps[r][3]);
        ss[r][0] = pack_frag(dp[r][0], dp[r][1]); ss[r][1] = pack_frag(dp[r][2], dp[r][3]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 a0 = trfrag(Om, 0, 16 * d), a1 = trfrag(Om, 32, 16 * d);
        const bf16x8 c0 = trfrag(Qm, 0, 16 * d), c1 = trfrag(Qm, 32, 16 * d);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          dv[r][d] = MFMA(a1, pp[r][1], MFMA(a0, pp[r][0], dv[r][d]));
          dk[r][d] = MFMA(c1, ss[r][1], MFMA(c0, ss[r][0], dk[r][d]));
        }
      }
    };
    // query tiles whose first query is past the wave's last key need no causal mask
    if (live && qt >= qtw) {
      if (qt * AQ >= k0w + 31) compute(smem + cur * BUF, std::false_type{});
      else compute(smem + cur * BUF, std::true_type{});
    }
    if (more) {
      attn_vm_drain();
      stash(cur ^ 1);
    }
    __syncthreads();
  };
  for (int qt = qs; qt < nqt; qt += 2) {
    step(qt, std::integral_constant<int, 0>{});
    if (qt + 1 < nqt) step(qt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
  // dK, dV (bf16) -> dqkv[b, key, 1|2, h, :]
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint16_t* dkb = dqkv + (int64_t)b * T * RS + (int64_t)(k0w + 16 * r + li) * RS + H * AD + (int64_t)h * AD;
    uint16_t* dvb = dkb + H * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 a, c;
      a[0] = pack_bf2(dk[r][d][0] * scale, dk[r][d][1] * scale);
      a[1] = pack_bf2(dk[r][d][2] * scale, dk[r][d][3] * scale);
      c[0] = pack_bf2(dv[r][d][0], dv[r][d][1]);
      c[1] = pack_bf2(dv[r][d][2], dv[r][d][3]);
      *(u32x2*)(dkb + 16 * d + 4 * g) = a;
      *(u32x2*)(dvb + 16 * d + 4 * g) = c;
    }
  }
}

// dQ: the forward's structure with the query on the lane (one workgroup = 128 queries,
// 4 waves x 32 queries, looping over key tiles <= the query tile).  S^T = K.Q^T and
// dP^T = V.dO^T are recomputed (A = K / V images, B = the wave's Q / dO in registers);
// P = exp2(S*sl2 - lse2) and dS = P (dP - delta) are lane-local (one query per lane);
// dQ^T += K^T . dS^T takes dS^T straight from the accumulators (permuted key order,
// K read transposed like V in the forward).  dQ is written once, in bf16, into
// dqkv[:, :, 0] -- no fp32 atomics across key tiles, no conversion pass.
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ o,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse2, float* __restrict__ delta,
                                                          uint16_t* __restrict__ dqkv, int B, int T, int H, float sl2,
                                                          float scale) {
  // per buffer: K (two d-halves, K-contig) 8K | V (same) 8K | K permuted-row image 8K
  constexpr int KI = 0, VI = 2 * AKV * 64, KP = 4 * AKV * 64, STG = KP + AKV * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nq = (T + FQ - 1) / FQ, BH = B * H;
  const int qt = nq - 1 - (int)(blockIdx.x / BH);  // heaviest query tiles first
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const int64_t ORS = (int64_t)H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const uint16_t* vb = qb + 2 * H * AD;
  const int q0w = qt * FQ + 32 * w;
  const bool live = q0w < T;
  const int ktw = live ? (q0w + 31) / AKV : -1;
  const int kd = (q0w + 1) / AKV;  // key tiles below kd need no causal mask
  const int nkt = min((qt * FQ + FQ - 1) / AKV, T / AKV - 1) + 1;

  // the wave's Q / dO rows as B operands; delta = rowsum(dO * O) from the same lanes (the
  // lane's 16 d-values, then the 4-group permlane reduce), published for the dK/dV kernel
  bf16x8 qf[2][2], of[2][2];
  float lq[2], ndl[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int myq = live ? q0w + 16 * r + li : 0;
    float dot = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int64_t oo = ((int64_t)b * T + myq) * ORS + (int64_t)h * AD + 32 * kk + 8 * g;
      const u32x4 dov = *(const u32x4*)(dout + oo);
      qf[r][kk] = __builtin_bit_cast(bf16x8, *(const u32x4*)(qb + (int64_t)myq * RS + 32 * kk + 8 * g));
      of[r][kk] = __builtin_bit_cast(bf16x8, dov);
      float fa[8], fb[8];
      unpack8(dov, fa);
      unpack8(*(const u32x4*)(o + oo), fb);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot = fmaf(fa[e], fb[e], dot);
    }
    dot = rowsum4(dot);
    if (live && g == 0) delta[(int64_t)bh * T + myq] = dot;
    lq[r] = lse2[(int64_t)bh * T + myq];
    ndl[r] = -dot;
  }

  KVStage st;
  st.init(kb, vb, RS);
  auto lstore = [&](int buf) {
    char* s = smem + buf * STG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, key = c >> 3, dc = c & 7;
      *(u32x4*)(s + KI + (dc >> 2) * (AKV * 64) + kimg(key, dc & 3)) = st.rk[i];
      *(u32x4*)(s + VI + (dc >> 2) * (AKV * 64) + kimg(key, dc & 3)) = st.rv[i];
      *(u32x4*)(s + KP + pimg(key, dc)) = st.rk[i];
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[r][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  st.load(0);
  lstore(0);
  __syncthreads();
  // the tile loop unrolled by two: the LDS buffer of each step is a compile-time constant, so every
  // fragment address is a hoisted per-lane offset plus an immediate
  auto step = [&](int kt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = kt + 1 < nkt;
    if (more) st.load(kt + 1);
    auto compute = [&](const char* s, auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      f32x4 sc[2][4], dp[2][4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x8 k0 = kfrag64(s + KI, 16 * nt), k1 = kfrag64(s + KI + AKV * 64, 16 * nt);
        const bf16x8 v0 = kfrag64(s + VI, 16 * nt), v1 = kfrag64(s + VI + AKV * 64, 16 * nt);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          sc[r][nt] = MFMA(k1, qf[r][1], MFMA(k0, qf[r][0], (f32x4{0.f, 0.f, 0.f, 0.f})));
          dp[r][nt] = MFMA(v1, of[r][1], MFMA(v0, of[r][0], (f32x4{ndl[r], ndl[r], ndl[r], ndl[r]})));
        }
      }
      bf16x8 dd[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int myq = q0w + 16 * r + li;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float p = __builtin_amdgcn_exp2f(fmaf(sc[r][nt][e], sl2, -lq[r]));
            if constexpr (MASK)
              if (kt * AKV + 16 * nt + 4 * g + e > myq) p = 0.f;
            dp[r][nt][e] = p * dp[r][nt][e];  // dS^T (unscaled); dP^T started from -delta
          }
        dd[r][0] = pack_frag(dp[r][0], dp[r][1]);
        dd[r][1] = pack_frag(dp[r][2], dp[r][3]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 a0 = trfrag(s + KP, 0, 16 * d), a1 = trfrag(s + KP, 32, 16 * d);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r][d] = MFMA(a1, dd[r][1], MFMA(a0, dd[r][0], acc[r][d]));
      }
    };
    if (kt < kd) compute(smem + cur * STG, std::false_type{});
    else if (kt <= ktw) compute(smem + cur * STG, std::true_type{});
    if (more) lstore(cur ^ 1);
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nkt) step(kt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint16_t* o = dqkv + ((int64_t)b * T + q0w + 16 * r + li) * RS + (int64_t)h * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 pk;
      pk[0] = pack_bf2(acc[r][d][0] * scale, acc[r][d][1] * scale);
      pk[1] = pack_bf2(acc[r][d][2] * scale, acc[r][d][3] * scale);
      *(u32x2*)(o + 16 * d + 4 * g) = pk;
    }
  }
}

// The same with the key tile's three images (K, V K-contiguous; K permuted-row) staged global -> LDS by
// LDS-DMA one tile ahead instead of through registers and ds_write_b128 (as attn_bwd_dma_kernel).
// (ATTN_DQ_WAVES=3 caps it at 168 VGPRs: 26 spilled registers, 88.5 vs 74.0 us for the backward pair)
#ifndef ATTN_DQ_WAVES
#define ATTN_DQ_WAVES 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ATTN_DQ_WAVES))) void attn_bwd_dq_dma_kernel(const uint16_t* __restrict__ qkv, const uint16_t* __restrict__ o,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse2, float* __restrict__ delta,
                                                          uint16_t* __restrict__ dqkv, int B, int T, int H, float sl2,
                                                          float scale) {
  // per buffer: K (two d-halves, K-contig) 8K | V (same) 8K | K permuted-row image 8K
  constexpr int KI = 0, VI = 2 * AKV * 64, KP = 4 * AKV * 64, STG = KP + AKV * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nq = (T + FQ - 1) / FQ, BH = B * H;
  const int qt = nq - 1 - (int)(blockIdx.x / BH);  // heaviest query tiles first
  const int bh = blockIdx.x % BH, b = bh / H, h = bh % H;
  const int64_t RS = 3LL * H * AD;
  const int64_t ORS = (int64_t)H * AD;
  const uint16_t* qb = qkv + (int64_t)b * T * RS + (int64_t)h * AD;
  const uint16_t* kb = qb + H * AD;
  const uint16_t* vb = qb + 2 * H * AD;
  const int q0w = qt * FQ + 32 * w;
  const bool live = q0w < T;
  const int ktw = live ? (q0w + 31) / AKV : -1;
  const int kd = (q0w + 1) / AKV;  // key tiles below kd need no causal mask
  const int nkt = min((qt * FQ + FQ - 1) / AKV, T / AKV - 1) + 1;

  // the wave's Q / dO rows as B operands; delta = rowsum(dO * O) from the same lanes (the
  // lane's 16 d-values, then the 4-group permlane reduce), published for the dK/dV kernel
  bf16x8 qf[2][2], of[2][2];
  float lq[2], ndl[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int myq = live ? q0w + 16 * r + li : 0;
    float dot = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int64_t oo = ((int64_t)b * T + myq) * ORS + (int64_t)h * AD + 32 * kk + 8 * g;
      const u32x4 dov = *(const u32x4*)(dout + oo);
      qf[r][kk] = __builtin_bit_cast(bf16x8, *(const u32x4*)(qb + (int64_t)myq * RS + 32 * kk + 8 * g));
      of[r][kk] = __builtin_bit_cast(bf16x8, dov);
      float fa[8], fb[8];
      unpack8(dov, fa);
      unpack8(*(const u32x4*)(o + oo), fb);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot = fmaf(fa[e], fb[e], dot);
    }
    dot = rowsum4(dot);
    if (live && g == 0) delta[(int64_t)bh * T + myq] = dot;
    lq[r] = lse2[(int64_t)bh * T + myq];
    ndl[r] = -dot;
  }

  // the sequence's qkv rows from K of head h on: one buffer resource, tile advance in soffset
  const __amdgpu_buffer_rsrc_t rkv =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(kb), (short)0, (int)(T * RS * 2), 0x00020000);
  uint32_t voff[6];  // piece w + 4 i of the 24 KiB image set: [K halves | V halves | K permuted-row]
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int oo = ((w + 4 * i) * 1024 + lane * 16) & 8191;
    int row, dc;
    if (i < 4) {  // (dc >> 2) * 4096 + kimg(row, dc & 3)
      const int o2 = oo & 4095;
      row = o2 >> 6;
      dc = 4 * (oo >> 12) + (((o2 >> 4) & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3));
    } else {      // pimg(row, dc)
      row = oo >> 7;
      dc = ((oo >> 4) & 7) ^ (((row >> 1) & 3) << 1);
    }
    voff[i] = (uint32_t)(((int64_t)row * RS + ((i & 6) == 2 ? H * AD : 0) + dc * 8) * 2);
  }
  auto dma_tile = [&](int kt, int buf) {
    char* base = smem + buf * STG;
    const uint32_t so = (uint32_t)((int64_t)kt * AKV * RS * 2);
#pragma unroll
    for (int i = 0; i < 6; ++i) attn_dma16(rkv, base + (w + 4 * i) * 1024, voff[i], so);
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[r][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  dma_tile(0, 0);
  attn_vm_drain();
  __syncthreads();
  // the tile loop unrolled by two: the LDS buffer of each step is a compile-time constant, so every
  // fragment address is a hoisted per-lane offset plus an immediate
  auto step = [&](int kt, auto bufc) {
    constexpr int cur = decltype(bufc)::value;
    const bool more = kt + 1 < nkt;
    if (more) dma_tile(kt + 1, cur ^ 1);  // cur ^ 1 last read before the previous barrier
    auto compute = [&](const char* s, auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      f32x4 sc[2][4], dp[2][4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x8 k0 = kfrag64(s + KI, 16 * nt), k1 = kfrag64(s + KI + AKV * 64, 16 * nt);
        const bf16x8 v0 = kfrag64(s + VI, 16 * nt), v1 = kfrag64(s + VI + AKV * 64, 16 * nt);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          sc[r][nt] = MFMA(k1, qf[r][1], MFMA(k0, qf[r][0], (f32x4{0.f, 0.f, 0.f, 0.f})));
          dp[r][nt] = MFMA(v1, of[r][1], MFMA(v0, of[r][0], (f32x4{ndl[r], ndl[r], ndl[r], ndl[r]})));
        }
      }
      bf16x8 dd[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int myq = q0w + 16 * r + li;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float p = __builtin_amdgcn_exp2f(fmaf(sc[r][nt][e], sl2, -lq[r]));
            if constexpr (MASK)
              if (kt * AKV + 16 * nt + 4 * g + e > myq) p = 0.f;
            dp[r][nt][e] = p * dp[r][nt][e];  // dS^T (unscaled); dP^T started from -delta
          }
        dd[r][0] = pack_frag(dp[r][0], dp[r][1]);
        dd[r][1] = pack_frag(dp[r][2], dp[r][3]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 a0 = trfrag(s + KP, 0, 16 * d), a1 = trfrag(s + KP, 32, 16 * d);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r][d] = MFMA(a1, dd[r][1], MFMA(a0, dd[r][0], acc[r][d]));
      }
    };
    if (kt < kd) compute(smem + cur * STG, std::false_type{});
    else if (kt <= ktw) compute(smem + cur * STG, std::true_type{});
    if (more) attn_vm_drain();
    __syncthreads();
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nkt) step(kt + 1, std::integral_constant<int, 1>{});
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint16_t* o = dqkv + ((int64_t)b * T + q0w + 16 * r + li) * RS + (int64_t)h * AD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      u32x2 pk;
      pk[0] = pack_bf2(acc[r][d][0] * scale, acc[r][d][1] * scale);
      pk[1] = pack_bf2(acc[r][d][2] * scale, acc[r][d][3] * scale);
      *(u32x2*)(o + 16 * d + 4 * g) = pk;
    }
  }
}

}  // namespace dpe

using namespace dpe;

extern "C" int dpe_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int T, int H, int D, float scale, int causal,
                            hipStream_t st) {
  if (D != AD || T % AKV != 0 || !causal) return -1;
  const float sl2 = scale * 1.4426950408889634f;
#ifdef DPE_ATTN_FWD_STAGED
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, lse, B, T, H, sl2);
#else
  // one sequence's qkv rows must fit the DMA kernel's 32-bit buffer range
  if ((int64_t)T * 3 * H * AD * 2 < (1LL << 31))
    hipLaunchKernelGGL(attn_fwd_dma_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, lse, B, T, H,
                       sl2);
  else
    hipLaunchKernelGGL(attn_fwd_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, lse, B, T, H, sl2);
#endif
  return 0;
}

extern "C" int dpe_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, float* delta,
                            float* dq_acc, uint16_t* dqkv, int B, int T, int H, int D, float scale, int causal,
                            hipStream_t st) {
  (void)dq_acc;  // dQ is not accumulated with atomics (attn_bwd_dq_kernel)
  if (D != AD || T % AKV != 0 || !causal) return -1;
  const float sl2 = scale * 1.4426950408889634f;
  // dQ first: it also writes delta = rowsum(dO * O), which the dK/dV kernel reads
#ifdef DPE_ATTN_BWD_STAGED
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, dout, lse, delta,
                     dqkv, B, T, H, sl2, scale);
#else
  if ((int64_t)T * 3 * H * AD * 2 < (1LL << 31))
    hipLaunchKernelGGL(attn_bwd_dq_dma_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, dout, lse,
                       delta, dqkv, B, T, H, sl2, scale);
  else
    hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(B * H * ((T + FQ - 1) / FQ)), dim3(256), 0, st, qkv, out, dout, lse, delta,
                       dqkv, B, T, H, sl2, scale);
#endif
#ifdef DPE_ATTN_BWD_STAGED
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(B * H * ((T + BKW - 1) / BKW)), dim3(256), 0, st, qkv, dout, lse, delta, dqkv, B,
                     T, H, sl2, scale);
#else
  // one sequence's qkv / dO rows must fit the DMA kernel's 32-bit buffer ranges
  if ((int64_t)T * 3 * H * AD * 2 < (1LL << 31))
    hipLaunchKernelGGL(attn_bwd_dma_kernel, dim3(B * H * ((T + BKW - 1) / BKW)), dim3(256), 0, st, qkv, dout, lse, delta,
                       dqkv, B, T, H, sl2, scale);
  else
    hipLaunchKernelGGL(attn_bwd_kernel, dim3(B * H * ((T + BKW - 1) / BKW)), dim3(256), 0, st, qkv, dout, lse, delta, dqkv,
                       B, T, H, sl2, scale);
#endif
  return 0;
}
