// Large-tile dense GEMM for gfx950: 256x256x64 tiles, 8 waves, LDS-DMA
// (global_load_lds_dwordx4) staging and an 8-phase K-loop with counted
// vmcnt, raw s_barrier and s_setprio around each MFMA cluster
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5).
//
// Used for the big GEMMs (GPT-2 projections/MLP/LM head, ResNet's wide 1x1
// convolutions); the 128-tile register-staged igemm stays for small, strided
// and convolution-gather shapes.
//
// Operands (same conventions as igemm, D^T issue so each lane holds 4
// consecutive output columns):
//   A: K-contiguous A[m][k] (lda)      or M-contiguous A[k][m] (lda)
//   B: K-contiguous B[n][k] (ldb)      or N-contiguous B[k][n] (ldb)
//   fwd   y = x w^T   : A K-contig, B K-contig   (NT)
//   dgrad dx = dy w   : A K-contig, B N-contig   (NN)
//   wgrad dw = dy^T x : A M-contig, B N-contig   (TN)
//
// Waves: 2 (M) x 4 (N); wave (wr, wc) owns rows wr*128 + [0,128) and columns
// wc*64 + [0,64) = 8 x 4 MFMA 16x16 tiles (128 fp32 accumulators / lane).
// Each operand tile is stored as two *half images*, one per accumulator
// half the waves consume in different phases:
//   A half h: tile rows {wr*128 + h*64 + [0,64)}   (128 rows)
//   B half h: tile cols {wc*64  + h*32 + [0,32)}   (128 cols)
// so a half image is exactly what one phase-quadrant of every wave reads,
// and staging it is 16 KiB = 2 LDS-DMA instructions per thread.
//
// Per K-tile: 4 phases = 4 accumulator quadrants (A half, B half):
//   (0,0) reads A0+B0, (0,1) reads B1, (1,1) reads A1, (1,0) reads B0 again.
// K-tile t lives in LDS buffer t&1 (one tile per loop iteration: a two-tile
// body spills under the 256-VGPR budget of 2 waves/SIMD).  Every phase
// restages one half image, exactly two phases after that half's last ds_read
// (WAR), and the vmcnt(4) in phase 4 retires the tile read next (RAW),
// leaving the two newest half-tiles in flight across the barrier.
//
// LDS-DMA writes lane-linearly (base + lane*16), so bank-conflict swizzles
// are applied to the per-lane SOURCE address and undone on the read:
//   K image  [128][64] bf16, 128-B rows:  chunk ^= (row >> 1) & 7
//   MN image [64][128] bf16, 256-B rows:  chunk ^= 2*((k&3) | ((k>>3)&1)<<2)
// both conflict-free for ds_read_b128 / ds_read_b64_tr_b16 lane groups.
#include "common.h"
#include "igemm.h"

namespace dpe {
namespace g256 {

constexpr int NT = 512;
constexpr int TK = 64;                 // K per tile
constexpr int HALF = 16384;            // bytes per half image
// LDS: A images at [0, 64K), B images at [64K, 128K); image (buf, h) of an
// operand at (buf*2 + h) * HALF, so every fragment read is one per-lane base
// VGPR + an immediate offset (< 64 KiB) and no address is rematerialised.
constexpr int B_REGION = 65536;
constexpr int LDS_MAIN = 2 * B_REGION; // 128 KiB
constexpr int CROW = 512 + 16;         // bf16 epilogue staging row (bytes)
constexpr int FROW = 256 + 4;          // fp32 atomic staging row (floats)
constexpr int LDS_BF16 = 128 * CROW;   // 66 KiB
constexpr int LDS_ATOM = 64 * FROW * 4;
constexpr int LDS_TOTAL = LDS_MAIN;
static_assert(LDS_BF16 <= LDS_TOTAL && LDS_ATOM <= LDS_TOTAL, "epilogue staging must fit");

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DPE_DEVICE int amap(int h, int r) { return (r & 63) + ((r >> 6) << 7) + h * 64; }
DPE_DEVICE int bmap(int h, int r) { return (r & 31) + ((r >> 5) << 6) + h * 32; }
DPE_DEVICE int kswz(int row) { return (row >> 1) & 7; }
DPE_DEVICE int mnswz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

template <int ACT>
DPE_DEVICE float act(float x) {
  if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  if constexpr (ACT == ACT_GELU) {
    // 0.5 x (1 + tanh(u)) == x / (1 + exp(-2u)),  u = sqrt(2/pi) (x + 0.044715 x^3)
    const float u2 = -1.5957691216057308f * (x + 0.044715f * x * x * x);
    return x * __builtin_amdgcn_rcpf(1.f + __expf(u2));
  }
  return x;
}

// ---- per-lane LDS-DMA source pointers of one operand (2 halves x 2 instructions)
template <bool KC, bool ISA>
DPE_DEVICE void stage_setup(int64_t ld, int dim, int d0, int kb, uint32_t (&g)[2][2]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = wid * 2 + i;
      if constexpr (KC) {
        const int r = 8 * u + (lane >> 3);
        const int t = ISA ? amap(h, r) : bmap(h, r);
        const int gr = min(d0 + t, dim - 1);
        const int ch = (lane & 7) ^ kswz(r);
        g[h][i] = (uint32_t)(((int64_t)gr * ld + kb + ch * 8) * 2);
      } else {
        const int k = 4 * u + (lane >> 4);
        const int c = (lane & 15) ^ mnswz(k);
        const int t = ISA ? amap(h, c * 8) : bmap(h, c * 8);
        const int gc = min(d0 + t, dim - 8);
        g[h][i] = (uint32_t)(((int64_t)(kb + k) * ld + gc) * 2);
      }
    }
}

DPE_DEVICE void glds(const char* src, char* dst) {
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 16, 0, 0);
}

// lane part of a K-image fragment read at rows r0 + [0,16) (r0 % 16 == 0), k-step s
DPE_DEVICE int kread_off(int r0, int s) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15), ch = s * 4 + (lane >> 4);
  return row * 128 + ((ch ^ kswz(row)) << 4);
}
// lane part of an MN-image fragment read at columns c0 + [0,16), k-step 0 (k-step 1 = +8192)
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

#define G256_BARRIER()                   \
  do {                                   \
    asm volatile("" ::: "memory");       \
    __builtin_amdgcn_s_barrier();        \
    asm volatile("" ::: "memory");       \
  } while (0)

template <bool AK, bool BK, int EPI, int ACT>
__global__ __launch_bounds__(NT) void gemm256_kernel(IgemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tilesN = (p.N + 255) >> 8, tilesM = (p.M + 255) >> 8;
  const int ntile = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntile, split = bid / ntile;
  const int m0 = (tile / tilesN) << 8, n0 = (tile % tilesN) << 8;
  const int kb = split * p.k_split;
  const int ke = min(p.K, kb + p.k_split);
  const int nt = (ke - kb) / TK;

  // LDS-DMA sources: uniform base (advanced per K-tile) + per-lane 32-bit byte offset
  uint32_t ga[2][2], gb[2][2];
  stage_setup<AK, true>(p.lda, p.M, m0, kb, ga);
  stage_setup<BK, false>(p.ldb, p.N, n0, kb, gb);
  const int64_t astep = AK ? (int64_t)TK * 2 : (int64_t)TK * p.lda * 2;
  const int64_t bstep = BK ? (int64_t)TK * 2 : (int64_t)TK * p.ldb * 2;
  const char* const Ab = (const char*)p.A;
  const char* const Bb = (const char*)p.B;
  char* const wdst = smem + wid * 2048;  // this wave's 2 KiB slot in every half image

  // fragment-read lane offsets (k-step 0 / 1 for K images; per fragment for MN images)
  int ra[4][2], rb[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) ra[i][s] = AK ? kread_off(wr * 64 + i * 16, s) : mnread_off(wr * 64 + i * 16) + s * 8192;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      rb[j][s] = B_REGION + (BK ? kread_off(wc * 32 + j * 16, s) : mnread_off(wc * 32 + j * 16) + s * 8192);

#define STAGE_A(h, buf, t)                                                                     \
  do {                                                                                         \
    const char* b_ = Ab + (int64_t)(t) * astep;                                                \
    glds(b_ + ga[h][0], wdst + ((buf) * 2 + (h)) * HALF);                                      \
    glds(b_ + ga[h][1], wdst + ((buf) * 2 + (h)) * HALF + 1024);                               \
  } while (0)
#define STAGE_B(h, buf, t)                                                                     \
  do {                                                                                         \
    const char* b_ = Bb + (int64_t)(t) * bstep;                                                \
    glds(b_ + gb[h][0], wdst + B_REGION + ((buf) * 2 + (h)) * HALF);                           \
    glds(b_ + gb[h][1], wdst + B_REGION + ((buf) * 2 + (h)) * HALF + 1024);                    \
  } while (0)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2];

#define LOAD_A(boff, h)                                                                       \
  do {                                                                                        \
    _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                          \
      _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                      \
        const char* a_ = smem + (boff) + ra[i_][s_] + (h) * HALF;                             \
        af[i_][s_] = AK ? lds_b128(a_) : lds_tr(a_);                                          \
      }                                                                                       \
  } while (0)
#define LOAD_B(boff, h)                                                                       \
  do {                                                                                        \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                          \
      _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_) {                                      \
        const char* a_ = smem + (boff) + rb[j_][s_] + (h) * HALF;                             \
        bfr[j_][s_] = BK ? lds_b128(a_) : lds_tr(a_);                                         \
      }                                                                                       \
  } while (0)
#define QUAD(mh, nh)                                                                          \
  do {                                                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                        \
    __builtin_amdgcn_s_setprio(1);                                                            \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                          \
      _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                        \
        _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                      \
          acc[(mh) * 4 + i_][(nh) * 2 + j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(        \
              bfr[j_][s_], af[i_][s_], acc[(mh) * 4 + i_][(nh) * 2 + j_], 0, 0, 0);           \
    __builtin_amdgcn_s_setprio(0);                                                            \
  } while (0)

  // prologue: tile 0 -> buf 0 (all halves), tile 1 -> buf 1 (A0, B1)
  if (nt > 0) {
    STAGE_A(0, 0, 0); STAGE_B(1, 0, 0); STAGE_A(1, 0, 0); STAGE_B(0, 0, 0);
    if (nt > 1) {
      STAGE_A(0, 1, 1); STAGE_B(1, 1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  G256_BARRIER();
  // Ping-pong: the two wave groups (wr = 0 / 1, one wave of each per SIMD) run
  // one barrier apart, so on every SIMD one wave issues its MFMA cluster while
  // the other issues its ds_reads and LDS-DMA.  RAW/WAR still hold: a group's
  // wait/ds_read retirement always precedes the other group's use by at least
  // one shared barrier (the "one barrier MORE" rule for staggered groups).
  if (wr) G256_BARRIER();

  // One K-tile per iteration, buffer b = t & 1.  Phase p restages one half
  // image: A1(t+1)->b^1, B0(t+1)->b^1, A0(t+2)->b, B1(t+2)->b; each target was
  // last read two phases earlier, and phase 4's vmcnt(4) retires tile t+1.
  for (int t = 0; t < nt; ++t) {
    const int b = t & 1;
    const int boff = b * 2 * HALF;
    const bool h1 = t + 1 < nt, h2 = t + 2 < nt;

    LOAD_A(boff, 0); LOAD_B(boff, 0);
    if (h1) STAGE_A(1, b ^ 1, t + 1);
    G256_BARRIER();
    QUAD(0, 0);
    G256_BARRIER();

    LOAD_B(boff, 1);
    if (h1) STAGE_B(0, b ^ 1, t + 1);
    G256_BARRIER();
    QUAD(0, 1);
    G256_BARRIER();

    LOAD_A(boff, 1);
    if (h2) STAGE_A(0, b, t + 2);
    G256_BARRIER();
    QUAD(1, 1);
    G256_BARRIER();

    LOAD_B(boff, 0);
    if (h2) {
      STAGE_B(1, b, t + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    G256_BARRIER();
    QUAD(1, 0);
    G256_BARRIER();
  }
  if (!wr) G256_BARRIER();  // rebalance the stagger (equal barrier counts)
#undef STAGE_A
#undef STAGE_B
#undef LOAD_A
#undef LOAD_B
#undef QUAD

  // ------------------------------------------------------------- epilogue
  // acc[i][j][e]: row m0 + wr*128 + 16i + (lane&15), col n0 + wc*64 + 16j + (lane>>4)*4 + e
  const float alpha = p.alpha * (p.alpha_ptr ? *p.alpha_ptr : 1.f);
  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  __syncthreads();
  if constexpr (EPI == EPI_F32) {
    float* C = (float*)p.C;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + 16 * i + lm;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + 16 * j + ln4;
        if (n >= p.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
          v[e] = act<ACT>(alpha * acc[i][j][e] + b);
        }
        float* dst = C + (int64_t)m * p.ldc + n;
        if (n + 4 <= p.N) {
          if (p.residual_f32) {
            const f32x4 r = *(const f32x4*)(p.residual_f32 + (int64_t)m * p.ldc + n);
            v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3];
          }
          *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) dst[e] = v[e] + (p.residual_f32 ? p.residual_f32[(int64_t)m * p.ldc + n + e] : 0.f);
        }
      }
    }
  } else if constexpr (EPI == EPI_ATOMIC_F32) {
    float* C = (float*)p.C;
    float* st = (float*)smem;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int srow = wr * 32 + ii * 16 + lm;
#pragma unroll
        for (int j = 0; j < 4; ++j) *(f32x4*)(st + srow * FROW + wc * 64 + 16 * j + ln4) = acc[2 * q + ii][j] * alpha;
      }
      __syncthreads();
      for (int s = wid; s < 64 * 4; s += 8) {
        const int srow = s >> 2, c = (s & 3) * 64 + lane;
        const int m = m0 + (srow >> 5) * 128 + q * 32 + (srow & 31), n = n0 + c;
        if (m < p.M && n < p.N) atomicAdd(C + (int64_t)m * p.ldc + n, st[srow * FROW + c]);
      }
      __syncthreads();
    }
  } else {  // EPI_BF16: stage half the rows at a time in LDS, then 16-B row stores
    uint16_t* C = (uint16_t*)p.C;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int srow = wr * 64 + 16 * i + lm;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int nl = wc * 64 + 16 * j + ln4, n = n0 + nl;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
            v[e] = act<ACT>(alpha * acc[hh * 4 + i][j][e] + b);
          }
          u32x2 pk;
          pk[0] = pack_bf2(v[0], v[1]);
          pk[1] = pack_bf2(v[2], v[3]);
          *(u32x2*)(smem + srow * CROW + nl * 2) = pk;
        }
      }
      __syncthreads();
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int c = tid + it * NT;
        const int srow = c >> 5, ch = c & 31;
        const int m = m0 + amap(hh, srow), n = n0 + ch * 8;
        if (m < p.M && n < p.N) {
          u32x4 v = *(const u32x4*)(smem + srow * CROW + ch * 16);
          uint16_t* dst = C + (int64_t)m * p.ldc + n;
          if (p.residual) {
            float a[8], r[8];
            unpack8(v, a);
            if (n + 8 <= p.N) {
              unpack8(*(const u32x4*)(p.residual + (int64_t)m * p.ldc + n), r);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) r[e] = n + e < p.N ? bf2f(p.residual[(int64_t)m * p.ldc + n + e]) : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += r[e];
            v = pack8(a);
          }
          if (n + 8 <= p.N) {
            *(u32x4*)dst = v;
          } else {
            const uint16_t* hv = (const uint16_t*)&v;
            for (int e = 0; e < 8 && n + e < p.N; ++e) dst[e] = hv[e];
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace g256
}  // namespace dpe

using namespace dpe;

// a_k / b_k: operand is K-contiguous (1) or M/N-contiguous (0).  K range per
// split (k_split) must be a multiple of 64; ld's multiples of 8; N % 8 == 0
// for N-contiguous B and M % 8 == 0 for M-contiguous A.
extern "C" int dpe_gemm256_launch(const IgemmArgs* a, int a_k, int b_k, int epi, int splits, hipStream_t st) {
  const IgemmArgs& p = *a;
  if (p.k_split % 64 || p.K % 64) return -1;
  if (p.act != ACT_NONE && p.act != ACT_GELU) return -3;
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const dim3 grid((unsigned)(tiles * splits)), block(g256::NT);
#define L(AK, BK, E, A) hipLaunchKernelGGL((g256::gemm256_kernel<AK, BK, E, A>), grid, block, 0, st, p)
#define LA(AK, BK, E)                              \
  do {                                             \
    if (p.act == ACT_GELU) L(AK, BK, E, ACT_GELU); \
    else if (p.act == ACT_NONE) L(AK, BK, E, ACT_NONE); \
    else return -3;                                \
  } while (0)
  if (a_k && b_k) {
    if (epi == EPI_BF16) LA(true, true, EPI_BF16);
    else if (epi == EPI_F32) LA(true, true, EPI_F32);
    else L(true, true, EPI_ATOMIC_F32, ACT_NONE);
  } else if (a_k && !b_k) {
    if (epi == EPI_BF16) LA(true, false, EPI_BF16);
    else if (epi == EPI_F32) L(true, false, EPI_F32, ACT_NONE);
    else L(true, false, EPI_ATOMIC_F32, ACT_NONE);
  } else if (!a_k && !b_k) {
    if (epi == EPI_F32) L(false, false, EPI_F32, ACT_NONE);
    else if (epi == EPI_ATOMIC_F32) L(false, false, EPI_ATOMIC_F32, ACT_NONE);
    else return -2;
  } else {
    return -2;
  }
#undef LA
#undef L
  return 0;
}
