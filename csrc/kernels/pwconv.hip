// Streaming pointwise (1x1, stride 1) convolution forward for the write-heavy ResNet
// shapes: y[M][N] = x[M][K] . W[N][K]^T, K in {64, 128, 256}, N a multiple of 4*WN, with the
// BatchNorm-forward statistics (sum, sum of squares of the stored bf16 values).
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
//   * the output goes straight from the accumulators: each lane owns 4 consecutive channels of
//     one pixel (8-B stores; the 4 lane groups complete each 128-B row segment in L2);
//   * BatchNorm sums accumulate in registers over all of the block's rows and are reduced once
//     at the end: one partial column per row group ([2][N][row groups]) instead of one per
//     128-row tile, and no per-tile LDS reduction or barrier.
#include <algorithm>

#include "common.h"
#include "igemm.h"

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
template <int K, int WN, int NS>
__global__ __launch_bounds__(256, K == 64 ? 3 : 2) void pw_stream_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ y, float* __restrict__ stats, int M,
                                                           int N, int RG) {
  constexpr int KC = K / 32;                  // 32-deep K chunks
  constexpr int TILE = BM * K * 2;            // bytes of one x tile in LDS ([KC][64 rows][64 B])
  constexpr int P = TILE / 1024 / 4;          // 1-KiB DMA pieces per wave per tile
  constexpr int NI = WN / 16, MI = BM / 16;
  static_assert(P >= 1 && P * 4096 == TILE, "pieces");
  // output staging: each wave stages half a tile (32 rows x WN channels, padded rows) in its own
  // LDS region and stores whole 16-B row chunks: one store instruction = RPP full row segments
  constexpr int ROWB = WN * 2 + 16, CPRW = WN / 8, RPP = 64 / CPRW;
  constexpr int STG = 32 * ROWB;
  // stores outstanding per wave per tile, for the counted vmcnt below
  constexpr int S = 2 * (32 / RPP);
  constexpr int VM = (NS - 1) * S + (NS - 2) * P;
  static_assert(VM < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NS * TILE + 4 * STG];

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbN = N / (4 * WN);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the nbN column slices of a row group share an XCD
  const int rg = bid / nbN, nb = bid % nbN;
  const int n0w = nb * 4 * WN + wid * WN;  // the wave's first output channel
  const int tiles = (M + BM - 1) / BM;

  // weights as MFMA A operands: wf[ni][kc] = W[n0w + 16 ni + li][32 kc + 8 g .. +7]
  bf16x8 wf[NI][KC];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      wf[ni][kc] = __builtin_bit_cast(bf16x8, *(const u32x4*)(w + (int64_t)(n0w + 16 * ni + li) * K + 32 * kc + 8 * g));

  // DMA pieces: piece q (of 4P per tile) = K chunk q / 4, rows 16 (q % 4) .. +15; lane -> (row, 16-B chunk)
  const __amdgpu_buffer_rsrc_t xr = rsrc(x, (uint32_t)((int64_t)M * K * 2));
  uint32_t voff[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int q = wid * P + i, kc = q >> 2, row = (q & 3) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
    voff[i] = (uint32_t)(row * K * 2 + kc * 64 + lc * 16);
  }
  auto issue = [&](int t, int slot) {
    char* dst = smem + slot * TILE;
    const int64_t base = (int64_t)t * BM * K * 2;
    const int valid_rows = M - t * BM;  // rows past M read as zeros (offset out of range)
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int q = wid * P + i, row = (q & 3) * 16 + (lane >> 2);
      const uint32_t v = row < valid_rows ? voff[i] + (uint32_t)base : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(dst + q * 1024), 16, v, 0, 0, 0);
    }
  };

  float s[NI][4], ss[NI][4];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int e = 0; e < 4; ++e) { s[ni][e] = 0.f; ss[ni][e] = 0.f; }

  // this row group's tiles: rg, rg + RG, ...
  const int nt = rg < tiles ? (tiles - 1 - rg) / RG + 1 : 0;
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nt) issue(rg + j * RG, j);
  for (int j = 0; j < nt; ++j) {
    // tile j landed (its DMA is older than NS-2 later tiles' DMAs and NS-1 tiles' stores)
    if (j + NS - 2 < nt) wait_vm<VM>(); else wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile j are in; slot (j-1)%NS is free
    asm volatile("" ::: "memory");
    if (j + NS - 1 < nt) issue(rg + (j + NS - 1) * RG, (j + NS - 1) % NS);
    const char* img = smem + (j % NS) * TILE;
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
    // next half's writes never overtake this half's reads)
    const int m0 = (rg + j * RG) * BM;
    char* stg = smem + NS * TILE + wid * STG;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        const int mi = 2 * hf + mh;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          u32x2 pk;
          pk[0] = pack_bf2(acc[mi][ni][0], acc[mi][ni][1]);
          pk[1] = pack_bf2(acc[mi][ni][2], acc[mi][ni][3]);
          // statistics of the stored (rounded) values; rows past M are zeros
          const float v0 = __uint_as_float(pk[0] << 16), v1 = __uint_as_float(pk[0] & 0xffff0000u);
          const float v2 = __uint_as_float(pk[1] << 16), v3 = __uint_as_float(pk[1] & 0xffff0000u);
          s[ni][0] += v0; ss[ni][0] = fmaf(v0, v0, ss[ni][0]);
          s[ni][1] += v1; ss[ni][1] = fmaf(v1, v1, ss[ni][1]);
          s[ni][2] += v2; ss[ni][2] = fmaf(v2, v2, ss[ni][2]);
          s[ni][3] += v3; ss[ni][3] = fmaf(v3, v3, ss[ni][3]);
          *(u32x2*)(stg + (16 * mh + li) * ROWB + (16 * ni + 4 * g) * 2) = pk;
        }
      }
#pragma unroll
      for (int ps = 0; ps < 32 / RPP; ++ps) {
        const int row = ps * RPP + lane / CPRW, ch = lane % CPRW;
        const u32x4 v = *(const u32x4*)(stg + row * ROWB + ch * 16);
        const int m = m0 + 32 * hf + row;
        if (m < M) *(u32x4*)(y + (int64_t)m * N + n0w + ch * 8) = v;
      }
    }
  }
  // statistics: reduce over the 16 pixels of each lane group, one partial column per row group
  if (stats) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s[ni][e] += __shfl_xor(s[ni][e], o, 64);
          ss[ni][e] += __shfl_xor(ss[ni][e], o, 64);
        }
      }
    if (li == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0w + 16 * ni + 4 * g + e;
          stats[(int64_t)n * RG + rg] = s[ni][e];
          stats[(int64_t)(N + n) * RG + rg] = ss[ni][e];
        }
    }
  }
}

}  // namespace pw
}  // namespace dpe

using namespace dpe;

// Shape of the launch for (M, N, K): row groups (= BatchNorm partial columns) or 0 when the
// problem is outside this kernel's envelope (the caller then uses the implicit-GEMM kernels).
static int pw_wn(int K) { return K <= 128 ? 64 : 32; }

// Every block carries the same number of tiles, so the grid must be exactly the resident
// capacity (blocks per CU from the occupancy API x CUs): a grid that lets the dispatcher put
// 3 blocks on some CUs and 1 on others finishes at the pace of the fullest CU.
template <int K, int WN, int NS>
static int pw_slots() {
  static int slots = [] {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pw::pw_stream_kernel<K, WN, NS>, 256, 0);
    return std::max(1, per) * std::max(1, cus);
  }();
  return slots;
}
static int pw_capacity(int K) {
  return K == 64 ? pw_slots<64, 64, 4>() : K == 128 ? pw_slots<128, 64, 3>() : pw_slots<256, 32, 2>();
}

extern "C" int dpe_pw_stream_rowgroups(int64_t M, int64_t N, int64_t K) {
  if (K != 64 && K != 128 && K != 256) return 0;
  const int bnb = 4 * pw_wn((int)K);
  if (N % bnb || N < 2 * K) return 0;  // write-heavy shapes only (N >= 2K)
  if (M * K * 2 >= (1ll << 31) - 4096 || M >= (1ll << 31)) return 0;
  const int64_t tiles = (M + pw::BM - 1) / pw::BM;
  const int64_t nbN = N / bnb;
  int64_t rg = pw_capacity((int)K) / nbN;  // one resident wave of blocks over the whole launch
  if (rg < 1) rg = 1;
  if (rg > tiles) rg = tiles;
  return (int)rg;
}

extern "C" int dpe_pw_stream_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int64_t M, int64_t N,
                                    int64_t K, int rg, hipStream_t st) {
  if (rg <= 0 || rg != dpe_pw_stream_rowgroups(M, N, K)) return -1;
  const int nbN = (int)(N / (4 * pw_wn((int)K)));
  const dim3 grid((unsigned)(rg * nbN)), block(256);
  if (K == 64) hipLaunchKernelGGL((pw::pw_stream_kernel<64, 64, 4>), grid, block, 0, st, x, w, y, stats, (int)M, (int)N, rg);
  else if (K == 128) hipLaunchKernelGGL((pw::pw_stream_kernel<128, 64, 3>), grid, block, 0, st, x, w, y, stats, (int)M, (int)N, rg);
  else hipLaunchKernelGGL((pw::pw_stream_kernel<256, 32, 2>), grid, block, 0, st, x, w, y, stats, (int)M, (int)N, rg);
  return 0;
}
