// 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels (ResNet-50 layer 1:
// the bottleneck conv2 forward and its stride-1 data grad, run as a forward conv of dy with the
// flipped filter), walking output rows.
//
// On the implicit-GEMM tiles these ran at ~500 TF (229 us forward at batch 512) with the L2 ~91 %
// busy: the im2col operand re-reads every input pixel once per tap (9x) and every tile re-reads the
// 72 KiB filter (profiles/pmc_conv3_r2.txt).  A tile-local halo in LDS (the filter in LDS too)
// measured slower: > 80 KiB per block left one block per CU with no overlap (docs/perf_notes.md).
// Here, as in the stem kernel (stem.hip):
//   * a block owns consecutive output rows of one image; wave (mh, nh) holds output channels
//     32 nh .. +31 of the filter in VGPRs (18 K-steps x 2 fragments, 144 VGPRs) for the whole block;
//   * the three input rows an output row needs sit in a 4-slot LDS ring ([W + 2][64 ch], 16-B
//     chunks XOR-swizzled by pixel, zero pixels at both ends); each input row is read from HBM once
//     per block (register prefetch two rows ahead, written into the free slot after the MFMAs);
//   * the output row is staged in one of two LDS buffers and stored as 16-B chunks of contiguous
//     pixels; the epilogue is the shared one's EPI_BF16 (BN-forward sums of the stored output) or
//     EPI_BF16_BNB (sum dz, sum dz*(x - mean) with the ReLU recomputed from the pre-BN input and its
//     coefficients), accumulated per thread and reduced once per block ([2][64][blocks]).
// One barrier per output row.  Same K order as the implicit GEMM (tap-major, 32-channel halves), so
// the stored output is bitwise identical to it.
#include "common.h"

namespace dpe {
namespace rowconv {

constexpr int CO = 64, KS = 18;           // channels, 32-wide K-steps (9 taps x 2 halves)
constexpr int SLOT_PX = 66;               // ring slot pixels: zero + <= 64 data + zero
constexpr int SLOT = SLOT_PX * 128;
constexpr int NSLOT = 4;
constexpr int OROW = 144;                 // staged output pixel stride (128 B + 16 pad)
constexpr int OBUF = 64 * OROW;
constexpr int LDS = NSLOT * SLOT + 2 * OBUF;
static_assert(LDS <= 163840 / 2, "two blocks per CU");

DPE_DEVICE u32x4 zero16() { return u32x4{0u, 0u, 0u, 0u}; }
DPE_DEVICE int pix_off(int sp, int chunk) { return sp * 128 + ((chunk ^ (sp & 7)) << 4); }

struct RowArgs {
  const uint16_t* x;      // [N][H][W][64] bf16
  const uint16_t* w;      // [64][3][3][64] bf16 (K-contiguous)
  uint16_t* y;            // [N][H][W][64] bf16
  float* stats;           // [2][64][blocks] or nullptr
  const uint16_t* st_x;   // BNB: pre-BN input [N][H][W][64]
  const float* st_coef;   // BNB: [4][64] scale, shift, mean, invstd
  int N, H, W, parts;
};

template <bool BNB>
__global__ __launch_bounds__(256, 2) void conv3x3_rows_kernel(RowArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* const ring = smem;
  char* const obuf = smem + NSLOT * SLOT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mh = wid & 1, nh = wid >> 1;  // pixels 32 mh .. +31, channels 32 nh .. +31
  const int H = p.H, W = p.W;
  const int blk = blockIdx.x;
  const int n = blk / p.parts, part = blk - n * p.parts;
  const int oh_beg = (int)((int64_t)H * part / p.parts), oh_end = (int)((int64_t)H * (part + 1) / p.parts);
  const int lm = lane & 15, kc = lane >> 4;

  // filter fragments: output channel 32 nh + 16 j + lm, K elements 32 ks + 8 kc .. +7
  bf16x8 wf[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      wf[ks][j] = __builtin_bit_cast(bf16x8, *(const u32x4*)(p.w + (32 * nh + 16 * j + lm) * 576 + 32 * ks + 8 * kc));

  for (int i = tid; i < NSLOT * SLOT / 16; i += 256) *(u32x4*)(ring + i * 16) = zero16();

  // one input row = W pixels x 8 chunks (<= 512): thread t owns chunks t and t + 256
  const int64_t img = (int64_t)n * H * W * 64;
  const int nch = W * 8;
  auto load_row = [&](int ih, u32x4 (&v)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      v[u] = (c < nch && (unsigned)ih < (unsigned)H) ? *(const u32x4*)(p.x + img + (int64_t)ih * W * 64 + c * 8) : zero16();
    }
  };
  auto write_row = [&](int ih, const u32x4 (&v)[2]) {  // input row ih -> slot (ih + 1) % 4, pixel iw + 1
    char* sl = ring + ((ih + 1 + 4 * NSLOT) % NSLOT) * SLOT;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      if (c < nch) *(u32x4*)(sl + pix_off((c >> 3) + 1, c & 7)) = v[u];
    }
  };
  __syncthreads();
  {
    u32x4 t0[2], t1[2], t2[2];
    load_row(oh_beg - 1, t0);
    load_row(oh_beg, t1);
    load_row(oh_beg + 1, t2);
    write_row(oh_beg - 1, t0);
    write_row(oh_beg, t1);
    write_row(oh_beg + 1, t2);
  }
  u32x4 pf0[2], pf1[2];
  load_row(oh_beg + 2, pf0);
  load_row(oh_beg + 3, pf1);
  __syncthreads();

  // store-phase channel chunk of this thread and its BN coefficients
  const int sc = tid & 7;
  float s[8], ss[8], bsc[8], bsh[8], bmu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = 0.f;
    ss[e] = 0.f;
    if constexpr (BNB) {
      bsc[e] = p.st_coef[sc * 8 + e];
      bsh[e] = p.st_coef[CO + sc * 8 + e];
      bmu[e] = p.st_coef[2 * CO + sc * 8 + e];
    }
  }
  // this wave's pixel fragments: 32 mh + 16 i + lm (rows >= W compute on zero pixels, never stored)
  const int nfr = min(2, max(0, (W - 32 * mh + 15) / 16));

  for (int oh = oh_beg; oh < oh_end; ++oh) {
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-step ks: tap t = ks / 2 (r = t / 3, s = t % 3), channel half ks & 1; input row
    // oh - 1 + r in slot (oh + r) % 4, pixel ow + s
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int t = ks >> 1, r = t / 3, s_ = t - 3 * (t / 3), hf = ks & 1;
      const char* sl = ring + ((oh + r) % NSLOT) * SLOT;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i < nfr) {
          const int sp = 32 * mh + 16 * i + lm + s_;
          const bf16x8 af = __builtin_bit_cast(bf16x8, *(const u32x4*)(sl + pix_off(sp, hf * 4 + kc)));
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][j], af, acc[i][j], 0, 0, 0);
        }
      }
    }
    // input row oh + 2 into the slot of row oh - 2 (free); prefetch row oh + 4
    write_row(oh + 2, pf0);
    pf0[0] = pf1[0];
    pf0[1] = pf1[1];
    load_row(oh + 4, pf1);
    // stage: acc[i][j][e] = pixel 32 mh + 16 i + lm, channel 32 nh + 16 j + 4 kc + e
    char* ob = obuf + (oh & 1) * OBUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < nfr) {
        const int ow = 32 * mh + 16 * i + lm;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x2 pk;
          pk[0] = pack_bf2(acc[i][j][0], acc[i][j][1]);
          pk[1] = pack_bf2(acc[i][j][2], acc[i][j][3]);
          *(u32x2*)(ob + ow * OROW + (32 * nh + 16 * j + 4 * kc) * 2) = pk;
        }
      }
    }
    __syncthreads();
    // store: thread t -> chunk t & 7 of pixels t / 8 and t / 8 + 32
    const int64_t rowoff = ((int64_t)n * H + oh) * W * CO;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int px = (tid >> 3) + 32 * k;
      if (px < W) {
        const int64_t off = rowoff + px * CO + sc * 8;
        const u32x4 v = *(const u32x4*)(ob + px * OROW + sc * 16);
        u32x4 xv;
        if constexpr (BNB) xv = *(const u32x4*)(p.st_x + off);
        *(u32x4*)(p.y + off) = v;
        if (p.stats) {
          float f[8];
          unpack8(v, f);
          if constexpr (BNB) {  // (sum dz, sum dz * (x - mean)), dz = f * relu'(x * scale + shift)
            float xf[8];
            unpack8(xv, xf);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dz = fmaf(xf[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
              s[e] += dz;
              ss[e] += dz * (xf[e] - bmu[e]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] = fmaf(f[e], f[e], ss[e]); }
          }
        }
      }
    }
  }
  if (p.stats) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s[e] += __shfl_xor(s[e], o, 64);
        ss[e] += __shfl_xor(ss[e], o, 64);
      }
    __syncthreads();
    float* red = (float*)ring;  // [2][4 waves][64]
    if (lane < 8)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid * CO + sc * 8 + e] = s[e];
        red[4 * CO + wid * CO + sc * 8 + e] = ss[e];
      }
    __syncthreads();
    if (tid < CO) {
      const int nb = gridDim.x;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) { a += red[q * CO + tid]; b += red[4 * CO + q * CO + tid]; }
      p.stats[(int64_t)tid * nb + blk] = a;
      p.stats[(int64_t)(CO + tid) * nb + blk] = b;
    }
  }
}

}  // namespace rowconv
}  // namespace dpe

// Blocks of the launch for an [N, H, W, 64] input (0: outside the kernel's envelope).
extern "C" int dpe_conv3x3_rows_blocks(int N, int H, int W) {
  if (N <= 0 || H < 2 || W < 1 || W > 64) return 0;
  return N * 2;
}

// y = conv3x3(x, w) (stride 1, pad 1, 64 -> 64 channels); bnb: stats are the BN-backward partials
// of the BN with pre-BN input st_x and coefficients st_coef, else the BN-forward sums of y.
extern "C" int dpe_conv3x3_rows_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const uint16_t* st_x,
                                       const float* st_coef, int N, int H, int W, int bnb, hipStream_t st) {
  const int nb = dpe_conv3x3_rows_blocks(N, H, W);
  if (nb <= 0 || (bnb && (!stats || !st_x || !st_coef))) return -1;
  dpe::rowconv::RowArgs a{x, w, y, stats, st_x, st_coef, N, H, W, 2};
  if (bnb) hipLaunchKernelGGL(dpe::rowconv::conv3x3_rows_kernel<true>, dim3(nb), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dpe::rowconv::conv3x3_rows_kernel<false>, dim3(nb), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
