// Host-visible argument block for the implicit-GEMM kernels (igemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpe {

// How the A operand (M x K) is fetched.
enum ALoad : int {
  A_DENSE_K = 0,     // A[m][k] at A + m*lda + k         (K contiguous)
  A_DENSE_M = 1,     // A[m][k] at A + k*lda + m         (M contiguous)
  A_CONV_FWD = 2,    // im2col of NHWC x: m=(n,oh,ow), k=(r,s,ci)
  A_CONV_DGRAD = 3,  // col2im-gather of NHWC dy: m=(n,h,w), k=(r,s,co)
};
// How the B operand (K x N) is fetched.
enum BLoad : int {
  B_DENSE_K = 0,     // B[k][n] at B + n*ldb + k         (K contiguous)
  B_DENSE_N = 1,     // B[k][n] at B + k*ldb + n         (N contiguous)
  B_CONV_DGRAD = 2,  // weights [Co][R][S][Ci] as B[k=(r,s,co)][n=ci]
  B_CONV_WGRAD = 3,  // im2col of NHWC x as B[k=(n,oh,ow)][n=(r,s,ci)]
};
enum Epi : int {
  EPI_BF16 = 0,        // C (bf16) = act(alpha*acc + bias) [+ residual]
  EPI_F32 = 1,         // C (f32)  = act(alpha*acc + bias)
  EPI_ATOMIC_F32 = 2,  // C (f32) += alpha*acc  (split-K / accumulate)
  EPI_BF16_BNB = 3,    // EPI_BF16 + BatchNorm-backward partials of dL/dy in the epilogue (data-grad of a BN+ReLU input)
};
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };
// LDS-DMA conv kernel, dense A: the A operand is the output of a BatchNorm pass that is never run
// on its own -- computed on the fragments from two bf16 tensors (A, a2) and per-K-channel
// coefficients, and stored once as a by-product (a_out, a_bits) by the blocks of the first N tile.
enum AXform : int {
  AX_NONE = 0,
  AX_BN_RES = 1,   // relu(A * s[k] + t[k] + a2)                  a_coef = [scale | shift] (BN forward coef [4][K])
  AX_BN_RES2 = 2,  // relu(A * s[k] + t[k] + bf16(a2 * s2[k] + t2[k]))   + a_coef2 (the downsample BN's)
  AX_BN_BWD = 3,   // a[k] * A + b[k] * a2 + c[k]                  a_coef = [a | b | c] (BN backward coef [3][K])
  AX_CAT = 4,      // concatenated K: columns [0, k1) of A are A[m][k] (lda), columns [k1, K) are
                   // a2[m][k - k1] (lda2), relu(a2 * s[k-k1] + t[k-k1]) when a_coef = [s | t] is given
                   // (nothing stored; the Gram-algebra data grad [dz3 | a2] x [diag(a) W3 ; Q], bngram.hip)
};

struct ConvGeom {
  int N, H, W, C;      // input  NHWC
  int OH, OW, K;       // output NHW(K)
  int R, S;            // filter
  int sh, sw, ph, pw, dh, dw;
  // Phase-decomposed data-grad (stride > 1): the GEMM runs on a virtual
  // stride-1 problem over one output parity (a, b); taps t map to real filter
  // rows r = pr0 + psh*t (same for columns), and output row (n, hh, ww) is
  // stored at dX[n, oa + psh*hh, ob + psw*ww].  remap = 0: identity.
  int RR, SS;          // real filter dims (weight addressing)
  int pr0, ps0, psh, psw;
  int remap, Hr, Wr, oa, ob;
};

struct IgemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const uint16_t* residual;  // bf16 [M][ldc] added in the EPI_BF16 epilogue (may alias C)
  const float* bias;         // [N] or nullptr
  const float* residual_f32; // f32 [M][ldc] added in the EPI_F32 epilogue (x + f(a) on an fp32 residual stream)
  float* col_stats;          // [2][N][stats_ld] per-(column, M-tile) partial statistics of the stored bf16 output, or nullptr:
                             //   EPI_BF16:      (sum v, sum v^2)                      (BatchNorm forward)
                             //   EPI_BF16_BNB:  (sum dz, sum dz*(x - mean)),  dz = v * [x*scale+shift > 0],
                             //                  x = st_x, [scale|shift|mean|invstd] = st_coef  (BN+ReLU backward)
  const uint16_t* st_x;      // [M][ldc] bf16 pre-BN input (row indexing as C, incl. phase remap)  (EPI_BF16_BNB)
  const float* st_coef;      // [4][N]                                                            (EPI_BF16_BNB)
  const uint8_t* st_mask;    // EPI_BF16_BNB variant for a BN whose ReLU follows a residual add
                             //   (y = relu(BN(x) + idn)): ReLU-mask BITS of the saved y, one byte per
                             //   8 columns ([M][ldc/8], bit e = column 8j+e, written by bn_apply), and
                             //   the STORED value is the masked dz, not v
  int res_nt;                // residual is at its last use: stream it (non-temporal loads)
  const uint8_t* res_mask;   // optional ReLU-mask bits ([M][ldc/8]) applied to the residual before the add
                             //   (residual = dy of a BN+residual+ReLU output: dz = dy * relu'(y) on the fly)
  int stats_ld;              // partial columns per channel (0 -> tilesM of this launch)
  int stats_off;             // first partial column written by this launch (phase-decomposed dgrad)
  int M, N, K;
  int64_t lda, ldb, ldc;
  float alpha;
  const float* alpha_ptr;     // optional device scalar multiplied into alpha (loss-scale from autograd)
  int act;
  int k_split;  // K elements per split (multiple of 32); >= K means no split
  ConvGeom g;
  const float* b_coef;  // LDS-DMA weight grad, B_DENSE_N: B is a pre-BN tensor; the operand is
                        //   relu(B * b_coef[n] + b_coef[N + n]) (the BN output is never stored)
  // A on-load transform (AXform; LDS-DMA kernel, A_DENSE_K only)
  int a_mode;
  const uint16_t* a2;       // [M][lda] second operand of the transform
  const float* a_coef;      // per-K coefficients (see AXform)
  const float* a_coef2;     // AX_BN_RES2: the second BatchNorm's forward coefficients [4][K]
  uint16_t* a_out;          // [M][lda] the transformed A, written by the tn == 0 blocks (required)
  uint8_t* a_bits;          // [M][lda/8] ReLU-mask bits of a_out (AX_BN_RES / _RES2), or nullptr
  int k1;                   // AX_CAT: K of the first segment (multiple of 32)
  int64_t lda2;             // AX_CAT: row stride of a2
  float* slab;              // LDS-DMA weight grad only: EPI_ATOMIC_F32 partials STORED to slab[split][M][N]
                            //   (summed in split order by a finalize pass: deterministic) instead of atomics
};

// Up to 4 problems of one LDS-DMA tile class and tile count in one grid (igemm_dma_group_kernel): the
// per-parity sub-GEMMs of a strided data grad.
constexpr int IGEMM_GROUP_MAX = 4;
struct IgemmGroup {
  IgemmArgs a[IGEMM_GROUP_MAX];
  int n;
};

}  // namespace dpe

// n problems (<= IGEMM_GROUP_MAX) with equal M and N, forward-form (A_CONV_FWD or A_DENSE_K) on the LDS-DMA
// kernel, one grid; -1 when any is outside the kernel's envelope (the caller then launches them one by one).
extern "C" int dpe_igemm_dma_group_launch(const dpe::IgemmArgs* args, int n, int bm, int bn, int aload, int bload, int epi,
                                          hipStream_t stream);

extern "C" int dpe_igemm_launch(const dpe::IgemmArgs* args, int bm, int bn, int aload, int bload, int epi,
                                int splits, hipStream_t stream);

// LDS-DMA implicit-GEMM (igemm.hip) for forward-form convolutions and dense K-contiguous A
// (B K- or N-contiguous; EPI_BF16 / EPI_BF16_BNB, no split-K); LDS ring depth 2 for tiles up to
// 128x128 (4 blocks per CU), 3 for the 8-wave tiles.  -1: outside its envelope.
extern "C" int dpe_igemm_dma_launch(const dpe::IgemmArgs* args, int bm, int bn, int aload, int bload, int epi,
                                    hipStream_t stream);

// LDS-DMA weight-grad kernel (igemm.hip): A = dy (A_DENSE_M), B = x (B_DENSE_N) or its im2col
// (B_CONV_WGRAD), EPI_ATOMIC_F32 with split-K.  -1: outside its envelope.
extern "C" int dpe_igemm_wgrad_dma_launch(const dpe::IgemmArgs* args, int bm, int bn, int bload, int splits,
                                          hipStream_t stream);
