// Host-visible argument block of the persistent dense GEMM (hgemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "igemm.h"  // ConvGeom

namespace dpe {

// Epilogue of one output tile (or K-split partial of it).
enum HEpi : int {
  HE_BF16 = 0,    // C bf16 = act(alpha*acc + bias)           (ACT_GELU: aux_out = pre-activation v)
  HE_F32 = 1,     // C f32  = alpha*acc + bias (+ residual_f32)
  HE_ACC_F32 = 2, // C f32 += alpha*acc                       (weight grads into fp32 buckets; no K split)
  HE_SLAB = 3,    // ws[split] f32 = acc (K-split partial; hgemm_finalize applies the real epilogue)
  HE_GROUP = 4,   // grouped TN weight grads: per problem g, C_g f32 (+)= alpha*acc (+ the fused bias grad)
};

// One problem of a grouped launch (HE_GROUP): several independent TN weight-gradient GEMMs sharing K
// (the token count), the 256x256 tile, no K split.  Units [tile_end of the previous problem,
// tile_end) are this problem's output tiles.
struct HgemmProblem {
  const uint16_t* A;  // dy, M-contiguous A[k][m] (lda)
  const uint16_t* B;  // x, N-contiguous B[k][n] (ldb)
  float* C;           // the fp32 weight gradient [M][ldc]
  float* dbias;       // [M] bias gradient (+= row sums of dy^T) or nullptr
  int64_t lda, ldb, ldc;
  int M, N, a_dim;    // a_dim: load extent of A's M (>= M; 0 = M)
  int tile_end;       // cumulative 256x256 tile count through this problem
  int overwrite;      // 1: C = alpha*acc (the gradient's first writer of the step), 0: C += alpha*acc
};
constexpr int HGEMM_MAX_GROUP = 12;
// act values beyond igemm.h's Act: gelu backward, C = (alpha*acc) * gelu'(aux_in)
constexpr int HACT_GELU_BWD = 3;
// HE_BF16 + the BatchNorm-backward partials of the stored values (a conv data grad dL/dy of a BN + ReLU
// output y = relu(BN(st_x))): per column (sum dz, sum dz*(st_x - mean)), dz = v * [st_x*scale+shift > 0],
// written to col_stats[2][N][stats_ld] at column stats_off + (m0 / BM) * WR + wave row (no atomics)
constexpr int HACT_BNB = 4;
// HE_BF16 + the BatchNorm-forward partials of the stored values (sum v, sum v^2), same layout as HACT_BNB
constexpr int HACT_BNF = 5;

constexpr int HGEMM_SCHED_BYTES = 17 * 1024;  // 17 counters, one 1 KB line each (hgemm.hip)

struct HgemmArgs {
  const uint16_t* A;        // bf16, K-contiguous A[m][k] (lda) or M-contiguous A[k][m] (lda)
  const uint16_t* B;        // bf16, K-contiguous B[n][k] (ldb) or N-contiguous B[k][n] (ldb)
  void* C;                  // output (ldc)
  const float* bias;        // [N] or nullptr
  const float* residual_f32;// HE_F32: [M][ldc] added to the result (may alias C)
  const uint16_t* aux_in;   // HACT_GELU_BWD: pre-activation v, bf16 [M][ldc]
  uint16_t* aux_out;        // HE_BF16 + ACT_GELU: v stored here, bf16 [M][ldc] (nullptr: not stored)
  float* ws;                // HE_SLAB: [splits][M][N] f32 partials
  const float* alpha_ptr;   // optional device scalar multiplied into alpha
  int M, N, K;
  int64_t lda, ldb, ldc;
  float alpha;
  int act;                  // ACT_NONE / ACT_GELU / HACT_GELU_BWD
  int splits;               // K splits (HE_SLAB when > 1)
  int kps;                  // K elements per split, multiple of 64
  int group_m;              // tile rows per grouped-order band (L2 reuse per XCD); <= 0: row-major
  int a_dim, b_dim;         // load extents of A's M / B's N (>= M / N; 0 = M / N): loads may read the
                            // zero-padded columns of a padded operand, stores stay inside M x N
  float* dbias;             // TN weight grads only: db[m] += alpha * sum_k A[k][m] (the bias gradient)
  float* ws_bias;           // dbias with splits > 1: [splits][M] partial row sums (summed by hgemm_finalize)
  unsigned* sched;          // dynamic unit claims (HGEMM_SCHED_BYTES zeroed, self-resetting; one per stream),
                            // or nullptr: static round-robin over the persistent grid
  // HACT_BNB / HACT_BNF (no K split): BN-backward / BN-forward partials
  float* col_stats;         // [2][N][stats_ld]
  const uint16_t* st_x;     // bf16 [M][ldc] pre-BN input of the BN whose output this GEMM's result is the gradient of
  const float* st_coef;     // [4][N]: scale, shift, mean, invstd
  int stats_ld;
  // HE_GROUP: the problems (A, B, C, M, N, lda, ldb, ldc, a_dim, dbias above are ignored)
  int ngroup;
  HgemmProblem grp[HGEMM_MAX_GROUP];
  // conv != 0 (K-contiguous A only): A is the implicit im2col of an NHWC tensor (conv_g: input N,H,W,C,
  // output OH,OW, filter R,S, stride / pad / dilation): row m = (n, oh, ow), column k = (r, s, ci);
  // C a power of two >= 64 (a 64-deep K-tile lies in one filter tap), conv_smagic = ceil(65536 / S)
  int conv;
  ConvGeom conv_g;
  int conv_smagic;
  // conv == 3 (K-contiguous A only): A is the concatenation [A (k1 columns, lda) | A2 (K - k1 columns,
  // lda2)] along K -- the Gram-algebra BN3 data grad [dz3 | a2] (bngram.hip); k1 % 64 == 0, no K split
  const uint16_t* A2;
  int64_t lda2;
  int k1;
  // Stream-K schedule (sk != 0; 1-block-per-CU tiles, no K split, static grid <= free CUs): the launch's T
  // tiles x K/64 K-steps are cut into gridDim.x equal contiguous ranges, one per block, so every block does
  // the same MFMA work whatever T mod grid is.  A tile cut over P blocks: the segment done last owns it;
  // the P - 1 others store fp32 partials (sk_ws: two [tile fragments][threads] x 16 B slabs per block,
  // write-through) and add to the tile's counter (sk_cnt[tile], zero before the launch); the owner waits
  // for P - 1, resets it, adds the partials in block order (run-to-run identical) and runs the epilogue.
  // sk_cnt[HGEMM_SK_MAX_TILES - 1] != 0: an owner gave up waiting (a block never ran; output invalid).
  int sk;
  float* sk_ws;
  unsigned* sk_cnt;
};
constexpr int HGEMM_SK_MAX_TILES = 8192;  // sk_cnt entries (one per output tile)

// Tile configurations (BMxBN, waves WRxWC).
enum HCfg : int {
  HC_256x256 = 0,  // 8 waves 2x4, 128 KiB LDS, 1 block/CU
  HC_128x256 = 1,  // 8 waves 2x4,  96 KiB LDS, 1 block/CU
  HC_256x128 = 2,  // 8 waves 4x2,  96 KiB LDS, 1 block/CU
  HC_128x128 = 3,  // 4 waves 2x2,  64 KiB LDS, 2 blocks/CU
};

}  // namespace dpe

// a_k / b_k: operand K-contiguous (1) or M/N-contiguous (0).  grid = persistent block count.
// Returns 0, or < 0 when the configuration is outside the kernel's envelope.
extern "C" int dpe_hgemm_launch(const dpe::HgemmArgs* args, int cfg, int a_k, int b_k, int epi, int grid,
                                hipStream_t stream);
// Grouped TN weight grads (HE_GROUP): args->ngroup problems, 256x256 tile, no K split.
extern "C" int dpe_hgemm_group_launch(const dpe::HgemmArgs* args, int grid, hipStream_t stream);
// Sum of `splits` f32 partial slabs [M][N] -> the real epilogue (bias, act, residual, bf16/f32 out).
extern "C" int dpe_hgemm_finalize(const dpe::HgemmArgs* args, int epi, hipStream_t stream);
