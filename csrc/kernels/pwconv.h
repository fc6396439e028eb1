// Host-visible arguments of the streaming pointwise-conv kernel (pwconv.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpe {

enum PwEpi : int {
  PW_FWD = 0,    // y = x . W^T; stats = BatchNorm-forward (sum, sum of squares) of the stored y
  PW_DGRAD = 1,  // y = x . W (+ residual [masked]); stats = BatchNorm-backward (sum dz, sum dz*(st_x - mean))
  PW_APPLY = 2,  // y = relu(BN(x . W^T) + residual): out_coef = the BN's [4][N] coefficients, known before the
                 // conv (Gram algebra, bngram.hip); the pre-BN tensor is never stored; out_bits = ReLU bits of y
  PW_DSUM = 3,   // PW_DGRAD with st_mask and no st_x: stats row 0 = sum dz only (row 1 left unwritten)
};

struct PwArgs {
  const uint16_t* x;         // [M][K] bf16 (forward: the conv input; data grad: dy)
  const uint16_t* w;         // PW_FWD: [N][K] (conv weight [Cout][Cin]); PW_DGRAD: [K][N] (the same tensor)
  uint16_t* y;               // [M][N] bf16
  float* stats;              // [2][N][row groups] partials, or nullptr
  const uint16_t* residual;  // PW_DGRAD: bf16 [M][N] added to y, or nullptr
  const uint8_t* res_mask;   // PW_DGRAD: ReLU bits of the residual's producer ([M][N/8]), or nullptr
  const uint16_t* st_x;      // PW_DGRAD BN backward: pre-BN input [M][N]; nullptr = no stats
  const float* st_coef;      // [4][N]: scale, shift, mean, invstd of that BatchNorm
  const uint8_t* st_mask;    // ReLU bits of the BN output ([M][N/8]); the stored y is then the masked dz
  int64_t M, N, K;
  int rg;                    // row groups (= partial columns), from dpe_pw_rowgroups
  const float* in_coef;      // PW_FWD: x is the pre-BN tensor; the operand is relu(x * in_coef[k] + in_coef[K + k])
  int res_h, res_w;          // PW_DGRAD, > 0: y is an [*, res_h, res_w] image and the residual is the compact
                             // [*, res_h/2, res_w/2] grid of a stride-2 1x1 conv's data grad, added at even (h, w) only
  const float* out_coef;     // PW_APPLY: [4][N] BN coefficients (scale, shift, ...) applied to the conv output
  const float* res_coef;     // PW_APPLY: the residual is BN'd first: bf16(residual * res_coef[n] + res_coef[N + n])
  uint8_t* out_bits;         // PW_APPLY: ReLU bits of y ([M][N/8]), or nullptr
  unsigned* sched;           // claim counters (HGEMM_SCHED_BYTES, zeroed, left zeroed) for the dynamic schedule,
                             // or nullptr: static (see dpe_pw_rowgroups)
};

// The concatenated-K data grad of the Gram-path BN3 backward (bngram.hip) on a streaming kernel:
//   y[M][N] = [dz | relu(h2 * s + t)] . Bcat + e,  N = K2 (the bottleneck width: 64 or 128), K1 = 4 N,
// with the BN2-backward partials (sum dz, sum dz*(h2 - mean)) of the stored y; mask and h2 from the raw h2
// tile the kernel already holds in LDS (the LDS-DMA implicit GEMM re-read h2 for its epilogue).
struct PwCatArgs {
  const uint16_t* dz;     // [M][K1] bf16
  const uint16_t* h2;     // [M][K2] bf16, pre-BN2
  const float* coef;      // BN2 [4][K2]: scale, shift, mean, invstd
  const uint16_t* bcat;   // [K1 + K2][N] bf16
  const float* ebias;     // [N]
  uint16_t* y;            // [M][N] bf16
  float* stats;           // [2][N][rg]
  int64_t M;
  int rg;                 // blocks (= partial columns)
};

}  // namespace dpe

// Blocks (= partial columns) of the concatenated-K data grad for (M, K1, K2), 0: outside the kernel's envelope.
extern "C" int dpe_pw_cat_blocks(int64_t M, int64_t K1, int64_t K2);
extern "C" int dpe_pw_cat_launch(const dpe::PwCatArgs* args, int64_t K1, int64_t K2, hipStream_t stream);

// Row groups of the launch for (M, N, K, epi), or 0 outside the kernel's envelope
// (K in {64, 128, 256}, N a multiple of the block's column slice, N >= 2K).  With a CU budget in force
// (dpe_cu_reserve() > 0: collectives in flight) there are three times as many row groups as resident block
// rows and the last two thirds are claimed at run time (PwArgs::sched); otherwise one per resident block row.
extern "C" int dpe_pw_rowgroups(int64_t M, int64_t N, int64_t K, int epi);
extern "C" int dpe_pw_launch(const dpe::PwArgs* args, int epi, hipStream_t stream);
