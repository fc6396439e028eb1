// Deterministic launch planning of the persistent GEMM (bindings/gemm.cpp).
#pragma once
#include <stdint.h>

#include "../kernels/hgemm.h"

namespace dpe_gemm {

struct Plan {
  int cfg;       // dpe::HCfg, -1 if none fits
  int splits;    // K splits (> 1: fp32 slabs + finalize)
  int kps;       // K elements per split
  int grid;      // persistent workgroups
  double est_s;  // modelled time
};

// A plan in up to two launches: `main` over output rows/columns [0, at) and `tail` over the rest
// (axis 0: columns, 1: rows; -1: a single launch, `main` covers everything).
struct Plan2 {
  Plan main{-1, 1, 0, 0, 1e30};
  Plan tail{-1, 1, 0, 0, 0.0};
  int axis = -1;
  int at = 0;
  double est_s = 1e30;
};

int num_cus();
// The per-(device, stream) zeroed claim-counter buffer of the dynamic schedules (HGEMM_SCHED_BYTES; the
// persistent GEMM's and the streaming pointwise conv's -- launches on one stream are ordered and each
// leaves it zeroed), or nullptr (dynamic schedules off, or the stream is being captured).
#include <hip/hip_runtime.h>
unsigned* sched_buffer(hipStream_t st);
bool layout_ok(int cfg, int ak, int bk);
// out_bytes: bytes per output element of the final epilogue (slab traffic estimate)
Plan plan(int64_t M, int64_t N, int64_t K, int ak, int bk, bool allow_split, int out_bytes, int force_cfg = -1,
          int force_splits = -1);
Plan2 plan2(int64_t M, int64_t N, int64_t K, int ak, int bk, bool allow_split, int out_bytes);
// Plans, allocates the split workspace if any and launches; returns the tile configuration used.
// fin_stream (K-split plans only): the slab reduction (hgemm_finalize) runs there, ordered after the
// slab kernel by an event -- a memory-bound pass co-resident with the next compute-bound GEMM on the
// current stream.  The caller makes every consumer of C wait for fin_stream.
int run(dpe::HgemmArgs& a, int ak, int bk, int epi, bool allow_split, int out_bytes, hipStream_t fin_stream = nullptr);
// The BN-backward-partials GEMM (HE_BF16 + HACT_BNB): one launch, no K split.  plan_bnb returns the
// plan and the number of partial columns it writes (tile rows x wave rows); run_bnb launches it.
Plan plan_bnb(int64_t M, int64_t N, int64_t K, int ak, int bk, int* partial_cols);
void run_bnb(dpe::HgemmArgs& a, const Plan& pl, int ak, int bk);  // a.act: HACT_BNB (default) or HACT_BNF
// dW (+)= dy^T im2col(x) (a.conv = 2: the TN layout with an implicit-im2col B), planned and launched in one
// piece (K-split slabs + finalize when the planner splits; fin_stream as run()).
void run_conv_wgrad(dpe::HgemmArgs& a, hipStream_t fin_stream);
// A plan's single launch, bf16 out, no epilogue extras (the implicit-im2col convs without statistics).
void launch_plain(dpe::HgemmArgs& a, const Plan& pl, int ak, int bk);

}  // namespace dpe_gemm
