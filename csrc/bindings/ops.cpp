// pybind11 bindings for the gfx950 kernels.  Every entry point validates
// device / dtype / layout and fails loudly (no silent fallback), picks the
// launch configuration (tile shape, split-K) and enqueues on torch's current
// HIP stream, so the ops compose with the caching allocator and hipGraph
// capture (no host sync, no hipMalloc inside).
#include <torch/extension.h>
#include <cstring>
#include <map>
#include <string>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "../kernels/igemm.h"
#include "../kernels/hgemm.h"
#include "../kernels/pwconv.h"
#include "gemm_plan.h"

using at::Tensor;

extern "C" {
int dpe_cu_reserve();  // comm.cpp: slots to leave to in-flight collectives
int dpe_gram_blocks(int64_t M, int C);
int64_t dpe_gram_ws_floats(int64_t M, int C);
int dpe_gram(const uint16_t* x, const float* coef, const float* scoef, int64_t M, int C, float* ws, float* G, float* s,
             hipStream_t st);
int dpe_gram_coef(const float* G, const float* s, const uint16_t* w, int Cin, int Cout, int64_t M, const float* gamma,
                  const float* beta, float* rmean, float* rvar, float momentum, float eps, float* coef, float* u,
                  hipStream_t st);
int64_t dpe_gram_bwd_ws_floats(int Cin, int Cout);
int dpe_gram_bwd(const float* part, int rg, const float* P, const uint16_t* w, const float* u, const float* s,
                 const float* coef3, const float* gamma, int Cin, int Cout, int64_t M, float* dgamma, float* dbeta,
                 float* dw, uint16_t* bcat, float* abc, float* ebias, float* qws, hipStream_t st);
int dpe_bn_stats_nblocks(int64_t M, int C);
int dpe_bn_bwd_nblocks(int64_t M, int C);

int dpe_bn_stats(const uint16_t* x, int64_t M, int C, int nb, float* part, hipStream_t st);
int dpe_bn_finalize(const float* part, int nb, int C, int64_t M, const float* gamma, const float* beta, float* rmean,
                    float* rvar, float momentum, float eps, float* coef, hipStream_t st);
int dpe_bn_eval_coeff(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                      float* coef, hipStream_t st);
int dpe_bn_apply(const uint16_t* x, const uint16_t* res, uint16_t* y, int64_t M, int C, const float* coef, int relu,
                 hipStream_t st);
int dpe_bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint8_t* ybits, const uint16_t* x, const float* coef, int64_t M, int C, int nb,
                      float* part, hipStream_t st);
int dpe_bn_bwd_reduce_apply(const uint16_t* dz, const uint16_t* x, const float* coef, const uint16_t* ax, const float* abcoef,
                            uint16_t* adx, int64_t M, int C, int nb, float* part, hipStream_t st);
int dpe_bn_bwd_finalize(const float* part, int nb, int C, int64_t M, const float* gamma, const float* coef, float* dgamma,
                        float* dbeta, float* bcoef, hipStream_t st);
int dpe_bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint8_t* ybits, const uint16_t* x, const float* bcoef, uint16_t* dx,
                     uint16_t* dz_out, int64_t M, int C, const float* mcoef, hipStream_t st);
int dpe_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH, int OW, int k, int s,
                    int p, hipStream_t st);
int dpe_bn_apply2(const uint16_t* x, const float* coef, const uint16_t* x2, const float* coef2, uint16_t* y, int64_t M, int C,
                  int relu, uint8_t* mbits, hipStream_t st);
int dpe_bn_apply_m(const uint16_t* x, const uint16_t* res, uint16_t* y, int64_t M, int C, const float* coef, int relu,
                   uint8_t* mbits, hipStream_t st);
void dpe_set_pool_legacy(int on);
int dpe_bnrelu_maxpool_fwd(const uint16_t* h, const float* coef, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH,
                           int OW, int k, int s, int p, hipStream_t st);
int dpe_stem_wgrad_launch2(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W,
                           float alpha, const uint16_t* dyp, const uint8_t* idx, const uint16_t* h, const float* coef,
                           const float* bcoef, hipStream_t st);
int dpe_maxpool_bn_bwd_reduce(const uint16_t* dy, const uint8_t* idx, const uint16_t* x, const float* coef, int N, int H, int W,
                              int C, int OH, int OW, int k, int s, int p, int nb, float* part, hipStream_t st);
int dpe_maxpool_bn_bwd_apply(const uint16_t* dy, const uint8_t* idx, const uint16_t* x, const float* coef, const float* bcoef,
                             uint16_t* dx, int N, int H, int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st);
int dpe_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int OH, int OW, int k,
                    int s, int p, hipStream_t st);
int dpe_gavgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st);
int dpe_gavgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st);
int dpe_cross_entropy_mean(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld,
                           float grad_scale, void* dlogits, int out_bf16, float* loss_rows, float* out4, int ignore_index,
                           hipStream_t st);
int dpe_ce_grad_scale(const void* d, void* o, int64_t n, int bf16, const float* g, const float* inv_n, hipStream_t st);
int dpe_cross_entropy(const void* logits, int in_bf16, const int64_t* labels, int B, int V, int64_t ld, float grad_scale,
                      void* dlogits, int out_bf16, float* loss_rows, float* loss_sum, float* correct, int ignore_index,
                      hipStream_t st);
int dpe_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st);
int dpe_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st);
int dpe_act(const void* a, const void* b, void* out, int64_t n, int op, int bf16, hipStream_t st);
int dpe_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, uint64_t offset, int bf16, hipStream_t st);
int dpe_cu_hog(int nblocks, int threads, int lds_bytes, double us, int vgprs, const unsigned* stop, float* sink,
               int sleepy, float* buf, hipStream_t st);
int64_t dpe_cu_hog_buf_floats(int nblocks);
int dpe_hog_stop(unsigned* stop, unsigned v, hipStream_t st);
int dpe_conv3x3_rows_blocks(int N, int H, int W);
int dpe_wgrad3x3_rows_blocks(int N, int H, int W);
int64_t dpe_wgrad3x3_rows_scratch(int nb);
int dpe_wgrad3x3_rows_launch(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W, int nb,
                             float alpha, const float* in_coef, hipStream_t st);
int dpe_conv3x3_rows_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const uint16_t* st_x,
                            const float* st_coef, int N, int H, int W, int nb, int bnb, const float* in_coef, hipStream_t st);
int dpe_stem_blocks(int N, int H, int W);
int64_t dpe_stem_wgrad_scratch(int N, int H, int W);
int dpe_stem_wgrad_launch(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W,
                          float alpha, hipStream_t st);
int dpe_stem_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H, int W, hipStream_t st);
int dpe_add(const void* a, const void* b, void* out, int64_t n, float alpha, int bf16, hipStream_t st);
int dpe_colsum(const void* dy, int64_t M, int N, int64_t ld, float* db, int accumulate, int bf16, hipStream_t st);
int dpe_nchw_to_s2d(const float* x, uint16_t* y, int N, int C, int H, int W, hipStream_t st);
int dpe_flip_desc_bytes();
int dpe_flip_blocks(int K, int C, int Rp, int Sp);
int dpe_conv_w_flipT_multi(const void* desc, const int* start, int n, int total_blocks, hipStream_t st);
int dpe_conv_w_flipT(const uint16_t* w, uint16_t* wt, int K, int R, int S, int C, int r0, int rs, int Rp, int s0, int ss,
                     int Sp, hipStream_t st);
int dpe_nchw_to_nhwc(const float* x, uint16_t* y, int N, int C, int HW, int Cp, hipStream_t st);
int dpe_embedding_fwd(const int64_t* idx, const uint16_t* wte, const uint16_t* wpe, float* out, int64_t rows, int T, int D,
                      hipStream_t st);
int dpe_embedding_bwd(const int64_t* idx, const float* dout, float* dwte, float* dwpe, int64_t rows, int T, int D,
                      hipStream_t st);
int dpe_optim_chunk_size();
int dpe_optim_desc_bytes();
int dpe_optim_step(int kind, const void* desc, const void* chunks, int nchunks, const float* hp, const float* steps,
                   hipStream_t st);
int dpe_layernorm_fwd(const void* x, int x_bf16, const float* w, const float* b, uint16_t* y, float* mean, float* rstd,
                      int64_t rows, int D, float eps, hipStream_t st);
int dpe_layernorm_bwd_nblocks(int64_t rows);
int64_t dpe_layernorm_bwd_scratch(int64_t rows, int D);
int dpe_layernorm_bwd(const uint16_t* dy, const void* x, int x_bf16, const float* w, const float* mean, const float* rstd,
                      void* dx, int dx_accumulate_f32, const float* res_in, uint16_t* dx_bf16, float* dw, float* db,
                      float* part, int64_t rows, int D, hipStream_t st);
int dpe_layernorm_bwd_finalize_group(const float* const* parts, const int64_t* rows, const int* Ds, float* const* dws,
                                     float* const* dbs, int n, hipStream_t st);
int dpe_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int T, int H, int D, float scale, int causal,
                 hipStream_t st);
int dpe_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, float* delta,
                 float* dq_acc, uint16_t* dqkv, int B, int T, int H, int D, float scale, int causal, hipStream_t st);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_RC(rc, what)                                                                          \
  do {                                                                                              \
    const int rc_ = (rc);                                                                           \
    const hipError_t e_ = hipGetLastError();                                                        \
    TORCH_CHECK(rc_ == 0 && e_ == hipSuccess, "dpe kernel launch failed: " what " rc=", rc_, " hip=", \
                hipGetErrorString(e_));                                                             \
  } while (0)

inline const uint16_t* bp(const Tensor& t) { return (const uint16_t*)t.data_ptr(); }
inline uint16_t* bpm(const Tensor& t) { return (uint16_t*)t.data_ptr(); }
inline float* fp(const Tensor& t) { return (float*)t.data_ptr(); }
inline const float* fpo(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? (const float*)t->data_ptr() : nullptr; }
inline float* fpom(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? (float*)t->data_ptr() : nullptr; }

// --------------------------------------------------------------- GEMM tiling
struct Cfg { int bm, bn, splits, k_split; };

Cfg pick_cfg(int64_t M, int64_t N, int64_t K, bool allow_split) {
  Cfg c{128, N <= 64 ? 64 : 128, 1, (int)((K + 31) / 32 * 32)};
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  const int64_t target = 512;  // >= 2 workgroups per CU on 256 CUs
  if (allow_split && K >= 32 * 64) {
    // split-K (weight-grad) GEMMs: big K, small output.  Keep the largest
    // tile (highest MFMA:LDS ratio) and let the K split supply parallelism.
    c.bm = M <= 64 ? 64 : 128;
    c.bn = N <= 64 ? 64 : 128;
    const int64_t t = tiles(c.bm, c.bn);
    const int64_t ksteps = (K + 31) / 32;
    // register-staged weight-grad tiles (1x1 with 128 channels): 512 blocks (768 / 1024 / 1536 measured
    // worse, docs/perf_notes.md); the LDS-DMA im2col weight-grad kernel re-derives its split (run_igemm)
    // (at the CU budget -- an overlapped RCCL collective holding `reserve` slots -- a slot fewer per
    // reserved workgroup, so the split still fits one resident wave: SURVEY §5.8 item 7)
    // (budget in force: two such rounds, as the LDS-DMA weight grads in run_igemm)
    const int64_t target_blocks =
        std::max<int64_t>(64, (dpe_cu_reserve() > 0 ? 2 : 1) * (2 * (int64_t)dpe_gemm::num_cus() - dpe_cu_reserve()));
    const int64_t per = dpe_cu_reserve() > 0 ? target_blocks / t : (target_blocks + t - 1) / t;
    int64_t splits = std::max<int64_t>(1, std::min<int64_t>(per, ksteps / 8));
    const int64_t kps = (ksteps + splits - 1) / splits;
    c.k_split = (int)(kps * 32);
    c.splits = (int)((ksteps + kps - 1) / kps);
    return c;
  }
  if (tiles(c.bm, c.bn) < target && M <= 64) c.bm = 64;
  if (tiles(c.bm, c.bn) < target && c.bn == 128 && c.bm == 128 && tiles(128, 64) <= tiles(64, 128)) c.bn = 64;
  if (tiles(c.bm, c.bn) < target && c.bm == 128) c.bm = 64;
  if (tiles(c.bm, c.bn) < target && c.bn == 128) c.bn = 64;
  if (allow_split) {
    const int64_t t = tiles(c.bm, c.bn);
    int64_t splits = (1024 + t - 1) / t;
    const int64_t ksteps = (K + 31) / 32;
    const int64_t max_splits = std::max<int64_t>(1, ksteps / 4);  // >= 4 K-steps per split
    splits = std::min(splits, max_splits);
    if (splits < 1) splits = 1;
    const int64_t kps = (ksteps + splits - 1) / splits;
    c.k_split = (int)(kps * 32);
    c.splits = (int)((ksteps + kps - 1) / kps);
  }
  return c;
}

// DPE_IGEMM_DMA=0: forward-form convolutions stay on the register-staged kernel (A/B reference)
bool igemm_dma_on() {
  static const bool on = [] { const char* e = getenv("DPE_IGEMM_DMA"); return !(e && e[0] == '0'); }();
  return on;
}

// DPE_WGRAD_DMA=0: im2col weight grads on the register-staged kernel (documented fallback)
bool wgrad_dma_on() {
  static const bool on = [] { const char* e = getenv("DPE_WGRAD_DMA"); return !(e && e[0] == '0'); }();
  return on;
}
// 64x256 weight-grad tile: 1 = for the C <= 16 stem, 2 = also for C > 16 (test hook set_wgrad_wide;
// measured slower there: 388 -> 512 us on the 64->64 3x3), 0 = never
int g_wgrad_wide = 1;

// Tile of the LDS-DMA conv kernel: 0 auto, 1 128-tile (pick_cfg), 2 256x128, 3 256x256
// (8 waves; only where pick_cfg chose a 128-row tile, so BN partial layouts never change).
// Forced tiles are a test hook (set_conv_tile): every one is numerics-tested, only "auto" is timed.
int g_dma_tile = [] { const char* e = getenv("DPE_CONV_TILE"); return e ? atoi(e) : 0; }();  // (env: A/B runs)
int dma_tile_mode() { return g_dma_tile; }

void dma_tile(const dpe::IgemmArgs& a, int aload, int bload, int& bm, int& bn) {
  if (bm != 128) return;
  // (1x1 data grads, N-contiguous weights: the 256x128 8-wave tile measured slower at K >= 1024,
  // ResNet-50 37.77-37.82 vs 37.63-37.67 ms: they stay on the 128-row tiles)
  if (bload != dpe::B_DENSE_K) return;
  int mode = dma_tile_mode();
  const bool taps = aload == dpe::A_CONV_FWD && a.g.R * a.g.S > 1;
  if (a.N <= 64) {
    // N = 64 with K >= 256 (layer-1 3x3 forward / data grad, 1x1 256->64): 256x64 tile, 4 waves of
    // 64x64 on a 2-stage ring (40 KiB, 4 blocks/CU): 236 -> 229 / 227 -> 213 / 215 -> 203 us
    // (profiles/conv_w64_ab_r2.txt; a 3-stage ring's 60 KiB halved the blocks per CU: 296 / 271 us).
    // Not the C = 16 s2d stem (short K: 519 -> 539 us on 256x64 with the 2-stage ring).
    const bool stem = aload == dpe::A_CONV_FWD && a.g.C == 16;
    if (mode >= 2 || (mode == 0 && a.K >= 256 && !stem)) { bm = 256; bn = 64; }
    return;
  }
  if (mode == 0) {
    // measured (scripts/bench_convs.py, batch 512): 256x128 wins on 3x3 convs with K >= 576 and
    // on K >= 1024; 256x256 (one block per CU) loses on most ResNet-50 shapes
    mode = (a.K >= 1024 || (taps && a.K >= 576)) ? 2 : 1;
  }
  if (mode == 3 && a.N > 128) { bm = 256; bn = 256; }
  else if (mode >= 2 && a.N > 64) { bm = 256; bn = 128; }
}

// Strided data grads: the per-parity sub-GEMMs in one grid (igemm_dma_group_kernel) with DPE_PHASE_GROUP=1 or
// set_phase_group(true); default one launch per parity.  Measured neutral (ResNet-50 31.07-31.13 vs
// 31.10-31.16 ms/step; per shape 492 / 334 / 251 vs 487 / 329 / 232 us with the BN epilogue, layers 2 / 3 / 4:
// the shared dy rows and the single launch are not what the parity sub-GEMMs lose their time to)
bool g_phase_group = [] { const char* e = getenv("DPE_PHASE_GROUP"); return e && e[0] == '1'; }();

// ---------------------------------------------------------- flipped filters
// The stride-1 / per-parity data grads run as forward convs of dy with flipped, transposed filters
// (conv_w_flipT).  A filter only changes when the optimizer (or a torch-side edit) rewrites the bf16 shadow,
// which bumps the weight epoch (set_weight_epoch, ops/_state.py).  The flipped copies are cached per (filter,
// tap subset) and, at the first request of a new epoch, ALL cached copies are refreshed in one launch (one
// instead of ~26 per ResNet-50 backward); a copy first requested in this epoch is flipped on its own.
struct FlipDescHost {
  const uint16_t* w;
  uint16_t* wt;
  int K, R, S, C, r0, rs, Rp, s0, ss, Sp;
};
struct FlipEntry {
  Tensor w, wt;
  FlipDescHost d;
  int64_t epoch;
};
std::vector<FlipEntry> g_flips;
int64_t g_weight_epoch = 0;
Tensor g_flip_desc, g_flip_start;  // device copies of the descriptor table (rebuilt when the set changes)
bool g_flip_table_dirty = true;
int g_flip_total = 0;

Tensor flipped(const Tensor& w, int K, int R, int S, int C, int r0, int rs, int Rp, int s0, int ss, int Sp) {
  static const bool cache_on = [] { const char* e = getenv("DPE_FLIP_CACHE"); return !(e && e[0] == '0'); }();
  if (!cache_on) {
    Tensor wt = at::empty({C, Rp, Sp, K}, w.options());
    CHECK_RC(dpe_conv_w_flipT(bp(w), bpm(wt), K, R, S, C, r0, rs, Rp, s0, ss, Sp, cur_stream()), "conv_w_flipT");
    return wt;
  }
  if (!g_flips.empty() && g_flips.front().w.device() != w.device()) {
    // one device per table: the batched refresh launches on the current device's stream
    g_flips.clear();
    g_flip_desc = Tensor();
    g_flip_start = Tensor();
    g_flip_table_dirty = true;
  }
  FlipEntry* hit = nullptr;
  for (auto& e : g_flips)
    if (e.d.w == bp(w) && e.w.is_same(w) && e.d.K == K && e.d.R == R && e.d.S == S && e.d.C == C && e.d.r0 == r0 &&
        e.d.rs == rs && e.d.Rp == Rp && e.d.s0 == s0 && e.d.ss == ss && e.d.Sp == Sp) {
      hit = &e;
      break;
    }
  if (hit && hit->epoch == g_weight_epoch) return hit->wt;
  if (hit) {
    // a new epoch: refresh every cached copy at once.  This first stale request comes from the first
    // flipped-filter user of the backward pass; every other cached filter's layer back-propagates after it,
    // so none of them can have been stepped yet -- with DDP.overlap_optimizer a bucket is stepped only after
    // every reader of its parameters returned -- and all cached weights are current (one device: below)
    if (g_flip_table_dirty) {
      std::vector<int> start(g_flips.size() + 1, 0);
      std::vector<FlipDescHost> desc(g_flips.size());
      for (size_t i = 0; i < g_flips.size(); ++i) {
        desc[i] = g_flips[i].d;
        start[i + 1] = start[i] + dpe_flip_blocks(desc[i].K, desc[i].C, desc[i].Rp, desc[i].Sp);
      }
      TORCH_CHECK((int)sizeof(FlipDescHost) == dpe_flip_desc_bytes(), "FlipDesc ABI mismatch");
      auto u8 = at::TensorOptions().dtype(at::kByte);
      Tensor hd = at::empty({(int64_t)(desc.size() * sizeof(FlipDescHost))}, u8);
      memcpy(hd.data_ptr(), desc.data(), desc.size() * sizeof(FlipDescHost));
      Tensor hs = at::empty({(int64_t)start.size()}, at::TensorOptions().dtype(at::kInt));
      memcpy(hs.data_ptr(), start.data(), start.size() * sizeof(int));
      g_flip_desc = hd.to(w.device());
      g_flip_start = hs.to(w.device());
      g_flip_total = start.back();
      g_flip_table_dirty = false;
    }
    CHECK_RC(dpe_conv_w_flipT_multi(g_flip_desc.data_ptr(), (const int*)g_flip_start.data_ptr(), (int)g_flips.size(),
                                    g_flip_total, cur_stream()),
             "conv_w_flipT_multi");
    for (auto& e : g_flips) e.epoch = g_weight_epoch;
    return hit->wt;
  }
  if (g_flips.size() >= 256) {  // (models come and go in tests: bounded, nothing stale is kept alive)
    g_flips.clear();
    g_flip_desc = Tensor();
    g_flip_start = Tensor();
  }
  Tensor wt = at::empty({C, Rp, Sp, K}, w.options());
  CHECK_RC(dpe_conv_w_flipT(bp(w), bpm(wt), K, R, S, C, r0, rs, Rp, s0, ss, Sp, cur_stream()), "conv_w_flipT");
  g_flips.push_back(FlipEntry{w, wt, FlipDescHost{bp(w), bpm(wt), K, R, S, C, r0, rs, Rp, s0, ss, Sp}, g_weight_epoch});
  g_flip_table_dirty = true;
  return wt;
}

void run_igemm(dpe::IgemmArgs& a, int aload, int bload, int epi, bool allow_split, bool conv = false,
               bool deterministic = false, bool overwrite = false) {
  Cfg c = pick_cfg(a.M, a.N, a.K, allow_split && epi == dpe::EPI_ATOMIC_F32);
  a.k_split = c.k_split;
  // weight grads over an im2col B (3x3 / strided; split-K fp32 atomics): LDS-DMA kernel, measured 1.3-1.5x
  // faster (scripts/bench_convs.py) (DPE_WGRAD_DMA=0: the im2col ones register-staged)
  // the dense 1x1 ones (< 256 channels) too: on the LDS-DMA kernel since its round-5 changes, same-box
  // ResNet-50 31.42-31.47 vs 31.48-31.60 ms/step (3 alternating pairs; the register-staged tile measured
  // 10-15 % faster in round 1).  DPE_WGRAD_DMA_1X1=0: register-staged (A/B)
  static const bool dma_1x1 = [] { const char* e = getenv("DPE_WGRAD_DMA_1X1"); return !(e && e[0] == '0'); }();
  if (conv && epi == dpe::EPI_ATOMIC_F32 && aload == dpe::A_DENSE_M &&
      ((igemm_dma_on() && wgrad_dma_on() && bload == dpe::B_CONV_WGRAD) ||
       (bload == dpe::B_DENSE_N && (a.b_coef || (dma_1x1 && igemm_dma_on()))))) {
    int bm = c.bm, bn = c.bn, splits = c.splits;
    {
      // ~3 resident 128x128 blocks per CU (4 fit): ResNet-50 step, alternating
      // (profiles/wgrad_blocks_ab_r2.txt, all split-K weight grads at one target): 256 -8 %, 384 -2.4 %,
      // 512 0, 768 +1.4-1.8 %, 1024 -0.5 %, 1536 -0.5 %, 2048 -1 %; 704-768 best of 640-896.  The
      // register-staged 1x1 tiles measured best at 512 and keep pick_cfg's split.
      // 3 per CU (768 on 256 CUs), less the slots an overlapped RCCL collective holds (CU budget,
      // comm.cpp): a split that needs more blocks than fit beside the collective's workgroups runs a
      // second, nearly empty wave (x1.56-1.60 per kernel next to 16 RCCL-sized workgroups,
      // profiles/cu_hog_probe_r3.txt in git history).  Rounded down, so tiles x splits <= the target.
      // With a CU budget in force the split targets TWO rounds of blocks: foreign workgroups do not take
      // our slots away (they fit beside them) but slow the CUs they share, and with one round the
      // slowest CU set the kernel's time (x1.27 next to 16 VALU-bound hogs, profiles/cu_hog_probe_r4.txt);
      // with two, the dispatcher gives those CUs fewer blocks.
      static const bool two_rounds = [] { const char* e = getenv("DPE_WGRAD_TWO_ROUNDS"); return !(e && e[0] == '0'); }();
      const int rsv = dpe_cu_reserve();
      const int64_t dma_target = std::max<int64_t>(64, (rsv > 0 && two_rounds ? 2 : 1) * (3 * (int64_t)dpe_gemm::num_cus() - rsv));
      const int64_t t = (int64_t)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn), ksteps = (a.K + 31) / 32;
      const int64_t rs = dpe_cu_reserve() > 0 ? dma_target / t : (dma_target + t - 1) / t;  // (unchanged at no reserve)
      const int64_t sp = std::max<int64_t>(1, std::min<int64_t>(rs, ksteps / 8));
      const int64_t kps = (ksteps + sp - 1) / sp;
      a.k_split = (int)(kps * 32);
      splits = (int)((ksteps + kps - 1) / kps);
    }
    if (c.bm == 64 && bload == dpe::B_CONV_WGRAD && a.N >= 256 && g_wgrad_wide && (a.g.C <= 16 || g_wgrad_wide > 1)) {
      // Cout = 64 with few channels per tap (the stem): 64x256 tile (4 waves across N), split-K
      // re-derived for its tile count.  Measured: stem 1167 -> 783 us; 64->64 3x3 388 -> 512 us
      // (2 instead of 4 blocks per CU), so C > 16 keeps 64x128 unless forced (set_wgrad_wide(2)).
      bn = 256;
      const int64_t t = (int64_t)((a.N + 255) / 256), ksteps = (a.K + 31) / 32;
      const int64_t sp = std::max<int64_t>(1, std::min<int64_t>((512 + t - 1) / t, ksteps / 8));
      const int64_t kps = (ksteps + sp - 1) / sp;
      a.k_split = (int)(kps * 32);
      splits = (int)((ksteps + kps - 1) / kps);
    }
    Tensor slab;
    if (deterministic && splits > 1) {
      // split partials stored to slabs, summed in split order below (no atomics: bitwise reproducible)
      slab = at::empty({(int64_t)splits * a.M * a.N}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
      a.slab = fp(slab);
    }
    if (overwrite && !slab.defined())  // atomics accumulate: start from zeros
      TORCH_CHECK(hipMemsetAsync(a.C, 0, (size_t)a.M * a.ldc * sizeof(float), cur_stream()) == hipSuccess, "memset");
    const int rc = dpe_igemm_wgrad_dma_launch(&a, bm, bn, bload, splits, cur_stream());
    a.slab = nullptr;
    TORCH_CHECK(rc == 0 || (!a.b_coef && !deterministic),
                "weight grad with BN on load / deterministic: outside the LDS-DMA kernel's envelope (rc=", rc, ")");
    static const bool skip_fin = [] {  // (timing diagnostic: gemm.cpp launch_planned)
      const char* e = getenv("DPE_AB_SKIP_FINALIZE");
      const bool on = e && e[0] == '1';
      if (on) fprintf(stderr, "[dpe] DPE_AB_SKIP_FINALIZE=1: deterministic weight-grad splits are NOT reduced (timing only)\n");
      return on;
    }();
    if (rc == 0 && slab.defined() && !skip_fin) {
      dpe::HgemmArgs f;
      memset(&f, 0, sizeof(f));
      f.C = a.C; f.ws = fp(slab); f.M = a.M; f.N = a.N; f.ldc = a.ldc; f.splits = splits; f.alpha = 1.f;
      // overwrite: the split sum IS the result (the caller's buffer needs no zero fill)
      CHECK_RC(dpe_hgemm_finalize(&f, overwrite ? dpe::HE_F32 : dpe::HE_ACC_F32, cur_stream()), "weight-grad slab finalize");
    }
    a.k_split = c.k_split;  // (register-staged fallback uses pick_cfg's split)
    if (rc == 0) {
      const hipError_t e = hipGetLastError();
      TORCH_CHECK(e == hipSuccess, "igemm_wgrad_dma launch failed: ", hipGetErrorString(e));
      return;
    }
  }
  // LDS-DMA kernel where it measured faster (2-stage ring, batch 512, profiles/convs_bs512_*):
  //   im2col A (3x3 / strided), K-contiguous B: always;
  //   dense 1x1 forward (A_DENSE_K x B_DENSE_K): unless K and N are both 64 (store-bound);
  //   1x1 data grads (A_DENSE_K x B_DENSE_N): for 128 <= N <= 512 (8-27 % faster; N = 64 and
  //   N >= 1024 measured 2-10 % slower in round 1).
  // Since the round-2 kernel changes every forward-form role on the LDS-DMA kernel measures +0.2 %
  // on the ResNet-50 step (5 alternating pairs: +0.14 / +0.29 / +0.17 / +0.63 / -0.16 %,
  // profiles/dma_all_ab_r2.txt), so that is the default (the round-1 role table is gone).
  constexpr bool dma_all = true;
  bool dma_role = false;
  if (aload == dpe::A_CONV_FWD) dma_role = bload == dpe::B_DENSE_K || dma_all;
  else if (aload == dpe::A_DENSE_K && bload == dpe::B_DENSE_K) dma_role = dma_all || a.K >= 128 || a.N >= 256;
  else if (aload == dpe::A_DENSE_K && bload == dpe::B_DENSE_N) dma_role = dma_all || (a.N >= 128 && a.N <= 512);
  if (conv && c.splits == 1 && dma_role && igemm_dma_on()) {
    // convolutions whose A is an im2col / dense K-contiguous operand: LDS-DMA kernel
    // (same tile shape, so BatchNorm partial layouts are unchanged)
    int bm = c.bm, bn = c.bn;
    dma_tile(a, aload, bload, bm, bn);
    const int rc = dpe_igemm_dma_launch(&a, bm, bn, aload, bload, epi, cur_stream());
    if (rc == 0) {
      const hipError_t e = hipGetLastError();
      TORCH_CHECK(e == hipSuccess, "igemm_dma launch failed: ", hipGetErrorString(e));
      return;
    }
  }
  const int rc = dpe_igemm_launch(&a, c.bm, c.bn, aload, bload, epi, c.splits, cur_stream());
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, "igemm launch failed: ", hipGetErrorString(e));
  TORCH_CHECK(rc == 0, "igemm: unsupported configuration (aload=", aload, " bload=", bload, " epi=", epi, ") rc=", rc);
}

// optional device scalar (f32, 1 element) multiplied into the GEMM alpha
const float* alpha_ptr_of(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_GPU((*t)); CHECK_F32((*t));
  TORCH_CHECK(t->numel() == 1, "alpha tensor must have one element");
  return (const float*)t->data_ptr();
}

dpe::IgemmArgs base_args() {
  dpe::IgemmArgs a;
  memset(&a, 0, sizeof(a));
  a.alpha = 1.f;
  return a;
}


// -------------------------------------------------------------- dense GEMMs
// Every Linear GEMM runs on our MFMA kernels: the persistent hgemm kernel
// (csrc/kernels/hgemm.hip; tile / K split from the deterministic planner in
// bindings/gemm.cpp, identical on every rank, no timing) whenever the shape is
// inside its envelope (K % 64, 16-B aligned rows, N % 8 for bf16 outputs), and
// the 128-tile implicit-GEMM kernel otherwise (SimpleNet's K = 784 input, odd
// classifier widths).  There is no vendor-library arm.
dpe::HgemmArgs hargs() {
  dpe::HgemmArgs a;
  memset(&a, 0, sizeof(a));
  a.alpha = 1.f;
  a.splits = 1;
  return a;
}

// y[M,N] = act(x[M,K] @ w[N,K]^T + bias) (+ residual);  aux_out (act = GELU): pre-activation v
Tensor linear_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, int64_t act, bool out_f32,
                  const c10::optional<Tensor>& residual, const c10::optional<Tensor>& out,
                  const c10::optional<Tensor>& aux_out) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(w);
  TORCH_CHECK(x.stride(-1) == 1, "x must have unit inner stride");
  const int64_t K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "linear: weight shape mismatch");
  TORCH_CHECK(K % 8 == 0, "linear: in_features must be a multiple of 8");
  Tensor x2 = x.reshape({-1, K});
  TORCH_CHECK(x2.stride(0) % 8 == 0, "x row stride must be a multiple of 8");
  const int64_t M = x2.size(0);
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    TORCH_CHECK(y.numel() == M * N && y.is_contiguous(), "linear: bad out tensor");
  } else {
    y = at::empty(sizes, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  const bool has_aux = aux_out.has_value() && aux_out->defined();
  if (has_aux) {
    TORCH_CHECK(act == dpe::ACT_GELU && !out_f32, "linear: aux_out (pre-activation) is for bf16 GELU outputs");
    CHECK_BF16((*aux_out)); CHECK_CONTIG((*aux_out));
    TORCH_CHECK(aux_out->numel() == M * N, "linear: aux_out shape mismatch");
  }
  const bool bf16_res = residual.has_value() && residual->defined() && !out_f32;
  if (K % 64 == 0 && N % 8 == 0 && !bf16_res && (out_f32 ? act == 0 : true)) {
    auto a = hargs();
    a.A = bp(x2); a.B = bp(w); a.C = y.data_ptr();
    a.M = (int)M; a.N = (int)N; a.K = (int)K;
    a.lda = x2.stride(0); a.ldb = K; a.ldc = N;
    a.bias = fpo(bias);
    a.act = (int)act;
    if (has_aux) a.aux_out = bpm(*aux_out);
    if (out_f32 && residual.has_value() && residual->defined()) {
      CHECK_F32((*residual)); CHECK_CONTIG((*residual));
      TORCH_CHECK(residual->numel() == M * N, "residual shape mismatch");
      a.residual_f32 = (const float*)residual->data_ptr();
    }
    dpe_gemm::run(a, 1, 1, out_f32 ? dpe::HE_F32 : dpe::HE_BF16, true, out_f32 ? 4 : 2);
    return y;
  }
  TORCH_CHECK(!has_aux, "linear: aux_out needs K % 64 == 0 and N % 8 == 0");
  auto a = base_args();
  a.A = bp(x2); a.B = bp(w); a.C = y.data_ptr();
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.lda = x2.stride(0); a.ldb = K; a.ldc = N;
  a.bias = fpo(bias);
  a.act = (int)act;
  if (residual.has_value() && residual->defined()) {
    CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->numel() == M * N, "residual shape mismatch");
    if (out_f32) {
      CHECK_F32((*residual));
      a.residual_f32 = (const float*)residual->data_ptr();
    } else {
      CHECK_BF16((*residual));
      a.residual = bp(*residual);
    }
  }
  run_igemm(a, dpe::A_DENSE_K, dpe::B_DENSE_K, out_f32 ? dpe::EPI_F32 : dpe::EPI_BF16, false);
  return y;
}

// dx[M,K] = dy[M,N] @ w[N,K]  (alpha_t: device scalar; gelu_in: dx *= gelu'(gelu_in), the
// backward of a GELU whose pre-activation gelu_in [M,K] produced this layer's input)
Tensor linear_dgrad(const Tensor& dy, const Tensor& w, const c10::optional<Tensor>& residual,
                    const c10::optional<Tensor>& alpha_t, const c10::optional<Tensor>& gelu_in) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(dy);
  const int64_t N = w.size(0), K = w.size(1);
  TORCH_CHECK(dy.size(-1) == N, "linear_dgrad: shape mismatch");
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "linear_dgrad: features must be multiples of 8");
  const int64_t M = dy.numel() / N;
  auto sizes = dy.sizes().vec();
  sizes.back() = K;
  Tensor dx = at::empty(sizes, dy.options());
  const bool has_res = residual.has_value() && residual->defined();
  const bool has_gelu = gelu_in.has_value() && gelu_in->defined();
  if (has_gelu) {
    CHECK_BF16((*gelu_in)); CHECK_CONTIG((*gelu_in));
    TORCH_CHECK(gelu_in->numel() == M * K, "linear_dgrad: gelu_in shape mismatch");
  }
  if (N % 64 == 0 && !has_res) {
    auto a = hargs();
    a.A = bp(dy); a.B = bp(w); a.C = dx.data_ptr();
    a.M = (int)M; a.N = (int)K; a.K = (int)N;
    a.lda = N; a.ldb = K; a.ldc = K;
    a.alpha_ptr = alpha_ptr_of(alpha_t);
    if (has_gelu) { a.act = dpe::HACT_GELU_BWD; a.aux_in = bp(*gelu_in); }
    dpe_gemm::run(a, 1, 0, dpe::HE_BF16, true, 2);
    return dx;
  }
  TORCH_CHECK(!has_gelu, "linear_dgrad: gelu_in needs out_features % 64 == 0 and no residual");
  auto a = base_args();
  a.A = bp(dy); a.B = bp(w); a.C = dx.data_ptr();
  a.M = (int)M; a.N = (int)K; a.K = (int)N;
  a.lda = N; a.ldb = K; a.ldc = K;
  if (has_res) { CHECK_BF16((*residual)); CHECK_CONTIG((*residual)); a.residual = bp(*residual); }
  a.alpha_ptr = alpha_ptr_of(alpha_t);
  run_igemm(a, dpe::A_DENSE_K, dpe::B_DENSE_N, dpe::EPI_BF16, false);
  return dx;
}

// dw[N,K] (+)= alpha * dy[M,N]^T @ x[M,K]   (fp32 accumulate into dw, e.g. a DDP bucket view).
// dy may be column-padded (row stride ldy >= N, ldy % 8 == 0, pad columns zero): then N need not be a
// multiple of 8 (vocab-padded LM head: N = 50257, ldy = 50304).
dpe::ConvGeom geom(const Tensor& x, const Tensor& w, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                   int64_t OH, int64_t OW);

// overwrite: dw = alpha dy^T x instead of dw += (the step's first writer of a gradient whose stale
// contents were not zeroed, ops/_state.py grad_fresh); the bias gradient always accumulates.
void linear_wgrad(const Tensor& dy, const Tensor& x, Tensor& dw, double alpha, const c10::optional<Tensor>& alpha_t,
                  const c10::optional<Tensor>& dbias, int64_t fin_stream, bool overwrite) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_BF16(x); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_F32(dw); CHECK_CONTIG(dw);
  const int64_t N = dw.size(0), K = dw.size(1), ldy = dy.size(-1);
  TORCH_CHECK(ldy >= N && x.size(-1) == K && dy.numel() / ldy == x.numel() / K, "linear_wgrad: shape mismatch");
  TORCH_CHECK(ldy % 8 == 0 && K % 8 == 0, "linear_wgrad: dy row stride and in_features must be multiples of 8");
  const int64_t M = dy.numel() / ldy;
  if (M % 64 == 0) {
    // TN: A = dy^T (M-contiguous, loads may read dy's zero pad columns up to ldy), B = x (N-contiguous)
    auto a = hargs();
    a.A = bp(dy); a.B = bp(x); a.C = dw.data_ptr();
    a.M = (int)N; a.N = (int)K; a.K = (int)M;
    a.lda = ldy; a.ldb = K; a.ldc = K;
    a.a_dim = (int)((N + 7) / 8 * 8);
    a.alpha = (float)alpha;
    a.alpha_ptr = alpha_ptr_of(alpha_t);
    if (dbias.has_value() && dbias->defined()) {
      // bias gradient from the same launch: row sums of dy^T taken from the A fragments (hgemm BG)
      CHECK_F32((*dbias)); CHECK_CONTIG((*dbias));
      TORCH_CHECK(dbias->numel() == N, "linear_wgrad: dbias must have out_features elements");
      a.dbias = fp(*dbias);
    }
    dpe_gemm::run(a, 0, 0, overwrite ? dpe::HE_F32 : dpe::HE_ACC_F32, true, 4, (hipStream_t)(uintptr_t)fin_stream);
    return;
  }
  if (overwrite) dw.zero_();  // the split-K fallback below accumulates with atomics
  if (dbias.has_value() && dbias->defined()) {
    CHECK_F32((*dbias)); CHECK_CONTIG((*dbias));
    TORCH_CHECK(dbias->numel() == N, "linear_wgrad: dbias must have out_features elements");
    TORCH_CHECK(alpha == 1.0 && !alpha_ptr_of(alpha_t), "linear_wgrad: dbias with M % 64 != 0 needs alpha == 1");
    CHECK_RC(dpe_colsum(dy.data_ptr(), M, (int)N, ldy, fp(*dbias), 1, 1, cur_stream()), "colsum");
  }
  auto a = base_args();
  a.A = bp(dy); a.B = bp(x); a.C = dw.data_ptr();
  a.M = (int)N; a.N = (int)K; a.K = (int)M;
  a.lda = ldy; a.ldb = K; a.ldc = K;
  a.alpha = (float)alpha;
  a.alpha_ptr = alpha_ptr_of(alpha_t);
  run_igemm(a, dpe::A_DENSE_M, dpe::B_DENSE_N, dpe::EPI_ATOMIC_F32, true);
}

// ------------------------------------------------------------------- conv
dpe::ConvGeom geom(const Tensor& x, const Tensor& w, int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                   int64_t OH, int64_t OW) {
  dpe::ConvGeom g;
  g.N = (int)x.size(0); g.H = (int)x.size(1); g.W = (int)x.size(2); g.C = (int)x.size(3);
  g.K = (int)w.size(0); g.R = (int)w.size(1); g.S = (int)w.size(2);
  g.sh = (int)sh; g.sw = (int)sw; g.ph = (int)ph; g.pw = (int)pw; g.dh = (int)dh; g.dw = (int)dw;
  g.OH = (int)OH; g.OW = (int)OW;
  g.RR = g.R; g.SS = g.S;
  g.pr0 = 0; g.ps0 = 0; g.psh = 1; g.psw = 1;
  g.remap = 0; g.Hr = g.H; g.Wr = g.W; g.oa = 0; g.ob = 0;
  return g;
}

// DPE_PW_STREAM=0 / set_pw_stream(false): the write-heavy pointwise convs stay on the implicit-GEMM
// kernels (A/B reference and the equivalence tests)
int g_pw_stream = -1;
bool pw_stream_on() {
  if (g_pw_stream < 0) {
    const char* e = getenv("DPE_PW_STREAM");
    g_pw_stream = (e && e[0] == '0') ? 0 : 1;
  }
  return g_pw_stream == 1;
}
void set_pw_stream(bool on) { g_pw_stream = on ? 1 : 0; }

// DPE_ROWCONV=0 / set_rowconv(false): the 64-channel 3x3 convs stay on the implicit-GEMM tiles
int g_rowconv = -1;
bool rowconv_on() {
  if (g_rowconv < 0) {
    const char* e = getenv("DPE_ROWCONV");
    g_rowconv = (e && e[0] == '0') ? 0 : 1;
  }
  return g_rowconv == 1;
}
void set_rowconv(bool on) { g_rowconv = on ? 1 : 0; }
// DPE_ROW_WGRAD=0 / set_row_wgrad(false): their weight grads stay on the im2col weight-grad tile
int g_row_wgrad = -1;
bool row_wgrad_on() {
  if (g_row_wgrad < 0) {
    const char* e = getenv("DPE_ROW_WGRAD");
    g_row_wgrad = (e && e[0] == '0') ? 0 : 1;
  }
  return g_row_wgrad == 1;
}
void set_row_wgrad(bool on) { g_row_wgrad = on ? 1 : 0; }
// 3x3 / stride 1 / pad 1 / dilation 1, 64 -> 64 channels, W <= 64: the row-walking kernel's envelope
bool rowconv_geom(const dpe::ConvGeom& g) {
  return rowconv_on() && g.C == 64 && g.K == 64 && g.R == 3 && g.S == 3 && g.sh == 1 && g.sw == 1 && g.ph == 1 &&
         g.pw == 1 && g.dh == 1 && g.dw == 1 && g.OH == g.H && g.OW == g.W &&
         dpe_conv3x3_rows_blocks(g.N, g.H, g.W) > 0;
}

// DPE_STEM=0 / set_stem_kernel(false): the s2d stem conv stays on the implicit-GEMM tile
int g_stem = -1;
bool stem_on() {
  if (g_stem < 0) {
    const char* e = getenv("DPE_STEM");
    g_stem = (e && e[0] == '0') ? 0 : 1;
  }
  return g_stem == 1;
}
void set_stem_kernel(bool on) { g_stem = on ? 1 : 0; }

// DPE_WGRAD_HGEMM=0 / set_wgrad_hgemm(false): every conv weight grad stays on the implicit GEMM
int g_wgrad_hgemm = -1;
bool wgrad_hgemm_on() {
  if (g_wgrad_hgemm < 0) {
    const char* e = getenv("DPE_WGRAD_HGEMM");
    g_wgrad_hgemm = (e && e[0] == '0') ? 0 : 1;
  }
  return g_wgrad_hgemm == 1;
}
void set_wgrad_hgemm(bool on) { g_wgrad_hgemm = on ? 1 : 0; }

// Forward-form convolutions with taps (3x3, stride 1 or 2, and the stride-1 data grads run as forward
// convs of dy with the flipped filter) and >= 256 output channels on the persistent GEMM with an
// implicit-im2col A (hgemm.hip AC): its BK-64 ping-pong schedule ran the dense GEMMs of these shapes at
// 818-1,102 TF where the implicit-GEMM kernel ran them at 668-829 (profiles/conv_as_gemm_r3.jsonl);
// with 128 output channels the 256-wide tiles lose (481 vs 680 TF), so those stay.
// DPE_HGEMM_CONV=0 (or set_hgemm_conv(false)): the implicit-GEMM kernel (A/B, tests).
int g_hgemm_conv = [] { const char* e = getenv("DPE_HGEMM_CONV"); return (e && e[0] == '0') ? 0 : 1; }();
// the weight-grad half (implicit-im2col B) separately: DPE_HGEMM_CONV_WGRAD=0/1 (A/B)
int g_hgemm_conv_wgrad = [] { const char* e = getenv("DPE_HGEMM_CONV_WGRAD"); return (e && e[0] == '0') ? 0 : 1; }();
void set_hgemm_conv(bool on) { g_hgemm_conv = on ? 1 : 0; }
// DPE_HGEMM_CONV_1X1S=0: the strided 1x1 convs (bottleneck downsamples) stay on the implicit-GEMM kernel (A/B)
bool g_hgemm_conv_1x1s = [] { const char* e = getenv("DPE_HGEMM_CONV_1X1S"); return !(e && e[0] == '0'); }();
bool hconv_ok(const dpe::ConvGeom& f, int64_t nout) {
  // 1x1 only when strided (a stride-1 1x1 conv is a dense GEMM, routed elsewhere) and at >= 512 input
  // channels: the layer-3/4 downsamples 185 -> 169 and 145 -> 139 us, the layer-2 one (K = 256) slower
  // there, 287 vs 272 us (scripts/bench_down_fwd.py, profiles/down_fwd_r4.jsonl)
  const bool one = f.R * f.S == 1 && (f.sh > 1 || f.sw > 1) && f.ph == 0 && f.pw == 0 && f.C >= 512 && g_hgemm_conv_1x1s;
  if (!g_hgemm_conv || (f.R * f.S <= 1 && !one) || f.R * f.S > 32 || f.C < 64 || (f.C & (f.C - 1)) || nout < 256 || nout % 8) return false;
  const int64_t abytes = (((int64_t)f.N * f.H * f.W * f.C) + ((int64_t)f.ph * f.W + f.pw) * f.C) * 2;
  return abytes < (1ll << 31) - 4096 && (int64_t)f.N * f.OH * f.OW < (1ll << 31);
}
// y [M = N*OH*OW][nout] = im2col(x) . w^T with the BN-forward sums (act HACT_BNF) or the BN-backward
// partials of dL/d relu(BN(st_x)) (HACT_BNB) or neither (ACT_NONE); stats sized by the plan.  Returns
// false when no plan fits.
bool run_hconv(const uint16_t* x, const uint16_t* w, uint16_t* y, const dpe::ConvGeom& f, int64_t nout, int act,
               const Tensor& like, Tensor* stats, const uint16_t* st_x, const float* st_coef) {
  const int64_t M = (int64_t)f.N * f.OH * f.OW, K = (int64_t)f.R * f.S * f.C;
  int pcols = 0;
  const auto pl = dpe_gemm::plan_bnb(M, nout, K, 1, 1, &pcols);
  if (pl.cfg < 0 || pl.splits != 1 || pcols <= 0) return false;
  auto h = hargs();
  h.A = x; h.B = w; h.C = y;
  h.M = (int)M; h.N = (int)nout; h.K = (int)K;
  h.lda = K; h.ldb = K; h.ldc = nout;
  h.conv = 1; h.conv_g = f; h.conv_smagic = (65536 + f.S - 1) / f.S;
  h.act = act;
  if (act != dpe::ACT_NONE) {
    *stats = at::empty({2, nout, pcols}, like.options().dtype(at::kFloat));
    h.col_stats = fp(*stats); h.stats_ld = pcols;
    h.st_x = st_x; h.st_coef = st_coef;
    dpe_gemm::run_bnb(h, pl, 1, 1);
  } else {
    dpe_gemm::launch_plain(h, pl, 1, 1);
  }
  return true;
}

// DPE_HGEMM_DGRAD=0: 1x1 convs (data grads, and forwards with BN statistics) with K >= 1024 stay on the
// implicit-GEMM kernel (A/B reference)
bool hgemm_dgrad_on() {
  static const bool on = [] { const char* e = getenv("DPE_HGEMM_DGRAD"); return !(e && e[0] == '0'); }();
  return on;
}

bool is_pointwise(const dpe::ConvGeom& g) {
  return g.R == 1 && g.S == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0;
}

// x NHWC bf16 [N,H,W,C], w [K,R,S,C] bf16 -> y NHWC [N,OH,OW,K]
// in_coef: x is the pre-BN tensor of a BatchNorm+ReLU whose output was never stored ([4][C] coefficients;
// relu(x * scale + shift) is applied on load) -- only on the row-walking 64-channel 3x3 kernel
std::vector<Tensor> conv_fwd(const Tensor& x, const Tensor& w, std::vector<int64_t> stride, std::vector<int64_t> pad,
                             std::vector<int64_t> dil, bool want_stats, const c10::optional<Tensor>& bias,
                             const c10::optional<Tensor>& in_coef) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && x.size(3) == w.size(3), "conv: NHWC x / KRSC w shape mismatch");
  TORCH_CHECK(x.size(3) % 8 == 0 && w.size(0) % 8 == 0, "conv: channels must be multiples of 8");
  TORCH_CHECK(pad.size() == 2 || pad.size() == 4, "conv: pad is [ph, pw] or [top, left, bottom, right]");
  const int64_t H = x.size(1), W = x.size(2), R = w.size(1), S = w.size(2);
  const int64_t pb = pad.size() == 4 ? pad[2] : pad[0], pr = pad.size() == 4 ? pad[3] : pad[1];
  const int64_t OH = (H + pad[0] + pb - dil[0] * (R - 1) - 1) / stride[0] + 1;
  const int64_t OW = (W + pad[1] + pr - dil[1] * (S - 1) - 1) / stride[1] + 1;
  Tensor y = at::empty({x.size(0), OH, OW, w.size(0)}, x.options());
  auto g = geom(x, w, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], OH, OW);
  auto a = base_args();
  a.g = g;
  a.A = bp(x); a.B = bp(w); a.C = y.data_ptr();
  a.M = (int)(x.size(0) * OH * OW); a.N = g.K; a.K = (int)(R * S * g.C);
  a.lda = g.C; a.ldb = a.K; a.ldc = g.K;
  a.bias = fpo(bias);
  Tensor stats;
  // the space-to-depth ResNet stem (16 channels, 4x4 / s1 / pad 2-2-1-1 -> 64): row-walking
  // kernel with the filter in VGPRs and each input row loaded once (csrc/kernels/stem.hip)
  const int stem_nb = (stem_on() && g.C == 16 && g.K == 64 && R == 4 && S == 4 && g.sh == 1 && g.sw == 1 && g.ph == 2 &&
                       g.pw == 2 && pb == 1 && pr == 1 && g.dh == 1 && g.dw == 1 && OH == H && OW == W && !a.bias)
                          ? dpe_stem_blocks(g.N, g.H, g.W) : 0;
  const float* icoef = fpo(in_coef);
  const int pw_rg_in = (pw_stream_on() && is_pointwise(g) && !a.bias) ? dpe_pw_rowgroups(a.M, a.N, a.K, dpe::PW_FWD) : 0;
  TORCH_CHECK(!icoef || (rowconv_geom(g) && pb == 1 && pr == 1 && !a.bias) || pw_rg_in > 0,
              "conv_fwd: in_coef (BN+ReLU on load) needs the row-walking 64-channel 3x3 kernel or the streaming "
              "pointwise kernel");
  if (rowconv_geom(g) && pb == 1 && pr == 1 && !a.bias) {
    // 64-channel 3x3 (layer 1 conv2): row-walking kernel, filter in VGPRs (csrc/kernels/rowconv.hip)
    const int nb = dpe_conv3x3_rows_blocks(g.N, g.H, g.W);
    if (want_stats) stats = at::empty({2, g.K, nb}, x.options().dtype(at::kFloat));
    CHECK_RC(dpe_conv3x3_rows_launch(bp(x), bp(w), bpm(y), want_stats ? fp(stats) : nullptr, nullptr, nullptr, g.N, g.H,
                                     g.W, nb, 0, icoef, cur_stream()),
             "conv3x3 rows fwd");
    return {y, stats};
  }
  if (stem_nb > 0) {
    if (want_stats) stats = at::empty({2, g.K, stem_nb}, x.options().dtype(at::kFloat));
    CHECK_RC(dpe_stem_launch(bp(x), bp(w), bpm(y), want_stats ? fp(stats) : nullptr, g.N, g.H, g.W, cur_stream()),
             "stem conv");
    return {y, stats};
  }
  // write-heavy pointwise convs (K <= 256, N >= 2K; the bottleneck conv3 shapes): persistent
  // streaming kernel (csrc/kernels/pwconv.hip), BN partials per row group.
  const int pw_rg = (pw_stream_on() && is_pointwise(g) && !a.bias) ? dpe_pw_rowgroups(a.M, a.N, a.K, dpe::PW_FWD) : 0;
  if (pw_rg > 0) {
    if (want_stats) stats = at::empty({2, g.K, pw_rg}, x.options().dtype(at::kFloat));
    dpe::PwArgs pa{};
    pa.x = bp(x); pa.w = bp(w); pa.y = bpm(y); pa.stats = want_stats ? fp(stats) : nullptr;
    pa.in_coef = icoef;
    pa.M = a.M; pa.N = a.N; pa.K = a.K; pa.rg = pw_rg; pa.sched = dpe_gemm::sched_buffer(cur_stream());
    CHECK_RC(dpe_pw_launch(&pa, dpe::PW_FWD, cur_stream()), "pw_stream fwd");
    return {y, stats};
  }
  // 1x1 stride-1 forward at depth >= 1024 (layers 3-4 conv1) with BN statistics: the persistent GEMM's
  // BN-forward-partials epilogue (hgemm.hip HACT_BNF; its GEMM alone 60-71 vs 79-89 us,
  // profiles/pw_vs_hgemm_r3.jsonl)
  // DPE_HG_BNF_MINK (default 1024): the smallest depth routed there (with >= 256 output channels below 1024)
  static const int bnf_min_k = [] { const char* e = getenv("DPE_HG_BNF_MINK"); return e ? atoi(e) : 1024; }();
  if (want_stats && is_pointwise(g) && !a.bias && !icoef && hgemm_dgrad_on() && a.K >= bnf_min_k &&
      (a.K >= 1024 || a.N >= 256) && a.K % 64 == 0 && a.N % 8 == 0) {
    int pcols = 0;
    const auto pl = dpe_gemm::plan_bnb(a.M, a.N, a.K, 1, 1, &pcols);
    if (pl.cfg >= 0 && pcols > 0) {
      stats = at::empty({2, g.K, pcols}, x.options().dtype(at::kFloat));
      auto h = hargs();
      h.A = bp(x); h.B = bp(w); h.C = y.data_ptr();
      h.M = a.M; h.N = a.N; h.K = a.K;
      h.lda = a.K; h.ldb = a.K; h.ldc = a.N;
      h.act = dpe::HACT_BNF;
      h.col_stats = fp(stats); h.stats_ld = pcols;
      dpe_gemm::run_bnb(h, pl, 1, 1);
      return {y, stats};
    }
  }
  if (!is_pointwise(g) && !a.bias && !icoef && hconv_ok(g, a.N) &&
      run_hconv(bp(x), bp(w), bpm(y), g, a.N, want_stats ? dpe::HACT_BNF : dpe::ACT_NONE, x, &stats, nullptr, nullptr))
    return {y, stats};
  if (want_stats) {
    // [2][K][tilesM] partial (sum, sumsq) per output channel and M-tile, reduced by bn_fwd_train
    const Cfg c = pick_cfg(a.M, a.N, a.K, false);
    const int64_t tilesM = (a.M + c.bm - 1) / c.bm;
    stats = at::empty({2, g.K, tilesM}, x.options().dtype(at::kFloat));
    a.col_stats = fp(stats);
  }
  run_igemm(a, is_pointwise(g) ? dpe::A_DENSE_K : dpe::A_CONV_FWD, dpe::B_DENSE_K, dpe::EPI_BF16, false, true);
  return {y, stats};
}

// dx NHWC [N,H,W,C] = conv_transpose(dy, w); optional residual added into dx.
// With bn_x/bn_coef (dx is dL/d relu(BN(bn_x))), the epilogue also emits the
// BatchNorm-backward partials [2][C][tiles] (sum dz, sum dz*(x-mean)).

// DPE_DGRAD_FWD=0: stride-1 data grads on the transposed-filter loaders (A/B reference)
bool dgrad_as_fwd() {
  static const bool on = [] { const char* e = getenv("DPE_DGRAD_FWD"); return !(e && e[0] == '0'); }();
  return on;
}

std::vector<Tensor> conv_dgrad_impl(const Tensor& dy, const Tensor& w, std::vector<int64_t> xshape,
                                    std::vector<int64_t> stride, std::vector<int64_t> pad, std::vector<int64_t> dil,
                                    const c10::optional<Tensor>& residual, const c10::optional<Tensor>& bn_x,
                                    const c10::optional<Tensor>& bn_coef, const Tensor* acc_into = nullptr,
                                    const c10::optional<Tensor>& bn_mask = c10::nullopt,
                                    const c10::optional<Tensor>& residual_mask = c10::nullopt,
                                    bool res_stride2 = false, const c10::optional<Tensor>& sum_mask = c10::nullopt) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_BF16(w); CHECK_CONTIG(dy); CHECK_CONTIG(w);
  // acc_into: dx += dgrad in place (the epilogue reads each element as its residual
  // right before overwriting it); parities no tap reaches are left untouched.
  Tensor dx = acc_into ? *acc_into : at::empty(xshape, dy.options());
  auto g = geom(dx, w, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], dy.size(1), dy.size(2));
  TORCH_CHECK(dy.size(3) == g.K && dy.size(0) == g.N, "conv_dgrad: dy shape mismatch");
  auto a = base_args();
  a.g = g;
  a.A = bp(dy); a.B = bp(w); a.C = dx.data_ptr();
  a.M = g.N * g.H * g.W; a.N = g.C; a.K = g.R * g.S * g.K;
  a.lda = g.K; a.ldb = g.C; a.ldc = g.C;
  if (residual.has_value() && residual->defined()) {
    CHECK_BF16((*residual)); CHECK_CONTIG((*residual));
    a.residual = bp(*residual);
    // the data-grad residual (a block's dz3 pass-through) is at its last use
    static const bool nt = [] { const char* e = getenv("DPE_EPI_NT"); return !(e && e[0] == '0'); }();
    a.res_nt = nt ? 1 : 0;
    if (residual_mask.has_value() && residual_mask->defined()) {
      // residual = dy of a BN + residual + ReLU output: masked by that output's bits in the epilogue
      CHECK_CONTIG((*residual_mask));
      TORCH_CHECK(residual_mask->scalar_type() == at::kByte && residual_mask->numel() * 8 == residual->numel() &&
                      residual->size(-1) % 8 == 0,
                  "conv_dgrad: residual_mask must be uint8 mask bits [.., C/8] of the residual");
      a.res_mask = (const uint8_t*)residual_mask->data_ptr();
    }
  }
  if (acc_into) {
    TORCH_CHECK(!a.residual && !(bn_x.has_value() && bn_x->defined()), "conv_dgrad_acc: no residual / BN with accumulate");
    CHECK_BF16(dx); CHECK_CONTIG(dx);
    TORCH_CHECK(dx.sizes().vec() == xshape, "conv_dgrad_acc: dx shape mismatch");
    a.residual = bp(dx);
  }
  const bool want_bn = bn_x.has_value() && bn_x->defined();
  if (want_bn) {
    CHECK_BF16((*bn_x)); CHECK_CONTIG((*bn_x)); CHECK_F32((*bn_coef));
    TORCH_CHECK(bn_x->sizes() == dx.sizes(), "conv_dgrad: bn_x must have dx's shape");
    TORCH_CHECK(bn_coef->numel() == 4 * g.C, "conv_dgrad: bn_coef must be [4][C]");
    a.st_x = bp(*bn_x);
    a.st_coef = fp(*bn_coef);
    if (bn_mask.has_value() && bn_mask->defined()) {
      // BN + residual + ReLU: ReLU-mask bits of the saved block output (bn_apply want_mask),
      // dx stored already masked
      CHECK_CONTIG((*bn_mask));
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() * 8 == dx.numel() && g.C % 8 == 0,
                  "conv_dgrad: bn_mask must be uint8 mask bits [N,H,W,C/8] of dx's shape");
      a.st_mask = (const uint8_t*)bn_mask->data_ptr();
    }
  }
  Tensor part;
  // write-heavy pointwise data grads (a bottleneck's conv1: K = Cout <= 256, N = Cin >= 2K), with the
  // residual / BN-backward epilogue: streaming kernel (pwconv.hip), BN partials per row group
  const int pw_rg = (pw_stream_on() && is_pointwise(g) && !acc_into) ? dpe_pw_rowgroups(a.M, a.N, a.K, dpe::PW_DGRAD) : 0;
  if (res_stride2) {
    // residual = the compact data grad of a downsample block's stride-2 1x1 conv ([N, H/2, W/2, C]),
    // added at even (h, w) by the streaming kernel's epilogue
    TORCH_CHECK(a.residual && !a.res_mask && (pw_rg > 0 || (sum_mask.has_value() && sum_mask->defined())) &&
                    g.H % 2 == 0 && g.W % 2 == 0,
                "conv_dgrad: residual_stride2 needs the streaming pointwise data grad, even H / W, no residual mask");
    TORCH_CHECK(residual->dim() == 4 && residual->size(0) == g.N && residual->size(1) == g.H / 2 &&
                    residual->size(2) == g.W / 2 && residual->size(3) == g.C,
                "conv_dgrad: residual_stride2 residual must be [N, H/2, W/2, C]");
  }
  if (sum_mask.has_value() && sum_mask->defined()) {
    // BN + residual + ReLU backward partials WITHOUT the pre-BN input (Gram algebra, bngram.hip): dx stored
    // masked by the output's bits, partials row 0 = sum dz (row 1 unwritten); streaming kernel only
    TORCH_CHECK(!want_bn && !acc_into && is_pointwise(g), "conv_dgrad: sum_mask excludes bn_x / accumulate");
    CHECK_CONTIG((*sum_mask));
    TORCH_CHECK(sum_mask->scalar_type() == at::kByte && sum_mask->numel() * 8 == dx.numel() && g.C % 8 == 0,
                "conv_dgrad: sum_mask must be uint8 mask bits [N,H,W,C/8] of dx's shape");
    const int rg = pw_stream_on() ? dpe_pw_rowgroups(a.M, a.N, a.K, dpe::PW_DSUM) : 0;
    TORCH_CHECK(rg > 0, "conv_dgrad: sum_mask needs the streaming pointwise data grad");
    dpe::PwArgs pa{};
    pa.x = bp(dy); pa.w = bp(w); pa.y = bpm(dx);
    pa.residual = a.residual; pa.res_mask = a.res_mask;
    if (res_stride2) { pa.res_h = g.H; pa.res_w = g.W; }
    pa.st_mask = (const uint8_t*)sum_mask->data_ptr();
    pa.M = a.M; pa.N = a.N; pa.K = a.K; pa.rg = rg; pa.sched = dpe_gemm::sched_buffer(cur_stream());
    part = at::empty({2, g.C, rg}, dy.options().dtype(at::kFloat));
    pa.stats = fp(part);
    CHECK_RC(dpe_pw_launch(&pa, dpe::PW_DSUM, cur_stream()), "pw_stream dgrad (sum dz)");
    return {dx, part};
  }
  if (pw_rg > 0) {
    dpe::PwArgs pa{};
    pa.x = bp(dy); pa.w = bp(w); pa.y = bpm(dx);
    pa.residual = a.residual; pa.res_mask = a.res_mask;
    if (res_stride2) { pa.res_h = g.H; pa.res_w = g.W; }
    pa.st_x = a.st_x; pa.st_coef = a.st_coef; pa.st_mask = a.st_mask;
    pa.M = a.M; pa.N = a.N; pa.K = a.K; pa.rg = pw_rg; pa.sched = dpe_gemm::sched_buffer(cur_stream());
    if (want_bn) {
      part = at::empty({2, g.C, pw_rg}, dy.options().dtype(at::kFloat));
      pa.stats = fp(part);
    }
    CHECK_RC(dpe_pw_launch(&pa, dpe::PW_DGRAD, cur_stream()), "pw_stream dgrad");
    return {dx, part};
  }
  // 1x1 data grads at depth >= 1024 (layers 3-4: conv3's) with the plain BN-backward epilogue: the
  // persistent GEMM (NN layout, hgemm.hip HACT_BNB) -- its GEMM alone 73 vs 112-118 us for layer 3's conv3
  // data grad (profiles/pw_vs_hgemm_r3.jsonl); ResNet-50 37.73-37.76 vs 37.81-37.88 ms/step.  At K = 512
  // (layer 2) it measured +0.3 ms/step, so that depth stays on the implicit GEMM.
  if (is_pointwise(g) && !a.residual && !a.res_mask && !a.st_mask && !acc_into && !res_stride2 && want_bn &&
      hgemm_dgrad_on() && a.K >= 1024 && a.K % 64 == 0 && g.C % 8 == 0) {
    int pcols = 0;
    const auto pl = dpe_gemm::plan_bnb(a.M, g.C, a.K, 1, 0, &pcols);
    if (pl.cfg >= 0 && pcols > 0) {
      part = at::empty({2, g.C, pcols}, dy.options().dtype(at::kFloat));
      auto h = hargs();
      h.A = bp(dy); h.B = bp(w); h.C = dx.data_ptr();
      h.M = a.M; h.N = g.C; h.K = a.K;
      h.lda = g.K; h.ldb = g.C; h.ldc = g.C;
      h.col_stats = fp(part); h.st_x = a.st_x; h.st_coef = a.st_coef; h.stats_ld = pcols;
      dpe_gemm::run_bnb(h, pl, 1, 0);
      return {dx, part};
    }
  }
  auto tiles_of = [&](int64_t M, int64_t K) { const Cfg c = pick_cfg(M, g.C, K, false); return (M + c.bm - 1) / c.bm; };
  if (!is_pointwise(g) && g.sh == 1 && g.sw == 1 && g.dh == 1 && g.dw == 1 && dgrad_as_fwd()) {
    // Stride-1 data grad as a forward conv: dx = conv(dy, flipT(w), pad R-1-p) on the
    // forward loaders (K-contiguous filter, im2col gather of dy).
    Tensor wt = flipped(w, g.K, g.R, g.S, g.C, 0, 1, g.R, 0, 1, g.S);
    auto f = geom(dy, wt, 1, 1, g.R - 1 - g.ph, g.S - 1 - g.pw, 1, 1, g.H, g.W);
    if (rowconv_geom(f) && !acc_into && !a.residual && !a.st_mask) {
      // 64-channel 3x3 data grad (layer 1): the row-walking forward kernel over dy with the flipped
      // filter; BN-backward partials per block
      const int nb = dpe_conv3x3_rows_blocks(f.N, f.H, f.W);
      if (want_bn) part = at::empty({2, g.C, nb}, dy.options().dtype(at::kFloat));
      CHECK_RC(dpe_conv3x3_rows_launch(bp(dy), bp(wt), bpm(dx), want_bn ? fp(part) : nullptr, a.st_x, a.st_coef, f.N, f.H,
                                       f.W, nb, want_bn ? 1 : 0, nullptr, cur_stream()),
               "conv3x3 rows dgrad");
      return {dx, part};
    }
    if (!acc_into && !a.residual && !a.st_mask && !a.res_mask && hconv_ok(f, g.C) &&
        run_hconv(bp(dy), bp(wt), bpm(dx), f, g.C, want_bn ? dpe::HACT_BNB : dpe::ACT_NONE, dy, &part, a.st_x, a.st_coef))
      return {dx, part};
    auto b = a;
    b.g = f;
    b.B = bp(wt);
    b.lda = g.K; b.ldb = a.K; b.ldc = g.C;
    if (want_bn) {
      const int64_t t = tiles_of(b.M, b.K);
      part = at::empty({2, g.C, t}, dy.options().dtype(at::kFloat));
      b.col_stats = fp(part);
      b.stats_ld = (int)t;
    }
    run_igemm(b, dpe::A_CONV_FWD, dpe::B_DENSE_K, want_bn ? dpe::EPI_BF16_BNB : dpe::EPI_BF16, false, true);
  } else if (is_pointwise(g) || (g.sh == 1 && g.sw == 1)) {
    if (want_bn) {
      const int64_t t = tiles_of(a.M, a.K);
      part = at::empty({2, g.C, t}, dy.options().dtype(at::kFloat));
      a.col_stats = fp(part);
      a.stats_ld = (int)t;
    }
    const int epi = want_bn ? dpe::EPI_BF16_BNB : dpe::EPI_BF16;
    if (is_pointwise(g)) run_igemm(a, dpe::A_DENSE_K, dpe::B_DENSE_N, epi, false, true);
    else run_igemm(a, dpe::A_CONV_DGRAD, dpe::B_CONV_DGRAD, epi, false, true);
  } else {
    // Strided: one stride-1 sub-GEMM per output parity (a, b) over only the
    // taps that reach it -- no MFMA work on structural zeros.  A parity with
    // no taps is a K = 0 GEMM that stores zeros (+ residual).
    TORCH_CHECK(g.dh == 1 && g.dw == 1, "strided dgrad with dilation is not supported");
    std::vector<dpe::IgemmArgs> subs;
    std::vector<bool> sub_fwd;
    std::vector<Tensor> phase_w;  // keeps the per-parity filters alive until the launches are queued
    int64_t total_tiles = 0;
    for (int pa = 0; pa < g.sh; ++pa) {
      for (int pb = 0; pb < g.sw; ++pb) {
        dpe::ConvGeom v = g;
        const int r0 = (pa + g.ph) % g.sh, s0 = (pb + g.pw) % g.sw;
        const int Rp = g.R > r0 ? (g.R - r0 + g.sh - 1) / g.sh : 0;
        const int Sp = g.S > s0 ? (g.S - s0 + g.sw - 1) / g.sw : 0;
        const int Hp = (g.H - pa + g.sh - 1) / g.sh, Wp = (g.W - pb + g.sw - 1) / g.sw;
        if (Hp <= 0 || Wp <= 0) continue;
        if (acc_into && (g.R <= r0 || g.S <= s0)) continue;  // no taps: dx += 0
        v.H = Hp; v.W = Wp; v.R = Rp; v.S = Sp;
        v.sh = 1; v.sw = 1;
        v.ph = (pa + g.ph - r0) / g.sh;  // oh = hh + ph' - t
        v.pw = (pb + g.pw - s0) / g.sw;
        v.pr0 = r0; v.ps0 = s0; v.psh = g.sh; v.psw = g.sw;
        v.remap = 1; v.Hr = g.H; v.Wr = g.W; v.oa = pa; v.ob = pb;
        auto b = a;
        b.g = v;
        b.M = g.N * Hp * Wp;
        b.K = Rp * Sp * g.K;
        b.stats_off = (int)total_tiles;
        total_tiles += tiles_of(b.M, b.K);
        bool fwd_form = false;
        if (Rp > 0 && Sp > 0 && dgrad_as_fwd()) {
          // this parity as a forward conv of dy with its own flipped tap subset:
          // oh = hh + ph' - t = hh - (Rp-1-ph') + (Rp-1-t)
          Tensor wt = flipped(w, g.K, g.R, g.S, g.C, r0, g.sh, Rp, s0, g.sw, Sp);
          phase_w.push_back(wt);
          auto f = geom(dy, wt, 1, 1, Rp - 1 - v.ph, Sp - 1 - v.pw, 1, 1, Hp, Wp);
          f.remap = 2; f.Hr = g.H; f.Wr = g.W; f.oa = pa; f.ob = pb; f.psh = g.sh; f.psw = g.sw;
          b.g = f;
          b.B = bp(wt);
          b.lda = g.K; b.ldb = b.K;
          fwd_form = true;
        }
        subs.push_back(b);
        sub_fwd.push_back(fwd_form);
      }
    }
    if (want_bn) part = at::empty({2, g.C, total_tiles}, dy.options().dtype(at::kFloat));
    const int epi = want_bn ? dpe::EPI_BF16_BNB : dpe::EPI_BF16;
    for (auto& b : subs)
      if (want_bn) { b.col_stats = fp(part); b.stats_ld = (int)total_tiles; }
    // g_phase_group: all parities in one grid (igemm_dma_group_kernel), on the first (shortest-K) parity's
    // tile -- one launch instead of four, an XCD's neighbouring blocks holding the four parities of the same
    // dy rows (measured neutral: off by default)
    bool grouped = false;
    if (g_phase_group && igemm_dma_on() && subs.size() > 1 && subs.size() <= (size_t)dpe::IGEMM_GROUP_MAX &&
        std::all_of(sub_fwd.begin(), sub_fwd.end(), [](bool f) { return f; })) {
      const Cfg c0 = pick_cfg(subs[0].M, subs[0].N, subs[0].K, false);
      int bm = c0.bm, bn = c0.bn;
      dma_tile(subs[0], dpe::A_CONV_FWD, dpe::B_DENSE_K, bm, bn);
      for (auto& b : subs) b.k_split = (int)((b.K + 31) / 32 * 32);
      grouped = dpe_igemm_dma_group_launch(subs.data(), (int)subs.size(), bm, bn, dpe::A_CONV_FWD, dpe::B_DENSE_K, epi,
                                           cur_stream()) == 0;
      if (grouped) {
        const hipError_t e = hipGetLastError();
        TORCH_CHECK(e == hipSuccess, "igemm_dma group launch failed: ", hipGetErrorString(e));
      }
    }
    for (size_t i = 0; i < subs.size() && !grouped; ++i) {
      auto& b = subs[i];
      if (sub_fwd[i]) run_igemm(b, dpe::A_CONV_FWD, dpe::B_DENSE_K, epi, false, true);
      else run_igemm(b, dpe::A_CONV_DGRAD, dpe::B_CONV_DGRAD, epi, false, true);
    }
  }
  return {dx, part};
}

void conv_dgrad_acc(const Tensor& dy, const Tensor& w, Tensor& dx, std::vector<int64_t> stride, std::vector<int64_t> pad,
                    std::vector<int64_t> dil) {
  conv_dgrad_impl(dy, w, dx.sizes().vec(), stride, pad, dil, c10::nullopt, c10::nullopt, c10::nullopt, &dx);
}

Tensor conv_dgrad(const Tensor& dy, const Tensor& w, std::vector<int64_t> xshape, std::vector<int64_t> stride,
                  std::vector<int64_t> pad, std::vector<int64_t> dil, const c10::optional<Tensor>& residual,
                  const c10::optional<Tensor>& residual_mask) {
  return conv_dgrad_impl(dy, w, xshape, stride, pad, dil, residual, c10::nullopt, c10::nullopt, nullptr, c10::nullopt,
                         residual_mask)[0];
}

// dw [K,R,S,C] fp32 (+)= alpha * dy^T (x) im2col(x)
// in_coef: as conv_fwd's (x pre-BN, BN+ReLU applied on load; row-walking 64-channel 3x3 kernel only)
void conv_wgrad(const Tensor& dy, const Tensor& x, Tensor& dw, std::vector<int64_t> stride, std::vector<int64_t> pad,
                std::vector<int64_t> dil, double alpha, const c10::optional<Tensor>& in_coef, int64_t fin_stream,
                bool deterministic, bool overwrite) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_BF16(x); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_F32(dw); CHECK_CONTIG(dw);
  auto g = geom(x, dw, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], dy.size(1), dy.size(2));
  TORCH_CHECK(dy.size(3) == g.K && dy.size(0) == g.N, "conv_wgrad: dy shape mismatch");
  auto a = base_args();
  a.g = g;
  a.A = bp(dy); a.B = bp(x); a.C = dw.data_ptr();
  a.M = g.K; a.N = g.R * g.S * g.C; a.K = g.N * g.OH * g.OW;
  a.lda = g.K; a.ldb = g.C; a.ldc = a.N;
  a.alpha = (float)alpha;
  // 64 -> 64 3x3 (ResNet layer 1): the row-walking weight-grad kernel (rowconv.hip)
  const float* icoef = fpo(in_coef);
  const int row_nb = rowconv_geom(g) ? dpe_wgrad3x3_rows_blocks(g.N, g.H, g.W) : 0;  // (depends on the CU budget)
  const bool row = row_nb > 0;
  if (icoef && !row) {
    // 1x1 weight grad over a pre-BN input: the LDS-DMA weight-grad kernel applies BN + ReLU to its
    // B fragments (b_coef); outside that kernel's envelope there is no such path
    TORCH_CHECK(is_pointwise(g), "conv_wgrad: in_coef needs a 1x1 conv or the row-walking 64-channel 3x3 kernel");
    a.b_coef = icoef;
    run_igemm(a, dpe::A_DENSE_M, dpe::B_DENSE_N, dpe::EPI_ATOMIC_F32, true, true, deterministic, overwrite);
    return;
  }
  const bool hgemm_1x1 = wgrad_hgemm_on() && is_pointwise(g) && a.K % 64 == 0 && g.K >= 256 && g.C >= 256 &&
                         g.K % 8 == 0 && g.C % 8 == 0;
  if (overwrite && !hgemm_1x1)  // the accumulating kernels below: start from zeros
    TORCH_CHECK(hipMemsetAsync(dw.data_ptr(), 0, dw.numel() * sizeof(float), cur_stream()) == hipSuccess, "memset");
  if (row && (row_wgrad_on() || icoef)) {
    auto scratch = at::empty({dpe_wgrad3x3_rows_scratch(row_nb)}, dw.options());
    CHECK_RC(dpe_wgrad3x3_rows_launch(bp(x), bp(dy), fp(dw), fp(scratch), g.N, g.H, g.W, row_nb, (float)alpha, icoef,
                                      cur_stream()),
             "wgrad3x3_rows");
    return;
  }
  // the s2d stem (16 channels, 4x4 / s1 / pad 2-2-1-1 -> 64): the row-walking weight grad (stem.hip)
  static const bool stem_wg_env = [] { const char* e = getenv("DPE_STEM_WGRAD"); return !(e && e[0] == '0'); }();
  if (stem_on() && stem_wg_env && g.C == 16 && g.K == 64 && g.R == 4 && g.S == 4 && g.sh == 1 && g.sw == 1 && g.ph == 2 && g.pw == 2 &&
      g.dh == 1 && g.dw == 1 && g.OH == g.H && g.OW == g.W && dpe_stem_wgrad_scratch(g.N, g.H, g.W) > 0) {
    auto scratch = at::empty({dpe_stem_wgrad_scratch(g.N, g.H, g.W)}, dw.options());
    CHECK_RC(dpe_stem_wgrad_launch(bp(x), bp(dy), fp(dw), fp(scratch), g.N, g.H, g.W, (float)alpha, cur_stream()),
             "stem wgrad");
    return;
  }
  // 1x1 stride-1 weight grads with both channel counts >= 256 (ResNet layers 3-4 and the 512->256
  // entry of layer 3: 53 GFLOP over a few output tiles) are a plain TN GEMM over the pixels: the
  // persistent hgemm kernel with the planner's K split and a deterministic slab finalize, as
  // linear_wgrad.  With 128 channels the TN layout's only tile (256x256) wastes half its MFMAs and
  // the implicit GEMM is faster (profiles/wgrad_hgemm_ab_r2.txt).
  if (hgemm_1x1) {
    auto h = hargs();
    h.A = bp(dy); h.B = bp(x); h.C = dw.data_ptr();
    h.M = a.M; h.N = a.N; h.K = a.K;
    h.lda = g.K; h.ldb = g.C; h.ldc = g.C;
    h.a_dim = (int)((g.K + 7) / 8 * 8);
    h.alpha = (float)alpha;
    dpe_gemm::run(h, 0, 0, overwrite ? dpe::HE_F32 : dpe::HE_ACC_F32, true, 4, (hipStream_t)(uintptr_t)fin_stream);
    return;
  }
  // 3x3 weight grads with >= 256 output channels (layers 3-4): the persistent GEMM's TN layout with an
  // implicit-im2col B (hgemm.hip CV = 2); dense TN GEMMs of these shapes ran at 846-960 TF where the
  // LDS-DMA im2col weight grad ran them at 648-748 (profiles/wgrad_as_gemm_r4.jsonl).  Split-K partials
  // in slabs summed in a fixed order (no atomics).  Not with BN-on-load inputs (none at these shapes).
  if (g_hgemm_conv && g_hgemm_conv_wgrad && !is_pointwise(g) && g.K >= 256 && g.K % 8 == 0 && g.C >= 8 && (g.C & (g.C - 1)) == 0 &&
      a.K % 64 == 0 && a.K < (1 << 24) && g.R * g.S <= 32 &&
      (((int64_t)g.N * g.H * g.W * g.C) + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2 < (1ll << 31) - 4096) {
    auto h = hargs();
    h.A = bp(dy); h.B = bp(x); h.C = dw.data_ptr();
    h.M = a.M; h.N = a.N; h.K = a.K;
    h.lda = g.K; h.ldb = a.N; h.ldc = a.N;
    h.alpha = (float)alpha;
    h.conv = 2; h.conv_g = g; h.conv_smagic = (65536 + g.S - 1) / g.S;
    dpe_gemm::run_conv_wgrad(h, (hipStream_t)(uintptr_t)fin_stream);
    return;
  }
  run_igemm(a, dpe::A_DENSE_M, is_pointwise(g) ? dpe::B_DENSE_N : dpe::B_CONV_WGRAD, dpe::EPI_ATOMIC_F32, true, true);
}

// --------------------------------------------------------------- BatchNorm
int64_t rows_of(const Tensor& x) { return x.numel() / x.size(-1); }

// returns (y, coef[4][C]); stats: optional precomputed [2][C] column sums (from conv epilogue)
std::vector<Tensor> bn_fwd_train(const Tensor& x, const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                                 const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar, double momentum,
                                 double eps, bool relu, const c10::optional<Tensor>& residual,
                                 const c10::optional<Tensor>& stats) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = rows_of(x);
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: C must be a multiple of 8 and <= 2048");
  auto fo = x.options().dtype(at::kFloat);
  Tensor coef = at::empty({4, C}, fo);
  hipStream_t st = cur_stream();
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->dim() == 3 && stats->size(0) == 2 && stats->size(1) == C, "stats must be [2][C][nb] partials");
    CHECK_RC(dpe_bn_finalize(fp(*stats), (int)stats->size(2), (int)C, M, fpo(gamma), fpo(beta), fpom(rmean), fpom(rvar),
                             (float)momentum, (float)eps, fp(coef), st), "bn_finalize");
  } else {
    const int nb = dpe_bn_stats_nblocks(M, (int)C);
    Tensor part = at::empty({nb, 2, C}, fo);
    CHECK_RC(dpe_bn_stats(bp(x), M, (int)C, nb, fp(part), st), "bn_stats");
    CHECK_RC(dpe_bn_finalize(fp(part), nb, (int)C, M, fpo(gamma), fpo(beta), fpom(rmean), fpom(rvar), (float)momentum,
                             (float)eps, fp(coef), st), "bn_finalize");
  }
  Tensor y = at::empty_like(x);
  const uint16_t* res = nullptr;
  if (residual.has_value() && residual->defined()) { CHECK_BF16((*residual)); CHECK_CONTIG((*residual)); res = bp(*residual); }
  CHECK_RC(dpe_bn_apply(bp(x), res, bpm(y), M, (int)C, fp(coef), relu ? 1 : 0, st), "bn_apply");
  return {y, coef};
}

Tensor bn_fwd_eval(const Tensor& x, const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                   const Tensor& rmean, const Tensor& rvar, double eps, bool relu, const c10::optional<Tensor>& residual) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = rows_of(x);
  Tensor coef = at::empty({4, C}, x.options().dtype(at::kFloat));
  hipStream_t st = cur_stream();
  CHECK_RC(dpe_bn_eval_coeff((int)C, fpo(gamma), fpo(beta), fp(rmean), fp(rvar), (float)eps, fp(coef), st), "bn_eval");
  Tensor y = at::empty_like(x);
  const uint16_t* res = nullptr;
  if (residual.has_value() && residual->defined()) res = bp(*residual);
  CHECK_RC(dpe_bn_apply(bp(x), res, bpm(y), M, (int)C, fp(coef), relu ? 1 : 0, st), "bn_apply");
  return y;
}

// returns (dx, dz or empty); dgamma/dbeta accumulated (+=) if given
std::vector<Tensor> bn_bwd(const Tensor& dy, const c10::optional<Tensor>& y, const Tensor& x,
                           const c10::optional<Tensor>& gamma, const Tensor& coef, const c10::optional<Tensor>& dgamma,
                           const c10::optional<Tensor>& dbeta, bool want_dz, const c10::optional<Tensor>& y_bits) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = rows_of(x);
  const uint16_t* yp = (y.has_value() && y->defined()) ? bp(*y) : nullptr;
  const uint8_t* yb = nullptr;
  if (y_bits.has_value() && y_bits->defined()) {
    // ReLU mask as bn_apply's bits (1/16 of y's bytes): y itself is not read
    CHECK_CONTIG((*y_bits));
    TORCH_CHECK(y_bits->scalar_type() == at::kByte && y_bits->numel() * 8 == x.numel() && C % 8 == 0,
                "bn_bwd: y_bits must be uint8 mask bits [.., C/8] of x's shape");
    yb = (const uint8_t*)y_bits->data_ptr();
    yp = nullptr;
  }
  hipStream_t st = cur_stream();
  auto fo = x.options().dtype(at::kFloat);
  const int nb = dpe_bn_bwd_nblocks(M, (int)C);
  Tensor part = at::empty({nb, 2, C}, fo);
  CHECK_RC(dpe_bn_bwd_reduce(bp(dy), yp, yb, bp(x), fp(coef), M, (int)C, nb, fp(part), st), "bn_bwd_reduce");
  Tensor bcoef = at::empty({3, C}, fo);
  CHECK_RC(dpe_bn_bwd_finalize(fp(part), nb, (int)C, M, fpo(gamma), fp(coef), fpom(dgamma), fpom(dbeta), fp(bcoef), st),
           "bn_bwd_finalize");
  Tensor dx = at::empty_like(x);
  Tensor dz;
  if (want_dz) dz = at::empty_like(x);
  CHECK_RC(dpe_bn_bwd_apply(bp(dy), yp, yb, bp(x), fp(bcoef), bpm(dx), want_dz ? bpm(dz) : nullptr, M, (int)C, nullptr, st),
           "bn_bwd_apply");
  return {dx, dz};
}

// ------------------------------------------------------------ BN3 by Gram algebra (bngram.hip)
// G = a'^T a' [C][C] and s = [colsum(a'), mu] [2][C] of a' = a2 - mu, a2 = relu(x * coef[0] + coef[1]) (coef: the
// BN's [4][C]) or x, centred on the pilot shift mu (bngram.hip relu_gauss_mean) of the BN coefficients
// shift_coef (default: coef; neither: mu = 0).
std::vector<Tensor> bn_gram(const Tensor& x, const c10::optional<Tensor>& coef, const c10::optional<Tensor>& shift_coef) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t C = x.size(-1), M = x.numel() / C;
  TORCH_CHECK(C == 64 || C == 128 || C == 256, "bn_gram: C must be 64, 128 or 256");
  if (coef.has_value() && coef->defined()) {
    CHECK_F32((*coef)); CHECK_CONTIG((*coef));
    TORCH_CHECK(coef->numel() >= 2 * C, "bn_gram: coef must be the BN's [4][C] coefficients");
  }
  const float* scoef = fpo(coef);
  if (scoef) TORCH_CHECK(coef->numel() == 4 * C, "bn_gram: the shift needs coef's full [4][C] (scale, shift, mean, invstd)");
  if (shift_coef.has_value() && shift_coef->defined()) {
    CHECK_F32((*shift_coef)); CHECK_CONTIG((*shift_coef));
    TORCH_CHECK(shift_coef->numel() == 4 * C, "bn_gram: shift_coef must be the BN's [4][C] coefficients");
    scoef = fp(*shift_coef);
  }
  auto fo = x.options().dtype(at::kFloat);
  Tensor ws = at::empty({dpe_gram_ws_floats(M, (int)C)}, fo);
  Tensor G = at::empty({C, C}, fo), sv = at::empty({2, C}, fo);
  CHECK_RC(dpe_gram(bp(x), fpo(coef), scoef, M, (int)C, fp(ws), fp(G), fp(sv), cur_stream()), "bn_gram");
  return {G, sv};
}

// BN coefficients [4][Cout] of h = a2 W^T (never computed) from G, s: mean = w.s / M, E[h^2] = w^T G w / M;
// running stats updated as bn_coef.  Also returns u = W G [Cout][Cin] (fp32) for the backward.
std::vector<Tensor> bn_gram_coef(const Tensor& G, const Tensor& sv, const Tensor& w, int64_t M,
                                 const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
                                 const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar, double momentum,
                                 double eps) {
  CHECK_GPU(G); CHECK_F32(G); CHECK_F32(sv); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(G);
  const int64_t Cin = G.size(0), Cout = w.size(0);
  TORCH_CHECK(w.numel() == Cout * Cin && sv.numel() == 2 * Cin, "bn_gram_coef: shapes (s is bn_gram's [2][C])");
  CHECK_CONTIG(sv);
  Tensor coef = at::empty({4, Cout}, G.options()), u = at::empty({Cout, Cin}, G.options());
  CHECK_RC(dpe_gram_coef(fp(G), fp(sv), bp(w), (int)Cin, (int)Cout, M, fpo(gamma), fpo(beta), fpom(rmean), fpom(rvar),
                         (float)momentum, (float)eps, fp(coef), fp(u), cur_stream()), "bn_gram_coef");
  return {coef, u};
}

// y = relu(BN(x' W^T) + residual) of a 1x1 conv (x' = relu(x * in_coef) or x), with the BN's coefficients known
// in advance (bn_gram_coef): streaming pointwise kernel, PW_APPLY.  res_coef: the residual is the pre-BN
// output of a downsample conv, BN'd (and rounded) on the fly.  Returns (y, ReLU bits of y).
std::vector<Tensor> conv1x1_apply(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& in_coef,
                                  const Tensor& out_coef, const Tensor& residual, const c10::optional<Tensor>& res_coef) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_F32(out_coef);
  CHECK_BF16(residual); CHECK_CONTIG(residual);
  const int64_t K = x.size(-1), M = x.numel() / K, N = w.size(0);
  TORCH_CHECK(w.numel() == N * K && out_coef.numel() == 4 * N, "conv1x1_apply: shapes");
  auto ysz = x.sizes().vec();
  ysz.back() = N;
  TORCH_CHECK(residual.sizes().vec() == ysz, "conv1x1_apply: residual must have the output's shape");
  const int rg = pw_stream_on() ? dpe_pw_rowgroups(M, N, K, dpe::PW_APPLY) : 0;
  TORCH_CHECK(rg > 0, "conv1x1_apply: outside the streaming pointwise kernel's envelope");
  Tensor y = at::empty(ysz, x.options());
  auto bsz = ysz;
  bsz.back() = N / 8;
  Tensor bits = at::empty(bsz, x.options().dtype(at::kByte));
  dpe::PwArgs pa{};
  pa.x = bp(x); pa.w = bp(w); pa.y = bpm(y);
  pa.in_coef = fpo(in_coef);
  pa.out_coef = fp(out_coef);
  pa.residual = bp(residual);
  pa.res_coef = fpo(res_coef);
  pa.out_bits = (uint8_t*)bits.data_ptr();
  pa.M = M; pa.N = N; pa.K = K; pa.rg = rg; pa.sched = dpe_gemm::sched_buffer(cur_stream());
  CHECK_RC(dpe_pw_launch(&pa, dpe::PW_APPLY, cur_stream()), "pw_stream apply");
  return {y, bits};
}

// BN3 backward by Gram algebra: from part (row 0: sum dz partials, [2][Cout][rg]), P = dz^T a2 [Cout][Cin], W,
// u = W G, s, the forward coef: dgamma / dbeta / dw accumulate; returns the data grad's B operand
// [Cout + Cin][Cin] bf16 (= [diag(a) W ; W^T diag(b) W]) and its bias c^T W [Cin].
std::vector<Tensor> bn_gram_bwd(const Tensor& part, const Tensor& P, const Tensor& w, const Tensor& u, const Tensor& sv,
                                const Tensor& coef, const c10::optional<Tensor>& gamma, int64_t M,
                                const c10::optional<Tensor>& dgamma, const c10::optional<Tensor>& dbeta, Tensor& dw) {
  CHECK_GPU(part); CHECK_F32(part); CHECK_F32(P); CHECK_F32(u); CHECK_F32(sv); CHECK_F32(coef); CHECK_F32(dw);
  CHECK_BF16(w); CHECK_CONTIG(w); CHECK_CONTIG(P); CHECK_CONTIG(dw); CHECK_CONTIG(part);
  const int64_t Cout = w.size(0), Cin = w.numel() / Cout;
  TORCH_CHECK(part.dim() == 3 && part.size(1) == Cout && P.numel() == Cout * Cin && u.numel() == Cout * Cin &&
                  dw.numel() == Cout * Cin && sv.numel() == 2 * Cin && coef.numel() == 4 * Cout && sv.is_contiguous(),
              "bn_gram_bwd: shapes");
  auto fo = P.options();
  Tensor bcat = at::empty({Cout + Cin, Cin}, w.options()), abc = at::empty({3, Cout}, fo), e = at::empty({Cin}, fo);
  Tensor qws = at::empty({dpe_gram_bwd_ws_floats((int)Cin, (int)Cout)}, fo);
  CHECK_RC(dpe_gram_bwd(fp(part), (int)part.size(2), fp(P), bp(w), fp(u), fp(sv), fp(coef), fpo(gamma), (int)Cin,
                        (int)Cout, M, fpom(dgamma), fpom(dbeta), fp(dw), bpm(bcat), fp(abc), fp(e), fp(qws), cur_stream()),
           "bn_gram_bwd");
  return {bcat, e};
}

// da2 = [dz | a2] x bcat + e with the BN-backward partials of the BN + ReLU that produced a2 (bn_x, bn_coef):
// the concatenated-K data grad of the Gram-algebra BN3 backward (igemm AX_CAT).  a2 = relu(a2src * a2_coef)
// when a2_coef is given (a2 never materialised), else a2src itself.  Returns (da2, partials).
std::vector<Tensor> conv1x1_dgrad_cat(const Tensor& dz, const Tensor& a2src, const c10::optional<Tensor>& a2_coef,
                                      const Tensor& bcat, const Tensor& e, const Tensor& bn_x, const Tensor& bn_coef) {
  CHECK_GPU(dz); CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_BF16(a2src); CHECK_CONTIG(a2src); CHECK_BF16(bcat);
  CHECK_CONTIG(bcat); CHECK_F32(e); CHECK_BF16(bn_x); CHECK_CONTIG(bn_x); CHECK_F32(bn_coef);
  const int64_t K1 = dz.size(-1), M = dz.numel() / K1, C = a2src.size(-1);
  TORCH_CHECK(a2src.numel() == M * C && bcat.size(0) == K1 + C && bcat.size(1) == C && e.numel() == C &&
                  bn_x.sizes() == a2src.sizes() && bn_coef.numel() == 4 * C && K1 % 32 == 0 && C % 32 == 0,
              "conv1x1_dgrad_cat: shapes");
  Tensor dx = at::empty_like(bn_x);
  // a2 materialised and >= 256 channels (layer 3): the persistent GEMM's NN layout with the two A segments
  // (hgemm.hip CV = 3) and its BN-backward-partials epilogue; 156-167 us per call on the LDS-DMA kernel
  // here (416 TF, profiles/resnet50_bs512_sequence_r4.txt in git history)
  if (g_hgemm_conv && !(a2_coef.has_value() && a2_coef->defined()) && C >= 256 && C % 64 == 0 && K1 % 64 == 0) {
    int pcols = 0;
    const auto pl = dpe_gemm::plan_bnb(M, C, K1 + C, 1, 0, &pcols);
    if (pl.cfg >= 0 && pl.splits == 1 && pcols > 0) {
      Tensor part = at::empty({2, C, pcols}, dz.options().dtype(at::kFloat));
      auto h = hargs();
      h.A = bp(dz); h.B = bp(bcat); h.C = dx.data_ptr();
      h.M = (int)M; h.N = (int)C; h.K = (int)(K1 + C);
      h.lda = K1; h.ldb = C; h.ldc = C;
      h.bias = fp(e);
      h.conv = 3; h.A2 = bp(a2src); h.lda2 = C; h.k1 = (int)K1;
      h.col_stats = fp(part); h.stats_ld = pcols; h.st_x = bp(bn_x); h.st_coef = fp(bn_coef);
      dpe_gemm::run_bnb(h, pl, 1, 0);
      return {dx, part};
    }
  }
  // a2 = relu(BN2(h2)) on load with h2 also the BN-backward input (layers 1-2): the streaming kernel
  // (pwconv.hip pw_cat_kernel) -- mask and h2 - mean from the h2 tile it holds, no second read of h2
  if (a2_coef.has_value() && a2_coef->defined() && a2src.data_ptr() == bn_x.data_ptr() && a2_coef->numel() == 4 * C &&
      bn_coef.data_ptr() == a2_coef->data_ptr()) {
    const int rg = dpe_pw_cat_blocks(M, K1, C);
    if (rg > 0) {
      Tensor part = at::empty({2, C, rg}, dz.options().dtype(at::kFloat));
      dpe::PwCatArgs pa{};
      pa.dz = bp(dz); pa.h2 = bp(a2src); pa.coef = fp(bn_coef); pa.bcat = bp(bcat); pa.ebias = fp(e);
      pa.y = bpm(dx); pa.stats = fp(part); pa.M = M; pa.rg = rg;
      CHECK_RC(dpe_pw_cat_launch(&pa, K1, C, cur_stream()), "pw_cat data grad");
      return {dx, part};
    }
  }
  auto a = base_args();
  a.A = bp(dz); a.B = bp(bcat); a.C = dx.data_ptr();
  a.M = (int)M; a.N = (int)C; a.K = (int)(K1 + C);
  a.lda = K1; a.ldb = C; a.ldc = C;
  a.k_split = a.K;
  a.bias = fp(e);
  a.a_mode = dpe::AX_CAT;
  a.a2 = bp(a2src); a.lda2 = C; a.k1 = (int)K1;
  a.a_coef = fpo(a2_coef);
  a.st_x = bp(bn_x); a.st_coef = fp(bn_coef);
  const int bm = 128, bn = C <= 64 ? 64 : 128;
  const int64_t tilesM = (M + bm - 1) / bm;
  Tensor part = at::empty({2, C, tilesM}, dz.options().dtype(at::kFloat));
  a.col_stats = fp(part);
  a.stats_ld = (int)tilesM;
  const int rc = dpe_igemm_dma_launch(&a, bm, bn, dpe::A_DENSE_K, dpe::B_DENSE_N, dpe::EPI_BF16_BNB, cur_stream());
  CHECK_RC(rc, "igemm_dma AX_CAT data grad");
  return {dx, part};
}

// BatchNorm coefficients [4][C] (scale, shift, mean, invstd) from conv-epilogue
// partials WITHOUT applying them: the consumer conv applies relu(x*scale+shift)
// in its load prologue.  Updates running stats like bn_fwd_train.
Tensor bn_coef(const Tensor& stats, int64_t M, const c10::optional<Tensor>& gamma, const c10::optional<Tensor>& beta,
               const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar, double momentum, double eps) {
  CHECK_GPU(stats); CHECK_F32(stats);
  TORCH_CHECK(stats.dim() == 3 && stats.size(0) == 2, "stats must be [2][C][nb] partials");
  const int64_t C = stats.size(1);
  Tensor coef = at::empty({4, C}, stats.options());
  CHECK_RC(dpe_bn_finalize(fp(stats), (int)stats.size(2), (int)C, M, fpo(gamma), fpo(beta), fpom(rmean), fpom(rvar),
                           (float)momentum, (float)eps, fp(coef), cur_stream()), "bn_finalize");
  return coef;
}

// Backward of y = relu(BN(x)) given the (sum dz, sum dz*(x-mean)) partials
// [2][C][nb] produced by the dgrad epilogue that computed dy; the ReLU mask is
// recomputed from x and the forward coefficients.  dgamma/dbeta accumulate.
// relu_mask=false: dy is already dz (masked by its producer, see conv_dgrad_bn's mask).
Tensor bn_bwd_partials(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& gamma, const Tensor& coef,
                       const Tensor& partials, const c10::optional<Tensor>& dgamma, const c10::optional<Tensor>& dbeta,
                       bool relu_mask) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_BF16(x);
  TORCH_CHECK(dy.sizes() == x.sizes(), "bn_bwd_partials: dy/x shape mismatch");
  const int64_t C = x.size(-1), M = rows_of(x);
  TORCH_CHECK(partials.dim() == 3 && partials.size(0) == 2 && partials.size(1) == C, "partials must be [2][C][nb]");
  hipStream_t st = cur_stream();
  Tensor bcoef = at::empty({3, C}, x.options().dtype(at::kFloat));
  CHECK_RC(dpe_bn_bwd_finalize(fp(partials), (int)partials.size(2), (int)C, M, fpo(gamma), fp(coef), fpom(dgamma),
                               fpom(dbeta), fp(bcoef), st), "bn_bwd_finalize");
  Tensor dx = at::empty_like(x);
  CHECK_RC(dpe_bn_bwd_apply(bp(dy), nullptr, nullptr, bp(x), fp(bcoef), bpm(dx), nullptr, M, (int)C, relu_mask ? fp(coef) : nullptr, st),
           "bn_bwd_apply");
  return dx;
}

// BatchNorm-backward coefficients [3][C] (dx = a*dz + b*x + c) from the (sum dz, sum dz*(x-mean))
// partials, without the apply pass (its consumer applies it on load: conv1x1_bnin_dgrad).
// dgamma/dbeta accumulate.
Tensor bn_bwd_coef(const Tensor& partials, int64_t M, const c10::optional<Tensor>& gamma, const Tensor& coef,
                   const c10::optional<Tensor>& dgamma, const c10::optional<Tensor>& dbeta) {
  CHECK_GPU(partials); CHECK_F32(partials);
  TORCH_CHECK(partials.dim() == 3 && partials.size(0) == 2, "partials must be [2][C][nb]");
  const int64_t C = partials.size(1);
  Tensor bcoef = at::empty({3, C}, partials.options());
  CHECK_RC(dpe_bn_bwd_finalize(fp(partials), (int)partials.size(2), (int)C, M, fpo(gamma), fp(coef), fpom(dgamma),
                               fpom(dbeta), fp(bcoef), cur_stream()), "bn_bwd_finalize");
  return bcoef;
}

// 1x1 stride-1 convolutions over a BatchNorm output that is never written by a pass of its own
// (igemm.h AXform): the LDS-DMA kernel computes the operand from two tensors on its fragments and
// stores it once as a by-product (x_out [+ x_bits]), so the consumer's own read of it disappears.
//
// forward: y = x . W^T,  x = relu(h * scale + shift + res)           (res_coef absent)
//                         x = relu(h * scale + shift + bf16(res * scale_d + shift_d))   (downsample identity)
// with the BN-forward partials of y when want_stats.  tile_m: 128 or 256 (N = 64 only).
std::vector<Tensor> conv1x1_bnin_fwd(const Tensor& h, const Tensor& res, const Tensor& coef,
                                     const c10::optional<Tensor>& res_coef, const Tensor& w, Tensor& x_out,
                                     Tensor& x_bits, bool want_stats, int64_t tile_m) {
  CHECK_GPU(h); CHECK_BF16(h); CHECK_BF16(res); CHECK_BF16(w); CHECK_BF16(x_out);
  CHECK_CONTIG(h); CHECK_CONTIG(res); CHECK_CONTIG(w); CHECK_CONTIG(x_out); CHECK_CONTIG(x_bits);
  CHECK_F32(coef);
  TORCH_CHECK(h.dim() == 4 && w.dim() == 4 && w.size(1) == 1 && w.size(2) == 1 && w.size(3) == h.size(3),
              "conv1x1_bnin_fwd: NHWC h / [K,1,1,C] w shape mismatch");
  TORCH_CHECK(res.sizes() == h.sizes() && x_out.sizes() == h.sizes(), "conv1x1_bnin_fwd: res / x_out must have h's shape");
  TORCH_CHECK(x_bits.scalar_type() == at::kByte && x_bits.numel() * 8 == h.numel(), "conv1x1_bnin_fwd: x_bits [.., C/8] u8");
  const int64_t C = h.size(3), K = w.size(0);
  TORCH_CHECK(coef.numel() == 4 * C && (!res_coef.has_value() || res_coef->numel() == 4 * C), "coef must be [4][C]");
  TORCH_CHECK(C % 32 == 0 && C <= 2048 && K % 8 == 0, "conv1x1_bnin_fwd: C % 32 == 0, C <= 2048");
  Tensor y = at::empty({h.size(0), h.size(1), h.size(2), K}, h.options());
  auto a = base_args();
  a.g = geom(h, w, 1, 1, 0, 0, 1, 1, h.size(1), h.size(2));
  a.A = bp(h); a.B = bp(w); a.C = y.data_ptr();
  a.M = (int)(h.numel() / C); a.N = (int)K; a.K = (int)C;
  a.lda = C; a.ldb = C; a.ldc = K;
  a.k_split = a.K;
  a.a_mode = (res_coef.has_value() && res_coef->defined()) ? dpe::AX_BN_RES2 : dpe::AX_BN_RES;
  a.a2 = bp(res); a.a_coef = fp(coef); a.a_coef2 = fpo(res_coef);
  a.a_out = bpm(x_out); a.a_bits = (uint8_t*)x_bits.data_ptr();
  Tensor stats;
  if (want_stats) {  // per-128-row partials: the layout every conv path produces (BN finalize is tile-agnostic)
    stats = at::empty({2, K, (a.M + 127) / 128}, h.options().dtype(at::kFloat));
    a.col_stats = fp(stats);
  }
  const int bm = (K == 64 && tile_m == 256) ? 256 : 128, bn = K <= 64 ? 64 : 128;
  CHECK_RC(dpe_igemm_dma_launch(&a, bm, bn, dpe::A_DENSE_K, dpe::B_DENSE_K, dpe::EPI_BF16, cur_stream()),
           "conv1x1_bnin_fwd");
  return {y, stats};
}

// data grad: dx = dh . W  with  dh = a * dz + b * h + c  (BN backward applied on load, dh stored as a
// by-product for the weight grad), plus the BN-backward partials of the BN + ReLU that produced this
// conv's input (bn_x, bn_coef: ReLU mask recomputed from bn_x), as conv_dgrad_bn.
std::vector<Tensor> conv1x1_bnin_dgrad(const Tensor& dz, const Tensor& h, const Tensor& bcoef, const Tensor& w,
                                       Tensor& dh_out, const Tensor& bn_x, const Tensor& bn_coef) {
  CHECK_GPU(dz); CHECK_BF16(dz); CHECK_BF16(h); CHECK_BF16(w); CHECK_BF16(dh_out); CHECK_BF16(bn_x);
  CHECK_CONTIG(dz); CHECK_CONTIG(h); CHECK_CONTIG(w); CHECK_CONTIG(dh_out); CHECK_CONTIG(bn_x);
  CHECK_F32(bcoef); CHECK_F32(bn_coef);
  TORCH_CHECK(dz.dim() == 4 && w.dim() == 4 && w.size(1) == 1 && w.size(2) == 1 && w.size(0) == dz.size(3),
              "conv1x1_bnin_dgrad: NHWC dz / [K,1,1,C] w shape mismatch");
  TORCH_CHECK(h.sizes() == dz.sizes() && dh_out.sizes() == dz.sizes(), "conv1x1_bnin_dgrad: h / dh_out must have dz's shape");
  const int64_t K = dz.size(3), C = w.size(3);
  TORCH_CHECK(bcoef.numel() == 3 * K, "bcoef must be [3][K]");
  TORCH_CHECK(K % 32 == 0 && K <= 2048 && C % 8 == 0, "conv1x1_bnin_dgrad: K % 32 == 0, K <= 2048");
  TORCH_CHECK(bn_x.dim() == 4 && bn_x.size(0) == dz.size(0) && bn_x.size(1) == dz.size(1) && bn_x.size(2) == dz.size(2) &&
                  bn_x.size(3) == C && bn_coef.numel() == 4 * C,
              "conv1x1_bnin_dgrad: bn_x must be [N,H,W,C], bn_coef [4][C]");
  Tensor dx = at::empty_like(bn_x);
  auto a = base_args();
  a.g = geom(dx, w, 1, 1, 0, 0, 1, 1, dz.size(1), dz.size(2));
  a.A = bp(dz); a.B = bp(w); a.C = dx.data_ptr();
  a.M = (int)(dz.numel() / K); a.N = (int)C; a.K = (int)K;
  a.lda = K; a.ldb = C; a.ldc = C;
  a.k_split = a.K;
  a.a_mode = dpe::AX_BN_BWD;
  a.a2 = bp(h); a.a_coef = fp(bcoef); a.a_out = bpm(dh_out);
  a.st_x = bp(bn_x); a.st_coef = fp(bn_coef);
  const int64_t tiles_m = (a.M + 127) / 128;
  Tensor part = at::empty({2, C, tiles_m}, dz.options().dtype(at::kFloat));
  a.col_stats = fp(part);
  a.stats_ld = (int)tiles_m;
  const int bn = C <= 64 ? 64 : 128;
  CHECK_RC(dpe_igemm_dma_launch(&a, 128, bn, dpe::A_DENSE_K, dpe::B_DENSE_N, dpe::EPI_BF16_BNB, cur_stream()),
           "conv1x1_bnin_dgrad");
  return {dx, part};
}

// Two BatchNorms fed by the same dz (a downsample bottleneck: BN3 and BN_d both see dz3):
// BN3's backward from its epilogue partials, BN_d's reduce fused into BN3's apply pass
// (dz read once for both), then BN_d's apply.  Returns (dx, dx2).
std::vector<Tensor> bn_bwd_dual(const Tensor& dz, const Tensor& x, const c10::optional<Tensor>& gamma, const Tensor& coef,
                                const Tensor& partials, const c10::optional<Tensor>& dgamma,
                                const c10::optional<Tensor>& dbeta, const Tensor& x2, const c10::optional<Tensor>& gamma2,
                                const Tensor& coef2, const c10::optional<Tensor>& dgamma2, const c10::optional<Tensor>& dbeta2) {
  CHECK_GPU(dz); CHECK_BF16(dz); CHECK_CONTIG(dz); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(x2); CHECK_CONTIG(x2);
  TORCH_CHECK(dz.sizes() == x.sizes() && dz.sizes() == x2.sizes(), "bn_bwd_dual: dz / x / x2 shape mismatch");
  const int64_t C = x.size(-1), M = rows_of(x);
  TORCH_CHECK(partials.dim() == 3 && partials.size(0) == 2 && partials.size(1) == C, "partials must be [2][C][nb]");
  hipStream_t st = cur_stream();
  auto fo = x.options().dtype(at::kFloat);
  Tensor bcoef = at::empty({3, C}, fo);
  CHECK_RC(dpe_bn_bwd_finalize(fp(partials), (int)partials.size(2), (int)C, M, fpo(gamma), fp(coef), fpom(dgamma),
                               fpom(dbeta), fp(bcoef), st), "bn_bwd_finalize");
  const int nb = dpe_bn_bwd_nblocks(M, (int)C);
  Tensor part2 = at::empty({2, C, nb}, fo);
  Tensor dx = at::empty_like(x);
  CHECK_RC(dpe_bn_bwd_reduce_apply(bp(dz), bp(x2), fp(coef2), bp(x), fp(bcoef), bpm(dx), M, (int)C, nb, fp(part2), st),
           "bn_bwd_reduce_apply");
  Tensor bcoef2 = at::empty({3, C}, fo);
  CHECK_RC(dpe_bn_bwd_finalize(fp(part2), nb, (int)C, M, fpo(gamma2), fp(coef2), fpom(dgamma2), fpom(dbeta2), fp(bcoef2), st),
           "bn_bwd_finalize");
  Tensor dx2 = at::empty_like(x2);
  CHECK_RC(dpe_bn_bwd_apply(bp(dz), nullptr, nullptr, bp(x2), fp(bcoef2), bpm(dx2), nullptr, M, (int)C, nullptr, st),
           "bn_bwd_apply");
  return {dx, dx2};
}

// ----------------------------------------------------------------- pooling
std::vector<Tensor> maxpool_fwd(const Tensor& x, int64_t k, int64_t s, int64_t p) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  Tensor y = at::empty({N, OH, OW, C}, x.options());
  Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  CHECK_RC(dpe_maxpool_fwd(bp(x), bpm(y), (uint8_t*)idx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k,
                           (int)s, (int)p, cur_stream()), "maxpool_fwd");
  return {y, idx};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& idx, std::vector<int64_t> xshape, int64_t k, int64_t s, int64_t p) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy);
  Tensor dx = at::empty(xshape, dy.options());
  CHECK_RC(dpe_maxpool_bwd(bp(dy), (const uint8_t*)idx.data_ptr(), bpm(dx), (int)xshape[0], (int)xshape[1], (int)xshape[2],
                           (int)xshape[3], (int)dy.size(1), (int)dy.size(2), (int)k, (int)s, (int)p, cur_stream()),
           "maxpool_bwd");
  return dx;
}

// y = act(BN(x; coef) + r), r = residual (bf16) or, with residual_coef, BN(residual; residual_coef)
// computed in the same pass (bottleneck output with a BN'd downsample branch).
// want_mask: also the ReLU-mask bits of y, uint8 [.., C/8] (bit e of byte j = y[.., 8j+e] > 0).
std::vector<Tensor> bn_apply(const Tensor& x, const Tensor& coef, const c10::optional<Tensor>& residual,
                             const c10::optional<Tensor>& residual_coef, bool relu, bool want_mask) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_F32(coef);
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && coef.numel() == 4 * C, "bn_apply: coef must be [4][C], C % 8 == 0");
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) {
    CHECK_BF16((*residual)); CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->sizes() == x.sizes(), "bn_apply: residual shape mismatch");
  }
  Tensor y = at::empty_like(x);
  Tensor bits;
  if (want_mask) {
    auto sz = x.sizes().vec();
    sz.back() = C / 8;
    bits = at::empty(sz, x.options().dtype(at::kByte));
  }
  uint8_t* mb = want_mask ? (uint8_t*)bits.data_ptr() : nullptr;
  if (residual_coef.has_value() && residual_coef->defined()) {
    TORCH_CHECK(has_res, "bn_apply: residual_coef needs a residual");
    CHECK_F32((*residual_coef));
    TORCH_CHECK(residual_coef->numel() == 4 * C, "bn_apply: residual_coef must be [4][C]");
    CHECK_RC(dpe_bn_apply2(bp(x), fp(coef), bp(*residual), fp(*residual_coef), bpm(y), rows_of(x), (int)C, relu ? 1 : 0, mb,
                           cur_stream()), "bn_apply2");
  } else {
    CHECK_RC(dpe_bn_apply_m(bp(x), has_res ? bp(*residual) : nullptr, bpm(y), rows_of(x), (int)C, fp(coef), relu ? 1 : 0, mb,
                            cur_stream()), "bn_apply");
  }
  return {y, bits};
}

// Stem fusion: maxpool(relu(BN(h))) with BN coefficients `coef` [4][C] (bn_coef);
// the BN+ReLU output is never materialised.  Returns (pooled, argmax bytes).
std::vector<Tensor> bnrelu_maxpool_fwd(const Tensor& h, const Tensor& coef, int64_t k, int64_t s, int64_t p) {
  CHECK_GPU(h); CHECK_BF16(h); CHECK_CONTIG(h); CHECK_F32(coef);
  const int64_t N = h.size(0), H = h.size(1), W = h.size(2), C = h.size(3);
  TORCH_CHECK(coef.numel() == 4 * C, "bnrelu_maxpool_fwd: coef must be [4][C]");
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  Tensor y = at::empty({N, OH, OW, C}, h.options());
  Tensor idx = at::empty({N, OH, OW, C}, h.options().dtype(at::kByte));
  CHECK_RC(dpe_bnrelu_maxpool_fwd(bp(h), fp(coef), bpm(y), (uint8_t*)idx.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)OH,
                                  (int)OW, (int)k, (int)s, (int)p, cur_stream()), "bnrelu_maxpool_fwd");
  return {y, idx};
}

// Backward of the fused stem: dh = BN'(relu'(h) * maxpool'(dy)); dgamma/dbeta accumulate.
Tensor maxpool_bn_bwd(const Tensor& dy, const Tensor& idx, const Tensor& h, const c10::optional<Tensor>& gamma,
                      const Tensor& coef, const c10::optional<Tensor>& dgamma, const c10::optional<Tensor>& dbeta, int64_t k,
                      int64_t s, int64_t p) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(h); CHECK_CONTIG(h); CHECK_F32(coef);
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.sizes() == dy.sizes(), "maxpool_bn_bwd: idx must be uint8 of dy's shape");
  const int64_t N = h.size(0), H = h.size(1), W = h.size(2), C = h.size(3);
  TORCH_CHECK(dy.size(0) == N && dy.size(3) == C, "maxpool_bn_bwd: dy/h shape mismatch");
  const int64_t M = N * H * W;
  hipStream_t st = cur_stream();
  auto fo = h.options().dtype(at::kFloat);
  // the gather makes each row latency-heavy: ~16 rows per thread-row-phase, up to 8192 partial blocks
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(8192, M / 512));
  Tensor part = at::empty({2, C, nb}, fo);
  CHECK_RC(dpe_maxpool_bn_bwd_reduce(bp(dy), (const uint8_t*)idx.data_ptr(), bp(h), fp(coef), (int)N, (int)H, (int)W, (int)C,
                                     (int)dy.size(1), (int)dy.size(2), (int)k, (int)s, (int)p, nb, fp(part), st),
           "maxpool_bn_bwd_reduce");
  Tensor bcoef = at::empty({3, C}, fo);
  CHECK_RC(dpe_bn_bwd_finalize(fp(part), nb, (int)C, M, fpo(gamma), fp(coef), fpom(dgamma), fpom(dbeta), fp(bcoef), st),
           "bn_bwd_finalize");
  Tensor dh = at::empty_like(h);
  CHECK_RC(dpe_maxpool_bn_bwd_apply(bp(dy), (const uint8_t*)idx.data_ptr(), bp(h), fp(coef), fp(bcoef), bpm(dh), (int)N,
                                    (int)H, (int)W, (int)C, (int)dy.size(1), (int)dy.size(2), (int)k, (int)s, (int)p, st),
           "maxpool_bn_bwd_apply");
  return dh;
}

// The stem's backward without dY: BN-backward coefficients of the pooled gradient (reduce + finalize; dgamma /
// dbeta accumulate), then the stem weight grad computing dY = a dz + b h + c on the fly (stem.hip FUSED).
// dw [64, 4, 4, 16] (s2d filter layout) += dW.  No dY tensor, no apply pass.
void stem_bwd_fused(const Tensor& dy, const Tensor& idx, const Tensor& h, const Tensor& xs,
                    const c10::optional<Tensor>& gamma, const Tensor& coef, const c10::optional<Tensor>& dgamma,
                    const c10::optional<Tensor>& dbeta, Tensor& dw) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_BF16(h); CHECK_CONTIG(h); CHECK_F32(coef); CHECK_BF16(xs);
  CHECK_CONTIG(xs); CHECK_F32(dw); CHECK_CONTIG(dw);
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.sizes() == dy.sizes(), "stem_bwd_fused: idx must be uint8 of dy's shape");
  const int64_t N = h.size(0), H = h.size(1), W = h.size(2), C = h.size(3);
  TORCH_CHECK(C == 64 && dy.size(0) == N && dy.size(1) == H / 2 && dy.size(2) == W / 2 && dy.size(3) == C && H % 2 == 0 &&
                  W % 2 == 0 && xs.size(0) == N && xs.size(1) == H && xs.size(2) == W && xs.size(3) == 16 &&
                  dw.numel() == 64 * 256,
              "stem_bwd_fused: shapes (h [N,H,W,64], dy/idx [N,H/2,W/2,64], xs [N,H,W,16], dw [64,4,4,16])");
  const int64_t M = N * H * W;
  hipStream_t st = cur_stream();
  auto fo = h.options().dtype(at::kFloat);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(8192, M / 512));
  Tensor part = at::empty({2, C, nb}, fo);
  CHECK_RC(dpe_maxpool_bn_bwd_reduce(bp(dy), (const uint8_t*)idx.data_ptr(), bp(h), fp(coef), (int)N, (int)H, (int)W, (int)C,
                                     (int)dy.size(1), (int)dy.size(2), 3, 2, 1, nb, fp(part), st),
           "maxpool_bn_bwd_reduce");
  Tensor bcoef = at::empty({3, C}, fo);
  CHECK_RC(dpe_bn_bwd_finalize(fp(part), nb, (int)C, M, fpo(gamma), fp(coef), fpom(dgamma), fpom(dbeta), fp(bcoef), st),
           "bn_bwd_finalize");
  auto scratch = at::empty({dpe_stem_wgrad_scratch(N, H, W)}, fo);
  CHECK_RC(dpe_stem_wgrad_launch2(bp(xs), nullptr, fp(dw), fp(scratch), (int)N, (int)H, (int)W, 1.f, bp(dy),
                                  (const uint8_t*)idx.data_ptr(), bp(h), fp(coef), fp(bcoef), st),
           "stem wgrad (fused BN / max-pool backward)");
}

Tensor gavgpool_fwd(const Tensor& x) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  const int64_t N = x.size(0), C = x.size(-1), HW = x.numel() / (N * C);
  Tensor y = at::empty({N, C}, x.options());
  CHECK_RC(dpe_gavgpool_fwd(bp(x), bpm(y), (int)N, (int)HW, (int)C, cur_stream()), "gavgpool_fwd");
  return y;
}

Tensor gavgpool_bwd(const Tensor& dy, std::vector<int64_t> xshape) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy);
  Tensor dx = at::empty(xshape, dy.options());
  const int64_t N = xshape[0], C = xshape.back(), HW = dx.numel() / (N * C);
  CHECK_RC(dpe_gavgpool_bwd(bp(dy), bpm(dx), (int)N, (int)HW, (int)C, cur_stream()), "gavgpool_bwd");
  return dx;
}

// ------------------------------------------------------------------- loss
// returns (loss_rows [B] f32, loss_sum [1], correct [1], dlogits or empty)
std::vector<Tensor> cross_entropy(const Tensor& logits, const Tensor& labels, int64_t V, double grad_scale, bool want_grad,
                                  bool grad_bf16, int64_t ignore_index, bool inplace) {
  CHECK_GPU(logits); CHECK_CONTIG(logits); CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  const bool in_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(in_bf16 || logits.scalar_type() == at::kFloat, "logits must be f32 or bf16");
  const int64_t ld = logits.size(-1), B = logits.numel() / ld;
  TORCH_CHECK(labels.numel() == B, "labels size mismatch");
  auto fo = logits.options().dtype(at::kFloat);
  Tensor rows = at::empty({B}, fo);
  Tensor sums = at::zeros({2}, fo);
  Tensor d;
  if (want_grad && inplace) {
    TORCH_CHECK(grad_bf16 == in_bf16, "cross_entropy: in-place gradient needs the logits dtype");
    d = logits;  // the row is held in registers: the gradient overwrites the logits
  } else if (want_grad) {
    d = at::empty(logits.sizes(), logits.options().dtype(grad_bf16 ? at::kBFloat16 : at::kFloat));
  }
  CHECK_RC(dpe_cross_entropy(logits.data_ptr(), in_bf16, (const int64_t*)labels.data_ptr(), (int)B, (int)V, ld,
                             (float)grad_scale, want_grad ? d.data_ptr() : nullptr, grad_bf16, fp(rows), fp(sums),
                             fp(sums) + 1, (int)ignore_index, cur_stream()), "cross_entropy");
  return {rows, sums.slice(0, 0, 1), sums.slice(0, 1, 2), d};
}

// Training form: (out4 = [loss_sum, correct, mean over non-ignored rows, 1 / their count], dlogits).  The
// mean and the backward scale come out of the reduction kernel itself (no torch count / clamp / divide
// launches at the forward -> backward seam).
std::vector<Tensor> cross_entropy_mean(const Tensor& logits, const Tensor& labels, int64_t V, bool grad_bf16,
                                       int64_t ignore_index, bool inplace) {
  CHECK_GPU(logits); CHECK_CONTIG(logits); CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  const bool in_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(in_bf16 || logits.scalar_type() == at::kFloat, "logits must be f32 or bf16");
  const int64_t ld = logits.size(-1), B = logits.numel() / ld;
  TORCH_CHECK(labels.numel() == B, "labels size mismatch");
  auto fo = logits.options().dtype(at::kFloat);
  Tensor rows = at::empty({B}, fo);
  Tensor out4 = at::zeros({4}, fo);
  Tensor d;
  if (inplace) {
    TORCH_CHECK(grad_bf16 == in_bf16, "cross_entropy: in-place gradient needs the logits dtype");
    d = logits;
  } else {
    d = at::empty(logits.sizes(), logits.options().dtype(grad_bf16 ? at::kBFloat16 : at::kFloat));
  }
  CHECK_RC(dpe_cross_entropy_mean(logits.data_ptr(), in_bf16, (const int64_t*)labels.data_ptr(), (int)B, (int)V, ld, 1.f,
                                  d.data_ptr(), grad_bf16, fp(rows), fp(out4), (int)ignore_index, cur_stream()),
           "cross_entropy_mean");
  return {out4, d};
}

// d * g * inv_n (g, inv_n: one-element fp32 device tensors) in the dtype of d
Tensor ce_grad_scale(const Tensor& d, const Tensor& g, const Tensor& inv_n) {
  CHECK_GPU(d); CHECK_CONTIG(d); CHECK_F32(g); CHECK_F32(inv_n);
  const bool bf = d.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || d.scalar_type() == at::kFloat, "ce_grad_scale: f32 or bf16");
  TORCH_CHECK(g.numel() == 1 && inv_n.numel() == 1 && g.is_cuda() && inv_n.is_cuda(), "ce_grad_scale: device scalars");
  Tensor o = at::empty_like(d);
  CHECK_RC(dpe_ce_grad_scale(d.data_ptr(), o.data_ptr(), d.numel(), bf ? 1 : 0, fp(g.contiguous()), fp(inv_n.contiguous()),
                             cur_stream()),
           "ce_grad_scale");
  return o;
}

// ---------------------------------------------------------------- eltwise
Tensor cast_bf16(const Tensor& x, const c10::optional<Tensor>& out) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  Tensor y = (out.has_value() && out->defined()) ? *out : at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  TORCH_CHECK(y.numel() == x.numel() && y.is_contiguous() && y.scalar_type() == at::kBFloat16, "cast_bf16: bad out");
  CHECK_RC(dpe_cast_f32_bf16(fp(x), bpm(y), x.numel(), cur_stream()), "cast");
  return y;
}

Tensor cast_f32(const Tensor& x) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x);
  Tensor y = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  CHECK_RC(dpe_cast_bf16_f32(bp(x), fp(y), x.numel(), cur_stream()), "cast");
  return y;
}

// op: 0 relu, 1 relu_bwd(dy, y), 2 gelu, 3 gelu_bwd(dy, x)
Tensor act(const Tensor& a, const c10::optional<Tensor>& b, int64_t op) {
  CHECK_GPU(a); CHECK_CONTIG(a);
  const bool bf = a.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || a.scalar_type() == at::kFloat, "act: f32/bf16 only");
  Tensor out = at::empty_like(a);
  const void* bpv = (b.has_value() && b->defined()) ? b->data_ptr() : nullptr;
  if (op == 1 || op == 3) TORCH_CHECK(bpv && b->is_contiguous() && b->scalar_type() == a.scalar_type(), "act: second operand");
  CHECK_RC(dpe_act(a.data_ptr(), bpv, out.data_ptr(), a.numel(), (int)op, bf, cur_stream()), "act");
  return out;
}

Tensor dropout(const Tensor& x, double p, int64_t seed, int64_t offset) {
  CHECK_GPU(x); CHECK_CONTIG(x);
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "dropout: f32/bf16 only");
  Tensor y = at::empty_like(x);
  CHECK_RC(dpe_dropout(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (uint64_t)seed, (uint64_t)offset, bf, cur_stream()),
           "dropout");
  return y;
}

Tensor add(const Tensor& a, const Tensor& b, double alpha) {
  CHECK_GPU(a); CHECK_CONTIG(a); CHECK_CONTIG(b);
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.numel() == b.numel(), "add: mismatch");
  const bool bf = a.scalar_type() == at::kBFloat16;
  Tensor out = at::empty_like(a);
  CHECK_RC(dpe_add(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), (float)alpha, bf, cur_stream()), "add");
  return out;
}

void colsum(const Tensor& dy, Tensor& db, bool accumulate) {
  CHECK_GPU(dy); CHECK_CONTIG(dy); CHECK_F32(db);
  const int64_t N = dy.size(-1), M = dy.numel() / N;
  const bool bf = dy.scalar_type() == at::kBFloat16;
  CHECK_RC(dpe_colsum(dy.data_ptr(), M, (int)N, N, fp(db), accumulate ? 1 : 0, bf, cur_stream()), "colsum");
}

Tensor nchw_to_nhwc(const Tensor& x, int64_t cpad) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cp = std::max<int64_t>(C, cpad);
  Tensor y = at::empty({N, H, W, Cp}, x.options().dtype(at::kBFloat16));
  CHECK_RC(dpe_nchw_to_nhwc(fp(x), bpm(y), (int)N, (int)C, (int)(H * W), (int)Cp, cur_stream()), "nchw_to_nhwc");
  return y;
}

Tensor nchw_to_s2d(const Tensor& x) {
  CHECK_GPU(x); CHECK_F32(x); CHECK_CONTIG(x);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C <= 4 && H % 2 == 0 && W % 2 == 0, "nchw_to_s2d: needs C <= 4 and even H, W");
  Tensor y = at::empty({N, H / 2, W / 2, 16}, x.options().dtype(at::kBFloat16));
  CHECK_RC(dpe_nchw_to_s2d(fp(x), bpm(y), (int)N, (int)C, (int)H, (int)W, cur_stream()), "nchw_to_s2d");
  return y;
}

Tensor embedding_fwd(const Tensor& idx, const Tensor& wte, const c10::optional<Tensor>& wpe) {
  CHECK_GPU(idx); CHECK_CONTIG(idx); CHECK_BF16(wte); CHECK_CONTIG(wte);
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 2, "embedding: idx must be int64 [B,T]");
  const int64_t B = idx.size(0), T = idx.size(1), D = wte.size(1);
  Tensor out = at::empty({B, T, D}, wte.options().dtype(at::kFloat));
  const uint16_t* pe = (wpe.has_value() && wpe->defined()) ? bp(*wpe) : nullptr;
  CHECK_RC(dpe_embedding_fwd((const int64_t*)idx.data_ptr(), bp(wte), pe, fp(out), B * T, (int)T, (int)D, cur_stream()),
           "embedding_fwd");
  return out;
}

void embedding_bwd(const Tensor& idx, const Tensor& dout, Tensor& dwte, const c10::optional<Tensor>& dwpe) {
  CHECK_GPU(dout); CHECK_F32(dout); CHECK_CONTIG(dout); CHECK_F32(dwte);
  const int64_t B = idx.size(0), T = idx.size(1), D = dwte.size(1);
  CHECK_RC(dpe_embedding_bwd((const int64_t*)idx.data_ptr(), fp(dout), fp(dwte), fpom(dwpe), B * T, (int)T, (int)D,
                             cur_stream()), "embedding_bwd");
}

// --------------------------------------------------------------- optimizer
void optim_step(int64_t kind, const Tensor& desc, const Tensor& chunks, const Tensor& hp, const Tensor& steps) {
  CHECK_GPU(desc); CHECK_GPU(chunks); CHECK_GPU(hp); CHECK_GPU(steps); CHECK_F32(hp); CHECK_F32(steps);
  TORCH_CHECK(chunks.scalar_type() == at::kInt && chunks.dim() == 2 && chunks.size(1) == 2, "chunks must be int32 [n,2]");
  CHECK_RC(dpe_optim_step((int)kind, desc.data_ptr(), chunks.data_ptr(), (int)chunks.size(0), fp(hp), fp(steps), cur_stream()),
           "optim_step");
}

// -------------------------------------------------------------- LayerNorm
// x [rows, D] (f32 or bf16) -> y bf16, mean/rstd f32 [rows]
std::vector<Tensor> layernorm_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, double eps) {
  CHECK_GPU(x); CHECK_CONTIG(x); CHECK_F32(w);
  const bool xb = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(xb || x.scalar_type() == at::kFloat, "layernorm: f32/bf16 input");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "layernorm: D must be a multiple of 8 and <= 8192");
  Tensor y = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  Tensor mean = at::empty({rows}, x.options().dtype(at::kFloat));
  Tensor rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  CHECK_RC(dpe_layernorm_fwd(x.data_ptr(), xb, fp(w), fpo(b), bpm(y), fp(mean), fp(rstd), rows, (int)D, (float)eps,
                             cur_stream()), "layernorm_fwd");
  return {y, mean, rstd};
}

// dx: if dx_out (f32) given, dx is ACCUMULATED into it (residual stream); else a new tensor of x's dtype
Tensor layernorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& mean, const Tensor& rstd, Tensor& dw,
                     const c10::optional<Tensor>& db, const c10::optional<Tensor>& dx_out) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_F32(dw);
  const bool xb = x.scalar_type() == at::kBFloat16;
  const int64_t D = x.size(-1), rows = x.numel() / D;
  Tensor dx;
  bool acc = false;
  if (dx_out.has_value() && dx_out->defined()) {
    dx = *dx_out;
    CHECK_F32(dx); CHECK_CONTIG(dx);
    acc = true;
  } else {
    dx = at::empty_like(x);
  }
  Tensor part = at::empty({dpe_layernorm_bwd_scratch(rows, (int)D)}, x.options().dtype(at::kFloat));
  CHECK_RC(dpe_layernorm_bwd(bp(dy), x.data_ptr(), xb, fp(w), fp(mean), fp(rstd), dx.data_ptr(), acc ? 1 : 0, nullptr,
                             nullptr, fp(dw), fpom(db), fp(part), rows, (int)D, cur_stream()), "layernorm_bwd");
  return dx;
}

// Residual-stream form (pre-LN transformer block): dx = res_in + dLN(dy) in fp32 (a new tensor,
// res_in untouched) plus its bf16 copy for the next data/weight-grad GEMMs -- one pass instead of
// LN-bwd + add + cast.
// defer: dw / db are not touched; the third output is the [nblocks][2][D] partial scratch, finalized into
// dw / db later by layernorm_bwd_finalize_group (several LayerNorms per launch).
std::vector<Tensor> layernorm_bwd_residual(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& mean,
                                           const Tensor& rstd, Tensor& dw, const c10::optional<Tensor>& db,
                                           const Tensor& res_in, bool defer) {
  CHECK_GPU(dy); CHECK_BF16(dy); CHECK_CONTIG(dy); CHECK_CONTIG(x); CHECK_F32(dw);
  CHECK_F32(res_in); CHECK_CONTIG(res_in);
  const bool xb = x.scalar_type() == at::kBFloat16;
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(res_in.numel() == x.numel(), "layernorm_bwd_residual: res_in shape mismatch");
  Tensor dx = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  Tensor dxb = at::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  Tensor part = at::empty({dpe_layernorm_bwd_scratch(rows, (int)D)}, x.options().dtype(at::kFloat));
  CHECK_RC(dpe_layernorm_bwd(bp(dy), x.data_ptr(), xb, fp(w), fp(mean), fp(rstd), dx.data_ptr(), 1, fp(res_in), bpm(dxb),
                             defer ? nullptr : fp(dw), defer ? nullptr : fpom(db), fp(part), rows, (int)D, cur_stream()),
           "layernorm_bwd_residual");
  if (defer) return {dx, dxb, part};
  return {dx, dxb};
}

// The deferred LayerNorm-backward finalizes: dw_i (+)= sum of part_i's dw partials (db_i likewise, when
// given), rows_i = the LayerNorm's row count; at most 8 per call.
void layernorm_bwd_finalize_group(const std::vector<Tensor>& parts, const std::vector<int64_t>& rows,
                                  const std::vector<Tensor>& dws, const std::vector<c10::optional<Tensor>>& dbs) {
  const size_t n = parts.size();
  TORCH_CHECK(n >= 1 && n <= 8 && rows.size() == n && dws.size() == n && dbs.size() == n,
              "layernorm_bwd_finalize_group: 1..8 problems, equal list lengths");
  std::vector<const float*> pp(n);
  std::vector<float*> pw(n), pb(n);
  std::vector<int> Ds(n);
  for (size_t i = 0; i < n; ++i) {
    CHECK_GPU(parts[i]); CHECK_F32(parts[i]); CHECK_F32(dws[i]); CHECK_CONTIG(dws[i]);
    const int64_t D = dws[i].numel();
    TORCH_CHECK(D > 0 && D % 8 == 0 && parts[i].numel() >= (int64_t)dpe_layernorm_bwd_nblocks(rows[i]) * 2 * D,
                "layernorm_bwd_finalize_group: partial scratch too small for rows / D");
    pp[i] = fp(parts[i]);
    pw[i] = fp(dws[i]);
    pb[i] = fpom(dbs[i]);
    if (pb[i]) TORCH_CHECK(dbs[i]->numel() == D, "layernorm_bwd_finalize_group: db size");
    Ds[i] = (int)D;
  }
  CHECK_RC(dpe_layernorm_bwd_finalize_group(pp.data(), rows.data(), Ds.data(), pw.data(), pb.data(), (int)n, cur_stream()),
           "layernorm_bwd_finalize_group");
}

// ---------------------------------------------------------------- attention
// qkv: [B, T, 3, H, D] bf16 -> out [B, T, H, D] bf16, lse [B, H, T] f32
std::vector<Tensor> attn_fwd(const Tensor& qkv, int64_t H, double scale, bool causal) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_CONTIG(qkv);
  const int64_t B = qkv.size(0), T = qkv.size(1), D = qkv.size(-1);
  TORCH_CHECK(qkv.numel() == B * T * 3 * H * D, "attn: qkv must be [B,T,3,H,D]");
  TORCH_CHECK(D == 64, "attn: head dim 64 supported");
  Tensor out = at::empty({B, T, H, D}, qkv.options());
  Tensor lse = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  CHECK_RC(dpe_attn_fwd(bp(qkv), bpm(out), fp(lse), (int)B, (int)T, (int)H, (int)D, (float)scale, causal, cur_stream()),
           "attn_fwd");
  return {out, lse};
}

Tensor attn_bwd(const Tensor& qkv, const Tensor& out, const Tensor& dout, const Tensor& lse, int64_t H, double scale,
                bool causal) {
  CHECK_GPU(qkv); CHECK_BF16(dout); CHECK_CONTIG(dout); CHECK_CONTIG(out);
  const int64_t B = qkv.size(0), T = qkv.size(1), D = qkv.size(-1);
  Tensor dqkv = at::empty_like(qkv);
  Tensor delta = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  CHECK_RC(dpe_attn_bwd(bp(qkv), bp(out), bp(dout), fp(lse), fp(delta), nullptr, bpm(dqkv), (int)B, (int)T, (int)H, (int)D,
                        (float)scale, causal, cur_stream()), "attn_bwd");
  return dqkv;
}

}  // namespace

void register_ops(pybind11::module& m) {
  namespace py = pybind11;
  using c10::optional;
  m.def("linear_fwd", &linear_fwd, py::arg("x"), py::arg("w"), py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("out_f32") = false, py::arg("residual") = py::none(), py::arg("out") = py::none(),
        py::arg("aux_out") = py::none());
  m.def("linear_dgrad", &linear_dgrad, py::arg("dy"), py::arg("w"), py::arg("residual") = py::none(),
        py::arg("alpha_t") = py::none(), py::arg("gelu_in") = py::none());
  m.def("linear_wgrad", &linear_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("alpha") = 1.0,
        py::arg("alpha_t") = py::none(), py::arg("dbias") = py::none(), py::arg("fin_stream") = 0,
        py::arg("overwrite") = false,
        "dw (+)= alpha dy^T x (+ db += alpha colsum(dy)); fin_stream: run a K-split's slab reduction on that HIP "
        "stream (the caller orders dw's consumers after it); overwrite: dw = instead of dw +=");
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("dil"),
        py::arg("want_stats") = false, py::arg("bias") = py::none(), py::arg("in_coef") = py::none());
  m.def("row_bn_on_load", [](std::vector<int64_t> xs, std::vector<int64_t> ws, std::vector<int64_t> stride,
                             std::vector<int64_t> pad, std::vector<int64_t> dil) {
          // the row-walking 64-channel 3x3 kernels (fwd + wgrad) take the pre-BN input (in_coef)
          if (xs.size() != 4 || ws.size() != 4 || stride.size() != 2 || pad.size() != 2 || dil.size() != 2) return false;
          dpe::ConvGeom g{};
          g.N = (int)xs[0]; g.H = (int)xs[1]; g.W = (int)xs[2]; g.C = (int)xs[3];
          g.K = (int)ws[0]; g.R = (int)ws[1]; g.S = (int)ws[2];
          g.sh = (int)stride[0]; g.sw = (int)stride[1]; g.ph = (int)pad[0]; g.pw = (int)pad[1];
          g.dh = (int)dil[0]; g.dw = (int)dil[1];
          g.OH = (g.H + 2 * g.ph - g.dh * (g.R - 1) - 1) / g.sh + 1;
          g.OW = (g.W + 2 * g.pw - g.dw * (g.S - 1) - 1) / g.sw + 1;
          return ws[3] == xs[3] && rowconv_geom(g) && dpe_wgrad3x3_rows_blocks(g.N, g.H, g.W) > 0;
        }, py::arg("x_shape"), py::arg("w_shape"), py::arg("stride"), py::arg("pad"), py::arg("dil"));
  m.def("pw_bn_on_load", [](std::vector<int64_t> xs, int64_t cout) {
          // a 1x1 / stride-1 conv over a pre-BN input [N, H, W, C]: the streaming pointwise forward and the
          // LDS-DMA weight grad (K = pixels % 32, M = Cout, N = C) take the BN coefficients (in_coef)
          if (xs.size() != 4) return false;
          const int64_t M = xs[0] * xs[1] * xs[2], C = xs[3];
          static const int cmax = [] { const char* e = getenv("DPE_PW_BNIN_CMAX"); return e ? atoi(e) : 128; }();
          return pw_stream_on() && (C == 64 || C == 128) && C <= cmax && cout % 8 == 0 && M % 32 == 0 &&
                 dpe_pw_rowgroups(M, cout, C, dpe::PW_FWD) > 0;
        }, py::arg("x_shape"), py::arg("cout"));
  m.def("gram_ok", [](std::vector<int64_t> h2shape, int64_t cout3, int64_t next_width) {
          // BN3 by Gram algebra for a bottleneck whose conv3 input is h2 [N, H, W, C2] (bngram.hip): conv3's
          // forward with the BN3 + residual + ReLU epilogue on the streaming kernel (PW_APPLY), its data
          // grad as the concatenated-K LDS-DMA GEMM, and the next block's conv1 data grad (K = next_width ->
          // cout3) emitting the sum-dz partials (PW_DSUM)
          if (h2shape.size() != 4 || !pw_stream_on()) return false;
          const int64_t M = h2shape[0] * h2shape[1] * h2shape[2], C2 = h2shape[3];
          if (C2 != 64 && C2 != 128 && C2 != 256) return false;
          if (cout3 % 128 || M % 32) return false;
          return dpe_pw_rowgroups(M, cout3, C2, dpe::PW_APPLY) > 0 &&
                 dpe_pw_rowgroups(M, cout3, next_width, dpe::PW_DSUM) > 0;
        }, py::arg("h2_shape"), py::arg("cout3"), py::arg("next_width"));
  m.def("pw_dgrad_strided_residual_ok", [](std::vector<int64_t> xshape, int64_t k) {
          // a downsample block's conv1 data grad (1x1, K = k -> N = xshape[3]) on the streaming kernel,
          // which can take the stride-2 branch's compact data grad as its residual
          if (xshape.size() != 4 || xshape[1] % 2 || xshape[2] % 2 || !pw_stream_on()) return false;
          return dpe_pw_rowgroups(xshape[0] * xshape[1] * xshape[2], xshape[3], k, dpe::PW_DGRAD) > 0;
        }, py::arg("xshape"), py::arg("k"));
  m.def("conv_dgrad_acc", &conv_dgrad_acc, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("stride"), py::arg("pad"),
        py::arg("dil"), "dx += data grad of conv(w) in place (parities without taps untouched)");
  m.def("conv_dgrad_bn", [](const Tensor& dy, const Tensor& w, std::vector<int64_t> xshape, std::vector<int64_t> stride,
                            std::vector<int64_t> pad, std::vector<int64_t> dil, const c10::optional<Tensor>& residual,
                            const c10::optional<Tensor>& bn_x, const c10::optional<Tensor>& bn_coef,
                            const c10::optional<Tensor>& bn_mask, const c10::optional<Tensor>& residual_mask,
                            bool residual_stride2, const c10::optional<Tensor>& sum_mask) {
          return conv_dgrad_impl(dy, w, xshape, stride, pad, dil, residual, bn_x, bn_coef, nullptr, bn_mask, residual_mask,
                                 residual_stride2, sum_mask);
        }, py::arg("dy"), py::arg("w"), py::arg("xshape"), py::arg("stride"),
        py::arg("pad"), py::arg("dil"), py::arg("residual") = py::none(), py::arg("bn_x") = py::none(),
        py::arg("bn_coef") = py::none(), py::arg("bn_mask") = py::none(), py::arg("residual_mask") = py::none(),
        py::arg("residual_stride2") = false, py::arg("sum_mask") = py::none(),
        "data grad; with bn_x/bn_coef also the BN-backward partials of the BN+ReLU that produced the conv input; "
        "with bn_mask (BN + residual + ReLU) the mask is bn_mask > 0 and dx is stored masked");
  m.def("bn_gram", &bn_gram, py::arg("x"), py::arg("coef") = py::none(), py::arg("shift_coef") = py::none(),
        "(G = a'^T a', s = [colsum(a'), mu]) of a' = a2 - mu, a2 = relu(x * coef[0] + coef[1]) (or x), centred on the "
        "pilot shift of shift_coef (default coef); fp32, deterministic");
  m.def("bn_gram_coef", &bn_gram_coef, py::arg("G"), py::arg("s"), py::arg("w"), py::arg("M"), py::arg("gamma"),
        py::arg("beta"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        "BN coefficients [4][Cout] of the never-computed h = a2 W^T from (G, s), and u = W G");
  m.def("conv1x1_apply", &conv1x1_apply, py::arg("x"), py::arg("w"), py::arg("in_coef"), py::arg("out_coef"),
        py::arg("residual"), py::arg("res_coef") = py::none(),
        "y = relu(BN(x' W^T) + residual [BN_d]) and its ReLU bits (pre-BN tensor never stored)");
  m.def("bn_gram_bwd", &bn_gram_bwd, py::arg("part"), py::arg("P"), py::arg("w"), py::arg("u"), py::arg("s"),
        py::arg("coef"), py::arg("gamma"), py::arg("M"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dw"),
        "BN3 backward from (sum dz partials, P = dz^T a2): dgamma/dbeta/dw +=, returns (B_cat bf16, bias)");
  m.def("conv1x1_dgrad_cat", &conv1x1_dgrad_cat, py::arg("dz"), py::arg("a2src"), py::arg("a2_coef"), py::arg("bcat"),
        py::arg("e"), py::arg("bn_x"), py::arg("bn_coef"),
        "[dz | a2] x bcat + e with the BN2-backward partials (concatenated-K data grad)");
  m.def("bn_bwd_coef", &bn_bwd_coef, py::arg("partials"), py::arg("M"), py::arg("gamma"), py::arg("coef"),
        py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none(),
        "BN-backward coefficients [3][C] from the dgrad-epilogue partials (no apply pass); dgamma/dbeta +=");
  m.def("conv1x1_bnin_fwd", &conv1x1_bnin_fwd, py::arg("h"), py::arg("res"), py::arg("coef"), py::arg("res_coef"),
        py::arg("w"), py::arg("x_out"), py::arg("x_bits"), py::arg("want_stats") = true, py::arg("tile_m") = 128,
        "1x1 conv over x = relu(BN(h) + res [BN_d]) computed on load; x (+ ReLU bits) stored as a by-product");
  m.def("conv1x1_bnin_dgrad", &conv1x1_bnin_dgrad, py::arg("dz"), py::arg("h"), py::arg("bcoef"), py::arg("w"),
        py::arg("dh_out"), py::arg("bn_x"), py::arg("bn_coef"),
        "1x1 data grad over dh = a*dz + b*h + c computed on load (dh stored as a by-product) + BN-backward partials");
  m.def("bn_coef", &bn_coef, py::arg("stats"), py::arg("M"), py::arg("gamma"), py::arg("beta"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("momentum"), py::arg("eps"));
  m.def("bn_apply", &bn_apply, py::arg("x"), py::arg("coef"), py::arg("residual") = py::none(),
        py::arg("residual_coef") = py::none(), py::arg("relu") = true, py::arg("want_mask") = false);
  m.def("bnrelu_maxpool_fwd", &bnrelu_maxpool_fwd, py::arg("h"), py::arg("coef"), py::arg("k"), py::arg("s"), py::arg("p"));
  m.def("set_pool_legacy", [](bool on) { dpe_set_pool_legacy(on ? 1 : 0); },
        "test hook: the stem max-pool on the reference (per-tap compare) kernel instead of the key-max one");
  m.def("stem_bwd_fused", &stem_bwd_fused, py::arg("dy"), py::arg("idx"), py::arg("h"), py::arg("xs"), py::arg("gamma"),
        py::arg("coef"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dw"),
        "stem backward without dY: BN-backward coefficients of the pooled gradient, then the stem weight grad "
        "(s2d filter layout) computing dY on the fly");
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd, py::arg("dy"), py::arg("idx"), py::arg("h"), py::arg("gamma"), py::arg("coef"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("k"), py::arg("s"), py::arg("p"));
  m.def("bn_bwd_partials", &bn_bwd_partials, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("coef"),
        py::arg("partials"), py::arg("dgamma") = py::none(), py::arg("dbeta") = py::none(), py::arg("relu_mask") = true);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("xshape"), py::arg("stride"), py::arg("pad"),
        py::arg("dil"), py::arg("residual") = py::none(), py::arg("residual_mask") = py::none());
  m.def("set_weight_epoch", [](int64_t e) { g_weight_epoch = e; }, py::arg("epoch"),
        "bf16 weight shadows changed (optimizer step / re-cast): cached flipped filters are refreshed at next use");
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("stride"), py::arg("pad"),
        py::arg("dil"), py::arg("alpha") = 1.0, py::arg("in_coef") = py::none(), py::arg("fin_stream") = 0,
        py::arg("deterministic") = false, py::arg("overwrite") = false,
        "dw (+)= alpha dW; fin_stream: a K-split hgemm's slab reduction runs on that stream (caller orders consumers); "
        "deterministic: 1x1 weight grads over a pre-BN input sum their K splits in a fixed order (no atomics); "
        "overwrite: dw = alpha dW (dw's old contents, e.g. torch.empty, are never read)");
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"),
        py::arg("momentum"), py::arg("eps"), py::arg("relu"), py::arg("residual") = py::none(), py::arg("stats") = py::none());
  m.def("bn_fwd_eval", &bn_fwd_eval, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"),
        py::arg("eps"), py::arg("relu"), py::arg("residual") = py::none());
  m.def("bn_bwd_dual", &bn_bwd_dual, py::arg("dz"), py::arg("x"), py::arg("gamma"), py::arg("coef"), py::arg("partials"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("x2"), py::arg("gamma2"), py::arg("coef2"), py::arg("dgamma2"),
        py::arg("dbeta2"), "backward of two BatchNorms fed by one dz (BN3 + downsample BN): dz read once for both");
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("gamma"), py::arg("coef"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("want_dz") = false, py::arg("y_bits") = py::none());
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("gavgpool_fwd", &gavgpool_fwd);
  m.def("gavgpool_bwd", &gavgpool_bwd);
  m.def("cross_entropy_mean", &cross_entropy_mean, py::arg("logits"), py::arg("labels"), py::arg("V"),
        py::arg("grad_bf16"), py::arg("ignore_index") = -100, py::arg("inplace") = false,
        "training CE: (out4 = [sum, correct, mean, 1/n_valid], softmax - onehot)");
  m.def("ce_grad_scale", &ce_grad_scale, py::arg("d"), py::arg("g"), py::arg("inv_n"), "d * g * inv_n (device scalars)");
  m.def("cross_entropy", &cross_entropy, py::arg("logits"), py::arg("labels"), py::arg("V"), py::arg("grad_scale"),
        py::arg("want_grad"), py::arg("grad_bf16"), py::arg("ignore_index") = -100, py::arg("inplace") = false);
  m.def("cast_bf16", &cast_bf16, py::arg("x"), py::arg("out") = py::none());
  m.def("cast_f32", &cast_f32);
  m.def("act", &act, py::arg("a"), py::arg("b") = py::none(), py::arg("op") = 0);
  m.def("dropout", &dropout);
  m.def("add", &add, py::arg("a"), py::arg("b"), py::arg("alpha") = 1.0);
  m.def("colsum", &colsum, py::arg("dy"), py::arg("db"), py::arg("accumulate") = false);
  m.def("nchw_to_s2d", &nchw_to_s2d, py::arg("x"));
  m.def("nchw_to_nhwc", &nchw_to_nhwc, py::arg("x"), py::arg("cpad") = 8);
  m.def("embedding_fwd", &embedding_fwd, py::arg("idx"), py::arg("wte"), py::arg("wpe") = py::none());
  m.def("embedding_bwd", &embedding_bwd, py::arg("idx"), py::arg("dout"), py::arg("dwte"), py::arg("dwpe") = py::none());
  m.def("optim_step", &optim_step);
  m.def("optim_chunk_size", []() { return dpe_optim_chunk_size(); });
  m.def("optim_desc_bytes", []() { return dpe_optim_desc_bytes(); });
  m.def("layernorm_bwd_residual", &layernorm_bwd_residual, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("dw"), py::arg("db"), py::arg("res_in"), py::arg("defer") = false);
  m.def("layernorm_bwd_finalize_group", &layernorm_bwd_finalize_group, py::arg("parts"), py::arg("rows"), py::arg("dws"),
        py::arg("dbs"));
  m.def("layernorm_fwd", &layernorm_fwd, py::arg("x"), py::arg("w"), py::arg("b") = py::none(), py::arg("eps") = 1e-5);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"), py::arg("rstd"),
        py::arg("dw"), py::arg("db") = py::none(), py::arg("dx_out") = py::none());
  m.def("set_pw_stream", &set_pw_stream, "streaming pointwise-conv kernel on/off (pwconv.hip)");
  m.def("cu_hog", [](int64_t nblocks, int64_t threads, int64_t lds_bytes, double us, int64_t vgprs,
                     const c10::optional<Tensor>& stop, bool sleepy, int64_t mode) {
          static Tensor sink = at::empty({1024}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
          static Tensor buf;
          const int md = mode >= 0 ? (int)mode : (sleepy ? 1 : 0);
          if (md == 2 && (!buf.defined() || buf.numel() < dpe_cu_hog_buf_floats((int)nblocks)))
            buf = at::zeros({dpe_cu_hog_buf_floats((int)nblocks)}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
          const unsigned* sp = nullptr;
          if (stop.has_value() && stop->defined()) {
            TORCH_CHECK(stop->is_cuda() && stop->scalar_type() == at::kInt && stop->numel() >= 1, "cu_hog: stop is an int32 GPU tensor");
            sp = (const unsigned*)stop->data_ptr();
          }
          CHECK_RC(dpe_cu_hog((int)nblocks, (int)threads, (int)lds_bytes, us, (int)vgprs, sp, (float*)sink.data_ptr(),
                              md, md == 2 ? (float*)buf.data_ptr() : nullptr, cur_stream()),
                   "cu_hog");
        }, py::arg("nblocks"), py::arg("threads") = 256, py::arg("lds_bytes") = 0, py::arg("us") = 1000.0,
        py::arg("vgprs") = 8, py::arg("stop") = py::none(), py::arg("sleepy") = false, py::arg("mode") = -1,
        "occupancy probe: nblocks workgroups holding a CU slot (threads, LDS, ~vgprs per lane) until stop[0] != 0 or `us` "
        "microseconds pass (current stream); mode 0 VALU-bound, 1 idle (= sleepy), 2 RCCL-like reduce-copy streaming");
  m.def("hog_stop", [](Tensor& stop, int64_t v) {
          TORCH_CHECK(stop.is_cuda() && stop.scalar_type() == at::kInt, "hog_stop: int32 GPU tensor");
          CHECK_RC(dpe_hog_stop((unsigned*)stop.data_ptr(), (unsigned)v, cur_stream()), "hog_stop");
        }, py::arg("stop"), py::arg("value") = 1, "set a cu_hog stop flag, ordered on the current stream");
  m.def("set_row_wgrad", &set_row_wgrad, "64-channel 3x3 weight grads on the row-walking kernel (rowconv.hip) on/off");
  m.def("set_rowconv", &set_rowconv, "64-channel 3x3 convs on the row-walking kernel (rowconv.hip) on/off");
  m.def("set_stem_kernel", &set_stem_kernel, "s2d stem conv on its row-walking kernel (stem.hip) on/off");
  m.def("set_wgrad_hgemm", &set_wgrad_hgemm, "1x1 conv weight grads on the persistent hgemm kernel on/off");
  m.def("set_hgemm_conv", &set_hgemm_conv,
        "3x3 forward-form convs with >= 256 output channels on the persistent GEMM (implicit im2col A) on/off");
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("H"), py::arg("scale"), py::arg("causal") = true);
  m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"), py::arg("H"),
        py::arg("scale"), py::arg("causal") = true);
  m.def("set_gemm_backend", [](int64_t mode) {
          TORCH_CHECK(mode == 1, "only the native MFMA GEMM backend exists (mode 1); the vendor-library arm was removed");
        }, "kept for API compatibility: 1 = native kernels (the only backend)");
  m.def("set_wgrad_wide", [](int64_t v) { g_wgrad_wide = (int)v; },
        "64x256 tile for Cout = 64 weight grads: 0 off, 1 when C <= 16 (default), 2 always");
  m.def("set_phase_group", [](bool on) { g_phase_group = on; },
        "strided data grads: all parity sub-GEMMs in one grid, or one launch per parity (default)");
  m.def("set_conv_tile", [](int64_t mode) { g_dma_tile = (int)mode; },
        "LDS-DMA conv tile: 0 auto, 1 128-tile, 2 256x128, 3 256x256 (8 waves)");
  m.def("pick_gemm_cfg", [](int64_t M, int64_t N, int64_t K, bool split) {
    auto c = pick_cfg(M, N, K, split);
    return std::make_tuple(c.bm, c.bn, c.splits, c.k_split);
  });
}
