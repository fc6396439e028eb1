// Launch planning for the persistent dense GEMM (csrc/kernels/hgemm.hip).
//
// The plan is a pure function of (M, N, K, operand layouts, device CU count):
// every rank of a DDP job computes the same kernel, tile and K split for the
// same GEMM without timing anything (no per-rank autotune, no host sync inside
// a training step).  A small analytic model picks, per shape, the tile
// (256x256 / 128x256 / 256x128 / 128x128) and the K split:
//   time = rounds * (unit FLOPs / per-block rate) + fixed prologue/epilogue
//          + (split > 1) slab traffic + the finalize launch,
// rounds = ceil(units / (CUs * blocks per CU)).  The per-tile rates are the
// measured single-shape throughputs of each tile (profiles/hgemm_*), relative
// to the 256x256 tile.
#include <torch/extension.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "../kernels/hgemm.h"
#include "../kernels/igemm.h"
#include "gemm_plan.h"

using at::Tensor;

extern "C" int dpe_cu_reserve();  // comm.cpp: slots to leave to in-flight collectives

namespace dpe_gemm {

namespace {
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

struct TileCfg { int cfg, bm, bn, bpc; double eff, eff_alone; };
// eff: per-CU throughput relative to the 256x256 tile with the CU fully occupied (bpc blocks);
// eff_alone: the same for ONE block of a 2-per-CU tile holding a CU by itself (a launch with no
// more units than CUs): 128x128 x 768 units ran in ~10 us alone vs 16.2 us two to a CU
// (scripts/bench_gemm_parts.py two-launch tails, GPT-2 shapes)
constexpr TileCfg kTiles[] = {
    {dpe::HC_256x256, 256, 256, 1, 1.00, 1.00},
    {dpe::HC_128x256, 128, 256, 1, 0.70, 0.70},
    {dpe::HC_256x128, 256, 128, 1, 0.70, 0.70},
    {dpe::HC_128x128, 128, 128, 2, 0.75, 0.65},
};
// per-CU main-loop rate of the 256x256 tile by operand layout (random bf16, 4096^3 / 8192^3 on 256
// CUs: NT 1318 / 1196, NN 1262 / 1274, TN 1187 / 1222 TF, scripts/bench_hgemm_layouts.py; before the
// LDS-DMA moved into inline asm the transposed-read layouts ran at NN 1047 / TN 885)
double layout_rate(int ak, int bk) { return ak && bk ? 5.2e12 : (ak ? 5.0e12 : 4.7e12); }
constexpr double kEpi = 5.0e-11;  // s per output byte per CU: the store tail is issue-bound (~20 GB/s per CU)
constexpr double kFix = 2.0e-6;   // first prologue + launch
// slab write + finalize read bandwidth (DPE_HGEMM_SLAB_GBPS: A/B)
const double kBw = [] { const char* e = getenv("DPE_HGEMM_SLAB_GBPS"); return e ? atof(e) * 1e9 : 4.0e12; }();
constexpr double kLaunch = 3.0e-6;

int g_force_cfg = -1, g_force_splits = -1;
// (off by default: with it the budgeted planner traded whole-K plans for K splits whose slab traffic
// cost more than the balance bought -- GPT-2 data grads x1.7 -> x3.0, profiles/cu_hog_probe_r4.txt)
bool g_budget_tail = [] { const char* e = getenv("DPE_HGEMM_BUDGET_TAIL"); return e && e[0] == '1'; }();  // A/B
bool g_dynamic = [] { const char* e = getenv("DPE_HGEMM_DYNAMIC"); return !(e && e[0] == '0'); }();  // A/B

// Dynamic-schedule state of the persistent GEMM (hgemm.hip: 8 per-XCD claim counters + exit
// counters), one zeroed buffer per (device, stream): launches on one stream are ordered, and the last
// block of each launch resets the counters, so the buffer is reused without a per-call memset.
// Launches on different streams may overlap and get different buffers.  A stream first seen while
// it is being captured into a graph gets none (its zeroing memset would only run at replay): such a
// launch uses the static schedule.
unsigned* sched_buffer_impl(hipStream_t st) {
  if (!g_dynamic) return nullptr;
  static std::mutex mu;
  static std::unordered_map<uint64_t, unsigned*> bufs;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t key = (uint64_t)(uintptr_t)st * 64 + (uint64_t)dev;
  std::lock_guard<std::mutex> lk(mu);
  auto it = bufs.find(key);
  if (it != bufs.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  unsigned* b = nullptr;
  TORCH_CHECK(hipMalloc(&b, dpe::HGEMM_SCHED_BYTES) == hipSuccess &&
                  hipMemsetAsync(b, 0, dpe::HGEMM_SCHED_BYTES, st) == hipSuccess,
              "hgemm: schedule buffer allocation failed");
  bufs.emplace(key, b);
  return b;
}

// Stream-K arrival counters (hgemm.h sk_cnt): one zeroed buffer of HGEMM_SK_MAX_TILES words per (device,
// stream), kept zero by each tile's last arriver; nullptr while the stream is being captured.
unsigned* sk_counters(hipStream_t st) {
  static std::mutex mu;
  static std::unordered_map<uint64_t, unsigned*> bufs;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t key = (uint64_t)(uintptr_t)st * 64 + (uint64_t)dev;
  std::lock_guard<std::mutex> lk(mu);
  auto it = bufs.find(key);
  if (it != bufs.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  unsigned* b = nullptr;
  const size_t bytes = sizeof(unsigned) * dpe::HGEMM_SK_MAX_TILES;
  TORCH_CHECK(hipMalloc(&b, bytes) == hipSuccess && hipMemsetAsync(b, 0, bytes, st) == hipSuccess,
              "hgemm: stream-K counter allocation failed");
  bufs.emplace(key, b);
  return b;
}
}  // namespace

// Stream-K for the implicit-im2col convolutions (DPE_HGEMM_SK=1 / set_hgemm_sk(true): on; default off): for
// plans whose whole-K tiles leave a partly empty last round -- ResNet-50's layer-3 3x3 convs at batch 512
// are 392 tiles of 256x256 on 256 CUs, 1.53 rounds run as 2 (scripts/bench_wave_quant.py).  Measured:
// that conv 142 -> 134 us alone, the ResNet-50 step -0.06 ms on average over 9 alternating pairs -- a partly
// filled round runs faster per CU, so the idle CUs cost less than their share.  Off by default: its owners
// wait on blocks of their own grid, which an RCCL kernel holding CUs can delay by a whole all-reduce
// (docs/perf_notes.md).
int g_sk = [] { const char* e = getenv("DPE_HGEMM_SK"); return (e && e[0] == '1') ? 1 : 0; }();

unsigned* sched_buffer(hipStream_t st) { return sched_buffer_impl(st); }

int num_cus() {
  static const int n = [] {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&pr, dev) != hipSuccess) {
      (void)hipGetLastError();
      return 256;  // no device (CPU planning / tests): MI355X
    }
    return pr.multiProcessorCount > 0 ? pr.multiProcessorCount : 256;
  }();
  return n;
}

bool layout_ok(int cfg, int ak, int bk) {
  if (ak && bk) return true;
  if (ak && !bk) return cfg == dpe::HC_256x256 || cfg == dpe::HC_128x256;
  if (!ak && !bk) return cfg == dpe::HC_256x256;
  return false;
}

Plan plan(int64_t M, int64_t N, int64_t K, int ak, int bk, bool allow_split, int out_bytes, int force_cfg,
          int force_splits) {
  const int ncu = num_cus();
  const int reserve = dpe_cu_reserve();
  const int64_t ktiles = K / 64;
  Plan best{-1, 1, (int)K, 0, 1e30};
  if (force_cfg < 0) force_cfg = g_force_cfg;
  if (force_splits < 0) force_splits = g_force_splits;
  for (const TileCfg& c : kTiles) {
    if (force_cfg >= 0 && c.cfg != force_cfg) continue;
    if (!layout_ok(c.cfg, ak, bk)) continue;
    const int64_t tiles = ((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    // resident slots, minus those left to RCCL channel blocks while a bucket all-reduce overlaps
    // (comm.cpp CU budget): a full-residency static grid would push blocks into a second wave
    const int64_t slots = std::max<int64_t>(c.bpc, (int64_t)ncu * c.bpc - reserve);
    // up to 8 K splits in general; more (<= 128) when the tiles alone leave most CUs idle (a 1x1 conv
    // weight grad: a few output tiles over 25K-400K pixels), so the split fills one round of slots
    // (cap swept 8-128: neutral, profiles/hgemm_split_cap_ab_r2.txt)
    const int max_split =
        allow_split ? (int)std::max<int64_t>(8, std::min<int64_t>(128, slots / std::max<int64_t>(1, tiles))) : 1;
    for (int s = 1; s <= max_split; ++s) {
      if (force_splits > 0 && s != force_splits) continue;
      const int64_t kt = (ktiles + s - 1) / s;
      const int64_t se = (ktiles + kt - 1) / kt;  // effective splits (no empty split)
      if (se != s) continue;
      if (s > 1 && (kt < 4 || (double)s * M * N * 4 > 2.0e9)) continue;
      const int64_t units = tiles * s;
      const int64_t rounds = (units + slots - 1) / slots;
      // blocks sharing a CU (bpc) each get 1/bpc of its rate; with no more units than CUs every
      // block has a CU to itself
      const bool alone = c.bpc > 1 && units <= (int64_t)ncu - (reserve + c.bpc - 1) / c.bpc;
      const double rate_blk = alone ? layout_rate(ak, bk) * c.eff_alone : layout_rate(ak, bk) * c.eff / c.bpc;
      const double t_unit = 2.0 * c.bm * c.bn * kt * 64 / rate_blk + kEpi * c.bm * c.bn * (s > 1 ? 4 : out_bytes) *
                                                                          (alone ? 1 : c.bpc);
      double t = rounds * t_unit + kFix;
      // CU budget in force (collectives in flight): a foreign workgroup fits beside our blocks and slows
      // the CU it shares, so the launch ends about one unit after its even share (the dynamic claims
      // balance everything but the last unit): favour more, shorter units.  Unchanged without a budget.
      // (whole-K plans only: with K splits the shorter units would buy balance with slab traffic)
      if (reserve > 0 && g_budget_tail && s == 1) t += t_unit;
      if (s > 1) t += ((double)s * M * N * 4 * 2 + (double)M * N * out_bytes) / kBw + kLaunch;
      if (t < best.est_s * 0.995) best = Plan{c.cfg, s, (int)(kt * 64), (int)std::min<int64_t>(units, slots), t};
    }
  }
  return best;
}

// Tile rows per grouped-order band.  An XCD runs grid/8 consecutive units at a time; with 4-row
// bands those 32 (1 block/CU) units form a 4 x 8 tile block sharing A rows and B columns in the
// XCD's L2.  Interleaved A/B (scripts/ab_hgemm.py, profiles/hgemm_group_ab_r2.jsonl in git history), TF/s vs
// row-major: 8192^3 NT 1340 -> 1478, NN 1054 -> 1201, TN 989 -> 1132; GPT-2 LM head fwd 973 ->
// 1055; 4096^3 and the small GPT-2 GEMMs neutral; 8-row bands equal on squares, worse on the LM
// head; 16-row bands worse everywhere.
int group_rows(const Plan& pl) { return pl.grid >= 64 ? 4 : 1; }

// Two-launch plans.  A GEMM whose tiles do not fill whole rounds of slots (GPT-2's QKV 8192x2304: 288
// tiles of 256^2 on 256 CUs) spends its last round mostly idle.  Splitting the output into a main part
// that fills whole rounds with one tile and a tail covered by a smaller tile (its own round) costs one
// extra launch and removes most of that idle round.  The cut is along N (whole tile columns of the
// main tile) or M (whole tile rows); both parts are planned by plan() and the split is taken only if
// the modelled time improves by > 2 % (measured two-launch wins on the GPT-2 shapes, 10-19 %:
// scripts/bench_gemm_parts.py).  Pure function of the shape, like plan().
Plan2 plan2(int64_t M, int64_t N, int64_t K, int ak, int bk, bool allow_split, int out_bytes) {
  Plan2 best;
  best.main = plan(M, N, K, ak, bk, allow_split, out_bytes);
  best.est_s = best.main.est_s;
  static const bool on = [] { const char* e = getenv("DPE_HGEMM_PLAN2"); return !(e && e[0] == '0'); }();  // A/B
  if (!on || best.main.cfg < 0 || g_force_cfg >= 0 || g_force_splits >= 0) return best;
  const int ncu = num_cus();
  const int reserve = dpe_cu_reserve();
  for (const TileCfg& c : kTiles) {
    if (!layout_ok(c.cfg, ak, bk)) continue;
    const int64_t slots = std::max<int64_t>(c.bpc, (int64_t)ncu * c.bpc - reserve);
    const int64_t tm = (M + c.bm - 1) / c.bm, tn = (N + c.bn - 1) / c.bn;
    for (int axis = 0; axis < 2; ++axis) {  // 0: cut along N (main = leading columns), 1: along M
      const int64_t lines = axis == 0 ? tn : tm, per = axis == 0 ? tm : tn;  // tiles per cut line
      const int64_t rounds = lines * per / slots;
      if (rounds < 1) continue;
      const int64_t keep = rounds * slots / per;  // whole lines that fit in `rounds` full rounds
      const int64_t at = keep * (axis == 0 ? c.bn : c.bm);
      const int64_t rest = (axis == 0 ? N : M) - at;
      if (keep < 1 || rest < 64) continue;
      const Plan pm = axis == 0 ? plan(M, at, K, ak, bk, false, out_bytes, c.cfg, 1) : plan(at, N, K, ak, bk, false, out_bytes, c.cfg, 1);
      const Plan pt = axis == 0 ? plan(M, rest, K, ak, bk, allow_split, out_bytes) : plan(rest, N, K, ak, bk, allow_split, out_bytes);
      if (pm.cfg < 0 || pt.cfg < 0) continue;
      const double t = pm.est_s + pt.est_s + kLaunch;
      if (t < best.est_s * 0.98 && t < best.main.est_s * 0.98) {
        best.main = pm;
        best.tail = pt;
        best.axis = axis;
        best.at = (int)at;
        best.est_s = t;
      }
    }
  }
  return best;
}

namespace {
// Stream-K grid for this launch (0: whole-K tiles as planned): conv GEMMs with a 1-block-per-CU tile whose
// tile count leaves >= 10 % of the last round idle, between one and three rounds of tiles, and enough
// K-steps per block (>= 8 of 64) that the cut costs little.  (A single partial round is left alone: with
// fewer CUs busy each runs faster -- layer 4's 196 tiles took the same time whole-K and stream-K.)
int sk_grid(const dpe::HgemmArgs& a, const Plan& pl, int epi) {
  if (!g_sk || a.conv != 1 || epi != dpe::HE_BF16 || pl.splits != 1 || pl.cfg < 0 || pl.cfg == dpe::HC_128x128) return 0;
  const int bm = pl.cfg == dpe::HC_128x256 ? 128 : 256, bn = pl.cfg == dpe::HC_256x128 ? 128 : 256;
  const int64_t tiles = ((int64_t)(a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  const int64_t G = std::max(8, num_cus() - dpe_cu_reserve());
  if (tiles >= dpe::HGEMM_SK_MAX_TILES || tiles <= G || tiles >= 3 * G || tiles * (a.K / 64) < 8 * G) return 0;
  const double r = (double)tiles / (double)G;
  if (std::ceil(r) / r < 1.10) return 0;
  return (int)G;
}

// one planned launch (+ its slab finalize when K-split)
void launch_planned(dpe::HgemmArgs a, const Plan& pl, int ak, int bk, int epi, hipStream_t fin_stream) {
  a.splits = pl.splits;
  a.kps = pl.kps;
  if (a.group_m == 0) a.group_m = group_rows(pl);
  a.sched = sched_buffer_impl(cur_stream());
  Tensor ws;
  if (pl.splits > 1) {
    // one allocation: [splits][M][N] partial slabs (+ [splits][M] bias-gradient partials)
    const int64_t slab = (int64_t)pl.splits * a.M * a.N;
    ws = at::empty({slab + (a.dbias ? (int64_t)pl.splits * a.M : 0)}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
    a.ws = (float*)ws.data_ptr();
    if (a.dbias) a.ws_bias = a.ws + slab;
    const int rc = dpe_hgemm_launch(&a, pl.cfg, ak, bk, dpe::HE_SLAB, pl.grid, cur_stream());
    hipError_t e = hipGetLastError();
    TORCH_CHECK(rc == 0 && e == hipSuccess, "hgemm (split) launch failed rc=", rc, " ", hipGetErrorString(e));
    hipStream_t fs = cur_stream();
    if (fin_stream && fin_stream != fs) {
      // slabs -> side stream: event order, and the workspace stays allocated until the finalize ran
      static thread_local hipEvent_t ev = [] {
        hipEvent_t x = nullptr;
        (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
        return x;
      }();
      TORCH_CHECK(hipEventRecord(ev, fs) == hipSuccess && hipStreamWaitEvent(fin_stream, ev, 0) == hipSuccess,
                  "hgemm: finalize stream ordering failed");
      int dev = 0;
      (void)hipGetDevice(&dev);
      c10::hip::HIPCachingAllocator::recordStream(ws.storage().data_ptr(),
                                                  c10::hip::getStreamFromExternal(fin_stream, (c10::DeviceIndex)dev));
      fs = fin_stream;
    }
    // DPE_AB_SKIP_FINALIZE=1: timing diagnostic only (what the slab reductions cost the step; gradients WRONG)
    static const bool skip = [] {
      const char* e = getenv("DPE_AB_SKIP_FINALIZE");
      const bool on = e && e[0] == '1';
      if (on) fprintf(stderr, "[dpe] DPE_AB_SKIP_FINALIZE=1: K-split weight gradients are NOT reduced (timing only)\n");
      return on;
    }();
    if (skip) return;
    const int rf = dpe_hgemm_finalize(&a, epi, fs);
    e = hipGetLastError();
    TORCH_CHECK(rf == 0 && e == hipSuccess, "hgemm finalize failed rc=", rf, " ", hipGetErrorString(e));
    return;
  }
  int grid = pl.grid;
  Tensor skw;
  if (const int G = sk_grid(a, pl, epi)) {
    if (unsigned* cnt = sk_counters(cur_stream())) {
      const int64_t tile_f32 = (pl.cfg == dpe::HC_256x256 ? 256 * 256 : 128 * 256);
      skw = at::empty({2 * (int64_t)G * tile_f32}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
      a.sk = 1;
      a.sk_ws = (float*)skw.data_ptr();
      a.sk_cnt = cnt;
      a.sched = nullptr;
      grid = G;
    }
  }
  const int rc = dpe_hgemm_launch(&a, pl.cfg, ak, bk, epi, grid, cur_stream());
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(rc == 0 && e == hipSuccess, "hgemm launch failed rc=", rc, " ", hipGetErrorString(e));
}

// the sub-GEMM of output rows [m1, M) or columns [n1, N): operand / output / epilogue pointers moved
dpe::HgemmArgs part_args(const dpe::HgemmArgs& a, int ak, int bk, int out_bytes, int axis, int at) {
  dpe::HgemmArgs b = a;
  const int64_t eo = axis == 0 ? (int64_t)at : (int64_t)at * a.ldc;  // output element offset
  b.C = (char*)a.C + eo * out_bytes;
  if (a.residual_f32) b.residual_f32 = a.residual_f32 + eo;
  if (a.aux_in) b.aux_in = a.aux_in + eo;
  if (a.aux_out) b.aux_out = a.aux_out + eo;
  if (axis == 0) {  // columns [at, N)
    b.N = a.N - at;
    b.B = bk ? a.B + (int64_t)at * a.ldb : a.B + at;
    if (a.bias) b.bias = a.bias + at;
    if (a.b_dim > 0) b.b_dim = a.b_dim - at;
    b.dbias = nullptr;  // the row sums come from the first tile column, which is in the main part
  } else {          // rows [at, M)
    b.M = a.M - at;
    b.A = ak ? a.A + (int64_t)at * a.lda : a.A + at;
    if (a.a_dim > 0) b.a_dim = a.a_dim - at;
    if (a.dbias) b.dbias = a.dbias + at;
  }
  return b;
}
}  // namespace

int run(dpe::HgemmArgs& a, int ak, int bk, int epi, bool allow_split, int out_bytes, hipStream_t fin_stream) {
  TORCH_CHECK(a.K % 64 == 0 && a.K > 0, "hgemm: K must be a positive multiple of 64 (got ", a.K, ")");
  const Plan2 p2 = plan2(a.M, a.N, a.K, ak, bk, allow_split, out_bytes);
  TORCH_CHECK(p2.main.cfg >= 0, "hgemm: no tile configuration for M=", a.M, " N=", a.N, " K=", a.K, " layout ", ak, bk);
  if (p2.axis < 0) {
    launch_planned(a, p2.main, ak, bk, epi, fin_stream);
    return p2.main.cfg;
  }
  const int ob = (epi == dpe::HE_BF16) ? 2 : 4;
  dpe::HgemmArgs m = a;
  if (p2.axis == 0) {
    m.N = p2.at;
    if (m.b_dim > 0) m.b_dim = p2.at;
  } else {
    m.M = p2.at;
    if (m.a_dim > 0) m.a_dim = p2.at;
  }
  launch_planned(m, p2.main, ak, bk, epi, fin_stream);
  launch_planned(part_args(a, ak, bk, ob, p2.axis, p2.at), p2.tail, ak, bk, epi, fin_stream);
  return p2.main.cfg;
}

Plan plan_bnb(int64_t M, int64_t N, int64_t K, int ak, int bk, int* partial_cols) {
  const Plan pl = plan(M, N, K, ak, bk, false, 2);
  int bm = 0, wr = 0;
  for (const TileCfg& c : kTiles)
    if (c.cfg == pl.cfg) bm = c.bm;
  wr = pl.cfg == dpe::HC_256x128 ? 4 : 2;  // wave rows of the configuration (hgemm.h HCfg)
  *partial_cols = pl.cfg >= 0 ? (int)((M + bm - 1) / bm) * wr : 0;
  return pl;
}

void run_conv_wgrad(dpe::HgemmArgs& a, hipStream_t fin_stream) {
  // one launch (no two-launch split: a column cut would shift the implicit im2col's tap / channel origin)
  const Plan pl = plan(a.M, a.N, a.K, 0, 0, true, 4);
  TORCH_CHECK(pl.cfg == dpe::HC_256x256, "hgemm conv weight grad: no plan");
  launch_planned(a, pl, 0, 0, dpe::HE_ACC_F32, fin_stream);
}

void launch_plain(dpe::HgemmArgs& a, const Plan& pl, int ak, int bk) {
  TORCH_CHECK(pl.cfg >= 0 && pl.splits == 1, "hgemm: bad single-launch plan");
  launch_planned(a, pl, ak, bk, dpe::HE_BF16, nullptr);
}

void run_bnb(dpe::HgemmArgs& a, const Plan& pl, int ak, int bk) {
  if (a.act != dpe::HACT_BNF) a.act = dpe::HACT_BNB;
  TORCH_CHECK(pl.cfg >= 0 && pl.splits == 1 && a.col_stats && (a.act == dpe::HACT_BNF || (a.st_x && a.st_coef)),
              "hgemm BN-statistics epilogue: bad plan / arguments");
  launch_planned(a, pl, ak, bk, dpe::HE_BF16, nullptr);
}

}  // namespace dpe_gemm

extern "C" int dpe_gemm_f32(const float* A, const float* B, float* C, int64_t sam, int64_t sak, int64_t sbk, int64_t sbn,
                            int64_t ldc, int M, int N, int K, const float* bias, float alpha, int relu, float drop_p,
                            uint64_t seed, uint64_t offset, const float* mask_src, float mask_scale, int accumulate,
                            hipStream_t st);

namespace dpe_gemm {
namespace {

// ------------------------------------------------ fp32 Linear (exact-f32 MFMA, gemm_f32.hip)
void check_f32(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), what,
              " must be a contiguous fp32 GPU tensor");
}
void launch_f32(int rc) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(rc == 0 && e == hipSuccess, "gemm_f32 launch failed rc=", rc, " ", hipGetErrorString(e));
}

// y[M,N] = dropout(relu(x[M,K] w[N,K]^T + b))  (relu / dropout optional; dropout mask = dpe_dropout's)
Tensor linear32_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, bool relu, double drop_p,
                    int64_t seed, int64_t offset) {
  check_f32(x, "x"); check_f32(w, "w");
  const int64_t K = x.size(-1), N = w.size(0), M = x.numel() / K;
  TORCH_CHECK(w.size(1) == K, "linear32_fwd: weight shape mismatch");
  const float* b = nullptr;
  if (bias && bias->defined()) { check_f32(*bias, "bias"); b = (const float*)bias->data_ptr(); }
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y = at::empty(sizes, x.options());
  launch_f32(dpe_gemm_f32((const float*)x.data_ptr(), (const float*)w.data_ptr(), (float*)y.data_ptr(), K, 1, 1, K, N,
                          (int)M, (int)N, (int)K, b, 1.f, relu, (float)drop_p, (uint64_t)seed, (uint64_t)offset, nullptr,
                          1.f, 0, cur_stream()));
  return y;
}

// dx[M,K] = (dy[M,N] w[N,K]) * (mask_src > 0) * mask_scale   (mask_src: the previous layer's output)
Tensor linear32_dgrad(const Tensor& dy, const Tensor& w, const c10::optional<Tensor>& mask_src, double mask_scale) {
  check_f32(dy, "dy"); check_f32(w, "w");
  const int64_t N = w.size(0), K = w.size(1), M = dy.numel() / N;
  TORCH_CHECK(dy.size(-1) == N, "linear32_dgrad: shape mismatch");
  const float* ms = nullptr;
  if (mask_src && mask_src->defined()) {
    check_f32(*mask_src, "mask_src");
    TORCH_CHECK(mask_src->numel() == M * K, "linear32_dgrad: mask_src shape mismatch");
    ms = (const float*)mask_src->data_ptr();
  }
  auto sizes = dy.sizes().vec();
  sizes.back() = K;
  Tensor dx = at::empty(sizes, dy.options());
  launch_f32(dpe_gemm_f32((const float*)dy.data_ptr(), (const float*)w.data_ptr(), (float*)dx.data_ptr(), N, 1, K, 1, K,
                          (int)M, (int)K, (int)N, nullptr, 1.f, 0, 0.f, 0, 0, ms, (float)mask_scale, 0, cur_stream()));
  return dx;
}

// dw[N,K] += alpha * dy[M,N]^T x[M,K]
void linear32_wgrad(const Tensor& dy, const Tensor& x, Tensor& dw, double alpha) {
  check_f32(dy, "dy"); check_f32(x, "x"); check_f32(dw, "dw");
  const int64_t N = dw.size(0), K = dw.size(1), M = dy.numel() / N;
  TORCH_CHECK(dy.size(-1) == N && x.size(-1) == K && x.numel() / K == M, "linear32_wgrad: shape mismatch");
  launch_f32(dpe_gemm_f32((const float*)dy.data_ptr(), (const float*)x.data_ptr(), (float*)dw.data_ptr(), 1, N, K, 1, K,
                          (int)N, (int)K, (int)M, nullptr, (float)alpha, 0, 0.f, 0, 0, nullptr, 1.f, 1, cur_stream()));
}

// Raw entry for tests and benchmarks: C (M x N, ldc) from A / B with explicit layouts.
Tensor hgemm_raw(const Tensor& A, const Tensor& B, Tensor C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                 int64_t ldc, bool ak, bool bk, int64_t epi, int64_t act, const c10::optional<Tensor>& bias,
                 const c10::optional<Tensor>& residual, const c10::optional<Tensor>& aux_in,
                 const c10::optional<Tensor>& aux_out, double alpha, int64_t cfg, int64_t splits, int64_t group_m,
                 const c10::optional<Tensor>& dbias) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "hgemm: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "hgemm: bf16 operands");
  TORCH_CHECK(C.scalar_type() == (epi == dpe::HE_BF16 ? at::kBFloat16 : at::kFloat), "hgemm: output dtype");
  TORCH_CHECK(A.numel() >= (ak ? M * lda : K * lda) - (ak ? lda - K : lda - M), "hgemm: A too small");
  TORCH_CHECK(B.numel() >= (bk ? N * ldb : K * ldb) - (bk ? ldb - K : ldb - N), "hgemm: B too small");
  TORCH_CHECK(C.numel() >= M * ldc - (ldc - N), "hgemm: C too small");
  dpe::HgemmArgs a;
  memset(&a, 0, sizeof(a));
  a.A = (const uint16_t*)A.data_ptr(); a.B = (const uint16_t*)B.data_ptr(); a.C = C.data_ptr();
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.alpha = (float)alpha; a.act = (int)act;
  if (bias && bias->defined()) { TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= N); a.bias = (const float*)bias->data_ptr(); }
  if (residual && residual->defined()) { TORCH_CHECK(residual->scalar_type() == at::kFloat); a.residual_f32 = (const float*)residual->data_ptr(); }
  if (aux_in && aux_in->defined()) { TORCH_CHECK(aux_in->scalar_type() == at::kBFloat16); a.aux_in = (const uint16_t*)aux_in->data_ptr(); }
  if (aux_out && aux_out->defined()) { TORCH_CHECK(aux_out->scalar_type() == at::kBFloat16); a.aux_out = (uint16_t*)aux_out->data_ptr(); }
  TORCH_CHECK(act != dpe::HACT_GELU_BWD || a.aux_in, "hgemm: gelu backward needs aux_in");
  if (dbias && dbias->defined()) {
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == at::kFloat && dbias->is_contiguous() && dbias->numel() >= M,
                "hgemm: dbias is a contiguous fp32 [M] GPU tensor");
    TORCH_CHECK(!ak && !bk, "hgemm: dbias (fused bias gradient) needs the TN layout");
    a.dbias = (float*)dbias->data_ptr();
  }
  const int out_bytes = epi == dpe::HE_BF16 ? 2 : 4;
  const Plan pl = plan(M, N, K, ak, bk, splits != 1, out_bytes, (int)cfg, (int)splits);
  TORCH_CHECK(pl.cfg >= 0, "hgemm: no configuration (cfg=", cfg, " splits=", splits, ")");
  a.splits = pl.splits;
  a.kps = pl.kps;
  a.group_m = group_m != 0 ? (int)group_m : group_rows(pl);
  a.sched = sched_buffer_impl(cur_stream());
  Tensor ws;
  if (pl.splits > 1) {
    const int64_t slab = (int64_t)pl.splits * M * N;
    ws = at::empty({slab + (a.dbias ? (int64_t)pl.splits * M : 0)}, A.options().dtype(at::kFloat));
    a.ws = (float*)ws.data_ptr();
    if (a.dbias) a.ws_bias = a.ws + slab;
    int rc = dpe_hgemm_launch(&a, pl.cfg, ak, bk, dpe::HE_SLAB, pl.grid, cur_stream());
    TORCH_CHECK(rc == 0 && hipGetLastError() == hipSuccess, "hgemm split launch rc=", rc);
    rc = dpe_hgemm_finalize(&a, (int)epi, cur_stream());
    TORCH_CHECK(rc == 0 && hipGetLastError() == hipSuccess, "hgemm finalize rc=", rc);
  } else {
    const int rc = dpe_hgemm_launch(&a, pl.cfg, ak, bk, (int)epi, pl.grid, cur_stream());
    TORCH_CHECK(rc == 0 && hipGetLastError() == hipSuccess, "hgemm launch rc=", rc);
  }
  return C;
}

// Grouped TN weight gradients (hgemm.hip HE_GROUP): dw_g (+)= dy_g^T x_g and db_g += colsum(dy_g) for up to
// HGEMM_MAX_GROUP problems sharing the token count K, in ONE persistent launch of whole-K 256x256 tiles.
// A transformer layer's weight-gradient GEMMs have few output tiles (GPT-2-small: 27 + 9 + 36 + 36 per
// layer at d = 768) over K = B*T = 8192 tokens: alone, each needs an 8-9-way K split to fill the chip,
// whose fp32 partial slabs (as many bytes as the GEMM's whole operand traffic) and finalize launch
// dominate.  Two layers' problems together are 216 tiles, one round on 256 CUs with no split.
void linear_wgrad_group(const std::vector<Tensor>& dys, const std::vector<Tensor>& xs, const std::vector<Tensor>& dws,
                        const std::vector<Tensor>& dbs, const std::vector<bool>& overwrite) {
  const size_t n = dys.size();
  TORCH_CHECK(n >= 1 && n <= (size_t)dpe::HGEMM_MAX_GROUP && xs.size() == n && dws.size() == n && dbs.size() == n &&
                  overwrite.size() == n, "linear_wgrad_group: 1..", dpe::HGEMM_MAX_GROUP, " problems, equal list lengths");
  dpe::HgemmArgs a;
  memset(&a, 0, sizeof(a));
  a.alpha = 1.f;
  a.splits = 1;
  a.ngroup = (int)n;
  int64_t K = -1;
  int tiles = 0;
  for (size_t g = 0; g < n; ++g) {
    const Tensor &dy = dys[g], &x = xs[g], &dw = dws[g], &db = dbs[g];
    TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dw.is_cuda(), "linear_wgrad_group: GPU tensors");
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && dy.is_contiguous() && x.is_contiguous(),
                "linear_wgrad_group: dy / x must be contiguous bf16");
    TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.dim() == 2, "linear_wgrad_group: dw contiguous fp32 [out, in]");
    const int64_t N = dw.size(0), Kin = dw.size(1), ldy = dy.size(-1);
    TORCH_CHECK(ldy >= N && ldy % 8 == 0 && N % 8 == 0 && Kin % 8 == 0 && x.size(-1) == Kin, "linear_wgrad_group: shapes");
    const int64_t T = dy.numel() / ldy;
    TORCH_CHECK(x.numel() / Kin == T && T % 64 == 0, "linear_wgrad_group: token counts (multiple of 64)");
    TORCH_CHECK(K < 0 || K == T, "linear_wgrad_group: every problem must have the same token count");
    K = T;
    dpe::HgemmProblem& q = a.grp[g];
    q.A = (const uint16_t*)dy.data_ptr();
    q.B = (const uint16_t*)x.data_ptr();
    q.C = (float*)dw.data_ptr();
    q.M = (int)N; q.N = (int)Kin; q.a_dim = (int)N;
    q.lda = ldy; q.ldb = Kin; q.ldc = Kin;
    q.overwrite = overwrite[g] ? 1 : 0;
    if (db.defined() && db.numel() > 0) {
      TORCH_CHECK(db.is_cuda() && db.scalar_type() == at::kFloat && db.is_contiguous() && db.numel() == N,
                  "linear_wgrad_group: db contiguous fp32 [out]");
      q.dbias = (float*)db.data_ptr();
    }
    tiles += (int)(((N + 255) / 256) * ((Kin + 255) / 256));
    q.tile_end = tiles;
  }
  a.K = (int)K;
  a.kps = (int)K;
  a.group_m = 4;
  const int slots = std::max(1, num_cus() - dpe_cu_reserve());
  a.sched = sched_buffer_impl(cur_stream());
  const int rc = dpe_hgemm_group_launch(&a, std::min(tiles, slots), cur_stream());
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(rc == 0 && e == hipSuccess, "hgemm group launch failed rc=", rc, " ", hipGetErrorString(e));
}

}  // namespace

void register_gemm(pybind11::module& m) {
  m.attr("HGEMM_MAX_GROUP") = dpe::HGEMM_MAX_GROUP;
  m.def("num_cus", &num_cus, "compute units of the current device (256 on MI355X; 256 without a device)");
  m.def("linear_wgrad_group", &linear_wgrad_group, pybind11::arg("dys"), pybind11::arg("xs"), pybind11::arg("dws"),
        pybind11::arg("dbs"), pybind11::arg("overwrite"),
        "grouped TN weight grads in one launch: dws[g] (+)= dys[g]^T xs[g], dbs[g] += colsum(dys[g]) "
        "(dbs[g] empty: none; overwrite[g]: the gradient's first writer)");
  namespace py = pybind11;
  m.def("hgemm", &hgemm_raw, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("a_k"), py::arg("b_k"), py::arg("epi") = 0,
        py::arg("act") = 0, py::arg("bias") = py::none(), py::arg("residual") = py::none(), py::arg("aux_in") = py::none(),
        py::arg("aux_out") = py::none(), py::arg("alpha") = 1.0, py::arg("cfg") = -1, py::arg("splits") = -1,
        py::arg("group_m") = 0, py::arg("dbias") = py::none(),
        "persistent MFMA GEMM with explicit layouts (cfg / splits -1: planner's choice; group_m 0: planner's, <0: row-major)");
  m.def("hgemm_plan", [](int64_t M, int64_t N, int64_t K, bool ak, bool bk, bool allow_split, int64_t out_bytes) {
          const Plan p = plan(M, N, K, ak, bk, allow_split, (int)out_bytes);
          return std::make_tuple(p.cfg, p.splits, p.kps, p.grid, p.est_s * 1e6);
        }, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("a_k"), py::arg("b_k"), py::arg("allow_split") = true,
        py::arg("out_bytes") = 2, "the planner's (cfg, splits, k per split, grid, estimated us) for a GEMM");
  m.def("hgemm_plan2", [](int64_t M, int64_t N, int64_t K, bool ak, bool bk, bool allow_split, int64_t out_bytes) {
          const Plan2 p = plan2(M, N, K, ak, bk, allow_split, (int)out_bytes);
          auto t = [](const Plan& q) { return std::make_tuple(q.cfg, q.splits, q.kps, q.grid, q.est_s * 1e6); };
          return std::make_tuple(t(p.main), p.axis, p.at, t(p.tail), p.est_s * 1e6);
        }, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("a_k"), py::arg("b_k"), py::arg("allow_split") = true,
        py::arg("out_bytes") = 2, "(main plan, cut axis (-1 none, 0 N, 1 M), cut at, tail plan, estimated us)");
  m.def("linear32_fwd", &linear32_fwd, py::arg("x"), py::arg("w"), py::arg("bias") = py::none(), py::arg("relu") = false,
        py::arg("drop_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0,
        "fp32 Linear on the exact-f32 MFMA: dropout(relu(x w^T + b)), mask identical to dropout()");
  m.def("linear32_dgrad", &linear32_dgrad, py::arg("dy"), py::arg("w"), py::arg("mask_src") = py::none(),
        py::arg("mask_scale") = 1.0, "fp32 dy w, times (mask_src > 0) * mask_scale (relu+dropout backward)");
  m.def("linear32_wgrad", &linear32_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("alpha") = 1.0,
        "fp32 dw += alpha dy^T x");
  m.def("set_hgemm_force", [](int64_t cfg, int64_t splits) { g_force_cfg = (int)cfg; g_force_splits = (int)splits; },
        py::arg("cfg") = -1, py::arg("splits") = -1, "pin the planner's tile / split (-1: free); A/B testing only");
  m.def("set_hgemm_sk", [](bool on) { const bool was = g_sk != 0; g_sk = on ? 1 : 0; return was; }, py::arg("on"),
        "stream-K schedule for the implicit-im2col conv GEMMs (DPE_HGEMM_SK); returns the previous setting");
  m.def("set_hgemm_dynamic", [](bool on) { const bool was = g_dynamic; g_dynamic = on; return was; }, py::arg("on"),
        "persistent GEMM: claim units beyond the grid at run time (default) or round-robin them statically; "
        "returns the previous setting");
}

}  // namespace dpe_gemm
