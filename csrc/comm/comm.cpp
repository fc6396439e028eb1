// RCCL communicator and bucketed DDP reducer.  See comm.h.
//
// Reference parity: C3 (init broadcast) -> Communicator::broadcast;
// C4 (per-backward bucket all-reduce, 25 MiB buckets, 1 MiB first) ->
// Reducer; C6/C8 barriers -> Communicator::barrier; C7 metric all-reduce ->
// Communicator::all_reduce.  Unlike gloo (host-staged TCP ring) the data
// never leaves HBM: RCCL moves it over xGMI from a side stream.
#include "comm.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>
#include <stdexcept>

#include <pybind11/functional.h>

extern "C" int dpe_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st);
extern "C" int dpe_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st);

// persistent-kernel slots to leave free right now (0 unless a collective may be resident)
extern "C" int dpe_cu_reserve() {
  return dpe::comm_active_reserve();
}

namespace dpe {

#define NCCL_CHECK(cmd)                                                                       \
  do {                                                                                        \
    ncclResult_t r_ = (cmd);                                                                  \
    if (r_ != ncclSuccess && r_ != ncclInProgress)                                            \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                    \
  } while (0)

#define HIP_CHECK(cmd)                                                                              \
  do {                                                                                              \
    hipError_t e_ = (cmd);                                                                          \
    if (e_ != hipSuccess)                                                                           \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + \
                               ":" + std::to_string(__LINE__));                                     \
  } while (0)

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: throw std::runtime_error("unsupported dtype for RCCL");
  }
}

ncclRedOp_t to_nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  throw std::runtime_error("unknown reduce op " + op);
}

std::string Communicator::unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

// ---------------------------------------------------------------- native watchdog backstop
// The Python watchdog (parallel/dist.py Watchdog) is a thread that needs the GIL and HIP's runtime
// locks to check progress.  A rank whose main thread is stuck inside a GIL-holding native call (a kernel
// launch blocked on a full launch queue behind a collective that can never complete, a stream sync)
// starves it, and the rank would hang forever.  This thread needs neither: the Python watchdog pets it
// on every check; when no pet has come for the armed limit, it reports, aborts the communicator
// (bounded) and exits the process non-zero.
namespace {
std::atomic<int64_t> g_wd_pet_ns{0};
std::atomic<int64_t> g_wd_limit_ns{0};  // 0: disarmed
std::atomic<Communicator*> g_wd_comm{nullptr};
// held by the abort thread for the whole abort and by ~Communicator while it unregisters: the
// communicator cannot be destroyed under a running abort (the process _exits 5 s after it starts)
std::mutex g_wd_mu;
std::once_flag g_wd_once;
int64_t wd_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void wd_loop() {
  while (true) {
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    const int64_t lim = g_wd_limit_ns.load(std::memory_order_relaxed);
    if (lim <= 0) continue;
    const int64_t idle = wd_now_ns() - g_wd_pet_ns.load(std::memory_order_relaxed);
    if (idle <= lim) continue;
    std::fprintf(stderr,
                 "[dpe native watchdog] watchdog: no check by the Python watchdog for %.0fs (starved or blocked); "
                 "aborting communicator\n",
                 (double)idle * 1e-9);
    std::fflush(stderr);
    if (g_wd_comm.load()) {
      std::thread([] {
        std::lock_guard<std::mutex> lk(g_wd_mu);
        if (Communicator* c = g_wd_comm.load()) c->abort();
      }).detach();
      std::this_thread::sleep_for(std::chrono::seconds(5));  // bounded: exit whether or not the abort returned
    }
    _exit(1);
  }
}
}  // namespace

void watchdog_backstop(double limit_s) {
  g_wd_pet_ns.store(wd_now_ns(), std::memory_order_relaxed);
  g_wd_limit_ns.store(limit_s > 0 ? (int64_t)(limit_s * 1e9) : 0, std::memory_order_relaxed);
  if (limit_s > 0) std::call_once(g_wd_once, [] { std::thread(wd_loop).detach(); });
}
void watchdog_pet() { g_wd_pet_ns.store(wd_now_ns(), std::memory_order_relaxed); }

Communicator::Communicator(const std::string& uid, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device), stream_(c10::hip::getStreamFromPool(true, device)) {
  if (uid.size() != sizeof(ncclUniqueId::internal)) throw std::runtime_error("bad RCCL unique id size");
  c10::hip::HIPGuard g(device);
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), sizeof(id.internal));
  NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
  HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device));
  g_wd_comm.store(this);
}

Communicator::~Communicator() {
  {
    std::lock_guard<std::mutex> lk(g_wd_mu);  // waits out a running backstop abort (then _exit follows)
    Communicator* self = this;
    g_wd_comm.compare_exchange_strong(self, nullptr);
  }
  if (comm_ && !aborted_) ncclCommDestroy(comm_);
  if (ev_in_) (void)hipEventDestroy(ev_in_);
  if (ev_out_) (void)hipEventDestroy(ev_out_);
}

void Communicator::pre(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "collective tensors must be contiguous GPU tensors");
  auto cur = c10::hip::getCurrentHIPStream(device_);
  HIP_CHECK(hipEventRecord(ev_in_, cur.stream()));
  HIP_CHECK(hipStreamWaitEvent(stream_.stream(), ev_in_, 0));
  c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
}

void Communicator::post(const at::Tensor&) {
  auto cur = c10::hip::getCurrentHIPStream(device_);
  HIP_CHECK(hipEventRecord(ev_out_, stream_.stream()));
  HIP_CHECK(hipStreamWaitEvent(cur.stream(), ev_out_, 0));
}

void Communicator::all_reduce(at::Tensor& t, const std::string& op) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  pre(t);
  NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_nccl_op(op), comm_,
                           stream_.stream()));
  post(t);
}

void Communicator::all_reduce_raw(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  NCCL_CHECK(ncclAllReduce(buf, buf, count, dt, op, comm_, s));
}

void Communicator::broadcast(at::Tensor& t, int root) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  pre(t);
  NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_.stream()));
  post(t);
}

void Communicator::all_gather(const at::Tensor& in, at::Tensor& out) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: out must hold world*in elements");
  pre(in);
  c10::hip::HIPCachingAllocator::recordStream(out.storage().data_ptr(), stream_);
  NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, stream_.stream()));
  post(out);
}

void Communicator::reduce_scatter(const at::Tensor& in, at::Tensor& out, const std::string& op) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: in must hold world*out elements");
  pre(in);
  c10::hip::HIPCachingAllocator::recordStream(out.storage().data_ptr(), stream_);
  NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()), to_nccl_op(op), comm_,
                               stream_.stream()));
  post(out);
}

void Communicator::all_to_all(const at::Tensor& in, at::Tensor& out) {
  TORCH_CHECK(!aborted_, "RCCL communicator was aborted");
  TORCH_CHECK(in.numel() == out.numel() && in.numel() % world_ == 0, "all_to_all: equal sizes divisible by world");
  pre(in);
  c10::hip::HIPCachingAllocator::recordStream(out.storage().data_ptr(), stream_);
  const size_t chunk = in.numel() / world_;
  const size_t esz = in.element_size();
  NCCL_CHECK(ncclGroupStart());
  for (int r = 0; r < world_; ++r) {
    NCCL_CHECK(ncclSend((char*)in.data_ptr() + r * chunk * esz, chunk, to_nccl(in.scalar_type()), r, comm_, stream_.stream()));
    NCCL_CHECK(ncclRecv((char*)out.data_ptr() + r * chunk * esz, chunk, to_nccl(in.scalar_type()), r, comm_, stream_.stream()));
  }
  NCCL_CHECK(ncclGroupEnd());
  post(out);
}

void Communicator::barrier() {
  all_reduce(barrier_buf_, "sum");
  HIP_CHECK(hipStreamSynchronize(c10::hip::getCurrentHIPStream(device_).stream()));
}

uint64_t Communicator::register_buffer(void* ptr, size_t bytes) {
  if (!comm_ || !ptr || bytes == 0) return 0;
  void* h = nullptr;
  const ncclResult_t r = ncclCommRegister(comm_, ptr, bytes, &h);
  if (r != ncclSuccess || !h) return 0;
  return (uint64_t)(uintptr_t)h;
}

void Communicator::deregister_buffer(uint64_t handle) {
  if (comm_ && handle && !aborted_) (void)ncclCommDeregister(comm_, (void*)(uintptr_t)handle);
}

std::string Communicator::async_error() {
  ncclResult_t st = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError(comm_, &st);
  if (r != ncclSuccess) return ncclGetErrorString(r);
  if (st != ncclSuccess && st != ncclInProgress) return ncclGetErrorString(st);
  return "";
}

void Communicator::abort() {
  // the flag first: an enqueue racing with the abort (a reducer launch) refuses instead of touching a
  // communicator being torn down
  if (comm_ && !aborted_.exchange(true)) ncclCommAbort(comm_);
  set_comm_active(false);  // no collective of this communicator is in flight any more
}

// ------------------------------------------------ CU budget while collectives overlap compute
// Every RCCL channel is one workgroup resident on a CU for the duration of a collective.  The
// persistent compute kernels (hgemm, pw_stream) size their grids to exactly the resident capacity and
// give every block a static share; a foreign workgroup on a CU whose slots they fill displaces one of
// their blocks into a second wave (x1.45-1.7 measured, profiles/cu_hog_probe_r2.txt in git history).  While the
// reducer has a bucket all-reduce in flight (first launch of a backward .. finalize) those kernels
// plan with `reserve` slots fewer (bindings/gemm.cpp plan(), pwconv.hip pw_capacity()).  The
// reserve is the communicator's channel count (parallel/dist.py).  Host-side state: every rank
// issues the same launch sequence, so every rank plans the same grids.
static std::atomic<int> g_cu_reserve{0};
static std::atomic<int> g_comm_active{0};

void set_comm_active(bool on) { g_comm_active.store(on ? 1 : 0, std::memory_order_relaxed); }
int comm_active_reserve() {
  return g_comm_active.load(std::memory_order_relaxed) ? g_cu_reserve.load(std::memory_order_relaxed) : 0;
}

// ------------------------------------------------ weight-grad side streams
// Per-device stream that the model's backward writes some gradients on
// (ops/_state.py run_on_aux); bucket all-reduces wait for it as well.
static hipStream_t g_aux_streams[64] = {};
hipStream_t aux_stream(int device) { return (device >= 0 && device < 64) ? g_aux_streams[device] : nullptr; }

// ------------------------------------------------------------------ Reducer
Reducer::Reducer(std::vector<at::Tensor> buckets, std::vector<std::vector<int64_t>> bucket_params, int64_t nparams,
                 std::shared_ptr<Communicator> comm, bool timing, bool force, bool comm_bf16, bool sync_debug,
                 bool register_buckets)
    : buckets_(std::move(buckets)), bparams_(std::move(bucket_params)), comm_(std::move(comm)), timing_(timing),
      force_(force), comm_bf16_(comm_bf16), sync_debug_(sync_debug) {
  for (auto& b : buckets_) TORCH_CHECK(b.is_cuda(), "bucket buffers must be GPU tensors (host transport: Reducer.host)");
  init_tracking(nparams);
  // timing-capable events whether or not timing is on now: set_timing() may switch it per step
  const unsigned flags = hipEventDefault;
  ev_ready_.resize(buckets_.size());
  ev_aux_.resize(buckets_.size());
  ev_start_.resize(buckets_.size());
  ev_end_.resize(buckets_.size());
  for (size_t b = 0; b < buckets_.size(); ++b) {
    HIP_CHECK(hipEventCreateWithFlags(&ev_ready_[b], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_aux_[b], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_start_[b], flags));
    HIP_CHECK(hipEventCreateWithFlags(&ev_end_[b], flags));
    if (comm_) c10::hip::HIPCachingAllocator::recordStream(buckets_[b].storage().data_ptr(), comm_->comm_stream());
    if (comm_bf16_) {
      TORCH_CHECK(buckets_[b].scalar_type() == at::kFloat, "comm_bf16 needs fp32 buckets");
      staging_.push_back(at::empty({buckets_[b].numel()}, buckets_[b].options().dtype(at::kBFloat16)));
      if (comm_) c10::hip::HIPCachingAllocator::recordStream(staging_.back().storage().data_ptr(), comm_->comm_stream());
    }
  }
  HIP_CHECK(hipEventCreateWithFlags(&ev_bwd_end_, flags));
  HIP_CHECK(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_step_begin_, flags));
  HIP_CHECK(hipEventCreateWithFlags(&ev_wait_, hipEventDisableTiming));
  // Register the buffers RCCL actually moves (fp32 buckets, or their bf16 staging copies) once per
  // (re)build; they live exactly as long as this reducer and are deregistered before release.
  if (register_buckets && comm_ && (comm_->world() > 1 || force_)) {
    auto& bufs = comm_bf16_ ? staging_ : buckets_;
    for (auto& t : bufs) reg_handles_.push_back(comm_->register_buffer(t.data_ptr(), t.numel() * t.element_size()));
  }
}

int64_t Reducer::registered_buffers() const {
  int64_t n = 0;
  for (uint64_t h : reg_handles_) n += h != 0;
  return n;
}

Reducer::Reducer(std::vector<at::Tensor> buckets, std::vector<std::vector<int64_t>> bucket_params, int64_t nparams,
                 int world, std::function<void(int64_t)> on_launch, std::function<void()> on_finalize)
    : buckets_(std::move(buckets)), bparams_(std::move(bucket_params)), timing_(false), force_(false), comm_bf16_(false),
      sync_debug_(false), host_launch_(std::move(on_launch)), host_finalize_(std::move(on_finalize)), host_world_(world) {
  TORCH_CHECK(host_launch_, "host-transport reducer needs an on_launch callable");
  TORCH_CHECK(world >= 1, "world must be >= 1");
  init_tracking(nparams);
}

void Reducer::init_tracking(int64_t nparams) {
  TORCH_CHECK(buckets_.size() == bparams_.size(), "bucket/param list size mismatch");
  param_bucket_.assign(nparams, -1);
  expected_.resize(buckets_.size());
  for (size_t b = 0; b < bparams_.size(); ++b) {
    TORCH_CHECK(buckets_[b].is_contiguous(), "bucket buffers must be contiguous");
    for (int64_t p : bparams_[b]) {
      TORCH_CHECK(p >= 0 && p < nparams && param_bucket_[p] == -1, "parameter in several buckets or out of range");
      param_bucket_[p] = (int64_t)b;
    }
    expected_[b] = (int)bparams_[b].size();
  }
  pending_ = expected_;
  ready_.assign(buckets_.size(), 0);
  seen_.assign(nparams, 0);
}

Reducer::~Reducer() {
  if (host_launch_) return;  // no HIP objects in host-transport mode
  set_comm_active(false);  // a backward that raised after its first launch never reached finalize()
  if (comm_) {
    // the last step's all-reduces may still be running on the comm stream (finalize only makes the
    // compute stream wait): drain them before their buffers are deregistered / released and a
    // rebuilt reducer registers its own
    if (!comm_->aborted()) (void)hipStreamSynchronize(comm_->comm_stream().stream());
    for (uint64_t h : reg_handles_) comm_->deregister_buffer(h);
  }
  for (auto* v : {&ev_ready_, &ev_aux_, &ev_start_, &ev_end_})
    for (auto e : *v) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ev_bwd_end_);
  (void)hipEventDestroy(ev_done_);
  (void)hipEventDestroy(ev_step_begin_);
  (void)hipEventDestroy(ev_wait_);
}

void Reducer::stream_wait_comm(uint64_t stream) {
  if (host_launch_ || !comm_ || (comm_->world() == 1 && !force_)) return;
  // (one event re-recorded each time: a wait captures the event's state when it is issued)
  HIP_CHECK(hipEventRecord(ev_wait_, comm_->comm_stream().stream()));
  HIP_CHECK(hipStreamWaitEvent((hipStream_t)(uintptr_t)stream, ev_wait_, 0));
}

void Reducer::prepare() {
  // a new step: clear a flag left set by a backward that raised after its first bucket launch (no
  // finalize ran), so compute kernels until this step's first launch plan with every slot
  if (!host_launch_) set_comm_active(false);
  pending_ = expected_;
  std::fill(ready_.begin(), ready_.end(), 0);
  std::fill(seen_.begin(), seen_.end(), 0);
  next_ = 0;
  launch_order_.clear();
  step_open_ = true;
  timed_ = timing_ && !host_launch_;
  timed_done_ = false;
  if (timed_) HIP_CHECK(hipEventRecord(ev_step_begin_, c10::hip::getCurrentHIPStream().stream()));
}

void Reducer::launch(int64_t b) {
  launch_order_.push_back(b);
  if (host_launch_) {
    host_launch_(b);
    return;
  }
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  if (!comm_ || (comm_->world() == 1 && !force_)) return;
  hipStream_t cs = comm_->comm_stream().stream();
  set_comm_active(true);  // compute kernels enqueued from here on may share the CUs with RCCL
  HIP_CHECK(hipEventRecord(ev_ready_[b], cur));
  HIP_CHECK(hipStreamWaitEvent(cs, ev_ready_[b], 0));
  // gradients written on the weight-grad side stream (set_aux_stream) are covered too
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (hipStream_t aux = aux_stream(dev)) {
    HIP_CHECK(hipEventRecord(ev_aux_[b], aux));
    HIP_CHECK(hipStreamWaitEvent(cs, ev_aux_[b], 0));
  }
  if (timed_) HIP_CHECK(hipEventRecord(ev_start_[b], cs));
  auto& t = buckets_[b];
  if (comm_bf16_) {
    auto& h = staging_[b];
    TORCH_CHECK(dpe_cast_f32_bf16((const float*)t.data_ptr(), (uint16_t*)h.data_ptr(), t.numel(), cs) == 0, "bf16 cast");
    comm_->all_reduce_raw(h.data_ptr(), h.numel(), ncclBfloat16, ncclAvg, cs);
    TORCH_CHECK(dpe_cast_bf16_f32((const uint16_t*)h.data_ptr(), (float*)t.data_ptr(), t.numel(), cs) == 0, "f32 cast");
  } else {
    comm_->all_reduce_raw(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), ncclAvg, cs);
  }
  if (timed_) HIP_CHECK(hipEventRecord(ev_end_[b], cs));
  if (sync_debug_) {
    HIP_CHECK(hipStreamSynchronize(cs));
    const std::string err = comm_->async_error();
    TORCH_CHECK(err.empty(), "RCCL error after bucket ", b, ": ", err);
  }
}

void Reducer::mark_ready(int64_t p) {
  TORCH_CHECK(p >= 0 && p < (int64_t)param_bucket_.size(), "mark_ready: bad parameter index");
  if (!step_open_) prepare();
  if (seen_[p]) return;  // a parameter used twice in one graph fires once (re-entrancy guard)
  seen_[p] = 1;
  const int64_t b = param_bucket_[p];
  if (b < 0) return;
  if (--pending_[b] == 0) ready_[b] = 1;
  while (next_ < (int64_t)buckets_.size() && ready_[next_]) launch(next_++);
}

void Reducer::finalize() {
  if (!step_open_) return;
  if (host_launch_) {
    while (next_ < (int64_t)buckets_.size()) launch(next_++);
    if (host_finalize_) host_finalize_();
    step_open_ = false;
    return;
  }
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  if (timed_) HIP_CHECK(hipEventRecord(ev_bwd_end_, cur));
  // Unused parameters: their (zero / stale-accumulated) slices are reduced
  // anyway so every rank issues the same collective sequence.
  while (next_ < (int64_t)buckets_.size()) launch(next_++);
  if (comm_ && (comm_->world() > 1 || force_)) {
    HIP_CHECK(hipEventRecord(ev_done_, comm_->comm_stream().stream()));
    HIP_CHECK(hipStreamWaitEvent(cur, ev_done_, 0));
  }
  set_comm_active(false);  // later compute kernels are ordered after the last collective
  step_open_ = false;
  timed_done_ = timed_;
}

bool Reducer::timings_ready() {
  if (host_launch_ || !timed_done_ || !comm_ || (comm_->world() == 1 && !force_)) return false;
  const hipError_t e = hipEventQuery(ev_done_);
  if (e == hipErrorNotReady) return false;
  HIP_CHECK(e);
  return true;
}

std::vector<std::tuple<int64_t, double, double>> Reducer::last_timings() {
  std::vector<std::tuple<int64_t, double, double>> out;
  if (host_launch_ || !timed_done_ || !comm_ || (comm_->world() == 1 && !force_)) return out;
  HIP_CHECK(hipEventSynchronize(ev_done_));
  for (size_t b = 0; b < buckets_.size(); ++b) {
    float ms = 0.f, rel = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_start_[b], ev_end_[b]));
    // start of this bucket's all-reduce relative to the end of backward (negative = overlapped)
    HIP_CHECK(hipEventElapsedTime(&rel, ev_bwd_end_, ev_start_[b]));
    out.emplace_back((int64_t)b, (double)ms, (double)rel);
  }
  return out;
}

void register_comm(pybind11::module& m) {
  namespace py = pybind11;
  m.def("rccl_unique_id", []() { return py::bytes(Communicator::unique_id()); });
  m.def("watchdog_backstop", &watchdog_backstop, py::arg("limit_s"),
        "arm (limit_s > 0) / disarm the native watchdog backstop: no watchdog_pet() for limit_s seconds -> "
        "report, abort the communicator (bounded), exit(1)");
  m.def("watchdog_pet", &watchdog_pet, "the Python watchdog made a check");
  m.def("set_aux_stream", [](int device, uint64_t stream) {
    TORCH_CHECK(device >= 0 && device < 64, "set_aux_stream: bad device");
    g_aux_streams[device] = (hipStream_t)(uintptr_t)stream;
  }, "register the weight-grad side stream of a device (bucket all-reduces wait for it)");
  m.def("set_cu_reserve", [](int64_t n) { g_cu_reserve.store((int)std::max<int64_t>(0, n), std::memory_order_relaxed); },
        py::arg("slots"), "persistent-kernel slots left free while a bucket all-reduce is in flight (0: none)");
  m.def("cu_reserve_config", []() { return g_cu_reserve.load(std::memory_order_relaxed); });
  m.def("set_comm_active", &set_comm_active, py::arg("on"),
        "mark collectives as (not) resident beside compute (the reducer does this itself; probes / tests)");
  m.def("cu_reserve", []() { return dpe_cu_reserve(); }, "slots the persistent kernels leave free right now");
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
             return std::make_shared<Communicator>(std::string(uid), rank, world, device);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def("all_reduce", &Communicator::all_reduce, py::arg("tensor"), py::arg("op") = "sum", py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &Communicator::broadcast, py::arg("tensor"), py::arg("root") = 0, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &Communicator::all_gather)
      .def("reduce_scatter", &Communicator::reduce_scatter, py::arg("input"), py::arg("output"), py::arg("op") = "sum")
      .def("all_to_all", &Communicator::all_to_all)
      .def("barrier", &Communicator::barrier, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &Communicator::async_error)
      // (abort keeps the GIL: Python-side collectives cannot be enqueued on the communicator meanwhile)
      .def("abort", &Communicator::abort)
      .def("comm_stream_ptr", [](Communicator& c) { return (uint64_t)(uintptr_t)c.comm_stream().stream(); })
      .def("register_buffer", [](Communicator& c, const at::Tensor& t) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "register_buffer: contiguous GPU tensor");
             return c.register_buffer(t.data_ptr(), t.numel() * t.element_size());
           }, "ncclCommRegister a tensor's bytes; returns a handle (0: RCCL declined)")
      .def("deregister_buffer", &Communicator::deregister_buffer);
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init<std::vector<at::Tensor>, std::vector<std::vector<int64_t>>, int64_t, std::shared_ptr<Communicator>, bool,
                    bool, bool, bool, bool>(),
           py::arg("buckets"), py::arg("bucket_params"), py::arg("nparams"), py::arg("comm"), py::arg("timing") = false,
           py::arg("force") = false, py::arg("comm_bf16") = false, py::arg("sync_debug") = false,
           py::arg("register_buckets") = true)
      .def_property_readonly("registered_buffers", &Reducer::registered_buffers)
      .def_static("host", [](std::vector<at::Tensor> buckets, std::vector<std::vector<int64_t>> bucket_params,
                             int64_t nparams, int world, std::function<void(int64_t)> on_launch,
                             std::function<void()> on_finalize) {
             return std::make_shared<Reducer>(std::move(buckets), std::move(bucket_params), nparams, world,
                                              std::move(on_launch), std::move(on_finalize));
           }, py::arg("buckets"), py::arg("bucket_params"), py::arg("nparams"), py::arg("world"), py::arg("on_launch"),
           py::arg("on_finalize"),
           "host-transport reducer: same C++ sequencing, collectives delegated to the callables (gloo on CPU)")
      .def_property_readonly("world", &Reducer::world)
      .def_property_readonly("host_mode", &Reducer::host_mode)
      .def("launch_order", &Reducer::launch_order)
      .def("prepare", &Reducer::prepare)
      .def("mark_ready", &Reducer::mark_ready)
      .def("finalize", &Reducer::finalize)
      .def("last_timings", &Reducer::last_timings)
      .def("set_timing", &Reducer::set_timing, py::arg("on"), "per-bucket timing events from the next prepare()")
      .def_property_readonly("timing", &Reducer::timing)
      .def("timings_ready", &Reducer::timings_ready,
           "the last finalized step was timed and its collectives completed (non-blocking)")
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("buckets_launched", &Reducer::buckets_launched)
      .def("stream_wait_comm", &Reducer::stream_wait_comm, py::arg("stream"),
           "the given HIP stream waits for every collective issued so far (no-op without collectives)");
}

}  // namespace dpe
