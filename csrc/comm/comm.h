// RCCL communicator + DDP gradient reducer (native replacement for the
// reference's ProcessGroupGloo + c10d::Reducer).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <functional>
#include <memory>
#include <atomic>
#include <string>
#include <vector>

namespace dpe {

// One RCCL communicator over all ranks of the job, bootstrapped from a
// unique id the Python side distributes through the c10d TCPStore.  All
// collectives run on a dedicated high-priority HIP stream (torch stream-pool
// stream, so the caching allocator can track cross-stream tensor use) and
// are ordered against the caller's current stream with events.
class Communicator {
 public:
  static std::string unique_id();
  Communicator(const std::string& uid, int rank, int world, int device);
  ~Communicator();

  int rank() const { return rank_; }
  int world() const { return world_; }
  c10::hip::HIPStream comm_stream() const { return stream_; }
  ncclComm_t handle() const { return comm_; }

  // Tensor collectives, enqueued after all prior work on the current stream;
  // the current stream waits for their completion (async w.r.t. the host).
  void all_reduce(at::Tensor& t, const std::string& op);
  void broadcast(at::Tensor& t, int root);
  void all_gather(const at::Tensor& in, at::Tensor& out);
  void reduce_scatter(const at::Tensor& in, at::Tensor& out, const std::string& op);
  void all_to_all(const at::Tensor& in, at::Tensor& out);
  void barrier();

  // Raw enqueue on the comm stream (no stream ordering): used by the reducer.
  void all_reduce_raw(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);

  // User-buffer registration (ncclCommRegister): RCCL may then move the buffer's bytes without
  // staging through its internal FIFOs.  Returns an opaque handle, or 0 when RCCL declined
  // (registration is an optimisation: never an error).  deregister(0) is a no-op.
  uint64_t register_buffer(void* ptr, size_t bytes);
  void deregister_buffer(uint64_t handle);

  // Non-blocking health check (ncclCommGetAsyncError); returns error string or "".
  std::string async_error();
  void abort();
  bool aborted() const { return aborted_; }

 private:
  void pre(const at::Tensor& t);
  void post(const at::Tensor& t);
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1, device_ = 0;
  c10::hip::HIPStream stream_;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  at::Tensor barrier_buf_;
  std::atomic<bool> aborted_{false};  // (set by the watchdog thread, read by every enqueue)
};

ncclDataType_t to_nccl(at::ScalarType t);
ncclRedOp_t to_nccl_op(const std::string& op);

// Bucketed gradient reducer.  Buckets are flat buffers whose slices are the
// parameters' .grad views (gradient-as-bucket-view), so no copy into or out
// of the buckets is ever made.  mark_ready(i) is called once per parameter
// per backward, after the kernel producing grad i was enqueued on the
// current stream; when every parameter of bucket b is ready the all-reduce
// (ncclAvg) is issued on the comm stream behind an event -- buckets are
// issued strictly in index order so all ranks enqueue identical sequences.
// finalize() issues any remaining buckets and makes the current stream wait
// for the last one (optimizer ordering).
class Reducer {
 public:
  // comm_bf16: all-reduce a bf16 copy of each fp32 bucket (cast -> ncclAvg in bf16 -> cast back, all on the
  //   comm stream): half the xGMI bytes, the gradient-compression hook of SURVEY §2.2 I5 / B3.
  // sync_debug: synchronise the comm stream after every bucket and raise on an RCCL async error (SURVEY §5.2
  //   stream-ordering assertion mode).
  Reducer(std::vector<at::Tensor> buckets, std::vector<std::vector<int64_t>> bucket_params, int64_t nparams,
          std::shared_ptr<Communicator> comm, bool timing, bool force = false, bool comm_bf16 = false,
          bool sync_debug = false, bool register_buckets = true);
  // Host-transport mode: the same readiness tracking / index-order issue / finalize sequencing with
  // the collective itself delegated to `on_launch(bucket)` and `on_finalize()` (the gloo control
  // plane on CPU, world >= 1).  No HIP call is made in this mode, so it runs on a GPU-less host.
  Reducer(std::vector<at::Tensor> buckets, std::vector<std::vector<int64_t>> bucket_params, int64_t nparams, int world,
          std::function<void(int64_t)> on_launch, std::function<void()> on_finalize);
  ~Reducer();
  void prepare();
  void mark_ready(int64_t param);
  void finalize();
  // (bucket, comm_ms, issued_before_backward_end) for the last finalized step
  std::vector<std::tuple<int64_t, double, double>> last_timings();
  // per-bucket timing on / off from the next prepare() (the adaptive CU budget times a few warm-up steps)
  void set_timing(bool on) { timing_ = on; }
  bool timing() const { return timing_; }
  // the last finalized step was timed and its collectives have completed (non-blocking)
  bool timings_ready();
  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  int64_t registered_buffers() const;
  int world() const { return host_launch_ ? host_world_ : (comm_ ? comm_->world() : 1); }
  bool host_mode() const { return (bool)host_launch_; }
  int64_t buckets_launched() const { return next_; }
  // make `stream` wait for every collective issued so far on the comm stream (no-op when none are issued:
  // world 1 without force, host transport) -- the overlapped optimizer's per-bucket ordering
  void stream_wait_comm(uint64_t stream);
  std::vector<int64_t> launch_order() const { return launch_order_; }

 private:
  void launch(int64_t b);
  std::vector<at::Tensor> buckets_;
  std::vector<std::vector<int64_t>> bparams_;
  std::vector<int64_t> param_bucket_;
  std::vector<int> pending_, expected_;
  std::vector<char> ready_, seen_;
  int64_t next_ = 0;
  std::shared_ptr<Communicator> comm_;
  bool timing_;
  bool timed_ = false;       // the step in flight (or last finalized) records timing events
  bool timed_done_ = false;  // ... and it reached finalize()
  bool force_;  // issue collectives even at world size 1 (exercises the comm path on a 1-GPU box)
  bool comm_bf16_, sync_debug_;
  std::vector<at::Tensor> staging_;  // bf16 copies of the buckets (comm_bf16)
  std::vector<int64_t> launch_order_;
  std::vector<hipEvent_t> ev_ready_, ev_aux_, ev_start_, ev_end_;
  hipEvent_t ev_bwd_end_ = nullptr, ev_done_ = nullptr, ev_step_begin_ = nullptr, ev_wait_ = nullptr;
  bool step_open_ = false;
  std::vector<uint64_t> reg_handles_;  // ncclCommRegister handles of the buckets / bf16 staging buffers
  std::function<void(int64_t)> host_launch_;
  std::function<void()> host_finalize_;
  int host_world_ = 1;
  void init_tracking(int64_t nparams);
};

// CU budget: mark collectives resident beside compute; slots persistent kernels leave free now
void set_comm_active(bool on);
int comm_active_reserve();

// weight-grad side stream registered for a device (nullptr: none)
hipStream_t aux_stream(int device);

void register_comm(pybind11::module& m);

}  // namespace dpe
