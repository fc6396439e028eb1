"""Process-group setup and the collective API used by the training loop.

Reference: `setup_distributed` / `cleanup_distributed` (`train.py:70-86`)
hard-code ``init_process_group("gloo")`` and run every GPU collective through
gloo's host-staged TCP ring.  Here:

* ``backend="gloo"``  -- exactly the reference (CPU plumbing, BASELINE config 1).
* ``backend="rccl"``  -- torch's c10d process group is initialised with gloo
  as a *control plane only* (rendezvous, object broadcast, host barriers), and
  a native RCCL communicator (``_C.Communicator``, C++) is bootstrapped from
  its TCPStore: rank 0 calls ``ncclGetUniqueId`` and publishes it, peers read
  it, everyone ``ncclCommInitRank``s.  All tensor collectives
  (DDP buckets, init broadcast, metric all-reduce, barriers) then run on RCCL
  over xGMI from a dedicated HIP stream.
* ``backend="auto"``  -- rccl when a GPU is present, else gloo.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.env import read_env
from ..utils.logging import get_logger

log = get_logger(__name__)

_state = {"backend": None, "comm": None, "device": None, "max_channels": None}


def resolve_backend(backend: str) -> str:
    b = backend.lower()
    if b == "nccl":
        b = "rccl"
    if b == "auto":
        b = "rccl" if torch.cuda.is_available() else "gloo"
    if b not in ("rccl", "gloo"):
        raise ValueError(f"unknown backend {backend!r} (expected rccl|gloo|auto)")
    if b == "rccl" and not torch.cuda.is_available():
        raise RuntimeError("backend 'rccl' requires a GPU")
    return b


def init_process_group(backend: str = "auto", timeout_s: float = 1800.0,
                       comm_max_channels: Optional[int] = None) -> tuple[int, int, int]:
    """Initialise the job.  Returns (rank, world_size, local_rank) like the reference's setup_distributed.

    ``comm_max_channels`` (or env ``DPE_RCCL_MAX_CHANNELS``): cap on RCCL's channels for the
    communicator.  Every RCCL channel is one workgroup resident on a CU for the duration of a
    collective, so while bucket all-reduces overlap backward this bounds how many of the 256 CUs
    the communication can take from the compute kernels.  Applied through
    ``NCCL_MAX_NCHANNELS`` before ``ncclCommInitRank`` (read once at communicator creation)."""
    env = read_env()
    backend = resolve_backend(backend)
    if comm_max_channels is None and os.environ.get("DPE_RCCL_MAX_CHANNELS"):
        comm_max_channels = int(os.environ["DPE_RCCL_MAX_CHANNELS"])
    _state["max_channels"] = None
    if comm_max_channels is None and os.environ.get("NCCL_MAX_NCHANNELS", "").strip().isdigit():
        # a cap the user set for RCCL directly: the CU budget follows it
        _state["max_channels"] = max(1, int(os.environ["NCCL_MAX_NCHANNELS"]))
    if comm_max_channels:
        n = max(1, int(comm_max_channels))
        os.environ["NCCL_MAX_NCHANNELS"] = str(n)
        if int(os.environ.get("NCCL_MIN_NCHANNELS", "0") or 0) > n:
            os.environ["NCCL_MIN_NCHANNELS"] = str(n)
        _state["max_channels"] = n
    if not dist.is_initialized():
        dist.init_process_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    rank, world = dist.get_rank(), dist.get_world_size()
    local_rank = env.local_rank
    _state["backend"] = backend
    if backend == "rccl":
        torch.cuda.set_device(local_rank)
        _state["device"] = torch.device("cuda", local_rank)
        _state["comm"] = _make_comm(rank, world, local_rank)
        set_cu_budget(cu_reserve_for(world, _state["max_channels"]))
    else:
        _state["device"] = torch.device("cpu")
    return rank, world, local_rank


# RCCL channel cap (each channel = one workgroup resident on a CU while a bucket all-reduce overlaps
# backward).  OPT-IN: without --comm-max-channels / DPE_RCCL_MAX_CHANNELS / NCCL_MAX_NCHANNELS, RCCL
# keeps its own topology-tuned channel count.  Suggested value 16 (bandwidth model: ResNet-50's 102 MB
# / GPT-2's 498 MB fp32 gradients need 2*7/8 of that per GPU over the ~25 / ~9 ms backward, i.e.
# < 100 GB/s of bus bandwidth to stay hidden, while 16 blocks are 1.6-6 % of the persistent kernels'
# slots) -- a model, not a measurement, so it is not the default until an 8-GPU sweep
# (bench.py --comm-max-channels) backs it.
SUGGESTED_MAX_CHANNELS = 16


def cu_reserve_for(world: int, channels: Optional[int]) -> int:
    """Persistent-kernel slots left free while a bucket all-reduce is in flight: one per RCCL channel
    block (a 256-thread RCCL workgroup displaces at most one block of ours per CU; the kernels' grid =
    channel blocks, 256 threads, 140 VGPRs, ~20 KB LDS: profiles/world8_1gpu_r6.txt, and round 3's
    footprint run in git history).  ``DPE_CU_RESERVE`` overrides; 0 at world 1."""
    if os.environ.get("DPE_CU_RESERVE"):
        return max(0, int(os.environ["DPE_CU_RESERVE"]))
    if world <= 1:
        return 0
    # RCCL's own channel count is not queryable from here: when uncapped assume 32 resident channel blocks
    # (an upper bound for an 8-GPU xGMI all-reduce; the one-GPU socket rehearsal ran 4).  DDP keeps this
    # reserve only while the measured all-reduce duty warrants it (DDP.settle_cu_budget).
    return int(channels) if channels else 32


def set_cu_budget(slots: int) -> None:
    """Slots the persistent compute kernels (hgemm, streaming pointwise convs) leave to RCCL while the
    reducer has a collective in flight (csrc/comm/comm.cpp, CU budget)."""
    from ..ops._ext import ext

    ext().set_cu_reserve(int(slots))


def _make_comm(rank: int, world: int, local_rank: int):
    from ..ops._ext import ext

    C = ext()
    store = dist.distributed_c10d._get_default_store()
    key = "dpe/rccl_uid"
    if rank == 0:
        uid = C.rccl_unique_id()
        store.set(key, uid)
    else:
        uid = store.get(key)
    comm = C.Communicator(bytes(uid), rank, world, local_rank)
    return comm


def comm_max_channels() -> Optional[int]:
    """The RCCL channel cap this process initialised with (None: RCCL's own choice)."""
    return _state["max_channels"]


def backend() -> Optional[str]:
    return _state["backend"]


def comm():
    """The native RCCL communicator (None on the gloo backend)."""
    return _state["comm"]


def is_initialized() -> bool:
    return dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def all_reduce(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce of a tensor (RCCL for GPU tensors on the rccl backend)."""
    c = _state["comm"]
    if c is not None and t.is_cuda:
        c.all_reduce(t, op)
        return t
    if not dist.is_initialized() or get_world_size() == 1:
        return t
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "avg": None}
    if op == "avg":
        dist.all_reduce(t, dist.ReduceOp.SUM)
        t /= get_world_size()
    else:
        dist.all_reduce(t, ops[op])
    return t


def broadcast(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    c = _state["comm"]
    if c is not None and t.is_cuda:
        c.broadcast(t, src)
        return t
    if dist.is_initialized() and get_world_size() > 1:
        dist.broadcast(t, src)
    return t


def barrier() -> None:
    c = _state["comm"]
    if c is not None:
        c.barrier()
    elif dist.is_initialized():
        dist.barrier()


def check_health() -> str:
    """RCCL async-error watchdog probe ('' if healthy)."""
    c = _state["comm"]
    return c.async_error() if c is not None else ""


class Watchdog:
    """Failure detector: a daemon thread that polls the RCCL
    communicator's async error (``ncclCommGetAsyncError``) and a heartbeat the
    training loop refreshes every step.  On an RCCL error, or no heartbeat for
    ``timeout_s`` (a peer died mid-collective, a hang), it logs, aborts the
    communicator (``ncclCommAbort`` releases ranks blocked in collectives) and
    exits the process non-zero so the launcher's fail-fast path tears the job
    down -- instead of the reference's 30-minute gloo timeout.

    The training loop beats every step and every validation batch; rank 0's
    checkpoint writes run under ``suspended()``, the barrier behind them under
    ``grace(extra_s)`` (a longer but still bounded stall deadline).  The timeout
    must still cover the first training step (kernel/module load, bucket build).
    GEMM dispatch is planned analytically, so there is no autotuning pause."""

    def __init__(self, timeout_s: float = 600.0, interval_s: float = 2.0, on_fail=None):
        import threading
        import time

        self.timeout_s, self.interval_s = timeout_s, interval_s
        self._time = time
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._paused = 0
        self._grace = 0.0
        self._pending: list = []  # (event, host time) of beats whose device work has not completed
        self._lock = threading.Lock()
        self._on_fail = on_fail
        self.failure: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="dpe-watchdog", daemon=True)
        # native backstop (csrc/comm/comm.cpp): this thread needs the GIL and HIP's locks to check anything;
        # if it is starved or blocked for timeout_s + 15 s (at least 3 check intervals + 15 s), a native thread
        # aborts the communicator and exits
        self._native = _native_watchdog()
        self._arm_native()
        self._thread.start()

    def _arm_native(self) -> None:
        """(Re-)arm the native backstop for the CURRENT deadline: timeout (+ the grace in force) + 15 s;
        disarmed while suspended -- the Python check is off there too, so a legitimately long checkpoint
        write or the barrier behind it never meets a shorter native limit than the Python one."""
        if self._native is None:
            return
        if self._paused:
            self._native.watchdog_backstop(0.0)
        else:
            self._native.watchdog_backstop(max(float(self.timeout_s), 3.0 * float(self.interval_s)) + self._grace + 15.0)

    def beat(self) -> None:
        """A step finished on the host.  On a GPU job progress is what the DEVICE completes: the beat
        records an event on the current stream and the heartbeat advances only when that event has
        completed -- the host enqueues steps far ahead of a device that is stuck in a collective
        whose peer died, so host-side beats alone would hide the stall until the next sync."""
        now = self._time.monotonic()
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            ev = torch.cuda.Event()
            ev.record()
            self._push(ev, now)
            return
        self._last = now

    def _push(self, ev, now: float) -> None:
        with self._lock:
            # bounded: keep the oldest pending events (they gate progress) and always the newest beat --
            # a full list replaces its last entry, so the most recent step keeps an event and the
            # heartbeat advances as soon as the device reaches it
            if len(self._pending) >= 64:
                self._pending[-1] = (ev, now)
            else:
                self._pending.append((ev, now))

    def _device_progress(self) -> None:
        with self._lock:
            while self._pending and self._pending[0][0].query():
                self._pending.pop(0)
                self._last = self._time.monotonic()

    def suspended(self):
        """Context: no stall check inside (checkpoint writes, the barrier behind them); RCCL async
        errors are still polled.  The heartbeat restarts when the block ends."""
        import contextlib

        @contextlib.contextmanager
        def _ctx():
            self._paused += 1
            self._arm_native()
            try:
                yield self
            finally:
                self._paused -= 1
                self.beat()
                self._arm_native()

        return _ctx()

    def grace(self, extra_s: float):
        """Context: the stall deadline is ``timeout_s + extra_s`` inside (a barrier that waits for a
        peer's checkpoint write).  Detection stays on, so a peer dying there still aborts the job."""
        import contextlib

        @contextlib.contextmanager
        def _ctx():
            old = self._grace
            self._grace = max(old, float(extra_s))
            self.beat()
            self._arm_native()  # the native limit follows the raised deadline
            try:
                yield self
            finally:
                self._grace = old
                self.beat()
                self._arm_native()

        return _ctx()

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=5)
        if self._native is not None:
            self._native.watchdog_backstop(0.0)

    def _run(self):
        import threading

        while not self._stop.wait(self.interval_s):
            if self._native is not None:
                self._native.watchdog_pet()
            err = check_health()
            self._device_progress()
            stalled = 0.0 if self._paused else self._time.monotonic() - self._last
            if err or stalled > self.timeout_s + self._grace:
                self.failure = f"RCCL async error: {err}" if err else f"no progress for {stalled:.0f}s"
                log.error(f"watchdog: {self.failure}; aborting communicator")
                c = _state["comm"]
                if c is not None:
                    # ncclCommAbort releases ranks blocked in collectives; bounded, so an abort that
                    # itself blocks cannot turn the failure into a hang
                    t = threading.Thread(target=_try_abort, args=(c,), daemon=True)
                    t.start()
                    t.join(timeout=10.0)
                if self._on_fail is not None:
                    if self._native is not None:
                        self._native.watchdog_backstop(0.0)  # the caller handles the failure
                    self._on_fail(self.failure)
                    return
                for h in log.handlers + __import__("logging").getLogger().handlers:
                    try:
                        h.flush()
                    except Exception:  # noqa: BLE001
                        pass
                os._exit(1)


def _native_watchdog():
    """The extension module for the native watchdog backstop (None where it is not built)."""
    try:
        from ..ops._ext import ext

        C = ext()
        return C if hasattr(C, "watchdog_backstop") else None
    except Exception:  # noqa: BLE001
        return None


def _try_abort(c) -> None:
    try:
        c.abort()
    except Exception:  # noqa: BLE001
        pass


# The reference's collectives run on gloo, whose process group times out after 30 min
# ($TORCH/distributed/constants.py:12).  On the rccl backend every tensor collective is RCCL, which has
# no timeout of its own: the watchdog is that bound, on by default at world > 1.
DEFAULT_COLLECTIVE_TIMEOUT_S = 1800.0


def default_watchdog_timeout(requested: Optional[float], backend_name: Optional[str], world: int) -> float:
    """Watchdog stall timeout in seconds (0 = off).  An explicit value wins (``0`` is the opt-out);
    otherwise 1800 s on the rccl backend at world > 1, off elsewhere (gloo keeps its own timeout)."""
    if requested is not None:
        return max(0.0, float(requested))
    return DEFAULT_COLLECTIVE_TIMEOUT_S if (backend_name == "rccl" and world > 1) else 0.0


def start_watchdog(timeout_s: float = 600.0, interval_s: float = 2.0, on_fail=None) -> Watchdog:
    return Watchdog(timeout_s, interval_s, on_fail)


def destroy_process_group() -> None:
    if _state["comm"] is not None:
        torch.cuda.synchronize()
        _state["comm"] = None
        set_cu_budget(0)
    if dist.is_initialized():
        dist.destroy_process_group()
    _state["backend"] = None
    _state["max_channels"] = None


def get_device(local_rank: int) -> torch.device:
    """Reference `get_device` (`train.py:89-98`)."""
    if torch.cuda.is_available():
        device = torch.device(f"cuda:{local_rank}")
        torch.cuda.set_device(device)
        log.info(f"Using GPU: {torch.cuda.get_device_name(device)}")
    else:
        device = torch.device("cpu")
        log.info("Using CPU for training")
    return device
