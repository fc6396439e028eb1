"""The native C++ Reducer at world 2, 4 and 8 over real RCCL collectives, on a 1-GPU box.

N processes share GPU 0.  Each gets its own NCCL_HOSTID, so RCCL sees N hosts
(no duplicate-GPU refusal) and connects them with its socket transport over
loopback: Reducer::launch runs with world() == N, the buckets are really
all-reduced (ncclAvg), the bucket rebuild (rank 0's order broadcast to N-1 peers),
no_sync accumulation and the bf16 compression path are checked against
rank-averaged plain-backward gradients (tests/_rccl_world2_worker.py), and a rank
killed mid-epoch must take every survivor down through its watchdog.  On an
8-GPU node the same code runs over xGMI.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_world(n, args, extra_env=None, timeout=100):
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "PYTHONPATH": ROOT,
                    "NCCL_HOSTID": f"dpe-test-host-{r}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0", "OMP_NUM_THREADS": "1",
                    "DPE_RCCL_MAX_CHANNELS": "4"})  # the CU cap for overlapped collectives, exercised
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, "-u", *args], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    import time

    outs = [None] * n
    deadline = time.time() + timeout
    try:
        for i, p in enumerate(procs):
            try:
                outs[i] = p.communicate(timeout=max(1.0, deadline - time.time()))[0]
            except subprocess.TimeoutExpired:
                break  # (every process still running is killed below; its output is kept for the report)
    finally:
        for i, p in enumerate(procs):
            if p.poll() is None:
                p.kill()
            if outs[i] is None:
                outs[i] = (p.communicate()[0] or "") + f"\n[killed by the test after {timeout}s]"
    return [p.returncode for p in procs], outs


def _run_world2(args, extra_env=None, timeout=100):
    return _run_world(2, args, extra_env, timeout)


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world2_rccl():
    codes, outs = _run_world2([os.path.join(ROOT, "tests", "_rccl_world2_worker.py")])
    assert codes == [0, 0], "\n".join(o[-3000:] for o in outs)
    assert all("ok: world-2 RCCL reducer" in o for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-2" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world2_rccl_gpt2():
    """The transformer path at world 2: tied wte written by two kernels, fused bias grads, rebuild,
    no_sync (tests/_rccl_world2_worker.py main_gpt2)."""
    codes, outs = _run_world2([os.path.join(ROOT, "tests", "_rccl_world2_worker.py"), "gpt2"])
    assert codes == [0, 0], "\n".join(o[-3000:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-2" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_overlap_optimizer_world2_rccl():
    """the optimizer-in-backward stream waits for each bucket's real RCCL
    all-reduce (fp32, and bf16 with the cast-back on the comm stream); parameters match the
    step-after run and are bitwise identical across ranks (tests/_rccl_world2_worker.py main_ovopt)."""
    codes, outs = _run_world2([os.path.join(ROOT, "tests", "_rccl_world2_worker.py"), "ovopt"], timeout=150)
    assert codes == [0, 0], "\n".join(o[-3000:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-2" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rank_death_mid_allreduce_aborts_survivor(tmp_path):
    """Failure detection on the real RCCL path: rank 1 SIGKILLs itself at batch 3 of
    epoch 0 (DPE_FAULT_INJECT) while rank 0 keeps issuing bucket all-reduces that can never complete.
    Rank 0's watchdog (device-progress heartbeat + ncclCommGetAsyncError) must ncclCommAbort and exit
    non-zero within its timeout instead of hanging; the launcher-level fail-fast is tested on gloo
    (test_distributed_cpu.py::test_fault_injection_fails_fast)."""
    import time

    t0 = time.time()
    codes, outs = _run_world2([os.path.join(ROOT, "train.py"), "--backend", "rccl", "--model", "resnet_tiny",
                               "--image-size", "32", "--batch-size", "8", "--num-samples", "2048", "--epochs", "2",
                               "--checkpoint-dir", str(tmp_path), "--watchdog-timeout", "15"],
                              extra_env={"DPE_FAULT_INJECT": "1:0:3:kill"}, timeout=110)
    dt = time.time() - t0
    assert codes[1] == -9, outs[1][-2000:]                     # the injected death
    assert codes[0] == 1, (codes, outs[0][-3000:])             # the survivor aborted, non-zero
    assert "watchdog:" in outs[0] and "aborting communicator" in outs[0], outs[0][-3000:]
    assert dt < 100, dt
    print(f"survivor exited rc={codes[0]} after {dt:.1f}s: "
          f"{[ln for ln in outs[0].splitlines() if 'watchdog:' in ln][0][-160:]}")


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world4_rccl():
    """world 4 -- RCCL's multi-peer ring, rank 0's bucket order broadcast to three
    peers, one rebuild, no_sync, registration and the bf16 hook, against rank-averaged grads."""
    codes, outs = _run_world(4, [os.path.join(ROOT, "tests", "_rccl_world2_worker.py")], timeout=170)
    assert codes == [0] * 4, "\n".join(o[-2000:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-4" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world4_rccl_gpt2():
    codes, outs = _run_world(4, [os.path.join(ROOT, "tests", "_rccl_world2_worker.py"), "gpt2"], timeout=170)
    assert codes == [0] * 4, "\n".join(o[-2000:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-4" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rank_death_world4_aborts_every_survivor(tmp_path):
    """Rank 2 SIGKILLs itself at batch 3 of epoch 0; ranks 0, 1 and 3 are blocked in bucket
    all-reduces of a 4-rank ring that can never complete.  Each survivor's watchdog must abort its
    communicator and exit non-zero within the timeout (several peers blocked at once)."""
    import time

    t0 = time.time()
    codes, outs = _run_world(4, [os.path.join(ROOT, "train.py"), "--backend", "rccl", "--model", "resnet_tiny",
                                 "--image-size", "32", "--batch-size", "8", "--num-samples", "2048", "--epochs", "2",
                                 "--checkpoint-dir", str(tmp_path), "--watchdog-timeout", "15"],
                             extra_env={"DPE_FAULT_INJECT": "2:0:3:kill"}, timeout=130)
    dt = time.time() - t0
    assert codes[2] == -9, outs[2][-2000:]
    for r in (0, 1, 3):
        assert codes[r] not in (0, None) and codes[r] != -9, (r, codes, outs[r][-2000:])
        assert "watchdog:" in outs[r] and "aborting communicator" in outs[r], (r, outs[r][-2000:])
    assert dt < 140, dt
    print(f"survivors rc={[codes[r] for r in (0, 1, 3)]} after {dt:.1f}s")


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world8_rccl():
    """the deployment's world size (NPROC_PER_NODE=8) -- an 8-rank RCCL
    ring (socket transport, 8 processes on GPU 0), rank 0's bucket order broadcast to seven peers, one
    rebuild, no_sync, registration and the bf16 hook, against rank-averaged grads (< 1e-4)."""
    codes, outs = _run_world(8, [os.path.join(ROOT, "tests", "_rccl_world2_worker.py")], timeout=280)
    assert codes == [0] * 8, "\n".join(o[-1500:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-8" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world8_rccl_gpt2():
    codes, outs = _run_world(8, [os.path.join(ROOT, "tests", "_rccl_world2_worker.py"), "gpt2"], timeout=280)
    assert codes == [0] * 8, "\n".join(o[-1500:] for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-8" in ln][0])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rank_death_world8_aborts_every_survivor(tmp_path):
    """Rank 5 SIGKILLs itself at batch 3 of epoch 0; the seven survivors are blocked in bucket
    all-reduces of an 8-rank ring that can never complete.  Every survivor's watchdog must abort its
    communicator and exit non-zero within the timeout."""
    import time

    t0 = time.time()
    codes, outs = _run_world(8, [os.path.join(ROOT, "train.py"), "--backend", "rccl", "--model", "resnet_tiny",
                                 "--image-size", "32", "--batch-size", "8", "--num-samples", "2048", "--epochs", "2",
                                 "--checkpoint-dir", str(tmp_path), "--watchdog-timeout", "15"],
                             extra_env={"DPE_FAULT_INJECT": "5:0:3:kill"}, timeout=200)
    dt = time.time() - t0
    assert codes[5] == -9, outs[5][-2000:]
    survivors = [r for r in range(8) if r != 5]
    for r in survivors:
        assert codes[r] not in (0, None) and codes[r] != -9, (r, codes, outs[r][-2000:])
        assert "watchdog:" in outs[r] and "aborting communicator" in outs[r], (r, outs[r][-2000:])
    assert dt < 200, dt
    print(f"7 survivors rc={[codes[r] for r in survivors]} after {dt:.1f}s")
