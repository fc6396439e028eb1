"""The native C++ Reducer at world 2 over real RCCL collectives, on a 1-GPU box.

Two processes share GPU 0.  Each gets its own NCCL_HOSTID, so RCCL sees two
hosts (no duplicate-GPU refusal) and connects them with its socket transport
over loopback: Reducer::launch runs with world() == 2, the buckets are really
all-reduced (ncclAvg), the bucket rebuild, no_sync accumulation and the bf16
compression path are checked against rank-averaged plain-backward gradients
(tests/_rccl_world2_worker.py).  On an 8-GPU node the same code runs over xGMI.
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


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_reducer_world2_rccl():
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": "2", "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": "2",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "PYTHONPATH": ROOT,
                    "NCCL_HOSTID": f"dpe-test-host-{r}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0", "OMP_NUM_THREADS": "1",
                    "DPE_RCCL_MAX_CHANNELS": "4"})  # the CU cap for overlapped collectives, exercised
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_rccl_world2_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=100)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    codes = [p.returncode for p in procs]
    assert codes == [0, 0], "\n".join(o[-3000:] for o in outs)
    assert all("ok: world-2 RCCL reducer" in o for o in outs)
    for o in outs:
        print([ln for ln in o.splitlines() if "ok: world-2" in ln][0])
