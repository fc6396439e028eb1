"""bench.py driver contract (task spec): launched exactly as the driver does
(`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
127.0.0.1 ... bench.py --gpus N --steps K --warmup W`), rank 0 prints ONE JSON
line with the whole-job aggregate.  Runs the CPU/gloo arm (SimpleNet)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_json_line_torchrun_world2():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--model", "simplenet"]
    p = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = lines[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 128
    # whole-job aggregate: samples/s = per-GPU batch * world * steps / time
    assert abs(d["value"] - 64 * 2 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.01


def test_bench_defaults_single_process():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "simplenet", "--steps", "2",
                        "--warmup", "1"], cwd="/tmp", stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    (d,) = _json_lines(p.stdout)
    assert d["n_gpus"] == 1 and d["config"]["parallelism"] == "dp1"
