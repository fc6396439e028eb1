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
    # a multi-rank run documents its communication by default (one untimed
    # instrumented step after the timed loop) and records where the CU-budget decision came from
    b = d["buckets"]
    assert b["count"] >= 1 and len(b["per_bucket"]) == b["count"] and b["comm_ms"] > 0
    assert all(r["allreduce_ms"] >= 0 and r["bytes"] > 0 for r in b["per_bucket"])
    assert "overlap_pct" in b
    assert "source" in d["config"]["cu_budget"]


def test_bench_bare_multi_gpu_refused():
    """`python bench.py --gpus 2` without a launcher must fail, not report a one-GPU number."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "simplenet",
                        "--steps", "1", "--warmup", "0"], cwd="/tmp", env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode != 0
    assert not _json_lines(p.stdout), p.stdout
    assert "torch.distributed.run" in p.stderr, p.stderr[-1000:]


def test_bench_defaults_single_process():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "simplenet", "--steps", "2",
                        "--warmup", "1"], cwd="/tmp", stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    (d,) = _json_lines(p.stdout)
    assert d["n_gpus"] == 1 and d["config"]["parallelism"] == "dp1"
