"""entrypoint.sh contract via PATH shims: fake `hostname` and a
fake launcher (`python3`/`torchrun`) that just echo their arguments."""
import os
import stat
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shim(dirpath, name, body):
    p = os.path.join(dirpath, name)
    with open(p, "w") as f:
        f.write("#!/bin/bash\n" + body + "\n")
    os.chmod(p, os.stat(p).st_mode | stat.S_IEXEC)


@pytest.fixture
def shims(tmp_path):
    _shim(str(tmp_path), "hostname", 'echo "$FAKE_HOST"')
    _shim(str(tmp_path), "python3", 'echo "LAUNCH $@"')
    _shim(str(tmp_path), "torchrun", 'echo "TORCHRUN $@"')
    return str(tmp_path)


def _run(shims, env):
    e = {"PATH": shims + ":/usr/bin:/bin"}
    e.update(env)
    return subprocess.run(["bash", os.path.join(ROOT, "entrypoint.sh")], env=e, capture_output=True, text=True)


def test_node_rank_and_master_from_hostname(shims):
    r = _run(shims, {"FAKE_HOST": "my-ddp-job-3", "NF_DISCOVERY_SERVICE": "ddp-headless", "REPLICAS": "4",
                     "NPROC_PER_NODE": "8", "SCRIPT_ARGS": "--epochs 2"})
    assert r.returncode == 0, r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("LAUNCH")][0]
    assert "--nnodes=4" in line and "--nproc-per-node=8" in line and "--node-rank=3" in line
    assert "--master-addr=my-ddp-job-0.ddp-headless" in line and "--master-port=29500" in line
    assert line.endswith("train.py --epochs 2")


def test_torchrun_mode(shims):
    r = _run(shims, {"FAKE_HOST": "job-1", "NF_DISCOVERY_SERVICE": "svc", "REPLICAS": "2", "LAUNCHER": "torchrun"})
    assert "TORCHRUN --nnodes=2 --nproc-per-node=1 --node-rank=1 --master-addr=job-0.svc" in r.stdout


@pytest.mark.parametrize("missing", ["NF_DISCOVERY_SERVICE", "REPLICAS"])
def test_required_env(shims, missing):
    env = {"FAKE_HOST": "job-0", "NF_DISCOVERY_SERVICE": "svc", "REPLICAS": "1"}
    del env[missing]
    r = _run(shims, env)
    assert r.returncode == 1 and f"ERROR: {missing} not set" in r.stdout


def test_single_node_local_master(shims):
    r = _run(shims, {"FAKE_HOST": "workstation", "NF_DISCOVERY_SERVICE": "svc", "REPLICAS": "1"})
    assert r.returncode == 0 and "--node-rank=0" in r.stdout and "--master-addr=127.0.0.1" in r.stdout


def test_bad_hostname_multi_node_is_an_error(shims):
    r = _run(shims, {"FAKE_HOST": "workstation", "NF_DISCOVERY_SERVICE": "svc", "REPLICAS": "2"})
    assert r.returncode == 1 and "cannot derive the node rank" in r.stdout
