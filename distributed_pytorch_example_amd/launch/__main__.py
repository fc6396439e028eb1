"""Local multi-process launcher with torchrun's CLI and worker env contract.

    python -m distributed_pytorch_example_amd.launch --nnodes=1 --nproc-per-node=8 \\
        --node-rank=0 --master-addr=127.0.0.1 --master-port=29500 train.py --epochs 2

Semantics reproduced from torchrun as the reference uses it:
static rendezvous (no agent store needed: the workers' ``env://`` init makes
global rank 0 host the TCPStore), worker env ``RANK / LOCAL_RANK /
WORLD_SIZE / LOCAL_WORLD_SIZE / GROUP_RANK / MASTER_ADDR / MASTER_PORT``,
``OMP_NUM_THREADS=1`` when more than one worker per node (and, unlike
torchrun, also for 1-proc-per-node multi-node jobs -- the survey measured a
29x slowdown without it), fail-fast: when any worker exits non-zero the
others get SIGTERM (then SIGKILL) and the launcher exits 1 with a root-cause
table; ``--max-restarts`` re-launches the whole worker group.
Each worker gets ``TORCHELASTIC_ERROR_FILE`` so a Python exception is recorded.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="dpe-launch")
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--node-rank", "--node_rank", type=int, default=0)
    ap.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    ap.add_argument("--master-port", "--master_port", type=int, default=29500)
    ap.add_argument("--standalone", action="store_true")
    ap.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    ap.add_argument("--monitor-interval", type=float, default=0.1)
    ap.add_argument("--term-timeout", type=float, default=10.0)
    ap.add_argument("-m", "--module", action="store_true", help="run the script as a module (python -m)")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker_env(args, local_rank: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    world = args.nnodes * args.nproc_per_node
    env.update({
        "RANK": str(args.node_rank * args.nproc_per_node + local_rank),
        "LOCAL_RANK": str(local_rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(args.nproc_per_node),
        "GROUP_RANK": str(args.node_rank),
        "MASTER_ADDR": args.master_addr,
        "MASTER_PORT": str(args.master_port),
        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    })
    if (args.nproc_per_node > 1 or args.nnodes > 1) and "OMP_NUM_THREADS" not in os.environ:
        env["OMP_NUM_THREADS"] = "1"
    return env


def _spawn(args, errdir):
    procs = []
    for lr in range(args.nproc_per_node):
        env = worker_env(args, lr)
        env["TORCHELASTIC_ERROR_FILE"] = os.path.join(errdir, f"error_{lr}.json")
        cmd = [sys.executable, "-u"] + (["-m", args.script] if args.module else [args.script]) + list(args.script_args)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    return procs


def _terminate(procs, timeout):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + timeout
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run(args) -> int:
    if args.standalone:
        args.nnodes, args.node_rank, args.master_addr = 1, 0, "127.0.0.1"
        args.master_port = _free_port()
    attempt = 0
    while True:
        errdir = tempfile.mkdtemp(prefix="dpe_launch_")
        procs = _spawn(args, errdir)
        failed = None
        interrupted = False
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    failed = bad
                    break
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(args.monitor_interval)
        except KeyboardInterrupt:
            interrupted = True
        _terminate(procs, args.term_timeout)
        if interrupted:
            return 130
        _report(args, failed, errdir)
        if attempt >= args.max_restarts:
            return 1
        attempt += 1
        print(f"[dpe-launch] restarting worker group ({attempt}/{args.max_restarts})", file=sys.stderr, flush=True)


def _report(args, failed, errdir):
    lines = ["[dpe-launch] worker group failed (fail-fast: remaining workers terminated)", "Root Cause:"]
    for lr, code in failed:
        grank = args.node_rank * args.nproc_per_node + lr
        sig = f" (signal {-code}: {signal.Signals(-code).name})" if code < 0 else ""
        msg = ""
        ef = os.path.join(errdir, f"error_{lr}.json")
        if os.path.exists(ef):
            try:
                msg = json.load(open(ef)).get("message", {}).get("message", "")
            except Exception:
                msg = open(ef).read()[:500]
        lines.append(f"  rank {grank} (local_rank {lr}): exitcode {code}{sig}{' error: ' + msg if msg else ''}")
    print("\n".join(lines), file=sys.stderr, flush=True)


def main(argv=None):
    sys.exit(run(parse(argv)))


if __name__ == "__main__":
    main()
