"""In-tree build of the native extension ``distributed_pytorch_example_amd/_C.so``.

* ``csrc/kernels/*.hip``  -> ``hipcc --offload-arch=gfx950 -O3`` (device code; no torch headers)
* ``csrc/bindings/*.cpp``, ``csrc/comm/*.cpp`` -> ``g++`` against torch's C++ API
* link against torch's own ``libamdhip64`` / ``librccl`` (one HIP runtime and one
  RCCL per process; SURVEY §7.4 "runtime/ABI skew").

Incremental (mtime vs. every header under csrc/) and parallel.  Run as
``python -m distributed_pytorch_example_amd._build`` or via ``__graft_entry__.build()``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_pytorch_example_amd")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


# per-file device flags.  attn.hip: max / sum / product chains over MFMA and v_exp results stay
# single-issue VALU (no NaN-quieting canonicalisation v_max before each fmaxf, no SLP packing into
# v_pk_*_f32, which costs extra issue cycles beside MFMAs) -- without inline asm, whose
# operands would miss the compiler's hazard wait states.  NaN inputs are not honoured there.
# hgemm.hip: the schedule's claim atomics are issued by one lane and consumed phases later; the
# atomic optimizer rewrites a uniform-address add into a wave-wide add plus a per-lane offset
# (readfirstlane of the result), which puts a vmcnt(0) wait right behind the atomic.
FILE_FLAGS = {"attn.hip": ["-fno-slp-vectorize", "-fno-honor-nans"],
              "hgemm.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def _torch_dirs():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib")


def _headers():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _needs(obj, src, hdr_mtime):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return t < os.path.getmtime(src) or t < hdr_mtime


def _run(cmd):
    t0 = time.time()
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build failed ({p.returncode}): {' '.join(cmd)}\n{p.stdout}")
    return time.time() - t0, p.stdout


def build_variant(defines, out_name: str, verbose: bool = True) -> str:
    """Build the extension with extra ``-D`` defines into ``<pkg>/<out_name>`` (own object dir):
    a compile-time variant for A/B runs, loaded with ``DPE_EXT_SO=<path>``."""
    global BUILD, OUT
    saved = BUILD, OUT
    tag = out_name.replace(".so", "")
    BUILD, OUT = os.path.join(ROOT, "build", tag), os.path.join(PKG, out_name)
    try:
        return build(verbose=verbose, extra_defines=[f"-D{d}" for d in defines])
    finally:
        BUILD, OUT = saved


def build(verbose: bool = True, jobs: int | None = None, force: bool = False, extra_defines=()) -> str:
    tdir, tinc, tlib = _torch_dirs()
    os.makedirs(BUILD, exist_ok=True)
    hdr = _headers()
    py_inc = sysconfig.get_paths()["include"]
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp")) + glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    common_defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C", "-D_GLIBCXX_USE_CXX11_ABI=1",
                   *extra_defines]
    jobs = jobs or int(os.environ.get("MAX_JOBS", min(16, os.cpu_count() or 4)))

    tasks = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _needs(obj, src, hdr):
            tasks.append([os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                          "-ffp-contract=fast", "-munsafe-fp-atomics",
                          # MFMA C/D in arch VGPRs (gfx950 unified file): avoids per-K-step
                          # v_accvgpr_read/write shuffles of the accumulators in the main loops
                          "-mllvm", "-amdgpu-mfma-vgpr-form", *FILE_FLAGS.get(os.path.basename(src), []),
                          *extra_defines, "-c", src, "-o", obj])
    for src in cpp_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _needs(obj, src, hdr):
            tasks.append(["g++", "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", *common_defs,
                          *[f"-I{d}" for d in tinc], f"-I{ROCM}/include", f"-I{py_inc}", "-c", src, "-o", obj])
    t0 = time.time()
    if tasks:
        if verbose:
            print(f"[dpe build] compiling {len(tasks)} translation unit(s) with {jobs} jobs", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for dt, _ in ex.map(_run, tasks):
                pass
    newest = max(os.path.getmtime(o) for o in objs)
    if force or tasks or not os.path.exists(OUT) or os.path.getmtime(OUT) < newest:
        link = [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs,
                f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                os.path.join(tlib, "libamdhip64.so"), os.path.join(tlib, "librccl.so"),
                f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]
        _run(link)
        os.replace(OUT + ".tmp", OUT)
    if verbose:
        print(f"[dpe build] {OUT} ready ({time.time() - t0:.1f}s)", flush=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
