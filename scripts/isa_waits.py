#!/usr/bin/env python3
"""Per-kernel count of full drains (s_waitcnt vmcnt(0)) and counted vmcnt waits in a .hip file's gfx950 ISA.

    python scripts/isa_waits.py csrc/kernels/pwconv.hip [name-filter]

Full drains are also listed by loop depth (the innermost depth is the hot loop).  A vmcnt(0) inside a streaming kernel's tile loop also waits for the ring's in-flight DMAs; it appears when a
load/store sits under a branch, a DMA issue is conditional, or a second __shared__ object hides the ring's
LDS-DMA destination from the compiler."""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-mllvm",
       "-amdgpu-mfma-vgpr-form", "--cuda-device-only", "-S", src, "-o", "-"]
asm = subprocess.run(cmd, capture_output=True, text=True).stdout
cur, rows, depth = None, {}, 0
for line in asm.splitlines():
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        rows[cur] = [0, 0, {}]
        depth = 0
        continue
    if line.startswith(".Lfunc_end"):
        cur = None
    if re.match(r"^(\.LBB\w+|; %bb\.\d+):", line):  # block label: its comment names the enclosing loop depth
        md = re.search(r"Depth=(\d+)", line)
        depth = int(md.group(1)) if md else 0
    if cur and "s_waitcnt" in line:
        for v in re.findall(r"vmcnt\((\d+)\)", line):
            rows[cur][0 if v == "0" else 1] += 1
            if v == "0" and depth:
                rows[cur][2][depth] = rows[cur][2].get(depth, 0) + 1
names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (k, (z, c, zl)), d in zip(rows.items(), names):
    if pat in d:
        dl = " ".join(f"d{k}:{v}" for k, v in sorted(zl.items())) or "-"
        print(f"vmcnt(0) {z:3d} (by loop depth {dl:12s})  counted {c:3d}  {d[:100]}")
