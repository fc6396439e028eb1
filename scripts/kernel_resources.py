#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS / occupancy table of a .hip file (hipcc -Rpass-analysis remarks)."""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-munsafe-fp-atomics",
       "-mllvm", "-amdgpu-mfma-vgpr-form", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/_kr.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
dm = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dm):
    if pat and pat not in d:
        continue
    print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','?'):>3} agpr spill {r.get('VGPRs Spill','?'):>4} "
          f"lds {r.get('LDS Size [bytes/block]','?'):>6} occ {r.get('Occupancy [waves/SIMD]','?')}  {d[:150]}")
