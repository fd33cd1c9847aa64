#!/usr/bin/env python3
"""Per-kernel register / spill / LDS table of izpi_gpu.hip for gfx950 (compile-time remarks).

    python tools/kres.py [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys

SRC = os.environ.get("KRES_SRC", "izpi_amd/csrc/izpi_gpu.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
       "-Iinclude", "--cuda-device-only", "-c", "-o", "/tmp/kres.o", SRC, "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: .*?(Function Name|VGPRs Spill|SGPRs Spill|VGPRs|AGPRs|SGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
demangle = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, demangle):
    name = re.sub(r"\(.*", "", d)
    if not re.search(r"k_(shade|tail|trace2|start)", name):
        continue
    print(f"{name:40s} vgpr {r.get('VGPRs','?'):>4} spill {r.get('VGPRs Spill','?'):>4} sgpr_spill {r.get('SGPRs Spill','?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]')} lds {r.get('LDS Size [bytes/block]')}")
