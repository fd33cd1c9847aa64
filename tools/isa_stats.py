"""Instruction mix of the main kernels in a device assembly file (hipcc --cuda-device-only -S):
    python tools/isa_stats.py x.s [name-filter ...]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
filt = sys.argv[2:] or ["k_shade", "k_trace2"]
for m in re.finditer(r"^(_Z\w+):.*?$(.*?)^\s*s_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if not any(f in name for f in filt):
        continue
    ops = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = Counter(ops)
    print(name[:48], "instrs", len(ops), "readlane", c["v_readlane_b32"], "writelane", c["v_writelane_b32"],
          "scratch", sum(v for k, v in c.items() if "scratch" in k), "div_scale", c["v_div_scale_f64"],
          "sqrt", c["v_sqrt_f64"], "fma64", c["v_fma_f64"], "s_load", sum(v for k, v in c.items() if k.startswith("s_load")),
          "global_ld", sum(v for k, v in c.items() if k.startswith("global_load")))
