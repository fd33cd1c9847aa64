"""Per-unit busy / stall counters of k_trace2 and k_shade (texture addresser TA, texture data
TD, vector L1 TCP) on one C3 frame, one rocprofv3 --pmc pass per group (on the GPU box):

    python tools/pmc_units.py [--config C3] [--spp 64] > gpurun_out/pmc_units.jsonl

Each counter is summed over the kernel's dispatches; GRBM_GUI_ACTIVE (the GPU's busy
cycles, summed over the XCDs) is the denominator the busy fractions are quoted against.
Counter groups that the profiler rejects are reported and skipped.
"""
import argparse
import csv
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
GROUPS = [["GRBM_GUI_ACTIVE", "GRBM_COUNT"],
          ["TA_TA_BUSY_sum", "TA_BUFFER_READ_WAVEFRONTS_sum"],
          ["TA_FLAT_READ_WAVEFRONTS_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"],
          ["TD_TD_BUSY_sum", "TD_TC_STALL_sum"],
          ["TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
           "TCP_TCR_TCP_STALL_CYCLES_sum"],
          ["TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_GATE_EN1_sum", "TCP_GATE_EN2_sum"],
          ["SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_BUSY_CYCLES"]]
KERNELS = {"k_trace2": "k_trace2<", "k_shade": "k_shade<"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C3")
    p.add_argument("--spp", type=int, default=64)
    a = p.parse_args()
    env = dict(os.environ, TMPDIR="/tmp")
    child = [sys.executable, str(ROOT / "tools" / "first_frame.py"), "--config", a.config, "--frames", "1", "--spp", str(a.spp)]
    sums = {}
    for grp in GROUPS:
        d = tempfile.mkdtemp(prefix="izpi_pmcu_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", *grp, "--output-format", "csv", "-d", d, "-o", "run", "--", *child]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=str(ROOT), env=env)
        except subprocess.TimeoutExpired:
            print(json.dumps({"group": grp, "error": "timeout"}), flush=True)
            continue
        if r.returncode != 0:
            print(json.dumps({"group": grp, "error": r.stderr[-600:]}), flush=True)
            continue
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                for short, pat in KERNELS.items():
                    if pat in row["Kernel_Name"]:
                        e = sums.setdefault(short, {})
                        e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for short, e in sums.items():
        out = {"kernel": short, "config": a.config, "spp": a.spp, **e}
        g = e.get("GRBM_GUI_ACTIVE")
        if g:
            for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TD_TC_STALL_sum",
                      "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
                      "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum"):
                if k in e:  # per-CU units summed over 256 CUs; GRBM over 8 XCDs
                    out[k.replace("_sum", "") + "_frac"] = round(e[k] / (g / 8.0 * 256.0), 4)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
