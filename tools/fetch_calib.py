"""Run tools/fetch_calib.hip's kernels under rocprofv3 PMC passes (on the GPU box) and print,
per kernel, FETCH_SIZE against the bytes it is known to read.

    python tools/fetch_calib.py > gpurun_out/fetch_calib.jsonl

FETCH_SIZE is reported in KiB; `fetch_over_lines` = FETCH_SIZE bytes / (128-B lines the
kernel touches x 128). The guide's gfx950 rule (MI355X_MICROARCH.md, HBM) is 0.5 for a
16-B-per-lane stream; this checks the same factor for the gathers k_trace2 issues.
"""
import csv
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "izpi_amd" / "_lib" / "fetch_calib"
PASSES = [["FETCH_SIZE"], ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"], ["TCC_HIT_sum", "TCC_MISS_sum"],
          # which SQ counter counts global_load issue on gfx950 (SQ_ACTIVE_INST_VMEM read 0.0 in r4's bench)
          ["SQ_INSTS_VMEM", "SQ_INSTS_FLAT", "SQ_INSTS_VMEM_RD", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_FLAT", "SQ_WAVE_CYCLES"]]


def main():
    env = dict(os.environ, TMPDIR="/tmp")
    runs, info = [], None
    for counters in PASSES:
        d = tempfile.mkdtemp(prefix="izpi_fc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--", str(EXE)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
        if r.returncode != 0:
            print(json.dumps({"pass": counters, "rc": r.returncode, "stderr": r.stderr[-800:]}), flush=True)
            continue
        info = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        per = {}
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                did = int(row["Dispatch_Id"])
                per.setdefault(did, {"kernel": row["Kernel_Name"]})
                per[did][row["Counter_Name"]] = per[did].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        runs.append(per)
    if not info:
        sys.exit("no run")
    for k in info:
        did = k["launch"] + 2  # dispatch ids start at 1, after fetch_calib's first table fill
        row = dict(k)
        for per in runs:
            e = per.get(did, {})
            for c, v in e.items():
                if c != "kernel":
                    row[c] = v
            row.setdefault("kernel_name", e.get("kernel"))
        if "FETCH_SIZE" in row:
            row["fetch_bytes"] = row["FETCH_SIZE"] * 1024
            row["fetch_over_lines"] = round(row["fetch_bytes"] / row["line_bytes"], 4)
        for c in ("SQ_INSTS_VMEM", "SQ_INSTS_FLAT", "SQ_INSTS_VMEM_RD"):
            if c in row and row.get("load_insts"):
                row[c + "_over_loads"] = round(row[c] / row["load_insts"], 4)
        if "TCC_EA0_RDREQ_sum" in row:
            rq, r32 = row["TCC_EA0_RDREQ_sum"], row.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            row["rdreq_per_line"] = round(rq / (row["line_bytes"] / 128), 4)
            row["rdreq_32B_frac"] = round(r32 / rq, 4) if rq else None
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
