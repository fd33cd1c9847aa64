"""Summarise rocprofv3 output of profiles/run_profile.sh into committed JSON/CSV.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag> [config]

Reads  <dir>/trace/**/run_kernel_stats.csv   (kernel-trace --stats pass)
       <dir>/pmc_fetch/**/run_counter_collection.csv  (FETCH_SIZE pass)
       <dir>/pmc_write/**/run_counter_collection.csv  (WRITE_SIZE pass)
Writes <out>/kernel_stats.csv (copy), <out>/pmc_traffic.json (per-kernel bytes per
launch) and merges {config: {"hbm_bytes_per_trace_launch": ...}} into
profiles/pmc_summary.json, which bench.py reports as roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE reports half of the bytes of wide (16 B/lane) reads, so it is
doubled; WRITE_SIZE is taken as is. Both count L2 memory-side requests, so
Infinity-Cache hits are included: "traffic" is bytes that left L2, an upper bound of
HBM bytes.
"""
import collections
import csv
import re
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in Path(d).rglob("run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return out, {k: len(v) for k, v in n.items()}


def main():
    src, dst = Path(sys.argv[1]).resolve(), Path(sys.argv[2]).resolve()
    config = sys.argv[3] if len(sys.argv) > 3 else "C3"
    dst.mkdir(parents=True, exist_ok=True)
    stats = list(src.rglob("run_kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], dst / "kernel_stats.csv")
    fetch, nf = _counters(src / "pmc_fetch")
    write, nw = _counters(src / "pmc_write")
    per = {}
    for k in sorted(set(fetch) | set(write)):
        launches = max(nf.get(k, 0), nw.get(k, 0), 1)
        fb = 2.0 * 1024.0 * fetch.get(k, {}).get("FETCH_SIZE", 0.0)
        wb = 1024.0 * write.get(k, {}).get("WRITE_SIZE", 0.0)
        per[k] = {"launches": launches, "fetch_bytes_per_launch": fb / launches,
                  "write_bytes_per_launch": wb / launches, "bytes_per_launch": (fb + wb) / launches}
    (dst / "pmc_traffic.json").write_text(json.dumps(per, indent=1))
    trace = [v for k, v in per.items() if re.search(r"\bk_trace2?<", k)]
    if trace:
        t = trace[0]
        summ_f = ROOT / "profiles" / "pmc_summary.json"
        summ = json.loads(summ_f.read_text()) if summ_f.exists() else {}
        summ[config] = {"hbm_bytes_per_trace_launch": t["bytes_per_launch"],
                        "fetch_bytes_per_trace_launch": t["fetch_bytes_per_launch"],
                        "write_bytes_per_trace_launch": t["write_bytes_per_launch"],
                        "trace_launches": t["launches"], "source": str(dst.relative_to(ROOT)),
                        "note": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KB->B; L2 memory-side bytes "
                                "(Infinity-Cache hits included)"}
        summ_f.write_text(json.dumps(summ, indent=1))
    for k, v in per.items():
        print("%-40s %6d launches %10.1f MB/launch" % (k[:40], v["launches"], v["bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main()
