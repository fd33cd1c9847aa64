"""k_trace2 / k_shade memory-side traffic of library variants (PMC passes on the GPU box).

    python tools/pmc_variants.py --config C3 --spp 64 [--tune k=v ...] base NAME[@k=v,...] ...

Each variant (`base`, or a build of tools/variants.py; `@k=v,...` adds izpi_render_tuning
fields for that run only) renders one frame of a fresh renderer under two rocprofv3 --pmc
passes of its own (FETCH_SIZE; WRITE_SIZE + TCC_HIT/MISS), and one JSON line gives the
bytes per traced ray of k_trace2 and k_shade: fetched (FETCH_SIZE x 2, the gfx950
correction of MI355X_MICROARCH.md, HBM section), written, and the L2 hit rate. Those
counters are L2 memory-side requests: Infinity-Cache hits included.
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
PASSES = [["FETCH_SIZE"], ["WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"]]
KERNELS = {"k_trace2": "k_trace2<", "k_shade": "k_shade<"}


def one(a, variant, tunes):
    base = [sys.executable, str(ROOT / "tools" / "variants.py"), "child", "--config", a.config, "--frames", "1",
            "--variant", variant]
    if a.spp:
        base += ["--spp", str(a.spp)]
    for kv in tunes:
        base += ["--tune", kv]
    sums, info = {}, None
    env = dict(os.environ, TMPDIR="/tmp")
    for counters in PASSES:
        d = tempfile.mkdtemp(prefix="izpi_pmcv_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--", *base]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=str(ROOT), env=env)
        if r.returncode != 0:
            sys.exit("variant %s pass %s: rc %d\n%s" % (variant, counters, r.returncode, r.stderr[-2000:]))
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                info = json.loads(line)
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                for short, pat in KERNELS.items():
                    if pat in row["Kernel_Name"]:
                        e = sums.setdefault(short, {})
                        e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    rays = max(info["rays"], 1) if info else 1
    out = {"variant": variant, "tune": tunes, "config": a.config, "spp": a.spp, "rays": rays,
           "trace_ms": info and info["trace_ms"], "shade_ms": info and info["shade_ms"], "digest": info and info["digest"],
           "nodes_per_ray": info and info["nodes_per_ray"], "tri_per_ray": info and info["tri_per_ray"]}
    for short, e in sums.items():
        hit, miss = e.get("TCC_HIT_sum", 0.0), e.get("TCC_MISS_sum", 0.0)
        out[short] = {"fetch_B_per_ray": round(2048.0 * e.get("FETCH_SIZE", 0.0) / rays, 2),
                      "write_B_per_ray": round(1024.0 * e.get("WRITE_SIZE", 0.0) / rays, 2),
                      "l2_req_per_ray": round((hit + miss) / rays, 3),
                      "l2_hit": round(hit / (hit + miss), 4) if hit + miss > 0 else None}
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C3")
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--timeout", type=int, default=240)
    p.add_argument("--tune", action="append", default=[])
    p.add_argument("variants", nargs="+")
    a = p.parse_args()
    for v in a.variants:
        name, _, extra = v.partition("@")
        one(a, name, a.tune + [kv for kv in extra.split(",") if kv])


if __name__ == "__main__":
    main()
