"""Per-kernel counter ratios from tools/pmc_kernels.sh output:
    python tools/pmc_report.py gpurun_out/pmc_TAG
SQ_* counters are summed over the frame's dispatches of each kernel; *_CYCLES ratios are
fractions of wave cycles; per-wave instruction counts are per wave launched."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, a in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = a.get("SQ_WAVE_CYCLES", 0)
    if not wc:
        continue
    g = lambda n: a.get(n, 0.0)  # noqa: E731
    waves = max(g("SQ_WAVES"), 1)
    print("%-44s waves %.3g  busy: wait_any %.2f active_any %.2f active_valu %.2f active_flat %.2f wait_inst %.2f" % (
        k[:44], waves, g("SQ_WAIT_ANY") / wc, g("SQ_ACTIVE_INST_ANY") / wc, g("SQ_ACTIVE_INST_VALU") / wc,
        g("SQ_ACTIVE_INST_FLAT") / wc, g("SQ_WAIT_INST_ANY") / wc))
    print("%-44s per wave: valu %.0f salu %.0f vmem_rd %.0f vmem_wr %.0f lds %.0f smem %.0f branch %.0f; "
          "vmem level/inst %.1f; L2 hit %.3f" % (
              "", g("SQ_INSTS_VALU") / waves, g("SQ_INSTS_SALU") / waves, g("SQ_INSTS_VMEM_RD") / waves,
              g("SQ_INSTS_VMEM_WR") / waves, g("SQ_INSTS_LDS") / waves, g("SQ_INSTS_SMEM") / waves,
              g("SQ_INSTS_BRANCH") / waves, g("SQ_INST_LEVEL_VMEM") / max(g("SQ_INSTS_VMEM_RD") + g("SQ_INSTS_VMEM_WR"), 1),
              g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1)))
