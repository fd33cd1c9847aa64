"""Per-kernel ratios from profiles/pmc_groups.sh output: python tools/pmc_report.py gpurun_out/pmc_TAG"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/g*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for k, a in agg.items():
    if "k_" not in k or not a.get("SQ_WAVE_CYCLES"):
        continue
    wc = a["SQ_WAVE_CYCLES"]
    print("%-28s wait_mem %.2f issue %.2f wait_dep %.2f lane_util %.2f L2hit %.2f valu %.3g salu %.3g vmem %.3g "
          "fetchGB %.2f writeGB %.2f" % (
              k, a["SQ_WAIT_ANY"] / wc, a["SQ_ACTIVE_INST_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc,
              a["SQ_THREAD_CYCLES_VALU"] / max(64 * a["SQ_ACTIVE_INST_VALU"], 1),
              a["TCC_HIT_sum"] / max(a["TCC_HIT_sum"] + a["TCC_MISS_sum"], 1), a["SQ_INSTS_VALU"], a["SQ_INSTS_SALU"],
              a["SQ_INSTS_VMEM_RD"], 2 * a["FETCH_SIZE"] / 1e6, a["WRITE_SIZE"] / 1e6))
